"""The gather's guessed due list (GSpec) pinned directly.

k_proc copies the chunk ids of the bucket it expects the next window to cover
whole; k_scatter's gather uses them only after checking the guess against the
window it planned (same step, one whole bucket, nothing straddling or spent),
and derives the due list from the bucket words otherwise.  Here configs[3]
(1M hosts, the bench's rounds) runs with the guess on, off (SG_GSPEC=0) and
deliberately wrong (SG_GSPEC=2: the bucket after the right one, which the
check must reject) against the oracle's per-round fixture, and the launch
counters show which path each run took."""
import json
import os

import pytest

from shadow_amd import phold
from shadow_amd.engine import Engine
from shadow_amd.trace import state_fingerprint

pytestmark = pytest.mark.gpu
FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "oracle_fixtures.json")))
ROWS = {r[0]: r for r in FIX["c4_1m"]["rounds"]}


@pytest.mark.parametrize("mode", ["1", "0", "2"])
def test_c4_gspec_modes_match_the_oracle(mode, monkeypatch):
    monkeypatch.setenv("SG_GSPEC", mode)  # read when the engine is created
    eng = Engine(phold.c4_config(n_hosts=1_000_000))
    eng.boot()
    done = 0
    for r in (25, 120):
        eng.run(r - done)
        done = r
        st = eng.stats()
        assert st["rounds"] == r and st["overflow"] == 0
        assert (st["pops"], st["window_start"], st["window_end"]) == (ROWS[r][1], ROWS[r][3], ROWS[r][4]), r
        hs = eng.host_state()
        assert state_fingerprint(eng.first_host, hs["digest"], hs["pops"], hs["rng"], hs["ev"]) == ROWS[r][2], r
    g = eng.gather_paths()
    assert g["guessed"] + g["listed"] >= 119  # every round but the boot's gathers
    if mode == "1":
        assert g["guessed"] >= 100, g  # steady rounds are one whole bucket each
    else:
        assert g["guessed"] == 0, g


def test_c4_64bit_bucket_arithmetic_matches_the_oracle(monkeypatch):
    """The calendar's bucket indices by 64-bit division (the path a calendar
    whose horizon passes 2^32 ns takes: k_scatter's planner, the insert and the
    bucket bins), forced on configs[3] with SG_NO_RING32=1, against the
    per-round fixture."""
    monkeypatch.setenv("SG_NO_RING32", "1")
    eng = Engine(phold.c4_config(n_hosts=1_000_000))
    eng.boot()
    eng.run(60)
    st = eng.stats()
    assert st["rounds"] == 60 and st["overflow"] == 0
    assert (st["pops"], st["window_start"], st["window_end"]) == (ROWS[60][1], ROWS[60][3], ROWS[60][4])
    hs = eng.host_state()
    assert state_fingerprint(eng.first_host, hs["digest"], hs["pops"], hs["rng"], hs["ev"]) == ROWS[60][2]


def test_ov_bug_guard_clamps_corrupt_staged_records():
    """The bounds guard of k_scatter's insert role (the round-4 fault,
    profiles/r04/ablation/README.md): two staged records are corrupted between
    a k_proc and its k_scatter (sg_engine_debug_inject: a host past the shard,
    a time beyond the calendar's horizon).  The launch must clamp both in
    bounds and flag OV_BUG (128) without faulting the GPU, the run must stop
    on it, and a new engine in the same process must run configs[3] to its
    fixture."""
    from shadow_amd._lib import SgError
    eng = Engine(phold.c4_config(n_hosts=40_000, V=64, end_time_s=0.2))
    eng.boot()
    eng.run(4)
    assert eng.stats()["overflow"] == 0
    eng.debug_inject()
    with pytest.raises(SgError):
        eng.run(4)  # stops at the next plan, which sees the flag
    st = eng.stats()
    assert st["overflow"] & 128, hex(st["overflow"])
    assert st["overflow"] & ~(128 | 32) == 0, hex(st["overflow"])  # nothing else ran out
    eng.close()
    eng = Engine(phold.c4_config(n_hosts=1_000_000))
    eng.boot()
    eng.run(25)
    st = eng.stats()
    assert st["rounds"] == 25 and st["overflow"] == 0
    hs = eng.host_state()
    assert state_fingerprint(eng.first_host, hs["digest"], hs["pops"], hs["rng"], hs["ev"]) == ROWS[25][2]
