"""CPU: the committed oracle fixtures (tests/golden/oracle_fixtures.json) are
what the oracle computes — re-derived here for the configs that finish in
seconds (C1, C3, the first rounds of C4 at 1M hosts) — and the product-side
fingerprint is additive over host shards, as the multi-GPU checks assume."""
import json
import os
import sys

import numpy as np

from oracle import oracle as O
from shadow_amd import phold
from shadow_amd.trace import state_fingerprint

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLDEN)
import make_fixtures as MF  # noqa: E402

FIX = json.load(open(os.path.join(GOLDEN, "oracle_fixtures.json")))


def test_fixture_c1_c3_reproduce():
    for name in ("c1", "c3"):
        assert MF.final_case(name) == FIX[name], name


def test_fixture_c4_first_rounds_reproduce():
    got = MF.per_round_case("c4_1m", 3)
    assert got["rounds"] == FIX["c4_1m"]["rounds"][:3]
    assert len(FIX["c4_1m"]["rounds"]) == MF.ROUNDS_C4


def test_fixture_c5_config_matches():
    cfg = phold.c5_config()
    assert FIX["c5"]["config"] == cfg["name"] and FIX["c5"]["n_hosts"] == 100_000
    st = FIX["c5"]["stats"]
    # every message reached (nearly) every host: pops = boots + origins + receipts
    assert st["boots"] == 100_000 and st["pops"] > 64 * 100_000 * 7
    assert st["drop_reliability"] > 0 and st["pending"] == 0


def test_fingerprint_additive_over_shards():
    cfg = phold.tiny_config(n_hosts=301, V=5, load=3, loss=0.2, end_time_s=0.2)
    sim = O.Sim(cfg)
    sim.boot()
    sim.run()
    hs = sim.host_state()
    whole = state_fingerprint(0, hs["digest"], hs["pops"], hs["rng"], hs["ev"])
    parts = 0
    for lo, hi in ((0, 100), (100, 101), (101, 301)):
        parts += state_fingerprint(lo, *(hs[k][lo:hi] for k in ("digest", "pops", "rng", "ev")))
    assert parts & ((1 << 64) - 1) == whole
    hs["rng"] = hs["rng"].copy()
    hs["rng"][7] ^= 1
    assert state_fingerprint(0, hs["digest"], hs["pops"], hs["rng"], hs["ev"]) != whole


def test_gossip_oracle_small_invariants():
    """The gossip body on a small instance: every message is seen at most once
    per host (a host forwards at most M * fan-out messages), the sharded oracle
    protocol is covered by test_dist_gloo."""
    cfg = phold.c5_config(n_hosts=500, V=8, msgs=16, fanout=4, end_time_s=2.0)
    sim = O.Sim(cfg)
    sim.boot()
    sim.run()
    st = sim.stats()
    hs = sim.host_state()
    assert st["pending"] == 0 and st["done"]
    # srcHostEventID counters: boot 1, one origin at most, fan-out per first receipt
    assert np.all(hs["ev"] <= 1 + 1 + 16 * 4)
    # every other id went to a kept send (worker.c:273-297: no event for a dropped packet)
    assert st["sends"] - st["drop_reliability"] == int(hs["ev"].sum()) - 500 - 16
