"""TEST INFRASTRUCTURE: writes tests/golden/oracle_fixtures.json from the CPU
oracle (oracle/orc.c, the line-cited restatement of the reference's round
semantics) for the BASELINE configs too large to re-run on the GPU box inside
a test or the bench:

  c1        configs[0]: the example's two hosts on its embedded one-vertex
            topology, the whole 3600 s run
  c3        configs[2]: 2k relays + 8k clients on the bundled topology, 10 s
  c5        configs[4]: gossip, 100k hosts, lossy links, the whole run
  c4_1m     configs[3]: PHOLD at 1M hosts, the state after every one of the
            first ROUNDS_C4 rounds (the bench's timed rounds are checked
            against it)
  c2_rounds configs[1]: PHOLD 10k hosts on the 50 ms mesh, every round of the
            whole run (bench.py --workload c2)
  c5_rounds configs[4]: the gossip run of c5, every round (bench.py --workload c5)

Per case: the oracle's counters and window, and a fingerprint of every host's
end state (shadow_amd.trace.state_fingerprint over trace digest, pops, rand_r
state and event counter; additive over hosts, so shards sum to it).  The data
are inputs and outputs only; run `python tests/golden/make_fixtures.py [case]`
to regenerate (about three minutes for all).
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from shadow_amd import phold  # noqa: E402
from shadow_amd.trace import state_fingerprint  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_fixtures.json")
ROUNDS_C4 = 600
STATS = ("rounds", "pops", "boots", "sends", "null_dst", "drop_reliability", "drop_endtime",
         "bumped", "same_round", "pending", "window_start", "window_end", "done", "jmin_ms")

CONFIGS = {
    "c1": lambda: phold.c1_config(),
    "c3": lambda: phold.c3_config(),
    "c5": lambda: phold.c5_config(),
    "c4_1m": lambda: phold.c4_config(n_hosts=1_000_000),
    "c2_rounds": lambda: phold.c2_config(),
    "c5_rounds": lambda: phold.c5_config(),
}
PER_ROUND = {"c4_1m": ROUNDS_C4, "c2_rounds": 1 << 30, "c5_rounds": 1 << 30}


def fingerprint(sim) -> int:
    hs = sim.host_state()
    return state_fingerprint(0, hs["digest"], hs["pops"], hs["rng"], hs["ev"])


def windows_fp(w) -> int:
    """Chained hash of the executed windows {start, end}."""
    h = 5381
    M = (1 << 64) - 1
    for s, e in w.tolist():
        h = ((h * 1000003) ^ s) & M
        h = ((h * 1000003) ^ e) & M
    return h


def final_case(name):
    cfg = CONFIGS[name]()
    sim = O.Sim(cfg)
    sim.boot()
    sim.run()
    st = sim.stats()
    return {"config": cfg["name"], "n_hosts": cfg["n_hosts"],
            "stats": {k: st[k] for k in STATS}, "fingerprint": fingerprint(sim),
            "windows_fp": windows_fp(sim.windows())}


def per_round_case(name, rounds):
    cfg = CONFIGS[name]()
    sim = O.Sim(cfg)
    sim.boot()
    out = []
    for r in range(1, rounds + 1):
        if sim.run(1) != 1:
            break
        st = sim.stats()
        out.append([r, st["pops"], fingerprint(sim), st["window_start"], st["window_end"]])
    return {"config": cfg["name"], "n_hosts": cfg["n_hosts"],
            "columns": ["rounds", "pops", "fingerprint", "next_window_start", "next_window_end"],
            "rounds": out}


def main(names):
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for name in names:
        t = time.time()
        data[name] = per_round_case(name, PER_ROUND[name]) if name in PER_ROUND else final_case(name)
        print(f"{name}: {time.time() - t:.1f} s", flush=True)
        json.dump(data, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CONFIGS))
