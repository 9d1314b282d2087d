"""Compare the GPU engine's pop trace with the oracle's; print the first
divergences (debug aid)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from shadow_amd import phold
from shadow_amd.engine import Engine
from oracle import oracle as O

cfg = phold.probe_config(n_hosts=int(sys.argv[1]) if len(sys.argv) > 1 else 50, jump_ms=5, end_time_s=0.2)
eng = Engine(cfg, trace_capacity=2_000_000, queue_cap=int(sys.argv[2]) if len(sys.argv) > 2 else 0)
eng.boot(); eng.run()
g = np.sort(eng.trace(), order=["host", "pos"])
orc = O.Sim(cfg, trace_capacity=2_000_000); orc.boot(); orc.run()
o = np.sort(orc.trace(), order=["host", "pos"])
print("lens", len(g), len(o))
bad = np.nonzero((g["time"] != o["time"]) | (g["src"] != o["src"]) | (g["seq"] != o["seq"]))[0]
print("mismatches", len(bad))
for i in bad[:12]:
    print("gpu", g[i], "orc", o[i])
