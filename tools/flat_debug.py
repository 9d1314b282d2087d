"""Debug aid: the configs[3] engine with and without k_proc's flat pass
(SG_FLAT=1 / 0), compared host by host after every round; the first round
with a difference prints the differing hosts and their traced pops.
python tools/flat_debug.py [rounds] [n_hosts]"""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
from shadow_amd import phold  # noqa: E402
from shadow_amd.engine import Engine  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 25
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
cfg = phold.c4_config(n_hosts=n)


def mk(flat):
    os.environ["SG_FLAT"] = str(flat)
    e = Engine(cfg, trace_capacity=14_000_000)
    e.boot()
    return e


A, B = mk(1), mk(0)
for r in range(1, rounds + 1):
    A.run(1)
    B.run(1)
    sa, sb = A.stats(), B.stats()
    ha, hb = A.host_state(), B.host_state()
    bad = {k: np.nonzero(ha[k] != hb[k])[0] for k in ("digest", "pops", "rng", "ev")}
    print(f"round {r}: pops {sa['pops']} / {sb['pops']}, differing hosts",
          {k: len(v) for k, v in bad.items()}, flush=True)
    if any(len(v) for v in bad.values()):
        ta, tb = A.trace(), B.trace()
        hosts = sorted(set(np.concatenate(list(bad.values())).tolist()))[:6]
        for h in hosts:
            print(f"host {h}:", {k: (int(ha[k][h]), int(hb[k][h])) for k in ha})
            for name, t in (("flat", ta), ("base", tb)):
                m = t[t["host"] == h]
                print(f"  {name} last pops:", [(int(x["time"]), int(x["src"]), int(x["seq"]), int(x["pos"]))
                                               for x in m[-6:]])
        break
