"""k_proc phase timing from in-kernel s_memrealtime stamps (SG_STAMPS=1):
per-workgroup phase durations over the last round of a 1M-host C4 run."""
import os
import sys

import numpy as np

os.environ["SG_STAMPS"] = "1"
sys.path.insert(0, ".")
from shadow_amd import phold  # noqa: E402
from shadow_amd.engine import Engine  # noqa: E402

cfg = phold.c4_config(n_hosts=int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000)
eng = Engine(cfg)
eng.boot()
eng.run(40)
for r in range(3):
    eng.run(1)
    st = eng.stamps().astype(np.int64)
    t0 = st[:, 0].min()
    ph = np.diff(st[:, :5], axis=1) * 10 / 1e3  # us (100 MHz ticks)
    print(f"round +{r}: kernel span {(st[:, 4].max() - t0) / 100:.1f} us; WG start spread "
          f"{(st[:, 0].max() - t0) / 100:.1f} us; end spread {(st[:, 4].max() - st[:, 4].min()) / 100:.1f} us")
    for i, nm in enumerate(["sort", "phaseA", "phaseB", "phaseC+part"]):
        v = ph[:, i]
        print(f"   {nm:<12} median {np.median(v):6.2f} us  p90 {np.percentile(v, 90):6.2f}  max {v.max():6.2f}")
    print("   due/active/sends per WG median", np.median(st[:, 5:8], axis=0), "max", st[:, 5:8].max(axis=0))
