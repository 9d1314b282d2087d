"""Mode P (drop-in gpu SchedulerPolicy) vs the host_steal restatement at several
worker counts on the bench workload (rounds 12..24 timed)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from shadow_amd import phold, policy  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(os.environ.get("HOSTS", "1000000"))
cfg = phold.c4_config(n_hosts=n)
# KPROF=1: the gpu policy's per-kernel device profile over rounds 12..24 (launches,
# ms, algorithmic bytes: DESIGN.md §7), one JSON line per run
kprof = os.environ.get("KPROF") == "1"
for w in [int(x) for x in os.environ.get("WORKERS", "1,4,16").split(",")]:
    for kind in os.environ.get("KINDS", "gpu,steal").split(","):
        ops = policy.gpu_ops(w, n) if kind == "gpu" else O.cpu_policy_ops(True, w, n)
        if kprof and kind == "gpu":
            policy.kernel_profile(ops, True, 12)
        t = time.perf_counter()
        r = policy.run_phold(cfg, w, ops, max_rounds=24, mark_round=12, free_ops=not (kprof and kind == "gpu"))
        print(f"{kind:5s} w={w:2d}: {r['marked_pops'] / r['marked_seconds']:.3e} events/s "
              f"({r['marked_seconds'] * 1e3 / 12:.1f} ms/round; total {time.perf_counter() - t:.1f} s)",
              flush=True)
        if kprof and kind == "gpu":
            ks = policy.kernel_stats(ops)
            ops.free(ops.data)
            print(json.dumps({"workers": w, "hosts": n, "kernels": ks}), flush=True)
