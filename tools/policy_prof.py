"""CPU-side profile of the drop-in `gpu` SchedulerPolicy beside the host_steal
restatement, on the bench workload (configs[3], 1M hosts): the Shadow-style
round driver's stage times (sg_sched_result.prof_*), per round and per call,
at -w 1 and -w W.  Writes one JSON document to stdout.

    python tools/policy_prof.py [workers] [warmup] [rounds]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402  (the CPU baseline policy)
from shadow_amd import phold, policy  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 16
WARM = int(sys.argv[2]) if len(sys.argv) > 2 else 12
ROUNDS = int(sys.argv[3]) if len(sys.argv) > 3 else 12
cfg = phold.c4_config(n_hosts=1_000_000)


def one(name, workers):
    ops = policy.gpu_ops(workers, cfg["n_hosts"]) if name == "gpu" else O.cpu_policy_ops(True, workers, cfg["n_hosts"])
    r = policy.run_phold(cfg, workers, ops, max_rounds=WARM + ROUNDS, mark_round=WARM, profile=True)
    n = r["marked_rounds"]
    us = {k: r["prof_" + k + "_s"] * 1e6 / n for k in ("push", "pop", "next", "exec", "barrier")}
    return {"policy": name, "workers": workers, "events_per_s": r["marked_pops"] / r["marked_seconds"],
            "round_ms": r["marked_seconds"] * 1e3 / n, "events_per_round": r["marked_pops"] / n,
            "cpu_us_per_round_by_stage": us,
            "ns_per_push": r["prof_push_s"] * 1e9 / max(r["prof_pushes"], 1),
            "ns_per_pop_call": r["prof_pop_s"] * 1e9 / max(r["prof_pops"], 1),
            "pushes": r["prof_pushes"], "pop_calls": r["prof_pops"]}


def glue(workers, variant="relabel"):
    """The Shadow-side glue (integration/scheduler_policy_gpu.c) over the same
    library, through tests/glue_phold.c's SchedulerPolicy adapter, if built."""
    import ctypes as C
    import numpy as np
    from shadow_amd import _lib as L
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "integration", "_bin",
                        f"libsgglue_{variant}.so")
    if not os.path.exists(path):
        return None
    L.lib()
    g = C.CDLL(path)
    p, t, _keep = policy.phold_args(cfg)
    res = policy.SchedResult()
    res.mark_round = WARM
    res.profile = 1
    rep = (C.c_int64 * 4)()
    n = cfg["n_hosts"]
    dig, pops, ev = (np.zeros(n, np.uint64) for _ in range(3))
    rng = np.zeros(n, np.uint32)
    L.check(g.glue_run_phold(C.byref(p), C.byref(t), C.c_uint32(workers), C.c_uint32(policy.default_scheduler_seed(cfg)),
                             C.c_uint64(WARM + ROUNDS), C.byref(res), C.c_void_p(dig.ctypes.data),
                             C.c_void_p(pops.ctypes.data), C.c_void_p(rng.ctypes.data), C.c_void_p(ev.ctypes.data), rep))
    r = res.as_dict()
    nr = r["marked_rounds"]
    return {"policy": f"gpu via scheduler_policy_gpu.c ({variant})", "workers": workers,
            "events_per_s": r["marked_pops"] / r["marked_seconds"], "round_ms": r["marked_seconds"] * 1e3 / nr,
            "cpu_us_per_round_by_stage": {k: r["prof_" + k + "_s"] * 1e6 / nr
                                          for k in ("push", "pop", "next", "exec", "barrier")},
            "ns_per_push": r["prof_push_s"] * 1e9 / max(r["prof_pushes"], 1),
            "ns_per_pop_call": r["prof_pop_s"] * 1e9 / max(r["prof_pops"], 1)}


out = [one(p, w) for w in (1, W) for p in ("steal", "gpu")]
out += [x for x in (glue(1), glue(W)) if x]
print(json.dumps({"workload": "configs[3] 1M hosts, rounds %d..%d" % (WARM, WARM + ROUNDS),
                  "note": "stage times are summed over workers (CPU seconds), two clock reads per call",
                  "runs": out}, indent=1))
