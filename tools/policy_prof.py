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


out = [one(p, w) for w in (1, W) for p in ("steal", "gpu")]
print(json.dumps({"workload": "configs[3] 1M hosts, rounds %d..%d" % (WARM, WARM + ROUNDS),
                  "note": "stage times are summed over workers (CPU seconds), two clock reads per call",
                  "runs": out}, indent=1))
