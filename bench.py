"""bench.py — committed events/s of the MI355X event-scheduling core on the
BASELINE.json metric's workload: synthetic PHOLD, 1M hosts x 16 events,
log-normal latency over 1024 vertices, runahead 1 ms (configs[3]).
--workload c2 / c5 measures configs[1] (10k-host PHOLD, 50 ms mesh) / configs[4]
(100k-host lossy gossip) the same way (shadow_amd/workloads.py).

A step is one conservative round (k_proc: pop + execute + stage; k_scatter:
insert + gather + next window) over the whole host population.  W warmup rounds (the boot round included) run untimed; K
rounds are timed between a barrier + device synchronisation on both sides.
value = committed events (executed pops) in the K rounds, all ranks, / max
rank time.  N > 1: hosts are block-sharded over ranks (one process per GPU)
and new events cross shards each round through RCCL all-to-all; the total
host count stays 1M (strong scaling, as the metric names it).

Also reported:
  roofline     dominant kernel (k_proc): algorithmic bytes (64 B per
               committed event + 24 B per active host-round)
               per launch / its average launch time (HIP events on the engine
               stream), against 8 TB/s HBM; roofline.per_kernel gives the same
               for every kernel of the round (k_scatter: 32 B per record it
               moves).
  cpu_baseline the CPU reference policy (oracle/host_steal.c, the host_steal
               restatement) on the same workload, timed on this machine's host
               cores over a bounded sample of rounds (rank 0, N=1): value with
               priority_queue.c's heap and its GLib position map (the
               reference's cost), plain_heap_value with plain binary heaps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from shadow_amd import workloads as WL  # noqa: E402
from shadow_amd.roofline import HBM_PEAK_GBS, kernel_line, proc_bytes, scatter_bytes  # noqa: E402
# PMC HBM bytes per launch of each kernel for each workload: rocprofv3
# FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh), corrected per
# MI355X_MICROARCH.md §HBM by tools/prof_summary.py.  Counters cannot be read
# from inside a timed run, so the bench quotes the committed measurement.
# The driver's own run (--steps 20 --warmup 5) has a profile of that window:
# its first rounds differ from the default run's steady state.
PMC_DIR = os.path.join(ROOT, "profiles", "r06", "final")
PMC_JSON = {w: os.path.join(PMC_DIR, f"prof_{w}", "pmc.json") for w in ("c4", "c2", "c5")}
PMC_JSON_WINDOW = {("c4", 20, 5): os.path.join(PMC_DIR, "prof_c4_driver", "pmc.json")}
DOMINANT = "k_proc"
_PMC_WINDOW = (None, None)


def pmc_traffic(workload, n_hosts, kernel=DOMINANT):
    """(corrected PMC bytes per launch of `kernel`, the bytes with FETCH_SIZE as
    counted, source) from the committed profile of this workload (of this
    run's window where one was profiled), or Nones."""
    path = PMC_JSON_WINDOW.get((workload,) + _PMC_WINDOW, PMC_JSON.get(workload))
    if (workload == "c4" and n_hosts != 1_000_000) or not path or not os.path.exists(path):
        return None, None, None
    ks = json.load(open(path))["kernels"]
    k = next((v for n, v in ks.items() if n == kernel or n.startswith(kernel + "<")), None)
    if not k:
        return None, None, None
    return k["traffic_bytes"], k.get("traffic_bytes_lower"), os.path.relpath(path, ROOT)


def kernel_roofline(workload, name, alg_bytes, avg_s, n_hosts):
    """One kernel's line of roofline.per_kernel: algorithmic bytes per launch
    over its average launch time against HBM peak, beside the committed PMC
    traffic per launch."""
    traffic, lower, src = pmc_traffic(workload, n_hosts, name)
    out = kernel_line(alg_bytes, avg_s)
    out.update(traffic=traffic, traffic_lower=lower,
               traffic_gbs=traffic / avg_s / 1e9 if traffic and avg_s else None, traffic_source=src)
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", default="c4", choices=sorted(WL.WORKLOADS),
                    help="c4: configs[3] (the BASELINE metric's, default); c2: configs[1]; c5: configs[4]")
    ap.add_argument("--steps", type=int, default=None, help="timed rounds (default: the workload's)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed rounds (default: the workload's)")
    ap.add_argument("--hosts", type=int, default=None, help="c4 only: the host count (default 1M)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-drop-in", action="store_true",
                    help="skip the Mode P (drop-in gpu SchedulerPolicy) leg")
    ap.add_argument("--cpu-rounds", type=int, default=12, help="CPU legs: rounds timed")
    ap.add_argument("--cpu-workers", type=int,
                    default=min(16, len(os.sched_getaffinity(0))),
                    help="CPU baseline worker threads (the GPU box's share is 16 cores)")
    ap.add_argument("--batch", type=int, default=32, help="rounds enqueued per host sync")
    ap.add_argument("--graph", type=int, default=int(os.environ.get("SG_GRAPH", "0")),
                    help="capture every GRAPH rounds / steps into a hipGraph and replay it (0: off)")
    ap.add_argument("--py-steps", action="store_true",
                    help="N > 1: drive each step from Python around torch's all_to_all_single "
                         "instead of sg_engine_run_steps")
    ap.add_argument("--kernel-rounds", type=int, default=50,
                    help="rounds after the timed region that are re-run with per-kernel HIP events")
    ap.add_argument("--kernel-timing", choices=("after", "replay", "inline"), default=None,
                    help="per-kernel durations from rounds after the timed region (c4's default), from "
                         "a second engine replaying the timed rounds (c2 / c5: their rounds change "
                         "along the run, and the run is deterministic) or from the timed rounds "
                         "themselves (their events then slow the timed region)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="N > 1: nccl (RCCL, the measured path) or gloo (rehearsal only)")
    ap.add_argument("--dist", action="store_true",
                    help="take the multi-rank step path even at N=1 (a world-1 RCCL job: "
                         "rehearses the collective path on a one-GPU box)")
    ap.add_argument("--exchange", choices=("auto", "xgmi", "rccl"), default="auto",
                    help="N > 1 (or --dist): the step's block exchange as xGMI peer stores into "
                         "the peers' receive regions (sg_xlink, after a self-test on every rank) or "
                         "the RCCL all-to-all; auto takes xgmi when its self-test passes")
    ap.add_argument("--same-device", action="store_true",
                    help="N > 1 rehearsal: every rank on GPU 0 (needs --dist-backend gloo)")
    a = ap.parse_args()
    w = WL.get(a.workload)
    if a.hosts is not None and a.workload != "c4":
        ap.error("--hosts applies to --workload c4 only")
    a.warmup = w["warmup"] if a.warmup is None else a.warmup
    a.steps = w["steps"] if a.steps is None else a.steps
    a.kernel_timing = a.kernel_timing or w["kernel_timing"]
    return a


def build_config(a):
    """The workload's config (a.cfg, a.hosts), built in the process that runs
    it (a self-launching parent never loads the native library)."""
    a.cfg = WL.get(a.workload)["build"](a.hosts)
    a.hosts = a.cfg["n_hosts"]


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_counts() -> dict:
    """The host's CPU counts: os.cpu_count() (nproc of the machine), this
    process's affinity set, and the cgroup's CPU quota where one is set (the
    GPU box shows the whole machine's CPUs to a 16-core share)."""
    out = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_cpus": None}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            out["cgroup_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return out


def cpu_baseline(cfg, warmup, rounds, workers):
    """The CPU reference policy: oracle/host_steal.c — the
    C restatement of scheduler_policy_host_steal.c — under the Shadow-style
    round driver (sg_sched.c, worker.c:149-216 semantics), same workload.
    Boot + `warmup` rounds untimed, the next `rounds` rounds timed.  value and
    single_thread_value (-w `workers`, -w 1): the per-host queues are
    priority_queue.c's heap with its GLib hash-table position map, updated on
    every swap (oracle/libhsglib.so), i.e. the reference's own cost;
    plain_heap_value: the same policy on plain binary heaps (liborc.so), a
    lower bound on it."""
    from oracle import oracle as O
    from shadow_amd import policy

    def one(w, faithful):
        ops = O.cpu_policy_ops(True, w, cfg["n_hosts"], faithful=faithful)
        r = policy.run_phold(cfg, w, ops, max_rounds=warmup + rounds, mark_round=warmup)
        return r["marked_pops"] / r["marked_seconds"], r

    faithful = O.faithful_available()
    counts = _cpu_counts()
    v, r = one(workers, faithful)
    v1, _ = one(1, faithful) if workers > 1 else (v, r)
    vp, _ = one(workers, False) if faithful else (v, r)
    # -w = every CPU this process may run on (-w nproc), when
    # that is more than the default share
    wall = counts["affinity"]
    vall, rall = one(wall, faithful) if wall > workers else (v, r)
    best_w, best_v, best_r = (wall, vall, rall) if vall > v else (workers, v, r)
    heap = ("priority_queue.c's heap with its GLib hash-table position map (oracle/libhsglib.so)"
            if faithful else "plain binary heaps (GLib absent: libhsglib.so not built)")
    return {"value": best_v, "unit": "events/s", "cores": best_w, "kind": "port",
            "share_value": v, "share_workers": workers,
            "all_cpus_value": vall, "all_cpus_workers": wall,
            "single_thread_value": v1, "plain_heap_value": vp, "faithful_heap": faithful,
            "cpu_model": _cpu_model(), **counts,
            "sample": f"oracle/host_steal.c (the C restatement of host_steal) under the Shadow round "
                      f"driver, per-host queues: {heap}; same config, rounds {warmup}..{warmup + rounds} "
                      f"timed ({best_r['marked_pops']} events, {best_r['marked_seconds']:.2f} s at "
                      f"-w {best_w}); value is the faster of -w {workers} (share_value, the box's CPU "
                      f"share) and -w {wall} (all_cpus_value, every CPU in the affinity set: nproc "
                      f"{counts['nproc']}, cgroup quota {counts['cgroup_cpus']}); single_thread_value is "
                      f"-w 1 on the same rounds; plain_heap_value is -w {workers} with plain binary heaps"}


def drop_in_policy(cfg, warmup, rounds, workers, fixture=None):
    """The drop-in `gpu` SchedulerPolicy (Mode P, sg_policy.c + sg_policy_dev.hip)
    under the same Shadow-style round driver and sample as cpu_baseline: CPU
    workers execute the PHOLD bodies and push/pop through the C-ABI, the GPU
    keeps the per-host queues.  PCIe-inclusive by construction (the boundary
    hands over host records), so it is reported beside `value`, never as it."""
    from shadow_amd import policy
    from shadow_amd.trace import state_fingerprint

    def one(w, kstats=None):
        ops = policy.gpu_ops(w, cfg["n_hosts"])
        if kstats is not None:  # the device half's kernels, timed rounds only
            policy.kernel_profile(ops, True, warmup)
        try:
            r = policy.run_phold(cfg, w, ops, max_rounds=warmup + rounds, mark_round=warmup, free_ops=False)
            if kstats is not None:
                kstats.update(policy.kernel_stats(ops))
        finally:
            ops.free(ops.data)
        return r

    ks = {}
    r = one(workers, ks)
    r1 = one(1) if workers > 1 else r
    out = {"value": r["marked_pops"] / r["marked_seconds"], "unit": "events/s",
           "workers": workers, "single_thread_value": r1["marked_pops"] / r1["marked_seconds"],
           "sample": f"gpu SchedulerPolicy (Mode P) with {workers} CPU workers under the Shadow "
                     f"round driver, same config, rounds {warmup}..{warmup + rounds} timed "
                     f"({r['marked_pops']} events, {r['marked_seconds']:.2f} s); single_thread_value "
                     f"is -w 1 on the same rounds"}
    # the device half's roofline: each kernel class's algorithmic bytes per
    # launch over its average launch time (dispatch-packet
    # timestamps) against 8 TB/s, over the timed rounds of the -w run
    per = {}
    for name, k in ks.items():
        if not k["launches"]:
            continue
        line = kernel_line(k["alg_bytes"] / k["launches"], k["ms"] / 1e3 / k["launches"])
        line["launches"] = k["launches"]
        per[name] = line
    dev_ms = sum(k["ms"] for k in ks.values())
    out["roofline"] = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "per_kernel": per,
                       "device_ms_per_round": dev_ms / max(rounds, 1),
                       "timing_method": "hipExtLaunchKernelGGL dispatch-packet timestamps of every device "
                                        "launch of the policy (sg_policy_kernel_profile), timed rounds only"}
    # the policy's end state against the oracle's per-round fixture (parity
    # checker only, after the timed rounds)
    if fixture and os.path.exists(FIXTURES):
        rows = {row[0]: row for row in json.load(open(FIXTURES))[fixture]["rounds"]}
        end = r["rounds"]
        if end in rows:
            fp = state_fingerprint(0, r["digest"], r["pops_per_host"], r["rng"], r["ev"])
            out["parity"] = {"round": end, "match": fp == rows[end][2] and r["pops"] == rows[end][1]}
    return out


def run_single(args):
    from shadow_amd.engine import Engine

    global _PMC_WINDOW
    _PMC_WINDOW = (args.steps, args.warmup)

    cfg = args.cfg
    wl = WL.get(args.workload)
    eng = Engine(cfg, device=0)
    eng.boot()
    eng.set_graph(args.graph)
    eng.run(args.warmup, batch=args.graph or args.batch)
    eng.prepare_graph()  # graphs on: the first timed batch replays, it does not capture
    inline = args.kernel_timing == "inline"
    s0 = eng.stats()
    if inline:  # the timed rounds' own kernel durations (dispatch-packet timestamps, no extra packets)
        a1, _ = eng.active_hosts()
        mv1 = eng.event_moves()
        eng.set_timing(True)
    eng.sync()
    # timed region: K rounds, nothing but the rounds on the stream (at most two
    # batches queued, no read-back)
    t0 = time.perf_counter()
    eng.enqueue_rounds(args.steps)
    eng.sync()
    dt = time.perf_counter() - t0
    if inline:
        kt = eng.kernel_times()
        eng.set_timing(False)
    s1 = eng.stats()
    if s1["overflow"]:
        raise SystemExit(f"device queue overflow during bench: {s1['overflow']:#x}")
    pops = s1["pops"] - s0["pops"]
    rounds = s1["rounds"] - s0["rounds"]
    if rounds != args.steps:
        raise SystemExit(f"simulation ended early: {rounds} of {args.steps} rounds")
    from shadow_amd.trace import state_fingerprint
    hs = eng.host_state()  # the state at the end of the timed region, for the parity check
    fp = state_fingerprint(0, hs["digest"], hs["pops"], hs["rng"], hs["ev"])
    del hs
    if inline:
        kr, s2, kpops = rounds, s1, pops
    elif args.kernel_timing == "replay":
        # the same rounds again on a second engine (the run is deterministic),
        # every launch carrying HIP events: the timed region stays event-free
        eng.close()
        eng = Engine(cfg, device=0)
        eng.boot()
        eng.run(args.warmup, batch=args.batch)
        r0 = eng.stats()
        a1, _ = eng.active_hosts()
        mv1 = eng.event_moves()
        eng.set_timing(True)
        eng.run(args.steps, batch=args.batch)
        kt = eng.kernel_times()
        eng.set_timing(False)
        s2 = eng.stats()
        kpops = s2["pops"] - r0["pops"]
        kr = s2["rounds"] - r0["rounds"]
        if kpops != pops or kr != rounds:
            raise SystemExit(f"replay diverged: {kpops} pops in {kr} rounds against {pops} in {rounds}")
    else:
        # kernel durations: the next rounds of the same run, every launch carrying
        # HIP events as its dispatch packet's start / stop timestamps
        # (hipExtLaunchKernelGGL) on the engine stream — kept out of the headline
        # region all the same
        a1, _ = eng.active_hosts()
        mv1 = eng.event_moves()
        kr = max(1, min(args.steps, args.kernel_rounds))
        eng.set_timing(True)
        eng.run(kr, batch=args.batch)
        kt = eng.kernel_times()
        eng.set_timing(False)
        s2 = eng.stats()
        kpops = s2["pops"] - s1["pops"]
        kr = s2["rounds"] - s1["rounds"]
    proc_ms, proc_n = kt["process"]
    a2, _ = eng.active_hosts()
    mv2 = eng.event_moves()
    alg_bytes = proc_bytes(kpops, a2 - a1)
    per_launch_bytes = alg_bytes / max(proc_n, 1)
    avg_launch_s = proc_ms / 1e3 / max(proc_n, 1)
    achieved = per_launch_bytes / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    traffic, traffic_lower, traffic_src = pmc_traffic(args.workload, args.hosts)
    kus = {k: v[0] * 1e3 / v[1] for k, v in kt.items() if v[1]}  # us per launch (one per round each)
    ins_ms, ins_n = kt["insert"]
    moves = {k: mv2[k] - mv1[k] for k in mv2}
    per_kernel = {
        DOMINANT: kernel_roofline(args.workload, DOMINANT, per_launch_bytes, avg_launch_s, args.hosts),
        "k_scatter": kernel_roofline(args.workload, "k_scatter", scatter_bytes(moves) / max(ins_n, 1),
                                     ins_ms / 1e3 / max(ins_n, 1), args.hosts),
    }
    res = {
        "metric": wl["metric"](cfg),
        "value": pops / dt,
        "unit": "events/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic",
        "config": {"workload": wl["describe"](cfg), "name": args.workload,
                   "n_hosts": args.hosts, "rounds_timed": rounds, "events_timed": pops,
                   "parallelism": "hosts sharded 1 way",
                   "round_loop": f"sg_engine_enqueue_rounds, hipGraph batch {args.graph}" if args.graph
                                 else "sg_engine_enqueue_rounds, eager launches"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_lower": traffic_lower,
                     "traffic_source": traffic_src,
                     "traffic_gbs": traffic / avg_launch_s / 1e9 if traffic and avg_launch_s else None,
                     "kernel": DOMINANT, "avg_launch_us": avg_launch_s * 1e6,
                     "alg_bytes_per_launch": per_launch_bytes,
                     "timing_rounds": kr,
                     "kernel_us_per_round": kus,
                     "per_kernel": per_kernel,
                     "gaps_us_per_round": dt * 1e6 / args.steps - sum(kus.values()),
                     "timing_method": "HIP events as each launch's dispatch-packet timestamps "
                                      "(hipExtLaunchKernelGGL), " +
                                      ("over the timed rounds themselves" if inline else
                                       "over the timed rounds replayed on a second engine (the run is "
                                       "deterministic; the timed region carries no events)"
                                       if args.kernel_timing == "replay" else
                                       "rounds after the timed region") +
                                      "; the rest of ms_per_step is launch gaps"},
        "_end_round": s1["rounds"], "_fingerprint": fp,
    }
    cw = wl["cpu_warmup"]
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(cfg, cw, args.cpu_rounds, args.cpu_workers)
    if not args.no_drop_in:
        res["drop_in_policy"] = drop_in_policy(cfg, cw, args.cpu_rounds, args.cpu_workers, wl["fixture"](cfg))
    return res


FIXTURES = os.path.join(ROOT, "tests", "golden", "oracle_fixtures.json")


def parity_check(res, args):
    """The state at the end of the timed region against the oracle: the host
    state fingerprint (shadow_amd.trace.state_fingerprint over every host's
    trace digest, pops, rand_r state and event counter, summed over ranks) and
    the executed-pop total, after the same number of rounds, from
    tests/golden/oracle_fixtures.json (tests/golden/make_fixtures.py ran the
    CPU oracle on this config).  "bit-exact" stays in the metric only on a match."""
    r, fp = res.pop("_end_round"), res.pop("_fingerprint")
    out = {"round": r, "fingerprint": f"{fp:016x}", "source": None, "match": None}
    fx = None
    key = WL.get(args.workload)["fixture"](args.cfg)
    metric = res["metric"]
    if key and os.path.exists(FIXTURES):
        fx = json.load(open(FIXTURES)).get(key)
    if fx:
        out["source"] = f"{os.path.relpath(FIXTURES, ROOT)} {key} (oracle, rounds 1..{len(fx['rounds'])})"
        row = next((x for x in fx["rounds"] if x[0] == r), None)
        if row is not None:
            out["match"] = bool(row[2] == fp)
            out["oracle_fingerprint"] = f"{row[2]:016x}"
    res["parity"] = out
    if out["match"] is False:
        res["metric"] = metric.replace("; bit-exact", "") + " (PARITY MISMATCH vs oracle)"
        print("bench: end-of-region state differs from the oracle fixture", file=sys.stderr)
    elif out["match"] is None:
        res["metric"] = metric.replace("; bit-exact", "") + " (parity unchecked)"
        out["note"] = "no oracle fixture for this round / host count: parity unchecked in this run"
    return out["match"] is not False


def self_launch(args) -> int:
    """`python bench.py --gpus N` without a launcher: start N ranks under
    torch.distributed.run as a child process (this process never touches the
    GPU, so nothing is exec'd from an initialised one) and return its exit code.
    Rank 0 prints the JSON line through the child's stdout."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 or args.gpus > 1 or args.dist:
        # dist.bench builds the config itself (args.cfg), after torch has set up
        # the device: a rank that loaded the native library first saw no device
        from shadow_amd import dist
        res = dist.bench(args)
    else:
        build_config(args)
        res = run_single(args)
    if res is None:
        return
    ok = parity_check(res, args)
    print(json.dumps(res), flush=True)
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
