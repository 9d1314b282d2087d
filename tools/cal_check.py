"""Debug aid (GPU box): run small configs on the engine and on the oracle and
print, per config, whether per-host state, counters and windows agree, with
the first diverging trace records."""
import sys
import time
import traceback

import numpy as np

sys.path.insert(0, ".")
from shadow_amd import _lib as L  # noqa: E402
from shadow_amd import phold  # noqa: E402
from shadow_amd.engine import Engine  # noqa: E402
from oracle import oracle as O  # noqa: E402

CFGS = {
    "smoke": lambda: phold.tiny_config(n_hosts=512, V=8, load=4, end_time_s=0.3, loss=0.02),
    "probe5": lambda: phold.probe_config(n_hosts=200, jump_ms=5, end_time_s=0.3),
    "probe10": lambda: phold.probe_config(n_hosts=200, jump_ms=10, end_time_s=0.3),
    "one_host": lambda: phold.tiny_config(n_hosts=1, V=1, load=3),
    "tiny_latency": lambda: phold.tiny_config(n_hosts=64, min_ms=0.2),
    "runahead": lambda: phold.tiny_config(n_hosts=96, runahead_ms=7),
    "c4_20k": lambda: phold.c4_config(n_hosts=20_000, end_time_s=0.1),
}


def one(name, mk):
    cfg = mk()
    t0 = time.time()
    eng = Engine(cfg, trace_capacity=2_000_000)
    eng.boot()
    eng.run()
    g, gs = eng.host_state(), eng.stats()
    orc = O.Sim(cfg, trace_capacity=2_000_000)
    orc.boot()
    orc.run()
    o, os_ = orc.host_state(), orc.stats()
    bad = [k for k in ("pops", "rng", "ev", "digest") if not np.array_equal(g[k], o[k])]
    sbad = [(k, gs[k], os_[k]) for k in ("rounds", "pops", "sends", "bumped", "same_round",
                                         "pending", "window_start", "window_end", "jmin_ms")
            if gs[k] != os_[k]]
    ok = not bad and not sbad and gs["overflow"] == 0
    print(f"{name}: {'PASS' if ok else 'FAIL'} pops={gs['pops']} rounds={gs['rounds']} "
          f"ovf={gs['overflow']:#x} geom={eng.geometry()} {time.time() - t0:.1f}s", flush=True)
    if not ok:
        print("  state mismatches:", bad, "stats:", sbad)
        gt = np.sort(eng.trace(), order=["host", "pos"])
        ot = np.sort(orc.trace(), order=["host", "pos"])
        n = min(len(gt), len(ot))
        diff = np.nonzero((gt["time"][:n] != ot["time"][:n]) | (gt["src"][:n] != ot["src"][:n])
                          | (gt["seq"][:n] != ot["seq"][:n]) | (gt["host"][:n] != ot["host"][:n]))[0]
        print("  trace lens", len(gt), len(ot), "first diffs:")
        for i in diff[:6]:
            print("   gpu", gt[i], "orc", ot[i])
        w1, w2 = eng.windows(), orc.windows()
        m = min(len(w1), len(w2))
        wd = np.nonzero((w1[:m] != w2[:m]).any(axis=1))[0]
        if len(wd):
            i = wd[0]
            print("  first window diff at round", i, w1[i], w2[i])
    return ok


if __name__ == "__main__":
    names = sys.argv[1:] or list(CFGS)
    fails = 0
    for n in names:
        try:
            fails += not one(n, CFGS[n])
        except L.SgError as e:
            fails += 1
            print(f"{n}: ERROR {e}", flush=True)
            if e.code == L.SG_ERR_HIP:
                break  # the device context is gone
        except Exception:
            fails += 1
            traceback.print_exc()
    sys.exit(1 if fails else 0)
