"""k_proc phase timing from in-kernel s_memrealtime stamps (SG_STAMPS=1):
per-workgroup phase durations over the last round of a 1M-host C4 run."""
import os
import sys

import numpy as np

os.environ["SG_STAMPS"] = "1"
sys.path.insert(0, ".")
from shadow_amd import phold  # noqa: E402
from shadow_amd.engine import Engine  # noqa: E402

# STAMPS_WL=c2 / c5: that workload (shadow_amd/workloads.py) after STAMPS_AT rounds
wl = os.environ.get("STAMPS_WL", "c4")
if wl == "c4":
    cfg = phold.c4_config(n_hosts=int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000)
else:
    from shadow_amd import workloads
    cfg = workloads.get(wl)["build"](None)
eng = Engine(cfg)
eng.boot()
eng.run(int(os.environ.get("STAMPS_AT", "40")))
for r in range(3):
    eng.run(1)
    st_all = eng.stamps().astype(np.int64)
    P = eng.geometry()["partitions"]
    st, pl, sc = st_all[:P], st_all[P], st_all[P + 1:]
    t0 = st[:, 0].min()
    ph = np.diff(st[:, :5], axis=1) * 10 / 1e3  # us (100 MHz ticks)
    print(f"round +{r}: kernel span {(st[:, 4].max() - t0) / 100:.1f} us; WG start spread "
          f"{(st[:, 0].max() - t0) / 100:.1f} us; end spread {(st[:, 4].max() - st[:, 4].min()) / 100:.1f} us")
    for i, nm in enumerate(["sort", "phaseA", "phaseB", "phaseC+part"]):
        v = ph[:, i]
        print(f"   {nm:<12} median {np.median(v):6.2f} us  p90 {np.percentile(v, 90):6.2f}  max {v.max():6.2f}")
    print("   due/active/sends per WG median", np.median(st[:, 5:8], axis=0), "max", st[:, 5:8].max(axis=0))
    a = np.diff(st[:, [1, 8, 9, 10, 11]], axis=1) / 100
    # stamp 12 is written only when that lane's first host recorded its sends
    # (phase B/C path); a light host commits inline and leaves it unset
    rec = st[:, 12] >= st[:, 11]
    r_s = "%.2f" % np.median((st[rec, 12] - st[rec, 11]) / 100) if rec.any() else "n/a"
    print("   phase A, lane 0 of wave 0, first host (median us): state loads %.2f  sort %.2f  count draws %.2f  "
          "reserve %.2f" % tuple(np.median(a, axis=0)) + f"  record+store {r_s} ({int(rec.sum())} WGs)")
    fl = st[:, 30] >= st[:, 1]
    if fl.any():  # k_proc's flat pass ran (stamp 30 at its end)
        print("   flat pass (median us): %.2f in %d WGs; phase A after it %.2f"
              % (np.median(st[fl, 30] - st[fl, 1]) / 100, int(fl.sum()), np.median(st[fl, 2] - st[fl, 30]) / 100))
        if os.environ.get("STAMPS_WL") == "c5":  # the gossip flat pass (stamps without waits)
            y = np.diff(st[fl][:, [1, 16, 31, 17, 18, 19, 30]], axis=1) / 100
            print("   gossip flat pass, lane 0 (median us): loads+pass 1 %.2f  barrier %.2f  pass 2 %.2f  "
                  "barrier %.2f  pass 3 %.2f  barrier %.2f" % tuple(np.median(y, axis=0)))
        x = np.diff(st[fl][:, [1, 16, 17, 18, 19, 30]], axis=1) / 100
        print("   flat pass, lane 0 (median us): start %.2f  draws %.2f  dst loads %.2f  sends %.2f  barrier %.2f"
              % tuple(np.median(x, axis=0)))
        w = (st[fl][:, 26:30] - st[fl][:, [1]]) / 100
        print("   flat pass end per wave 0/4/8/12 (median us after its start):", np.round(np.median(w, axis=0), 2))
    t = np.diff(st[:, [3, 13, 14, 15, 4]], axis=1) / 100
    print("   after phase B (median us): phase C %.2f  partials %.2f  reservations %.2f  tail %.2f"
          % tuple(np.median(t, axis=0)))
    g = np.diff(st[:, [0, 20, 21, 22, 1]], axis=1) / 100
    print("   sort (median us): part loads %.2f  histogram %.2f  scan %.2f  prefetch+scatter %.2f"
          % tuple(np.median(g, axis=0)))
    f = np.diff(st[:, [9, 16, 17, 18, 19]], axis=1) / 100
    print("   light host, lane 0 (median us): pop+draws %.2f  dst loads %.2f  pair loads %.2f  commit %.2f"
          % tuple(np.median(f, axis=0)))
    sc = sc[sc[:, 0] > 0]
    s0 = sc[:, 0].min()
    print(f"   k_scatter: span {(sc[:, 3].max() - s0) / 100:.1f} us, WG start spread {(sc[:, 0].max() - s0) / 100:.1f} us")
    if (sc[:, 16] > 0).all():  # entry stamps: dispatch spread, prologue (round state + plan), launch gap
        e0 = sc[:, 16].min()
        print(f"   k_scatter entry: spread {(sc[:, 16].max() - e0) / 100:.1f} us, prologue (entry -> start) median "
              f"{np.median(sc[:, 0] - sc[:, 16]) / 100:.2f} max {(sc[:, 0] - sc[:, 16]).max() / 100:.2f} us; "
              f"first entry {(e0 - st[:, 4].max()) / 100:.2f} us after k_proc's last workgroup ended")
        for role, nm in enumerate(["insert", "received", "gather", "rmin", "refill"]):
            x = sc[sc[:, 4] == role]
            if len(x):
                print(f"     {nm:<9} prologue median {np.median(x[:, 0] - x[:, 16]) / 100:5.2f} us "
                      f"(round state {np.median(x[:, 17] - x[:, 16]) / 100:.2f}, plan "
                      f"{np.median(x[:, 18] - x[:, 17]) / 100:.2f}, rest {np.median(x[:, 0] - x[:, 18]) / 100:.2f}), "
                      f"entry median {np.median(x[:, 16] - e0) / 100:5.2f} us")
    for role, nm in enumerate(["insert", "received", "gather", "rmin", "refill"]):
        x = sc[sc[:, 4] == role]
        if not len(x):
            continue
        print(f"     {nm:<9} {len(x):4d} WGs  start med {np.median(x[:, 0] - s0) / 100:6.2f}  "
              f"setup {np.median(x[:, 1] - x[:, 0]) / 100:5.2f}  events {np.median(x[:, 2] - x[:, 1]) / 100:5.2f}  "
              f"finish {np.median(x[:, 3] - x[:, 2]) / 100:5.2f}  end med {np.median(x[:, 3] - s0) / 100:6.2f} "
              f"max {(x[:, 3].max() - s0) / 100:6.2f}  n med {np.median(x[:, 5]):.0f}")
    x = sc[sc[:, 4] == 2]
    if len(x):
        g0 = x[0]
        print("     due list: %d entries in %d segments, %d freed; window [%d, %d) buckets %d..%d, straddling %d, "
              "previous straddling %d" % (g0[5], g0[7], g0[8], g0[13], g0[14], g0[9], g0[10],
                                          np.int64(g0[11]), np.int64(g0[12])))
        q = np.diff(x[:, [0, 1, 2, 6, 3]], axis=1) / 100
        print("     gather (median us): rs+due loads %.2f  pool loads+count %.2f  reserve %.2f  scatter %.2f" % tuple(np.median(q, axis=0)),
              " chunks/WG med", np.median(x[:, 5]) / len(x))
    dur = (st[:, 4] - st[:, 0]) / 100
    print("   k_proc WG duration: median %.2f  p90 %.2f  max %.2f us; end offsets median %.2f max %.2f"
          % (np.median(dur), np.percentile(dur, 90), dur.max(), np.median(st[:, 4] - t0) / 100, (st[:, 4].max() - t0) / 100))
    for nm, col in (("due", 5), ("active", 6), ("sends", 7)):
        print(f"     corr(duration, {nm}) = {np.corrcoef(dur, st[:, col])[0, 1]:.2f}")
    # workgroup p runs on XCD p % 8 (round-robin dispatch): a slow XCD shows here
    xcd = np.arange(len(st)) % 8
    print("     per XCD: dur med", [round(float(np.median(dur[xcd == k])), 2) for k in range(8)],
          " start med", [round(float(np.median(st[xcd == k, 0] - t0)) / 100, 2) for k in range(8)],
          " due med", [int(np.median(st[xcd == k, 5])) for k in range(8)])
    for k in range(8):
        print(f"       XCD {k} phases med", np.round(np.median(ph[xcd == k], axis=0), 2))
    top = np.argsort(-(st[:, 4] - t0))[:6]
    for w in top:
        print("     slow WG %3d end %.2f start %.2f dur %.2f  phases %s  due/active/sends %s" % (
            w, (st[w, 4] - t0) / 100, (st[w, 0] - t0) / 100, dur[w], np.round(ph[w], 2), st[w, 5:8]))
    q1 = st[:, 23] > 0
    if q1.any():
        x = st[q1]
        print("   phase A second host (lane 0, median us): start %.2f after phase A start, reserve done +%.2f, record+store +%.2f"
              % (np.median(x[:, 23] - x[:, 1]) / 100, np.median(x[:, 25] - x[:, 23]) / 100,
                 np.median(x[:, 24] - x[:, 25]) / 100))
    if wl == "c5":  # the gossip record path, lane 0's first host (no store waits in 16-18)
        g = st[(st[:, 16] >= st[:, 11]) & (st[:, 17] >= st[:, 16]) & (st[:, 18] >= st[:, 17]) & (st[:, 12] >= st[:, 18])]
        if len(g):
            print("   gossip record path, lane 0 (median us): reserve->loop %.2f  receipts loop %.2f  seen+pads+state %.2f  "
                  "store drain %.2f  (%d WGs)" % (np.median(g[:, 16] - g[:, 11]) / 100, np.median(g[:, 17] - g[:, 16]) / 100,
                                                 np.median(g[:, 18] - g[:, 17]) / 100, np.median(g[:, 12] - g[:, 18]) / 100, len(g)))
    wend = (st[:, 26:30] - st[:, [1]]) / 100
    print("   phase A end per wave 0/4/8/12 (median us after phase A start):", np.round(np.median(wend, axis=0), 2),
          " barrier at %.2f" % np.median((st[:, 2] - st[:, 1]) / 100))
