"""Summarise a tools/profile.sh run: kernel stats + per-kernel PMC averages.

Usage: python tools/prof_summary.py gpurun_out/prof [last_n] [out.json]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) is
doubled (gfx950 tallies 128-B read requests at 64 B), WRITE_SIZE (KiB) is
taken as is.  Only the last `last_n` launches of each kernel are averaged (the
bench's timed, steady-state rounds; the boot round and warmup are skipped).
"""
from __future__ import annotations

import collections
import csv
import os
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def load_counters(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    out = []
    ks = os.path.join(d, "kt", "kt_kernel_stats.csv")
    if os.path.exists(ks):
        out.append("== kernel stats (rocprofv3 --kernel-trace --stats)")
        for r in csv.DictReader(open(ks)):
            out.append(f"{short(r['Name']):<22} calls {int(r['Calls']):>5}  avg {float(r['AverageNs']) / 1e3:9.2f} us  "
                       f"min {float(r['MinNs']) / 1e3:9.2f} us  total {float(r['TotalDurationNs']) / 1e6:8.3f} ms "
                       f"({float(r['Percentage']):.1f}%)")
    kt = os.path.join(d, "kt", "kt_kernel_trace.csv")
    if os.path.exists(kt):
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(kt)):
            per[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        out.append(f"== steady-state durations (last {last} launches)")
        for k, v in per.items():
            v = v[-last:]
            out.append(f"{k:<22} avg {sum(v) / len(v) / 1e3:9.2f} us over {len(v)}")
    steady = {}
    if os.path.exists(kt):
        steady = {k: sum(v[-last:]) / len(v[-last:]) for k, v in per.items()}
    counters = {}
    for sub in ("fetch", "write", "sq", "grbm", "l2"):
        for k, cs in load_counters(os.path.join(d, sub, f"{sub}_counter_collection.csv")).items():
            counters.setdefault(k, {}).update({c: v[-last:] for c, v in cs.items()})
    if counters:
        out.append(f"== PMC per launch (last {last} launches; separate --pmc passes)")
    js = {}
    for k, cs in sorted(counters.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items() if v}
        parts = []
        if "FETCH_SIZE" in avg:
            parts.append(f"FETCH_SIZE {avg['FETCH_SIZE'] / 1024:.1f} MiB raw -> read {2 * avg['FETCH_SIZE'] / 1024:.1f} MiB")
        if "WRITE_SIZE" in avg:
            parts.append(f"WRITE_SIZE {avg['WRITE_SIZE'] / 1024:.1f} MiB")
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            parts.append(f"HBM traffic {(2 * avg['FETCH_SIZE'] + avg['WRITE_SIZE']) * 1024 / 1e6:.1f} MB")
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            tot = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
            parts.append(f"L2 hit {avg['TCC_HIT_sum'] / tot:.3f}" if tot else "L2 idle")
        if "SQ_WAVES" in avg:
            parts.append(f"waves {avg['SQ_WAVES']:.0f}")
        if "SQ_BUSY_CYCLES" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_BUSY_CYCLES"]:
            parts.append(f"avg waves in flight/SE {avg['SQ_WAVE_CYCLES'] / avg['SQ_BUSY_CYCLES']:.1f}")
        if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            parts.append(f"wait frac {avg['SQ_WAIT_ANY'] / avg['SQ_WAVE_CYCLES']:.2f}")
        if "SQ_ACTIVE_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            parts.append(f"issue frac {avg['SQ_ACTIVE_INST_ANY'] / avg['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_INSTS_VMEM" in avg and "SQ_WAVES" in avg and avg["SQ_WAVES"]:
            parts.append(f"vmem/wave {avg['SQ_INSTS_VMEM'] / avg['SQ_WAVES']:.1f} valu/wave {avg.get('SQ_INSTS_VALU', 0) / avg['SQ_WAVES']:.1f}")
        if "GRBM_GUI_ACTIVE" in avg:
            parts.append(f"GRBM_GUI_ACTIVE {avg['GRBM_GUI_ACTIVE']:.0f}")
        out.append(f"{k:<22} " + "; ".join(parts))
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            js[k] = {"read_bytes": 2 * avg["FETCH_SIZE"] * 1024, "write_bytes": avg["WRITE_SIZE"] * 1024,
                     "traffic_bytes": (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024,
                     # tools/calib_fetch.py on this pool: streaming 16-B reads are counted
                     # at half their bytes, random narrow reads of distinct lines at 64 B
                     # each (= the bytes fetched): FETCH_SIZE x1 bounds the reads below
                     "traffic_bytes_lower": (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024,
                     "avg_ns": steady.get(k)}
    print("\n".join(out))
    if len(sys.argv) > 3:
        import json
        with open(sys.argv[3], "w") as f:
            json.dump({"source": d, "launches_averaged": last,
                       "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts 128-B "
                               "reads at 64 B); WRITE_SIZE as is; KiB -> bytes.  traffic_bytes_lower "
                               "takes FETCH_SIZE as is: the calibration (tools/calib_fetch.py, "
                               "profiles/r02/calib/) counts random narrow reads at the 64 B "
                               "actually fetched, so x2 over-counts them",
                       "kernels": js}, f, indent=1)


if __name__ == "__main__":
    main()
