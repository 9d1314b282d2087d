"""Per-kernel call count, median / p90 / max duration (us) of a rocprofv3
kernel_trace.csv.  python tools/kt_median.py FILE [name-filter]"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if len(sys.argv) > 2 and sys.argv[2] not in name:
        continue
    d[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2]):
    v.sort()
    print(f"{k:40s} n={len(v):5d} med={v[len(v) // 2]:9.2f} p90={v[int(len(v) * 0.9)]:9.2f} max={v[-1]:9.2f}")
