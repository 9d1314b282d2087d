"""Per-kernel durations and the idle gaps between consecutive launches over the
last N launches of a rocprofv3 kernel trace (where a step's time goes)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
dur = defaultdict(list)
gap_before = defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0][:40]
    dur[k].append(e - s)
    if prev_end is not None:
        gap_before[k].append(s - prev_end)
    prev_end = e
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
busy = sum(sum(v) for v in dur.values())
print(f"last {len(rows)} launches: span {span/1e3:.1f} us, busy {busy/1e3:.1f} us, idle {100*(span-busy)/span:.1f}%")
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    g = gap_before[k]
    print(f"  {k:40s} n {len(dur[k]):4d}  avg {sum(dur[k])/len(dur[k])/1e3:7.2f} us  "
          f"gap before {sum(g)/max(1,len(g))/1e3:6.2f} us")
