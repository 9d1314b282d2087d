"""Per-round timeline from a rocprofv3 kernel trace: average busy time per
kernel and the idle gap in front of it, over the last rounds (debug aid);
a round starts at k_proc."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").split("<")[0]
seq = [(name(r), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
first = next((i for i, s in enumerate(seq) if s[0] == "k_proc"), None)
if first is None:
    sys.exit(0)
busy, gap, cnt = collections.defaultdict(int), collections.defaultdict(int), collections.Counter()
tail = seq[-min(len(seq), 40 * 6):]
for prev, cur in zip(tail, tail[1:]):
    busy[cur[0]] += cur[2] - cur[1]
    gap[cur[0]] += max(0, cur[1] - prev[2])
    cnt[cur[0]] += 1
starts = [s[1] for s in tail if s[0] == "k_proc"]
if len(starts) > 1:
    print(f"round period {(starts[-1] - starts[0]) / (len(starts) - 1) / 1e3:.1f} us over {len(starts) - 1} rounds")
for k in cnt:
    print(f"{k:<12} busy {busy[k] / cnt[k] / 1e3:7.2f} us  gap before {gap[k] / cnt[k] / 1e3:6.2f} us  (n={cnt[k]})")
