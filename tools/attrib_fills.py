"""Attribute the runtime's helper kernels (fillBufferAligned / copyBuffer) in a
rocprofv3 run made with --kernel-trace --hip-runtime-trace: which HIP API call
launched each one, on which stream, and how many fall inside the timed steps
(between the first and last k_proc). python tools/attrib_fills.py DIR"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
kt = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
api = {}
for f in glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        api[r["Correlation_Id"]] = r
kt.sort(key=lambda r: int(r["Start_Timestamp"]))
procs = [r for r in kt if "k_proc" in r["Kernel_Name"]]
t0, t1 = int(procs[10]["Start_Timestamp"]), int(procs[-1]["End_Timestamp"])
n_steps = sum(1 for r in procs if t0 <= int(r["Start_Timestamp"]) <= t1)
by = collections.Counter()
dur = collections.defaultdict(int)
for r in kt:
    name = r["Kernel_Name"]
    if "rocclr" not in name:
        continue
    ts = int(r["Start_Timestamp"])
    inside = t0 <= ts <= t1
    a = api.get(r["Correlation_Id"], {})
    key = (name.split("_")[-1], a.get("Function", "?"), r.get("Stream_Id", "?"), inside)
    by[key] += 1
    dur[key] += int(r["End_Timestamp"]) - ts
print(f"steps inside the window: {n_steps}")
for k, n in by.most_common():
    print(f"{k[0]:20s} api={k[1]:28s} stream={k[2]:4s} timed={k[3]!s:5s} n={n:6d} "
          f"per_step={n / max(n_steps, 1):5.2f} avg_us={dur[k] / n / 1e3:6.2f}")
# what runs right before / after each helper kernel inside the window
seq = collections.Counter()
for i, r in enumerate(kt):
    if "rocclr" in r["Kernel_Name"] and t0 <= int(r["Start_Timestamp"]) <= t1:
        prev = kt[i - 1]["Kernel_Name"][:40] if i else "-"
        seq[(r["Kernel_Name"].split("_")[-1], prev)] += 1
for k, n in seq.most_common(8):
    print("after", k, n)
