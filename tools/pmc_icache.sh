#!/bin/bash
# Instruction-fetch and wait counters for the bench's kernels, one pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ic
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_IFETCH_LEVEL SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/ic/p$i -o p$i --output-format csv -- python bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-drop-in > gpurun_out/ic/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/ic/p$i.log; exit 1; }
done
python - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob("gpurun_out/ic/p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        per[r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in per.items():
        if "k_" not in k:
            continue
        print(k, {c: round(sum(v[-10:]) / len(v[-10:]), 1) for c, v in cs.items()})
PY
