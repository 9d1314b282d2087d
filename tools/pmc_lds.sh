#!/bin/bash
# Wait / LDS / TA counters for k_proc, one pass each (SG_FLAT from the caller).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lds${SG_FLAT:-}
mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
           "TA_BUSY_avr TA_FLAT_WRITE_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- python bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-drop-in > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
python - "$OUT" <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in per.items():
        if k.startswith("k_proc"):
            print(k, {c: round(sum(v[-8:]) / len(v[-8:]), 1) for c, v in cs.items()})
PY
