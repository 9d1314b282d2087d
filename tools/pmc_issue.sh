#!/bin/bash
# Instruction-mix PMC passes over a short bench run (k_proc / k_scatter /
# k_plan): instruction counts by type, and issue-active cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_issue
mkdir -p $OUT
pass() {
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-drop-in > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
}
pass mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INSTS_SMEM
pass act SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY
python - <<'PY'
import csv, glob, collections
for g in ("mix", "act"):
    f = glob.glob(f"gpurun_out/pmc_issue/{g}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        per[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, cs in per.items():
        if not n.startswith(("k_proc", "k_scatter", "k_count")):
            continue
        print(g, n, {c: round(sum(v[-8:]) / len(v[-8:])) for c, v in cs.items()})
PY
