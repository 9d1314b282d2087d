#!/bin/bash
# rocprofv3 passes over a short bench run (run on the GPU box via gpurun).
# Pass 1: kernel trace + stats.  Then one PMC group per pass (never combined
# with tracing domains), each under its own hard time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
ARGS="${PROF_ARGS:---steps 200 --warmup 20 --no-cpu-baseline --no-drop-in}"
# the profiled program: bench.py by default; PROF_CMD (e.g. "python tools/modep_scan.py") otherwise
CMD="${PROF_CMD:-python bench.py $ARGS}"
echo "== kernel trace"; date
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $CMD > $OUT/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -2 $OUT/kt.log
case $rc in 124|137|134|139) exit $rc;; esac
pass() {  # name counters...
  local name=$1; shift
  echo "== pmc $name: $*"; date
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- $CMD > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass l2 TCC_HIT_sum TCC_MISS_sum
find $OUT -name "*.csv" | head -20
