#!/bin/bash
# PMC passes (one counter group per run, never with tracing) over a short bench
# run, then the per-kernel summary.  Run on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/prof}
mkdir -p $OUT
BARGS="${PMC_BENCH_ARGS:---steps 20 --warmup 20 --kernel-rounds 1 --no-cpu-baseline --no-drop-in}"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python bench.py $BARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass l2 TCC_HIT_sum TCC_MISS_sum
python tools/prof_summary.py $OUT 16 $OUT/pmc.json > $OUT/pmc_summary.txt; sed -n '/PMC/,$p' $OUT/pmc_summary.txt
