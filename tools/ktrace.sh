#!/bin/bash
# Kernel-trace pass only (no counters) over a short bench run + per-kernel
# steady-state summary and per-round gap analysis.  Run on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="${PROF_ARGS:---steps 60 --warmup 20 --no-cpu-baseline --no-drop-in}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python bench.py $ARGS > $OUT/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -1 $OUT/kt.log | cut -c1-400
case $rc in 0) ;; *) exit $rc;; esac
python tools/prof_summary.py $OUT 40 > $OUT/summary.txt && cat $OUT/summary.txt
python tools/round_gaps.py $OUT/kt/kt_kernel_trace.csv
