#!/bin/bash
# Kernel trace of the world-1 RCCL step path at a shard's host count (the N=8
# per-GPU share by default): per-kernel steady state and per-step gaps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_dist1
mkdir -p $OUT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=${MASTER_PORT:-29557} RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- \
  python bench.py --dist --hosts ${HOSTS:-125000} --steps 60 --warmup 10 > $OUT/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; tail -1 $OUT/kt.log | cut -c1-300
case $rc in 0) ;; *) exit $rc;; esac
python tools/prof_summary.py $OUT 40 > $OUT/summary.txt && cat $OUT/summary.txt
python tools/round_gaps.py $OUT/kt/kt_kernel_trace.csv
