#!/bin/bash
# Kernel trace of the world-1 multi-rank step path (native steps over RCCL) at
# HOSTS hosts, without a launcher process: RANK/WORLD_SIZE come from the env.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=${PORT:-29561}
HOSTS=${HOSTS:-125000}
OUT=gpurun_out/prof_steps_$HOSTS
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- \
  python bench.py --gpus 1 --dist --hosts $HOSTS --steps 200 --warmup 10 ${EXTRA} > $OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $OUT/run.log | cut -c1-400
[ $rc = 0 ] || exit $rc
python tools/gaps.py $(find $OUT -name "kt_kernel_trace.csv" | head -1) 120
