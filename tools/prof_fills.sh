#!/bin/bash
# Kernel + HIP runtime trace of the world-1 step path, then attribute the
# runtime's fill/copy kernels (tools/attrib_fills.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=${PORT:-29563}
HOSTS=${HOSTS:-125000}
OUT=gpurun_out/fills_$HOSTS
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $OUT -o kt --output-format csv -- \
  python bench.py --gpus 1 --dist --hosts $HOSTS --steps 200 --warmup 10 ${EXTRA} > $OUT/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $OUT/run.log | cut -c1-300
[ $rc = 0 ] || exit $rc
python tools/attrib_fills.py $OUT | tee $OUT/attrib.txt
