#!/bin/bash
# One-GPU rehearsal of the multi-rank bench path (2 ranks on GPU 0, gloo
# staging through host memory; RCCL itself needs one GPU per rank).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 40 --warmup 10 \
  --dist-backend gloo --same-device --hosts ${HOSTS:-200000} > gpurun_out/dist_rehearsal.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; tail -3 gpurun_out/dist_rehearsal.log; exit $rc
