#!/bin/bash
# World-1 RCCL rehearsal of the multi-rank bench path on a one-GPU box: the
# step API, the engine stream shared with the collective, RCCL all-to-all and
# all-reduce (RCCL needs one GPU per rank, so N > 1 is not runnable here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --dist ${RCCL_ARGS:---steps 100 --warmup 10} \
  > gpurun_out/rccl1.log 2>&1
rc=$?; echo "rccl1 rc=$rc"; tail -2 gpurun_out/rccl1.log | cut -c1-1500; exit $rc
