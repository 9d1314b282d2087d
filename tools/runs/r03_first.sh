#!/bin/bash
# Round 3 first GPU call: the new two-process dist tests, the full GPU suite,
# an RCCL duplicate-GPU probe, one bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r03
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03/dist_tests.log 2>&1; rc=$?; tail -8 gpurun_out/r03/dist_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  --deselect tests/test_gpu_dist.py > gpurun_out/r03/gpu_suite.log 2>&1; rc=$?; tail -4 gpurun_out/r03/gpu_suite.log
[ $rc -eq 0 ] || exit $rc
NCCL_DEBUG=WARN timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 tools/rccl_dup_probe.py > gpurun_out/r03/rccl_dup.log 2>&1
echo "probe rc=$?"; grep -h "rank" gpurun_out/r03/rccl_dup.log | tail -4
timeout -k 10 300 python bench.py --no-cpu-baseline --no-drop-in > gpurun_out/r03/bench_n1.json 2> gpurun_out/r03/bench_n1.err
rc=$?; cat gpurun_out/r03/bench_n1.json | cut -c1-600; exit $rc
