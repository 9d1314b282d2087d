#!/bin/bash
# GPU tests, then the multi-shard tests again with SG_CHECK=1: every step the
# plan re-derives the MIN terms k_proc's last workgroup put in the headers from
# the workgroups' plain partials, and a mismatch is an OV_BUG overflow.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/chk2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk2/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/chk2/pytest.log; [ $rc = 0 ] || exit $rc
SG_CHECK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "shard or rccl or eight" > gpurun_out/chk2/pytest_check.log 2>&1
rc=$?; tail -2 gpurun_out/chk2/pytest_check.log; exit $rc
