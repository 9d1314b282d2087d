#!/bin/bash
# Mode P: GPU policy tests, then a kernel trace of the gpu policy at 1M hosts
# with 16 workers (the calendar insert, extraction and MIN kernels) and the
# serial-section split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/modep
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_configs.py -k "policy" -x -q --timeout 200 --timeout-method thread > gpurun_out/modep/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/modep/pytest.log; [ $rc = 0 ] || exit $rc
SG_POLICY_PROF=1 WORKERS=16 KINDS=gpu,steal timeout -k 10 300 python tools/modep_scan.py > gpurun_out/modep/scan.log 2>&1 || exit $?
cat gpurun_out/modep/scan.log
SG_POLICY_PROF=1 WORKERS=16 KINDS=gpu timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/modep/kt -o kt --output-format csv -- python tools/modep_scan.py > gpurun_out/modep/kt.log 2>&1 || exit $?
tail -3 gpurun_out/modep/kt.log
f=$(find gpurun_out/modep/kt -name "*kernel_stats.csv" | head -1); head -12 "$f"
