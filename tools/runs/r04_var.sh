#!/bin/bash
# For each variant library: the configs[3] per-round parity test against it,
# then interleaved round times against the working tree's library.
# Usage: tools/runs/r04_var.sh v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/var
for v in "$@"; do
  SG_LIB=libshadowgpu_$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_configs.py -x -q -k c4_1m_bench --timeout 120 --timeout-method thread > gpurun_out/var/pytest_$v.log 2>&1
  rc=$?; echo "$v parity: $(tail -1 gpurun_out/var/pytest_$v.log)"; [ $rc = 0 ] || exit $rc
done
REPS=${REPS:-3} bash tools/runs/qt_ab.sh ${REPS:-3} "$@"
