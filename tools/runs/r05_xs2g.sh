#!/bin/bash
# Two bucket sub-lists (SG_XS=2) with the GSpec guess extended to both:
# GSpec / config parity tests on the variant library, then an interleaved A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/xs2g
SG_LIB=libshadowgpu_xs2g.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_gspec.py tests/test_gpu_configs.py tests/test_gpu_parity.py > gpurun_out/xs2g/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/xs2g/pytest.log; [ $rc = 0 ] || exit $rc
NO_TESTS=1 bash tools/runs/ab.sh base:SG_X=0 xs2:SG_LIB=libshadowgpu_xs2.so xs2g:SG_LIB=libshadowgpu_xs2g.so \
  base2:SG_X=0 xs2g2:SG_LIB=libshadowgpu_xs2g.so xs2b:SG_LIB=libshadowgpu_xs2.so
