#!/bin/bash
# Round 5: k_scatter's planning thread reading the round state by readlane
# (SG_RS_LANES=1) against the LDS copy (libshadowgpu_prev.so), interleaved, with
# the parity / gspec / sharded tests on the new build first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g12}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gspec.py tests/test_gpu_parity.py \
  tests/test_gpu_sharded.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for v in prev base; do
    lib=libshadowgpu.so; [ $v = base ] || lib=libshadowgpu_$v.so
    echo -n "$v: "
    SG_LIB=$lib timeout -k 10 120 python tools/quick_time.py 200 2>&1 | tail -1 || exit 2
  done
done
