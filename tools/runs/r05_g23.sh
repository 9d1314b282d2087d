#!/bin/bash
# Round 5: the xGMI arrival fenced across devices by default (SG_XFENCE unset:
# unfenced on one device): the sharded and multi-rank tests, incl. the fenced
# two-process run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g23}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py \
  tests/test_gpu_dist.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
