#!/bin/bash
# Round 6, thirty-ninth call: the new send-records-in-HBM parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g39}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "send_records_in_hbm or gossip or lossy" \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 12 $O/pytest.log
