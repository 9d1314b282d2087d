#!/bin/bash
# Round 6, fortieth call: the whole GPU suite and the smoke on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g40}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
tail -n 1 $O/smoke.log
