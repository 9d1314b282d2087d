#!/bin/bash
# Round 6, seventh call: configs[4] stamps with non-waiting stamps through the
# gossip flat pass's passes and barriers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g7}
mkdir -p $O
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 5; }
head -n 14 $O/stamps_c5.txt
