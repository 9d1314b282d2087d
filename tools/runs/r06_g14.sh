#!/bin/bash
# Round 6, fourteenth call: k_scatter's prologue split by two more stamps (round
# state in, step planned): configs[3] stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g14}
mkdir -p $O
STAMPS_WL=c4 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c4.txt 2>&1 || { tail $O/stamps_c4.txt; exit 5; }
head -n 28 $O/stamps_c4.txt
