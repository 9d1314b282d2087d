#!/bin/bash
# Round 6, twenty-eighth call: stamps of configs[1] (k_proc phases, k_scatter roles).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g28}
mkdir -p $O
STAMPS_WL=c2 STAMPS_AT=100 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c2.txt 2>&1 || { tail $O/stamps_c2.txt; exit 5; }
head -n 30 $O/stamps_c2.txt
