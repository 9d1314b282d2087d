#!/bin/bash
# Mode P A/B on one box: pinned vs pageable worker arenas, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for v in 1 0 1 0; do
  echo "SG_POLICY_PINNED=$v"
  SG_POLICY_PINNED=$v SG_POLICY_PROF=1 WORKERS=16 KINDS=gpu timeout -k 10 200 python tools/modep_scan.py 2>&1 | grep -E "gpu|serial" || exit 1
done
