#!/bin/bash
# GPU suite, then a gather-grid knob scan (bench lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/it
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/it/pytest.log; [ $rc = 0 ] || exit $rc
bash tools/runs/knob_scan.sh "SG_GATHER_GRID=128" "SG_GATHER_GRID=96" "SG_GATHER_GRID=160" "SG_GATHER_GRID=192" "SG_GATHER_GRID=256" "SG_GATHER_GRID=128" "SG_GATHER_GRID=96" "SG_GATHER_GRID=160" "SG_GATHER_GRID=192" "SG_GATHER_GRID=256"
