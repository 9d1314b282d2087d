#!/bin/bash
# GPU suite + world-1 RCCL step path + one bench line (tools/runs/gpu_check.sh),
# then the rocprofv3 kernel-trace pass and the PMC passes (tools/profile.sh)
# and their summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/runs/gpu_check.sh || exit $?
bash tools/profile.sh || exit $?
python tools/prof_summary.py gpurun_out/prof 40 gpurun_out/prof/pmc.json > gpurun_out/prof/summary.txt && cat gpurun_out/prof/summary.txt | head -40
