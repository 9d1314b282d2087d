#!/bin/bash
# Round 5: rocprofv3 kernel trace + PMC passes of the drop-in policy's device
# half (1M hosts, 16 workers, tools/modep_scan.py) and of the configs[3] bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
if [ -z "$NO_MODEP" ]; then
  OUT=gpurun_out/prof_modep PROF_CMD="python tools/modep_scan.py" KPROF=1 WORKERS=16 KINDS=gpu HOSTS=1000000 bash tools/profile.sh || exit $?
  python tools/prof_summary.py gpurun_out/prof_modep 12 gpurun_out/prof_modep/pmc.json > gpurun_out/prof_modep/summary.txt
  cat gpurun_out/prof_modep/summary.txt
fi
OUT=gpurun_out/prof_c4 bash tools/profile.sh || exit $?
python tools/prof_summary.py gpurun_out/prof_c4 40 gpurun_out/prof_c4/pmc.json > gpurun_out/prof_c4/summary.txt
cat gpurun_out/prof_c4/summary.txt
