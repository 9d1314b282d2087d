#!/bin/bash
# Round 5: rocprofv3 kernel trace + PMC passes for configs[1] and configs[4]
# (bench.py --workload c2 / c5) and for the drop-in policy's device half at 1M
# hosts / 16 workers (tools/modep_scan.py), each summarised per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for wl in ${WLS:-c2 c5}; do
  OUT=gpurun_out/prof_$wl PROF_ARGS="--workload $wl --no-cpu-baseline --no-drop-in" bash tools/profile.sh || exit $?
  python tools/prof_summary.py gpurun_out/prof_$wl 40 gpurun_out/prof_$wl/pmc.json > gpurun_out/prof_$wl/summary.txt
  cat gpurun_out/prof_$wl/summary.txt
done
if [ -z "$NO_MODEP" ]; then
  OUT=gpurun_out/prof_modep PROF_CMD="python tools/modep_scan.py" WORKERS=16 KINDS=gpu HOSTS=1000000 bash tools/profile.sh || exit $?
  python tools/prof_summary.py gpurun_out/prof_modep 12 gpurun_out/prof_modep/pmc.json > gpurun_out/prof_modep/summary.txt
  cat gpurun_out/prof_modep/summary.txt
fi
