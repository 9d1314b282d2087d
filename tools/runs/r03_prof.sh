#!/bin/bash
# Round 3 measurement call: the bench's rocprofv3 kernel trace + PMC passes over
# the bench's own default rounds (tools/profile.sh), summarised over the last
# 40 launches (the bench's kernel-timing rounds) into gpurun_out/prof.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/profile.sh || exit $?
python tools/prof_summary.py gpurun_out/prof 40 gpurun_out/prof/pmc.json > gpurun_out/prof/summary.txt || exit $?
cat gpurun_out/prof/summary.txt
