#!/bin/bash
# Final measurement pass: rocprof kernel trace + PMC passes, the full bench
# line, the world-1 step path, and stamps at 1M and 125k hosts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/profile.sh > gpurun_out/profile.log 2>&1 || { tail -5 gpurun_out/profile.log; exit 1; }
grep "rc=" gpurun_out/profile.log
bash tools/runs/final_check.sh || exit 1
NO_TESTS=1 bash tools/runs/r02b_check.sh > /dev/null 2>&1 || exit 1
head -3 gpurun_out/r02b/stamps_1m.log
