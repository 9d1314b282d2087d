set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || exit $?; tail -8 gpurun_out/stamps.log
bash tools/rccl1.sh || exit $?
bash tools/profile.sh > gpurun_out/profile.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof 40 gpurun_out/prof/pmc.json > gpurun_out/prof/summary.txt && cat gpurun_out/prof/summary.txt
