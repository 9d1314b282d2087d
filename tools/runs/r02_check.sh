#!/bin/bash
# GPU tests (verbose, durations), then a short bench with the parity check.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 ${PYTEST_ARGS:-} > gpurun_out/r02/pytest.log 2>&1
rc=$?; tail -30 gpurun_out/r02/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-drop-in > gpurun_out/r02/bench.json 2> gpurun_out/r02/bench.err
rc=$?; cat gpurun_out/r02/bench.json; tail -3 gpurun_out/r02/bench.err; exit $rc
