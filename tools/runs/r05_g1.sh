set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gspec.py::test_ov_bug_guard_clamps_corrupt_staged_records tests/test_gpu_sharded.py::test_graph_prepare_runs_nothing_when_eager "tests/test_gpu_policy.py::test_gpu_policy_matches_oracle" tests/test_gpu_dist.py > gpurun_out/g1_pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c2 > gpurun_out/g1_c2.json 2> gpurun_out/g1_c2.err || exit 2
timeout -k 10 400 python -u bench.py --workload c5 > gpurun_out/g1_c5.json 2> gpurun_out/g1_c5.err || exit 3
