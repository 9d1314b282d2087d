cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/wt
SG_LIB=libshadowgpu_wt.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wt/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/wt/pytest.log; [ $rc = 0 ] || exit $rc
NO_TESTS=1 STAMP_LIBS="libshadowgpu_wt.so" bash tools/r04_iter.sh wt
