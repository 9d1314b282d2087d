#!/bin/bash
# A/B of engine switches on the GPU box: GPU tests, then one bench per
# variant ("NAME:ENV=V,ENV=V" arguments), then stamps for the first variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/pytest.log; [ $rc = 0 ] || exit $rc
fi
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  env ${envs//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > gpurun_out/ab/bench_$name.log 2>&1 || { tail -5 gpurun_out/ab/bench_$name.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/bench_$name.log'));print('$name value %.4g'%d['value'], {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()})"
done
if [ -n "$STAMPS" ]; then
  env ${STAMPS//,/ } timeout -k 10 120 python tools/stamps.py > gpurun_out/ab/stamps.log 2>&1 || exit 1
  tail -18 gpurun_out/ab/stamps.log
fi
