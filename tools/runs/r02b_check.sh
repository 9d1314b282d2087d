#!/bin/bash
# GPU tests (quiet), a short bench, then in-kernel stamps at 1M and 125k hosts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/r02b
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/r02b/pytest.log; [ $rc = 0 ] || exit $rc
fi
timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > gpurun_out/r02b/bench.json 2> gpurun_out/r02b/bench.err || { tail -5 gpurun_out/r02b/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02b/bench.json'));print('value %.4g'%d['value'], round(d['ms_per_step']*1e3,2),'us/round', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'parity', d['parity']['match'])"
timeout -k 10 120 python tools/stamps.py > gpurun_out/r02b/stamps_1m.log 2>&1 || { tail -5 gpurun_out/r02b/stamps_1m.log; exit 1; }
head -24 gpurun_out/r02b/stamps_1m.log
timeout -k 10 120 python tools/stamps.py 125000 > gpurun_out/r02b/stamps_125k.log 2>&1 || { tail -5 gpurun_out/r02b/stamps_125k.log; exit 1; }
head -24 gpurun_out/r02b/stamps_125k.log
