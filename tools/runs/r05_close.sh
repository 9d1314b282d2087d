#!/bin/bash
# Round 5 close: the committed tree's GPU suite, the smoke and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/close; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 2; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 3; }
python -c "import json;d=json.load(open('$out/bench.json'));print('c4 %.4g'%d['value'], round(d['ms_per_step']*1e3,2), {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], d['roofline']['traffic_source'], d['parity']['match'])"
