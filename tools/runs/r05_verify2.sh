#!/bin/bash
# The tree after XS=2 + TICK8: GPU suite, then the default bench line and
# in-kernel stamps of configs[3] (phase breakdown for the next change).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/v2; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > $out/c4.json 2> $out/c4.err || { tail -5 $out/c4.err; exit 1; }
python -c "import json;d=json.load(open('$out/c4.json'));print('c4 %.4g'%d['value'], round(d['ms_per_step']*1e3,2), {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
timeout -k 10 150 python tools/stamps.py > $out/stamps.txt 2>&1 || { tail -5 $out/stamps.txt; exit 1; }
head -40 $out/stamps.txt
