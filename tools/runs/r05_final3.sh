#!/bin/bash
# Round 5, final tree after XS=2 + TICK8: the GPU suite, the smoke, the full
# bench lines (CPU baselines, drop-in policy), then rocprofv3 kernel trace + PMC
# passes of each workload's bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/final3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
for wl in c4 c2 c5; do
  timeout -k 10 400 python -u bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail $O/bench_$wl.err; exit 3; }
  python -c "import json;d=json.load(open('$O/bench_$wl.json'));print('$wl %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], 'cpu %.3g'%d['cpu_baseline']['value'], 'plain %.3g'%d['cpu_baseline'].get('plain_heap_value',0), 'dropin %.3g'%d.get('drop_in_policy',{}).get('value',0), d['parity']['match'])"
done
for wl in c4 c2 c5; do
  OUT=$O/prof_$wl PROF_ARGS="--workload $wl --no-cpu-baseline --no-drop-in" bash tools/profile.sh > $O/prof_$wl.log 2>&1 || { tail $O/prof_$wl.log; exit 4; }
  python tools/prof_summary.py $O/prof_$wl 40 $O/prof_$wl/pmc.json > $O/prof_$wl/summary.txt
  echo "== $wl"; grep -E "steady|k_proc|k_scatter" $O/prof_$wl/summary.txt | head -8
done
