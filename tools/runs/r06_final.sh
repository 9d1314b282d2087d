#!/bin/bash
# Round 6 final tree: the GPU suite, the smoke, then the bench lines with CPU
# baselines and the drop-in policy: the driver's own command (configs[3],
# --steps 20 --warmup 5), then each workload's default run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06final3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
show() {
  python -c "import json;d=json.load(open('$1'));c=d['cpu_baseline'];print('$2 %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], 'traffic', d['roofline'].get('traffic'), 'cpu %.3g x%s'%(c['value'], c['cores']), 'dropin %.3g'%d.get('drop_in_policy',{}).get('value',0), d['parity']['match'])"
}
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c4_driver.json 2> $O/bench_c4_driver.err || { tail $O/bench_c4_driver.err; exit 3; }
show $O/bench_c4_driver.json "c4 driver"
for wl in c4 c2 c5; do
  timeout -k 10 400 python -u bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail $O/bench_$wl.err; exit 4; }
  show $O/bench_$wl.json $wl
done
