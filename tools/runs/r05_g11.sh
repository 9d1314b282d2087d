#!/bin/bash
# Round 5: kernel durations of c2 / c5 from a replaying engine (the timed region
# carries no events): the bench tests, then inline against replay lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g11}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for wl in c2 c5; do
  for kt in inline replay inline replay; do
    timeout -k 10 300 python -u bench.py --workload $wl --kernel-timing $kt --no-cpu-baseline --no-drop-in > $O/${wl}_$kt.json 2> $O/${wl}_$kt.err || { tail $O/${wl}_$kt.err; exit 3; }
    python -c "import json;d=json.load(open('$O/${wl}_$kt.json'));print('$wl $kt %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'gaps %.1f'%d['roofline']['gaps_us_per_round'], d['parity']['match'])"
  done
done
