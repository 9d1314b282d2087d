#!/bin/bash
# Round 5: gossip record path drawing after phase A (SG_SKIP=1) with the
# null-draw redraw, against phase A's draws (SG_SKIP=0): gossip parity (incl. a
# fifth of the draws selecting no host), c5 fixtures, two-process c5, then c5
# interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g20}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gossip or skip" \
  tests/test_gpu_configs.py tests/test_gpu_dist.py -k "gossip or c5 or skip" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sk in 0 1 0 1; do
  SG_SKIP=$sk timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_s$sk.json 2> $O/c5_s$sk.err || { tail $O/c5_s$sk.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_s$sk.json'));print('c5 skip $sk %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
