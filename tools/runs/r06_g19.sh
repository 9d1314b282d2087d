#!/bin/bash
# Round 6, nineteenth call: the row reset from the round state in registers (g18: scalar
# loads of it, c5 k_proc +2 us?); parity tests and the bench lines twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g19}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for wl in c5 c4 c2 c5 c4 c2; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/$wl.json 2> $O/$wl.err || { tail $O/$wl.err; exit 3; }
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
