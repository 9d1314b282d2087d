#!/bin/bash
# Round 6, eighteenth call: each k_proc workgroup resets its own row of bucket
# minima (nb * P stores in one workgroup before); the GPU suite and
# the three bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g18}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for wl in c4 c2 c5; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/$wl.json 2> $O/$wl.err || { tail $O/$wl.err; exit 3; }
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
