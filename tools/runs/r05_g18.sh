#!/bin/bash
# Round 5 (measurement): rand_r skip-ahead forced on (SG_SKIP=2) in the flat pass
# (c2, c4) and the gossip record path (c5) against the serial draws.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g18}
mkdir -p $O
for wl in c2 c5 c4; do
  for sk in 0 2 0 2; do
    SG_SKIP=$sk timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/${wl}_s$sk.json 2> $O/${wl}_s$sk.err || { tail $O/${wl}_s$sk.err; exit 3; }
    python -c "import json;d=json.load(open('$O/${wl}_s$sk.json'));print('$wl skip $sk %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
