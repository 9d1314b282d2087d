#!/bin/bash
# Round 5: hipGraph replay of the configs[3] bench's timed rounds (batches of
# 25 / 50 / 100 / 200) against eager launches, interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g15}
mkdir -p $O
for rep in 1 2; do
  for g in 0 50 100 200 25; do
    timeout -k 10 300 python -u bench.py --graph $g --no-cpu-baseline --no-drop-in > $O/c4_g${g}_$rep.json 2> $O/c4_g${g}_$rep.err || { tail $O/c4_g${g}_$rep.err; exit 3; }
    python -c "import json;d=json.load(open('$O/c4_g${g}_$rep.json'));print('graph $g %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
