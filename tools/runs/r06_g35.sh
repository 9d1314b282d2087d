#!/bin/bash
# Round 6, thirty-fifth call: bisecting configs[3] within the first gossip commits
# (C..E of g34) and HEAD with the path rows through registers (L0), on one box (_bis/, not
# committed), the driver's command each, in order and then in reverse.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g35}
mkdir -p $O
R=$PWD
for n in C D1 D2 D3 E L L0 L0 L E D3 D2 D1 C; do
  (cd $R/_bis/$n && timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-drop-in) > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 3; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
