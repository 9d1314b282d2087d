#!/bin/bash
# Round 6, twenty-fifth call: k_scatter's gather grid (SG_GATHER_GRID, runtime;
# default 128) at 96 / 128 / 192 / 256 workgroups, interleaved on configs[3] and
# configs[4].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g25}
mkdir -p $O
for wl in c4 c5; do
  for g in 128 192 256 96 128 192 256 96; do
    SG_GATHER_GRID=$g timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/${wl}_g$g.json 2> $O/${wl}_g$g.err || { tail $O/${wl}_g$g.err; exit 3; }
    python -c "import json;d=json.load(open('$O/${wl}_g$g.json'));print('$wl G1=$g %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
