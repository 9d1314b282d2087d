#!/bin/bash
# k_scatter's gather grid (SG_GATHER_GRID) on the final tree, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/g1scan; mkdir -p $out
for r in a b; do
  for g in 128 112 160 192; do
    SG_GATHER_GRID=$g timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > $out/c4_$g$r.json 2> $out/c4_$g$r.err || { tail -5 $out/c4_$g$r.err; exit 1; }
    python -c "import json;d=json.load(open('$out/c4_$g$r.json'));print('G1 $g$r %.4g'%d['value'], round(d['ms_per_step']*1e3,2), {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
