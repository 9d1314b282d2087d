#!/bin/bash
# The bench line (no CPU legs) with eager launches and hipGraph batches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/graph
for g in 0 20 40 100 0; do
  SG_GRAPH=$g timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > gpurun_out/graph/b_$g.json 2> gpurun_out/graph/b_$g.err || { tail -5 gpurun_out/graph/b_$g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/graph/b_$g.json'));print('graph $g', '%.4g'%d['value'], round(d['ms_per_step']*1e3,2),'us/round', d['parity']['match'], d['config']['round_loop'])"
done
