#!/bin/bash
# Round time of the N=1 bench with hipGraph batches of G rounds (0: plain
# launches), interleaved; the first timed batch replays a graph captured after
# the warmup (sg_engine_graph_prepare).  Usage: tools/runs/graph_ab.sh [STEPS WARMUP]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
steps=${1:-200}; warm=${2:-20}
mkdir -p gpurun_out/gab
for r in 1 2; do
  for g in ${GS:-0 10 20 40 100}; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in --steps $steps --warmup $warm --graph $g > gpurun_out/gab/b_${steps}_${g}_$r.json 2> gpurun_out/gab/b_${steps}_${g}_$r.err || { tail -5 gpurun_out/gab/b_${steps}_${g}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/gab/b_${steps}_${g}_$r.json'));print('steps $steps graph $g', '%.4g'%d['value'], round(d['ms_per_step']*1e3,2),'us/round', d.get('parity',{}).get('match'))"
  done
done
