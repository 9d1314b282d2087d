#!/bin/bash
# The default bench line (with the CPU baseline and the drop-in policy legs),
# then the world-1 RCCL step path at 125k and 1M hosts with a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/final
timeout -k 10 400 python bench.py > gpurun_out/final/bench_n1.json 2> gpurun_out/final/bench_n1.err || { tail -5 gpurun_out/final/bench_n1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final/bench_n1.json'));print('value %.4g'%d['value'], round(d['ms_per_step']*1e3,2),'us/round', d['cpu_baseline']['value'], d['drop_in_policy']['value'], d['parity']['match'])"
bash tools/steps_check.sh
