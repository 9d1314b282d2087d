#!/bin/bash
# Round-end evidence: GPU suite, the default bench line (CPU baseline and the
# drop-in policy legs included), the world-1 RCCL step path, the rocprofv3
# kernel-trace and PMC passes with their summary, and stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/final/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/final/bench_n1.json 2> gpurun_out/final/bench_n1.err || { tail -5 gpurun_out/final/bench_n1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final/bench_n1.json'));print('value %.4g'%d['value'], round(d['ms_per_step']*1e3,2),'us/round', d['cpu_baseline']['value'], d['drop_in_policy']['value'], d['parity']['match'])"
port=29581
for hosts in 125000 1000000; do
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 > gpurun_out/final/d_$hosts.log 2>&1 || { tail -20 gpurun_out/final/d_$hosts.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/final/d_$hosts.log').read().strip().splitlines()[-1]);print('dist $hosts', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step', d['per_rank_us_per_step']['rows'][0])"
done
bash tools/profile.sh > gpurun_out/final/profile.log 2>&1 || { tail -5 gpurun_out/final/profile.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof 40 gpurun_out/prof/pmc.json > gpurun_out/prof/summary.txt && head -12 gpurun_out/prof/summary.txt
timeout -k 10 120 python tools/stamps.py > gpurun_out/final/stamps.log 2>&1 && grep -E "kernel span|k_scatter|insert  |gather  " gpurun_out/final/stamps.log | head -4
