#!/bin/bash
# World-1 RCCL step path (the N>1 bench path) at 125k and 1M hosts, then a
# kernel trace of the 125k case (tools/prof_steps.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/steps
port=29581
for hosts in 125000 1000000; do
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 > gpurun_out/steps/d_$hosts.log 2>&1 || { tail -20 gpurun_out/steps/d_$hosts.log; exit 1; }
  python - <<PY
import json
d = json.loads(open('gpurun_out/steps/d_$hosts.log').read().strip().splitlines()[-1])
print('dist $hosts', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step', d['config']['step_loop'],
      d['config']['drain_steps'], 'drains', {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0])},
      'parity', d['parity'].get('match'))
PY
done
PORT=29599 HOSTS=125000 bash tools/prof_steps.sh
