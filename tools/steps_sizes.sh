#!/bin/bash
# GPU suite, then the world-1 RCCL step path at the per-GPU sizes of configs[3]
# on 8, 4, 2 and 1 GPUs (125k, 250k, 500k, 1M hosts).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sizes
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sizes/pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/sizes/pytest.log; [ $rc = 0 ] || exit $rc
fi
port=29621
for hosts in 125000 250000 500000 1000000; do
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 > gpurun_out/sizes/d_$hosts.log 2>&1 || { tail -20 gpurun_out/sizes/d_$hosts.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sizes/d_$hosts.log').read().strip().splitlines()[-1]);print('dist $hosts', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step', [round(x,2) for x in d['per_rank_us_per_step']['rows'][0]])"
done
