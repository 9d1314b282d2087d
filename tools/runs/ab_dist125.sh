#!/bin/bash
# World-1 RCCL step path at HOSTS (default 125k) hosts under different engine env settings:
# each argument is NAME:ENV=V,ENV=V (as tools/runs/variants.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab125
port=29611
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}; port=$((port+1))
  env ${envs//,/ } timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts ${HOSTS:-125000} --steps 200 --warmup 10 > gpurun_out/ab125/$name.log 2>&1 || { tail -20 gpurun_out/ab125/$name.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab125/$name.log').read().strip().splitlines()[-1]);print('$name', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step')"
done
