#!/bin/bash
# World-1 step path at 250k and 500k hosts for two partition sizes each, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/hp2
port=29641
for rep in 1 2; do
  for cfg in "250000 0" "250000 2048" "500000 0" "500000 3907"; do
    set -- $cfg; hosts=$1; hp=$2; port=$((port+1))
    SG_HP=$hp timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
      bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 > gpurun_out/hp2/d_${hosts}_${hp}_$rep.log 2>&1 || { tail -20 gpurun_out/hp2/d_${hosts}_${hp}_$rep.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/hp2/d_${hosts}_${hp}_$rep.log').read().strip().splitlines()[-1]);print('hosts $hosts SG_HP=$hp', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step', [round(x,2) for x in d['per_rank_us_per_step']['rows'][0]])"
  done
done
