#!/bin/bash
# Round 6, forty-second call: the N > 1 step path at world 1 on the final tree
# (the per-GPU shard of configs[3] at N = 8 and N = 1): xGMI and RCCL exchange
# bench lines at 125k and 1M hosts, and a rocprofv3 kernel trace of the 125k
# xGMI run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g42}
mkdir -p $O
port=29851
for hx in 125000:xgmi 125000:rccl 1000000:xgmi 1000000:rccl; do
  h=${hx%%:*}; x=${hx##*:}; port=$((port+1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --dist --hosts $h --steps 200 --warmup 10 --exchange $x > $O/d_${h}_$x.log 2>&1 || { tail -20 $O/d_${h}_$x.log; exit 6; }
  python - <<PY
import json
d = json.loads(open('$O/d_${h}_$x.log').read().strip().splitlines()[-1])
print('dist $h $x', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0]) if v},
      d['config'].get('exchange'), d.get('parity', {}).get('match'))
PY
done
port=$((port+1))
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port $port bench.py --gpus 1 --dist --hosts 125000 --steps 200 --warmup 10 --exchange xgmi > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 7; }
find $O/kt -name "*kernel_stats.csv" | head -2
