#!/bin/bash
# Round 5: hosts per partition for the small shards of the N > 1 step (the
# 2048-host floor was chosen in round 4 for the RCCL step): world-1 xGMI steps
# at 125k / 250k / 500k hosts with SG_HP overrides, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g13}
mkdir -p $O
port=29781
for hosts in 125000 250000 500000; do
  for hp in 0 1024 512 0 1024 512; do
    port=$((port+1))
    SG_HP=$hp timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 \
      > $O/d_${hosts}_hp$hp.log 2>&1 || { tail -20 $O/d_${hosts}_hp$hp.log; exit 2; }
    python - <<PY
import json
d = json.loads(open('$O/d_${hosts}_hp$hp.log').read().strip().splitlines()[-1])
print('dist $hosts hp $hp', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0]) if v},
      'parity', d['parity'].get('match'))
PY
  done
done
