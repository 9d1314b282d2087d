#!/bin/bash
# Round 6, twenty-sixth call: hosts per partition (SG_HP, runtime) on the world-1
# xGMI step at 125k hosts (one of eight shards of configs[3]): 512 / 1024 / 2048
# (default) / 4096, twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g26}
mkdir -p $O
port=29811
for hp in 2048 512 1024 4096 2048 512 1024 4096; do
  port=$((port+1))
  SG_HP=$hp timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --dist --hosts 125000 --steps 200 --warmup 10 --exchange xgmi > $O/d_hp$hp.log 2>&1 || { tail -20 $O/d_hp$hp.log; exit 6; }
  python - <<PY
import json
d = json.loads(open('$O/d_hp$hp.log').read().strip().splitlines()[-1])
print('HP $hp', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0]) if v})
PY
done
