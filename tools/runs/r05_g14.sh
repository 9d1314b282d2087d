#!/bin/bash
# Round 5: step_view reading the G block headers by readlane (G <= 8): the
# multi-rank GPU tests, then world-1 xGMI steps at 125k and 1M hosts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g14}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py \
  tests/test_gpu_dist.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
port=29881
for hosts in 125000 1000000 125000 1000000; do
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 > $O/d_$hosts.log 2>&1 || { tail -20 $O/d_$hosts.log; exit 2; }
  python - <<PY
import json
d = json.loads(open('$O/d_$hosts.log').read().strip().splitlines()[-1])
print('dist $hosts', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0]) if v},
      'parity', d['parity'].get('match'), d['config']['exchange'])
PY
done
