#!/bin/bash
# Round 5, first GPU pass: the new / changed GPU tests, the split step against
# the unsplit one on the world-1 RCCL path (125k and 1M hosts), and the c2 / c5
# bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/g2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  ${TESTS:-tests/test_gpu_sharded.py tests/test_gpu_gspec.py tests/test_gpu_policy.py tests/test_gpu_dist.py} \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
port=29581
for hosts in 125000 1000000; do
  for split in 1 0 1 0; do
    port=$((port+1))
    SG_SPLIT=$split timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 \
      > $O/d_${hosts}_s$split.log 2>&1 || { tail -20 $O/d_${hosts}_s$split.log; exit 2; }
    python - <<PY
import json
d = json.loads(open('$O/d_${hosts}_s$split.log').read().strip().splitlines()[-1])
print('dist $hosts split $split', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      d['config']['drain_steps'], 'drains', {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0])},
      'parity', d['parity'].get('match'))
PY
  done
done
timeout -k 10 300 python -u bench.py --workload c2 > $O/c2.json 2> $O/c2.err || { tail $O/c2.err; exit 3; }
timeout -k 10 400 python -u bench.py --workload c5 > $O/c5.json 2> $O/c5.err || { tail $O/c5.err; exit 4; }
echo done
