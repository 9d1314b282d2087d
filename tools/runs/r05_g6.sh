#!/bin/bash
# Round 5: the xGMI peer exchange (sg_xlink).  Its GPU tests, then the world-1
# step with the block exchanged by k_xpush / k_xwait against the RCCL
# all-to-all (125k and 1M hosts, interleaved), a 2-rank same-device bench over
# the link, and configs[3] stamps with the per-XCD breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g6}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  ${TESTS:-tests/test_gpu_sharded.py tests/test_gpu_dist.py} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
port=29581
for hosts in 125000 1000000; do
  for x in ${VARIANTS:-xgmi xgmi0 rccl xgmi xgmi0 rccl}; do
    port=$((port+1))
    ex=$x; fu=1; [ $x = xgmi0 ] && { ex=xgmi; fu=0; }
    SG_XFUSE=$fu timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 --exchange $ex \
      > $O/d_${hosts}_$x.log 2>&1 || { tail -20 $O/d_${hosts}_$x.log; exit 2; }
    python - <<PY
import json
d = json.loads(open('$O/d_${hosts}_$x.log').read().strip().splitlines()[-1])
print('dist $hosts $x', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      d['config']['drain_steps'], 'drains', {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0])},
      'parity', d['parity'].get('match'), d['config']['exchange'])
PY
  done
done
timeout -k 10 300 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 100 --warmup 10 \
  > $O/two_xgmi.log 2>&1 || { tail -20 $O/two_xgmi.log; exit 3; }
python -c "import json;d=json.loads(open('$O/two_xgmi.log').read().strip().splitlines()[-1]);print('2 ranks same device', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', d['config']['exchange'], d['parity']['match'])"
timeout -k 10 200 python tools/stamps.py > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 4; }
grep -A9 "per XCD" $O/stamps.txt | head -24
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 200 python tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 5; }
head -30 $O/stamps_c5.txt
