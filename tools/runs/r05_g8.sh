#!/bin/bash
# Round 5: the xGMI exchange without the system-scope fence (SG_XFENCE=0: the
# blocks are uncached, a store's acknowledgement orders it) against the fence
# and RCCL at world 1, the arrival wait folded into the round-state load, and
# configs[4] with partitions sized for gossip (no 2048-host floor) against the
# old floor.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g8}
mkdir -p $O
for f in 1 0; do
  SG_XFENCE=$f timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_sharded.py -k xlink tests/test_gpu_dist.py > $O/pytest_f$f.log 2>&1 || { tail -40 $O/pytest_f$f.log; exit 1; }
  tail -1 $O/pytest_f$f.log
done
port=29681
for hosts in 125000 1000000; do
  for x in xgmi_f1 xgmi_f0 rccl xgmi_f1 xgmi_f0 rccl; do
    port=$((port+1))
    ex=${x%%_*}; fe=${x##*_f}; [ $x = rccl ] && fe=1
    SG_XFENCE=$fe timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 --exchange $ex \
      > $O/d_${hosts}_$x.log 2>&1 || { tail -20 $O/d_${hosts}_$x.log; exit 2; }
    python - <<PY
import json
d = json.loads(open('$O/d_${hosts}_$x.log').read().strip().splitlines()[-1])
print('dist $hosts $x', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0]) if v},
      'parity', d['parity'].get('match'))
PY
  done
done
for hp in 0 2048 800 0; do
  SG_HP=$hp timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_hp$hp.json 2> $O/c5_hp$hp.err || { tail $O/c5_hp$hp.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_hp$hp.json'));print('c5 hp $hp %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
