#!/bin/bash
# Round 6, second call: the cross-GPU form of the xGMI exchange as
# system-coherent stores (sc0 sc1) of every handed-off row and header, drained
# before each ticket / arrival, in place of a per-wave system release; the
# xGMI tests forced fenced and unfenced; the world-1 step at 125k and 1M hosts
# fenced / unfenced / RCCL; then configs[3]'s bench with the CPU baseline at
# the box's share and at every CPU of the affinity set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for f in 1; do
  SG_XFENCE=$f timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_sharded.py -k xlink tests/test_gpu_dist.py > $O/pytest_f$f.log 2>&1 || { tail -40 $O/pytest_f$f.log; exit 1; }
  tail -n 1 $O/pytest_f$f.log
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
      'parity', d['parity'].get('match'), d['config'].get('xlink', {}).get('fenced'))
PY
  done
done
/usr/bin/time -v timeout -k 10 600 python -u bench.py --no-drop-in > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 3; }
grep -E "Elapsed|Maximum resident" $O/bench_c4.err
python -c "import json;d=json.load(open('$O/bench_c4.json'));c=d['cpu_baseline'];print('c4 %.4g'%d['value'], round(d['ms_per_step']*1e3,2), d['parity']['match'], {k:c[k] for k in ('value','cores','share_value','share_workers','all_cpus_value','all_cpus_workers','single_thread_value','plain_heap_value','nproc','affinity','cgroup_cpus')})"
