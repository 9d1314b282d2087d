#!/bin/bash
# Round 6, second call, on the pruned tree (split step, SG_NT, SG_ABL,
# SG_SORT_LDS, SG_PART_LATE, partition halves removed) with the gossip flat
# pass (one lane per receipt, SG_GFLAT=1):
#  1. the xGMI tests forced fenced (system-coherent sc0 sc1 peer stores);
#  2. the world-1 step at 125k hosts fenced / unfenced / RCCL, 1M fenced / unfenced;
#  3. configs[4] bench, gossip flat pass off / on, interleaved, then its stamps;
#  4. the whole GPU suite;
#  5. configs[3]'s bench with the CPU baseline at the share and at every CPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g2}
mkdir -p $O
SG_XFENCE=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_sharded.py -k xlink tests/test_gpu_dist.py > $O/pytest_f1.log 2>&1 || { tail -40 $O/pytest_f1.log; exit 1; }
tail -n 1 $O/pytest_f1.log
port=29681
for run in 125000:xgmi_f1 125000:xgmi_f0 125000:rccl 125000:xgmi_f1 125000:xgmi_f0 125000:rccl 1000000:xgmi_f1 1000000:xgmi_f0; do
  hosts=${run%%:*}; x=${run##*:}
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
for v in 0 1 0 1; do
  SG_GFLAT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_gflat$v.json 2> $O/c5_gflat$v.err || { tail $O/c5_gflat$v.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_gflat$v.json'));print('c5 gflat $v %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], d['parity']['match'])"
done
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 4; }
head -n 12 $O/stamps_c5.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 5; }
tail -n 2 $O/pytest.log
/usr/bin/time -v timeout -k 10 600 python -u bench.py --no-drop-in > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 6; }
grep -E "Elapsed|Maximum resident" $O/bench_c4.err
python -c "import json;d=json.load(open('$O/bench_c4.json'));c=d['cpu_baseline'];print('c4 %.4g'%d['value'], round(d['ms_per_step']*1e3,2), d['parity']['match'], {k:c[k] for k in ('value','cores','share_value','share_workers','all_cpus_value','all_cpus_workers','single_thread_value','plain_heap_value','nproc','affinity','cgroup_cpus')})"
