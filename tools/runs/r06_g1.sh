#!/bin/bash
# Round 6, first call: the N > 1 exchange hardening (fail-fast waits, the fused
# self-test, a release by every storing workgroup when fenced, the drain
# step's arrival after its reads) through the whole GPU suite and the smoke,
# the default bench, the world-1 xGMI step at 125k hosts fenced / unfenced /
# RCCL, then the ptick8 variant (k_proc's two-level header ticket) on the
# two-process xGMI test that hung in round 5, now failing fast if it does.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g1}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-drop-in > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench_c4.json'));print('c4 %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], d['parity']['match'])"
port=29681
for x in xgmi_f1 xgmi_f0 rccl xgmi_f1 xgmi_f0 rccl; do
  port=$((port+1))
  ex=${x%%_*}; fe=${x##*_f}; [ $x = rccl ] && fe=1
  SG_XFENCE=$fe timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --dist --hosts 125000 --steps 200 --warmup 10 --exchange $ex \
    > $O/d_125k_$x.log 2>&1 || { tail -20 $O/d_125k_$x.log; exit 4; }
  python - <<PY
import json
d = json.loads(open('$O/d_125k_$x.log').read().strip().splitlines()[-1])
print('dist 125k $x', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0]) if v},
      'parity', d['parity'].get('match'), d['config'].get('xlink'))
PY
done
SG_LIB=libshadowgpu_ptick8.so timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_dist.py -k "test_c4_1m_two_processes and xgmi" > $O/ptick8.log 2>&1
echo "ptick8 rc $?"; tail -n 30 $O/ptick8.log
