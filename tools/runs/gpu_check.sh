#!/bin/bash
# GPU tests, then world-1 RCCL dist bench (native steps) at 125k and 1M hosts
# and the 1-GPU bench without the CPU baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/chk
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chk/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/chk/pytest.log; [ $rc = 0 ] || exit $rc
port=29571
for hosts in 125000 1000000; do
  port=$((port+1))
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 > gpurun_out/chk/d_$hosts.log 2>&1 || { tail -20 gpurun_out/chk/d_$hosts.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/chk/d_$hosts.log').read().strip().splitlines()[-1]);print('dist $hosts', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step')"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > gpurun_out/chk/single.json 2> gpurun_out/chk/single.err || { tail -5 gpurun_out/chk/single.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/chk/single.json'));print('single', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/round', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()})"
