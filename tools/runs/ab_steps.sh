#!/bin/bash
# A/B of the step loops on the GPU box: the new GPU tests, the 1-GPU round
# bench eager vs hipGraph, and world-1 RCCL runs of the multi-rank path
# (python steps / native steps / native + graph) at 1M and 125k hosts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread -k "native or graph" > gpurun_out/ab/pytest_new.log 2>&1
rc=$?; tail -3 gpurun_out/ab/pytest_new.log; [ $rc = 0 ] || exit $rc
for g in 0 32; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in --graph $g > gpurun_out/ab/single_g$g.json 2> gpurun_out/ab/single_g$g.err || { tail -5 gpurun_out/ab/single_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/single_g$g.json'));print('single graph=$g', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/round')"
done
port=29541
for hosts in 1000000 125000; do
  for v in "py:--py-steps" "native:--graph 0" "graph:--graph 16"; do
    name=${v%%:*}; a=${v#*:}; port=$((port+1))
    timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
      bench.py --gpus 1 --dist --hosts $hosts --steps 200 --warmup 10 $a > gpurun_out/ab/d_${hosts}_$name.log 2>&1 || { tail -20 gpurun_out/ab/d_${hosts}_$name.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab/d_${hosts}_$name.log').read().strip().splitlines()[-1]);print('dist $hosts $name', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step')"
  done
done
