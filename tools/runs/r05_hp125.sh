#!/bin/bash
# World-1 xGMI step: k_proc's header ticket in two levels (libshadowgpu_kt8.so)
# against the default at 125k and 1M hosts, and SG_HP partition sizes at 125k,
# interleaved; multi-shard GPU tests on the kt8 build first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/hp125; mkdir -p $out
SG_LIB=libshadowgpu_kt8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_sharded.py tests/test_gpu_dist.py > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc = 0 ] || exit $rc
port=29800
run() {  # name hosts env...
  local name=$1 h=$2; shift 2; port=$((port+1))
  env "$@" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts $h --steps 200 --warmup 10 > $out/d${h}_$name.log 2>&1 || { tail -20 $out/d${h}_$name.log; exit 1; }
  python -c "import json;d=json.loads(open('$out/d${h}_$name.log').read().strip().splitlines()[-1]);print('dist $h $name', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step')"
}
for r in a b; do
  run base$r 125000 SG_X=0
  run kt8$r 125000 SG_LIB=libshadowgpu_kt8.so
  run hp1024$r 125000 SG_HP=1024
  run hp1536$r 125000 SG_HP=1536
done
for r in a b; do
  run base$r 1000000 SG_X=0
  run kt8$r 1000000 SG_LIB=libshadowgpu_kt8.so
done
