#!/bin/bash
# k_proc's partials after its reservations (SG_PART_LATE) and k_scatter's
# two-level plan ticket (SG_TICK8): parity tests on the combined build, then
# configs[3] benches and the 125k world-1 step, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/tick; mkdir -p $out
SG_LIB=libshadowgpu_both.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_gspec.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_dist.py > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc = 0 ] || exit $rc
for v in base:libshadowgpu.so plate:libshadowgpu_plate.so tick8:libshadowgpu_tick8.so both:libshadowgpu_both.so \
         base2:libshadowgpu.so plate2:libshadowgpu_plate.so tick8b:libshadowgpu_tick8.so both2:libshadowgpu_both.so; do
  name=${v%%:*}; lib=${v#*:}
  SG_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > $out/c4_$name.json 2> $out/c4_$name.err || { tail -5 $out/c4_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$out/c4_$name.json'));print('c4 $name %.4g'%d['value'], round(d['ms_per_step']*1e3,2), {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
port=29770
for v in base:libshadowgpu.so both:libshadowgpu_both.so base2:libshadowgpu.so both2:libshadowgpu_both.so; do
  name=${v%%:*}; lib=${v#*:}; port=$((port+1))
  SG_LIB=$lib timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts 125000 --steps 200 --warmup 10 > $out/d125_$name.log 2>&1 || { tail -20 $out/d125_$name.log; exit 1; }
  python -c "import json;d=json.loads(open('$out/d125_$name.log').read().strip().splitlines()[-1]);print('dist 125000 $name', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step')"
done
