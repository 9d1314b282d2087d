#!/bin/bash
# k_proc MIN accumulators in eight copies (SG_XACC8): parity subset on the
# variant, then configs[3] interleaved with the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/xacc8b; mkdir -p $out
SG_LIB=libshadowgpu_xacc8.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_gspec.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_sharded.py > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc = 0 ] || exit $rc
for v in base:libshadowgpu.so x8:libshadowgpu_xacc8.so base2:libshadowgpu.so x8b:libshadowgpu_xacc8.so base3:libshadowgpu.so x8c:libshadowgpu_xacc8.so; do
  name=${v%%:*}; lib=${v#*:}
  SG_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > $out/c4_$name.json 2> $out/c4_$name.err || { tail -5 $out/c4_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$out/c4_$name.json'));print('c4 $name %.4g'%d['value'], round(d['ms_per_step']*1e3,2), {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
