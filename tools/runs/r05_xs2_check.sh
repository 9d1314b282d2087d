#!/bin/bash
# SG_XS=2 as the default: the GPU suite, then each workload and the world-1
# xGMI step path against the XS=1 build (libshadowgpu_xs1.so), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/xs2c; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc = 0 ] || exit $rc
for w in c2 c5; do
  for v in xs1:libshadowgpu_xs1.so xs2:libshadowgpu.so xs1b:libshadowgpu_xs1.so xs2b:libshadowgpu.so; do
    name=${v%%:*}; lib=${v#*:}
    SG_LIB=$lib timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-drop-in > $out/${w}_$name.json 2> $out/${w}_$name.err || { tail -5 $out/${w}_$name.err; exit 1; }
    python -c "import json;d=json.load(open('$out/${w}_$name.json'));print('$w $name %.4g'%d['value'], round(d['ms_per_step']*1e3,2), {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
port=29700
for h in 125000 1000000; do
  for v in xs1:libshadowgpu_xs1.so xs2:libshadowgpu.so xs1b:libshadowgpu_xs1.so xs2b:libshadowgpu.so; do
    name=${v%%:*}; lib=${v#*:}; port=$((port+1))
    SG_LIB=$lib timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
      bench.py --gpus 1 --dist --hosts $h --steps 200 --warmup 10 > $out/d_${h}_$name.log 2>&1 || { tail -20 $out/d_${h}_$name.log; exit 1; }
    python -c "import json;d=json.loads(open('$out/d_${h}_$name.log').read().strip().splitlines()[-1]);print('dist $h $name', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step', d['parity'].get('match') if isinstance(d.get('parity'),dict) else None)"
  done
done
