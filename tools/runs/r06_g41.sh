#!/bin/bash
# Round 6, forty-first call: the AMDGPU machine scheduler's strategy for the
# whole engine (-mllvm -amdgpu-sched-strategy=max-ilp / max-memory-clause, variant
# libraries) against the default, interleaved; parity tests on each first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g41}
mkdir -p $O
for lib in libshadowgpu_maxilp.so libshadowgpu_maxmemoryclause.so; do
  SG_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    > $O/pytest_$lib.log 2>&1 || { tail -20 $O/pytest_$lib.log; exit 1; }
  echo "$lib $(tail -n 1 $O/pytest_$lib.log)"
done
for i in 1 2; do
  for lib in libshadowgpu.so libshadowgpu_maxilp.so libshadowgpu_maxmemoryclause.so; do
    for a in "drv:--gpus 1 --steps 20 --warmup 5" "c4:--workload c4" "c5:--workload c5" "c2:--workload c2"; do
      tag=${a%%:*}; args=${a#*:}
      [ $i = 2 ] && [ $tag != drv ] && [ $tag != c4 ] && continue
      SG_LIB=$lib timeout -k 10 300 python -u bench.py $args --no-cpu-baseline --no-drop-in > $O/${tag}_${lib}_$i.json 2> $O/${tag}_${lib}_$i.err || { tail $O/${tag}_${lib}_$i.err; exit 3; }
      python -c "import json;d=json.load(open('$O/${tag}_${lib}_$i.json'));print('$tag $lib %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
    done
  done
done
