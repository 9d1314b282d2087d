#!/bin/bash
# Round 6, thirty-seventh call: the Dev kernel argument in round 5's field order (this tree)
# against HEAD before it (_bis/L, not
# committed): parity tests, then configs[3] in the driver's window and at the
# default run, configs[1] and configs[4], interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g37}
mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
run() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-drop-in) > $O/$tag.json 2> $O/$tag.err || { tail $O/$tag.err; exit 3; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
}
for i in 1 2; do
  run old_drv_$i $R/_bis/L --gpus 1 --steps 20 --warmup 5
  run new_drv_$i $R --gpus 1 --steps 20 --warmup 5
  run old_c4_$i $R/_bis/L --workload c4
  run new_c4_$i $R --workload c4
done
run old_c2 $R/_bis/L --workload c2
run new_c2 $R --workload c2
run old_c5 $R/_bis/L --workload c5
run new_c5 $R --workload c5
