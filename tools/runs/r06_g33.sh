#!/bin/bash
# Round 6, thirty-third call: round 5's final tree (commit 703a779, extracted and
# built under _r5/, not committed) against this tree on one box, interleaved:
# configs[3] in the driver's window and at the default run, configs[4], configs[1].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g33}
mkdir -p $O
R=$PWD
run() {  # tag dir args...
  local tag=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --no-drop-in) > $O/$tag.json 2> $O/$tag.err || { tail $O/$tag.err; exit 3; }
  python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
}
for i in 1 2; do
  run r5_c4drv_$i $R/_r5 --gpus 1 --steps 20 --warmup 5
  run r6_c4drv_$i $R --gpus 1 --steps 20 --warmup 5
  run r5_c4_$i $R/_r5 --workload c4
  run r6_c4_$i $R --workload c4
  run r5_c5_$i $R/_r5 --workload c5
  run r6_c5_$i $R --workload c5
  run r5_c2_$i $R/_r5 --workload c2
  run r6_c2_$i $R --workload c2
done
