#!/bin/bash
# Round 6, tenth call: the gossip flat pass takes its start loads into registers
# before its stores (no vmcnt(0) after them); parity tests, configs[4] off / on, stamps,
# configs[3] and configs[1].
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g10}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
for v in 0 1 0 1; do
  SG_GFLAT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_gflat$v.json 2> $O/c5_gflat$v.err || { tail $O/c5_gflat$v.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_gflat$v.json'));print('c5 gflat $v %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], d['parity']['match'])"
done
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 5; }
head -n 14 $O/stamps_c5.txt
for wl in c4 c2; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/$wl.json 2> $O/$wl.err || { tail $O/$wl.err; exit 4; }
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
