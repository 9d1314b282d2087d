#!/bin/bash
# Round 6, eighth call: the gossip flat pass's per-host sums by LDS atomics
# in pass 1 and its active index from the sort's scan (no per-host loops or
# binary search in pass 2): parity tests, the whole suite, configs[4] off /
# on, its stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g8}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -n 1 $O/pytest.log
for v in 0 1 0 1; do
  SG_GFLAT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_gflat$v.json 2> $O/c5_gflat$v.err || { tail $O/c5_gflat$v.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_gflat$v.json'));print('c5 gflat $v %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], d['parity']['match'])"
done
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 5; }
head -n 14 $O/stamps_c5.txt
