#!/bin/bash
# Round 6, thirtieth call: reserve_buckets' chunk ids from the stash in a loop of
# their own (LDS only: no vmcnt(0) before each btab store); parity tests and the
# bench lines twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g30}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
for wl in c4 c2 c5 c4 c2 c5; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/$wl.json 2> $O/$wl.err || { tail $O/$wl.err; exit 3; }
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
STAMPS_WL=c4 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c4.txt 2>&1 || { tail $O/stamps_c4.txt; exit 5; }
head -n 14 $O/stamps_c4.txt
