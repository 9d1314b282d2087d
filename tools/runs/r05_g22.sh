#!/bin/bash
# Round 5: the gossip draw-after-phase-A variant with the header fix (a header
# record's .a is not an active index in phase B): its tests and the other gossip
# parity tests first (each run stops at its first failure), then configs[4]
# A/B (SG_GSKIP=1 against 0), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g22}
mkdir -p $O
SG_DEBUG_SYNC=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "test_gossip_draws_after_phase_a" > $O/pytest_new.log 2>&1 || { tail -30 $O/pytest_new.log; exit 1; }
grep -cE "PASSED" $O/pytest_new.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  tests/test_gpu_dist.py tests/test_gpu_policy.py -k "gossip or c5" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for sk in 0 1 0 1; do
  SG_GSKIP=$sk timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_g$sk.json 2> $O/c5_g$sk.err || { tail $O/c5_g$sk.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_g$sk.json'));print('c5 gskip $sk %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
