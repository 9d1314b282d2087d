#!/bin/bash
# Experiment: hosts dealt round-robin over the partitions (SG_SLOT_STRIPE=1)
# against the vertex-sorted slots: parity at configs[3] and on the small
# sweep, then interleaved round times (with the LDS path rows off alone for
# reference), then stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/stripe
SG_SLOT_STRIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_random_sweep.py -x -q -m gpu -k "c4_1m_bench or tiny_variants or unsharded or large" --timeout 120 --timeout-method thread > gpurun_out/stripe/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/stripe/pytest.log; [ $rc = 0 ] || exit $rc
for r in 1 2 3; do
  for v in base rows0 stripe; do
    case $v in base) e="";; rows0) e="SG_NO_LDS_ROWS=1";; stripe) e="SG_SLOT_STRIPE=1";; esac
    out=$(env $e timeout -k 10 120 python tools/quick_time.py 300 2>&1) || { echo "$v failed: $out" | tail -3; exit 1; }
    echo "$r $v $out" | tail -1
  done
done
SG_SLOT_STRIPE=1 timeout -k 10 120 python tools/stamps.py > gpurun_out/stripe/stamps_stripe.log 2>&1 || { tail -5 gpurun_out/stripe/stamps_stripe.log; exit 1; }
grep -E "kernel span|sort  |phaseA|phaseC|flat pass, lane|WG duration|k_scatter|insert  |gather  " gpurun_out/stripe/stamps_stripe.log | head -12
