#!/bin/bash
# Round 5: k_scatter's plan arrival at the end (SG_LATE_TICKET), per-row bucket
# minima (SG_PMIN) and the flat pass for hosts of up to 64 events
# (SG_FLAT_CMAX): interleaved configs[3] round times per variant, c2 / c5 bench
# lines, the whole GPU suite on the default build, then stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/g5
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
for rep in 1 2; do
  for v in old lt pmin base; do
    lib=libshadowgpu.so; [ $v = base ] || lib=libshadowgpu_$v.so
    echo -n "$v: "
    SG_LIB=$lib timeout -k 10 120 python tools/quick_time.py 200 2>&1 | tail -1 || exit 1
  done
done
for wl in c2 c5; do
  for v in old base; do
    lib=libshadowgpu.so; [ $v = base ] || lib=libshadowgpu_$v.so
    SG_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/${wl}_$v.json 2> $O/${wl}_$v.err || { tail $O/${wl}_$v.err; exit 2; }
    python -c "import json;d=json.load(open('$O/${wl}_$v.json'));print('$wl $v %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
timeout -k 10 200 python tools/stamps.py > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 4; }
grep -B2 -A14 "k_scatter: span" $O/stamps.txt | head -60
