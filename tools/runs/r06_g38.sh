#!/bin/bash
# Round 6, thirty-eighth call: the PHOLD sort's host counts read in one batch (SG_SCAN_BATCH=1, default)
# against one branch per host (libshadowgpu_sb0.so), interleaved
# on configs[3], configs[1] and configs[4]; parity tests first; configs[3] stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g38}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py \
  > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
tail -n 1 $O/pytest_parity.log
for wl in c4 c2 c5; do
  for lib in libshadowgpu_sb0.so libshadowgpu.so libshadowgpu_sb0.so libshadowgpu.so; do
    t=${lib#libshadowgpu}; t=${t%.so}
    SG_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/${wl}$t.json 2> $O/${wl}$t.err || { tail $O/${wl}$t.err; exit 3; }
    python -c "import json;d=json.load(open('$O/${wl}$t.json'));print('$wl $lib %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
