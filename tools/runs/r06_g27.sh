#!/bin/bash
# Round 6, twenty-seventh call (measurement only): the per-event digest's cost —
# libshadowgpu_nd.so replaces digest_mix's five 64-bit multiplies by xors (parity
# is expected to fail there), interleaved with the product library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g27}
mkdir -p $O
for wl in c4 c5 c2; do
  for lib in libshadowgpu_nd.so libshadowgpu.so libshadowgpu_nd.so libshadowgpu.so; do
    t=${lib#libshadowgpu}; t=${t%.so}
    SG_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/${wl}$t.json 2> $O/${wl}$t.err || [ "$t" = "_nd" ] || { tail $O/${wl}$t.err; exit 3; }
    python -c "import json;d=json.load(open('$O/${wl}$t.json'));print('$wl $lib %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
