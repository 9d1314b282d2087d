#!/bin/bash
# Round 6, eleventh call: the LLVM atomic optimizer's DPP strategy
# (libshadowgpu_dpp.so) against its default iterative one, interleaved on
# configs[4], configs[3] and configs[1]; stamps of configs[4] with DPP.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g11}
mkdir -p $O
SG_LIB=libshadowgpu_dpp.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  > $O/pytest_parity_dpp.log 2>&1 || { tail -40 $O/pytest_parity_dpp.log; exit 1; }
tail -n 1 $O/pytest_parity_dpp.log
for wl in c5 c4 c2; do
  for lib in libshadowgpu.so libshadowgpu_dpp.so libshadowgpu.so libshadowgpu_dpp.so; do
    t=${lib#libshadowgpu}; t=${t%.so}
    SG_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/${wl}$t.json 2> $O/${wl}$t.err || { tail $O/${wl}$t.err; exit 3; }
    python -c "import json;d=json.load(open('$O/${wl}$t.json'));print('$wl $lib %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
SG_LIB=libshadowgpu_dpp.so STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 5; }
head -n 14 $O/stamps_c5.txt
