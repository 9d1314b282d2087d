#!/bin/bash
# GPU suite on the working tree's library, one bench line, an interleaved
# round-time A/B against variant libraries (tools/runs/qt_ab.sh), then stamps.
# Usage: tools/runs/r04_iter.sh [variant ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/it
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/it/pytest.log; [ $rc = 0 ] || exit $rc
fi
timeout -k 10 200 python bench.py --no-cpu-baseline --no-drop-in > gpurun_out/it/bench.json 2> gpurun_out/it/bench.err || { tail -5 gpurun_out/it/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/it/bench.json'));print('bench %.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/round', d['parity']['match'], {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()})"
if [ $# -gt 0 ]; then bash tools/runs/qt_ab.sh ${REPS:-3} "$@" || exit 1; fi
for lib in libshadowgpu.so ${STAMP_LIBS:-}; do
  SG_LIB=$lib timeout -k 10 120 python tools/stamps.py > gpurun_out/it/stamps_$lib.log 2>&1 || { tail -5 gpurun_out/it/stamps_$lib.log; exit 1; }
  echo "== stamps $lib"
  grep -E "kernel span|sort  |phaseA|phaseC|k_scatter|insert  |gather  |sort \(median|after phase B|flat pass, lane" gpurun_out/it/stamps_$lib.log | head -11
done
