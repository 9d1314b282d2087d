#!/bin/bash
# Interleaved round-time A/B of variant libraries (tools/quick_time.py, no
# parity check): base, then each variant, repeated.  Usage: tools/runs/qt_ab.sh REPS v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
reps=$1; shift
mkdir -p gpurun_out/qt
for r in $(seq 1 $reps); do
  for v in base "$@"; do
    lib=libshadowgpu.so; [ "$v" = base ] || lib=libshadowgpu_$v.so
    out=$(SG_LIB=$lib timeout -k 10 120 python tools/quick_time.py 300 2>&1) || { echo "$v failed: $out" | tail -3; exit 1; }
    echo "$r $v $out" | tail -1
  done
done
