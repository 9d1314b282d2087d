#!/bin/bash
# Interleaved round times of ablation variants (results intentionally wrong):
# SG_ABL=64 no bucket-minimum atomics in k_proc's reservations, 128 no
# returning reservation atomics, 192 both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/abl
for rep in 1 2; do
  for v in base abl64 abl128 abl192; do
    lib=libshadowgpu.so; [ $v = base ] || lib=libshadowgpu_$v.so
    echo -n "$v: "
    SG_LIB=$lib timeout -k 10 120 python tools/quick_time.py 200 2>&1 | tail -1 || exit 1
  done
done
