#!/bin/bash
# Round time of variant libraries / engine switches (no tests): each argument
# is NAME:ENV=V,ENV=V (SG_LIB=libshadowgpu_<v>.so selects a variant build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/var
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  env ${envs//,/ } timeout -k 10 120 python tools/quick_time.py 200 > gpurun_out/var/$name.log 2>&1 || { tail -5 gpurun_out/var/$name.log; exit 1; }
  echo "$name $(tail -1 gpurun_out/var/$name.log)"
done
