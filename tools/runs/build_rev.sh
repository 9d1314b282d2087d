#!/bin/bash
# Build libshadowgpu_<name>.so from git revision <rev>'s native sources (same
# ABI as the working tree), for A/B runs with SG_LIB=libshadowgpu_<name>.so.
set -e
rev=$1; name=$2
cd "$(dirname "$0")/../.."
tmp=$(mktemp -d)
git archive "$rev" shadow_amd/csrc include | tar -x -C "$tmp"
objs=""
for f in sg_host.c sg_policy.c sg_sched.c sg_topology.c; do
  gcc -O2 -std=c11 -fPIC -ffp-contract=off -fno-fast-math -I$tmp/include -c $tmp/shadow_amd/csrc/$f -o $tmp/$f.o
  objs="$objs $tmp/$f.o"
done
for f in sg_engine.hip sg_policy_dev.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -I$tmp/include -I$tmp/shadow_amd/csrc $EXTRA -c $tmp/shadow_amd/csrc/$f -o $tmp/$f.o
  objs="$objs $tmp/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o shadow_amd/libshadowgpu_$name.so $objs -lpthread
rm -rf "$tmp"
echo shadow_amd/libshadowgpu_$name.so
