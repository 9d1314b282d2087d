#!/bin/bash
# Round 6, fifth call: the gossip flat pass with every global load at its
# start (the rng after the draws written by the last send's lane); k_proc's
# path rows by global_load_lds (SG_ROWS_GLDS=1, default) against register
# staging (noglds), and the flat pass's state loads after the sort's scan
# (late); the whole GPU suite first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g5}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for v in 0 1; do
  SG_GFLAT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_gflat$v.json 2> $O/c5_gflat$v.err || { tail $O/c5_gflat$v.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_gflat$v.json'));print('c5 gflat $v %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], d['parity']['match'])"
done
for v in base late noglds base late noglds; do
  lib=libshadowgpu.so; [ $v != base ] && lib=libshadowgpu_$v.so
  SG_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-drop-in > $O/c4_$v.json 2> $O/c4_$v.err || { tail $O/c4_$v.err; exit 4; }
  python -c "import json;d=json.load(open('$O/c4_$v.json'));print('c4 $v %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 5; }
head -n 12 $O/stamps_c5.txt
timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c4.txt 2>&1 || { tail $O/stamps_c4.txt; exit 6; }
head -n 12 $O/stamps_c4.txt
SG_LIB=libshadowgpu_late.so timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c4_late.txt 2>&1 || { tail $O/stamps_c4_late.txt; exit 7; }
head -n 12 $O/stamps_c4_late.txt
