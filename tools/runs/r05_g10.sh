#!/bin/bash
# Round 5: gossip seen words loaded with the host state (phase A); parity on the
# gossip tests, then c5 A/B against the committed build (libshadowgpu_prev.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g10}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k gossip \
  tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in prev base prev base; do
  lib=libshadowgpu.so; [ $v = base ] || lib=libshadowgpu_$v.so
  SG_LIB=$lib timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_$v.json 2> $O/c5_$v.err || { tail $O/c5_$v.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));print('c5 $v %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
