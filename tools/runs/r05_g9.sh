#!/bin/bash
# Round 5: the GPU suite's multi-rank files with the unfenced xGMI exchange
# (the new default), then configs[4] partition sizes around the new automatic one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g9}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sharded.py tests/test_gpu_dist.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for hp in 256 320 0 512 192 0; do
  SG_HP=$hp timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_hp$hp.json 2> $O/c5_hp$hp.err || { tail $O/c5_hp$hp.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_hp$hp.json'));print('c5 hp $hp %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
done
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 200 python tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 5; }
head -12 $O/stamps_c5.txt
