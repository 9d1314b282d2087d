#!/bin/bash
# Round 5: rand_r skip-ahead in the flat pass (SG_SKIP=1) against the replay
# loop (SG_SKIP=0): parity suites, then c2 / c4 / c5 interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=${O:-gpurun_out/g16}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_random_sweep.py tests/test_gpu_configs.py tests/test_gpu_gspec.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for wl in c2 c4; do
  for sk in 0 1 0 1; do
    SG_SKIP=$sk timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --no-drop-in > $O/${wl}_s$sk.json 2> $O/${wl}_s$sk.err || { tail $O/${wl}_s$sk.err; exit 3; }
    python -c "import json;d=json.load(open('$O/${wl}_s$sk.json'));print('$wl skip $sk %.4g'%d['value'], round(d['ms_per_step']*1e3,2), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, d['parity']['match'])"
  done
done
