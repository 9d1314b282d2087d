#!/bin/bash
# Round 6, fourth call: the gossip seen words kept in registers (the select
# chain had become an indexed private array: a scratch round trip per
# receipt in phase A and in the flat pass); gossip parity tests, configs[4]
# flat pass off / on, its stamps, the whole suite, then configs[3]'s bench
# with the CPU baseline at every CPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06g4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "gossip" > $O/pytest_gossip.log 2>&1 || { tail -40 $O/pytest_gossip.log; exit 1; }
tail -n 1 $O/pytest_gossip.log
for v in 0 1 0 1; do
  SG_GFLAT=$v timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --no-drop-in > $O/c5_gflat$v.json 2> $O/c5_gflat$v.err || { tail $O/c5_gflat$v.err; exit 3; }
  python -c "import json;d=json.load(open('$O/c5_gflat$v.json'));print('c5 gflat $v %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'frac %.3f'%d['roofline']['frac'], d['parity']['match'])"
done
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 300 python -u tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 4; }
head -n 12 $O/stamps_c5.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 5; }
tail -n 2 $O/pytest.log
T0=$(date +%s); timeout -k 10 600 python -u bench.py --no-drop-in > $O/bench_c4.json 2> $O/bench_c4.err || { tail $O/bench_c4.err; exit 6; }
echo "bench_c4 wall $(( $(date +%s) - T0 )) s"
python -c "import json;d=json.load(open('$O/bench_c4.json'));c=d['cpu_baseline'];print('c4 %.4g'%d['value'], round(d['ms_per_step']*1e3,2), d['parity']['match'], {k:c[k] for k in ('value','cores','share_value','share_workers','all_cpus_value','all_cpus_workers','single_thread_value','plain_heap_value','nproc','affinity','cgroup_cpus')})"
