#!/bin/bash
# Round 5: the split step's cost split (SG_SPLIT 0 / 1 / 2 on the world-1 RCCL
# path at 125k hosts), the reservation microbenchmark, the c2 / c5 bench lines
# with their timed rounds' kernel durations, and k_proc / k_scatter stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1
O=gpurun_out/g4
mkdir -p $O
timeout -k 10 60 ./tools/resv_bench > $O/resv.txt 2>&1 || { cat $O/resv.txt; exit 1; }
cat $O/resv.txt
port=29611
for rep in 1 2; do
  for split in 0 1 2; do
    port=$((port+1))
    SG_SPLIT=$split timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 1 --dist --hosts 125000 --steps 200 --warmup 10 \
      > $O/d_125000_s${split}_$rep.log 2>&1 || { tail -20 $O/d_125000_s${split}_$rep.log; exit 2; }
    python - <<PY
import json
d = json.loads(open('$O/d_125000_s${split}_$rep.log').read().strip().splitlines()[-1])
print('dist 125000 split $split', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step',
      {k: round(v, 2) for k, v in zip(d['per_rank_us_per_step']['classes'], d['per_rank_us_per_step']['rows'][0])})
PY
  done
done
for wl in c2 c5; do
  timeout -k 10 400 python -u bench.py --workload $wl > $O/$wl.json 2> $O/$wl.err || { tail $O/$wl.err; exit 3; }
  python -c "import json;d=json.load(open('$O/$wl.json'));print('$wl %.4g'%d['value'], round(d['ms_per_step']*1e3,1), 'us/step', {k:round(v,2) for k,v in d['roofline']['kernel_us_per_round'].items()}, 'gaps', round(d['roofline']['gaps_us_per_round'],2), d['parity']['match'])"
done
timeout -k 10 200 python tools/stamps.py > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 4; }
grep -A3 "k_scatter" $O/stamps.txt | head -30
STAMPS_WL=c2 timeout -k 10 200 python tools/stamps.py > $O/stamps_c2.txt 2>&1 || { tail $O/stamps_c2.txt; exit 5; }
head -25 $O/stamps_c2.txt
STAMPS_WL=c5 STAMPS_AT=150 timeout -k 10 200 python tools/stamps.py > $O/stamps_c5.txt 2>&1 || { tail $O/stamps_c5.txt; exit 6; }
head -25 $O/stamps_c5.txt
