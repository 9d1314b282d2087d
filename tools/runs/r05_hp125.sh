#!/bin/bash
# World-1 xGMI step at 125k hosts (one of eight shards of configs[3]): SG_HP
# partition sizes against the default (2048 hosts, 62 partitions), interleaved,
# on the tree after XS=2 + TICK8; 1M for reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/hp125; mkdir -p $out
port=29800
run() {  # name hosts env...
  local name=$1 h=$2; shift 2; port=$((port+1))
  env "$@" timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 --dist --hosts $h --steps 200 --warmup 10 > $out/d${h}_$name.log 2>&1 || { tail -20 $out/d${h}_$name.log; exit 1; }
  python -c "import json;d=json.loads(open('$out/d${h}_$name.log').read().strip().splitlines()[-1]);print('dist $h $name', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1),'us/step')"
}
for r in a b; do
  run base$r 125000 SG_X=0
  run hp1024$r 125000 SG_HP=1024
  run hp1536$r 125000 SG_HP=1536
done
run base 1000000 SG_X=0
