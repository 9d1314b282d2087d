#!/bin/bash
# The multi-shard step path (world-1 RCCL communicator, native step loop,
# parity checked at 1M hosts) while another process keeps the same GPU busy
# with matmuls: k_scatter's bounded cross-workgroup wait (plan_when_read) and
# the RCCL kernel then run beside competing kernels.  The load process stops
# itself after LOAD_S seconds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/contention
LOAD_S=${LOAD_S:-90}
timeout -k 10 $((LOAD_S + 30)) python - > gpurun_out/contention/load.log 2>&1 <<PY &
import time, torch
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
b = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
t0 = time.time(); n = 0
while time.time() - t0 < $LOAD_S:
    for _ in range(20):
        c = a @ b
    torch.cuda.synchronize(); n += 20
print("matmuls", n, "in", round(time.time() - t0, 1), "s", flush=True)
PY
LOAD=$!
sleep 15  # the load is running (first torch import included)
rc=0
for hosts in 1000000 125000; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $((29700 + hosts % 97)) bench.py --gpus 1 --dist --hosts $hosts --steps 400 --warmup 10 \
    > gpurun_out/contention/d_$hosts.log 2>&1 || { rc=$?; tail -5 gpurun_out/contention/d_$hosts.log; break; }
  python - <<PY
import json
d = json.loads(open('gpurun_out/contention/d_$hosts.log').read().strip().splitlines()[-1])
print('under load: $hosts hosts', '%.4g' % d['value'], round(d['ms_per_step'] * 1e3, 1), 'us/step', d['config']['step_loop'],
      'drains', d['config']['drain_steps'], 'parity', d['parity'].get('match'), d['parity'].get('note', ''))
PY
done
wait $LOAD
cat gpurun_out/contention/load.log
exit $rc
