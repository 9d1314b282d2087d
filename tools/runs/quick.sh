#!/bin/bash
# debug trace + GPU tests + bench + traffic counters for k_process / k_insert
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 120 python tools/debug_trace.py 50 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/q/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "^E  |passed|failed" gpurun_out/q/pytest.log | head -20
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/q/bench.log 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/q/bench.log'));print('value %.3g ms/step %.4f'%(d['value'],d['ms_per_step']), {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items()})"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d gpurun_out/q/$c -o $c --output-format csv -- python bench.py --steps 10 --warmup 20 --no-cpu-baseline > gpurun_out/q/$c.log 2>&1 || exit $?
done
python - <<'PY'
import csv, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = list(csv.DictReader(open(f"gpurun_out/q/{c}/{c}_counter_collection.csv")))
    per = collections.defaultdict(list)
    for r in rows:
        per[r["Kernel_Name"].split("(")[0][-24:]].append(float(r["Counter_Value"]))
    for k, v in per.items():
        if len(v) > 5:
            v = v[-10:]
            print(c, k, "steady MB/launch %.1f" % (sum(v) / len(v) / 1024))
PY
