#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_proc and k_scatter for two builds (SG_LIB
# variants), one PMC pass each, over the bench's default-length run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fab
for v in "$@"; do
  name=${v%%:*}; lib=${v#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    SG_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc $c -d gpurun_out/fab/${name}_$c -o p --output-format csv -- \
      python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-drop-in > gpurun_out/fab/${name}_$c.log 2>&1 || exit $?
  done
  python - "$name" <<'PY'
import csv, glob, sys, collections
name = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/fab/{name}_{c}/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f))]
    by = collections.defaultdict(list)
    for r in rows:
        k = "k_proc" if "k_proc" in r["Kernel_Name"] else "k_scatter" if "k_scatter" in r["Kernel_Name"] else None
        if k: by[k].append(float(r["Counter_Value"]))
    print(name, c, {k: round(sum(v[-40:]) / len(v[-40:]) / 1024, 1) for k, v in by.items()}, "KiB/launch")
PY
done
