#!/bin/bash
# GPU box: k_gather grid sweep on the default bench, then the full profile
# (kernel trace + PMC passes) and its per-kernel summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for g in ${GRIDS:-128 256 512}; do
  SG_GATHER_GRID=$g timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/sweep_$g.json || exit $?
  python - "$g" gpurun_out/sweep_$g.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(sys.argv[1], round(d["value"] / 1e9, 3), {k: round(v, 1) for k, v in d["roofline"]["kernel_us_per_round"].items()})
PY
done
[ -n "$NO_PROFILE" ] && exit 0
bash tools/profile.sh > gpurun_out/profile.log 2>&1 || exit $?
python tools/prof_summary.py gpurun_out/prof 40 gpurun_out/prof/pmc.json > gpurun_out/prof/summary.txt && cat gpurun_out/prof/summary.txt
