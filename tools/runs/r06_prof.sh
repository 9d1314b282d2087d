#!/bin/bash
# Round 6 final tree: rocprofv3 kernel trace + PMC passes (tools/profile.sh) of
# configs[3] in the driver's window (--steps 20 --warmup 5) and at the bench
# default, of configs[1] and of configs[4]; each summarised over its timed launches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=${O:-gpurun_out/r06final3}
mkdir -p $O
run() {  # name last_n args...
  local name=$1 last=$2; shift 2
  OUT=$O/prof_$name PROF_ARGS="$* --no-cpu-baseline --no-drop-in" bash tools/profile.sh > $O/prof_$name.log 2>&1 || { tail $O/prof_$name.log; exit 4; }
  python tools/prof_summary.py $O/prof_$name $last $O/prof_$name/pmc.json > $O/prof_$name/summary.txt
  echo "== $name"; grep -E "steady|k_proc|k_scatter" $O/prof_$name/summary.txt | head -8
}
run c4_driver 20 --workload c4 --steps 20 --warmup 5
run c4 200 --workload c4
run c2 150 --workload c2
run c5 120 --workload c5
