#!/bin/bash
# Iteration loop on the GPU box: parity spot-check → bench → kernel trace.
# Every GPU step has its own time limit; a crash-like exit ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-12} "gpurun_out/$name.log" | cut -c1-600
  case $rc in 0) return 0;; *) echo "stopping after $name"; exit $rc;; esac
}
run cal 300 python -u tools/cal_check.py ${CAL_ARGS:-}
run bench 300 python -u bench.py --no-cpu-baseline --no-drop-in ${BENCH_ARGS:-}
[ -n "$NO_TRACE" ] || TAILN=30 run ktrace 400 bash tools/ktrace.sh
