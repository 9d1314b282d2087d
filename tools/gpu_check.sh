#!/bin/bash
# GPU-box check: smoke, GPU parity tests, bench.  Each GPU step has its own
# time limit; a crash-like exit (timeout, abort, segfault) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -5 "gpurun_out/$name.log"
  case $rc in 124|137|134|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
  return 0
}
step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 600 python -u bench.py ${BENCH_ARGS:-}
