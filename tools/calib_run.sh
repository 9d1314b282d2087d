#!/bin/bash
# FETCH_SIZE calibration pass (tools/calib_fetch.py) under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o calib --output-format csv -- python tools/calib_fetch.py > gpurun_out/calib/run.log 2>&1
rc=$?; echo "calib rc=$rc"; tail -1 gpurun_out/calib/run.log
[ $rc = 0 ] || exit $rc
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/calib/**/calib_counter_collection.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Dispatch_Id"], r["Kernel_Name"][:60], r["Counter_Name"], r["Counter_Value"])
PY
