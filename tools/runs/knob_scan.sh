# Engine knob scan: one bench line per setting (no CPU legs). Usage: bash tools/runs/knob_scan.sh "ENV=.. ENV=.." ...
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for cfg in "$@"; do
  line=$(env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --no-drop-in 2> gpurun_out/knob.err) || { echo "FAIL $cfg"; tail -5 gpurun_out/knob.err; exit 1; }
  python - "$cfg" "$line" <<'PY'
import json, sys
r = json.loads(sys.argv[2])
k = r["roofline"]["kernel_us_per_round"]
print(f"{sys.argv[1]:40s} {r['value']:.4g} ev/s  {r['ms_per_step']*1e3:6.1f} us/round  " + " ".join(f"{a}={b:.1f}" for a, b in k.items()), flush=True)
PY
done
