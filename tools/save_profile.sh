#!/bin/bash
# Copy a tools/profile.sh result (gpurun_out/prof) into profiles/<dest>: the
# rocprofv3 kernel-trace stats, the PMC counter CSVs, the corrected per-kernel
# summary and pmc.json (bench.py quotes its traffic figure).
set -e
cd "$(dirname "$0")/.."
SRC=${SRC:-gpurun_out/prof}
DEST=profiles/${1:?usage: save_profile.sh <dest under profiles/>}
mkdir -p "$DEST"
rm -f "$DEST"/*.csv "$DEST"/*.txt "$DEST"/*.json
cp "$SRC/kt/kt_kernel_stats.csv" "$DEST/kernel_stats.csv"
for g in sq fetch write grbm l2; do
  [ -f "$SRC/$g/${g}_counter_collection.csv" ] && cp "$SRC/$g/${g}_counter_collection.csv" "$DEST/pmc_$g.csv"
done
cp "$SRC/summary.txt" "$DEST/summary.txt"
cp "$SRC/pmc.json" "$DEST/pmc.json"
sed -i "s#\"source\": \"[^\"]*\"#\"source\": \"$DEST (rocprofv3 --pmc passes of tools/profile.sh)\"#" "$DEST/pmc.json"
ls -la "$DEST"
