cd "${GRAFT_REPO_ROOT:-.}"
set -o pipefail
for v in 1 0; do
  export SG_FLAT=$v
  bash tools/pmc_issue.sh > gpurun_out/pmc_issue_$v.txt 2>&1 || { cat gpurun_out/pmc_issue_$v.txt; exit 1; }
  bash tools/pmc_icache.sh > gpurun_out/pmc_icache_$v.txt 2>&1 || { cat gpurun_out/pmc_icache_$v.txt; exit 1; }
  mv gpurun_out/pmc_issue gpurun_out/pmc_issue_d$v; mv gpurun_out/ic gpurun_out/ic_d$v
done
grep -h "k_proc" gpurun_out/pmc_issue_1.txt gpurun_out/pmc_icache_1.txt gpurun_out/pmc_issue_0.txt gpurun_out/pmc_icache_0.txt
