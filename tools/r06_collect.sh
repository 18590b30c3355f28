#!/bin/bash
# copies one tools/r06_measure.sh set (gpurun_out/<tag>_*) into profiles/r06_*
set -e
TAG=${1:?tag}
cd "$(dirname "$0")/.."
for w in gp gp_eigen glm mulchol hvp normal glm_rank; do
  [ -f gpurun_out/${TAG}_bench_$w.json ] && cp gpurun_out/${TAG}_bench_$w.json profiles/r06_bench_$w.json
done
python3 tools/rocpd_summary.py gpurun_out/${TAG}_prof/run_results.db 60 > profiles/r06_gp4096_kernel_stats.txt
python3 tools/mfma_busy.py gpurun_out/pmc_${TAG}_gp_mfma/run_results.db > profiles/r06_gp4096_mfma_busy.json
python3 tools/pmc_traffic.py $TAG > profiles/r06_pmc_traffic.json
cp gpurun_out/${TAG}_ubp.txt profiles/r06_panel_trace.txt
cp gpurun_out/${TAG}_factor.txt profiles/r06_factor_variants.txt
cp gpurun_out/${TAG}_ubt.txt profiles/r06_panel_timeline.txt
grep -E "passed|failed" gpurun_out/${TAG}_pytest.log | tail -1 > profiles/r06_gpu_suite.txt || true
echo collected $TAG
