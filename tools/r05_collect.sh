#!/bin/bash
# copies one tools/r05_measure.sh set (gpurun_out/<tag>_*) into profiles/r05_*
set -e
TAG=${1:?tag}
cd "$(dirname "$0")/.."
for w in gp gp_eigen glm mulchol hvp normal glm_rank; do
  [ -f gpurun_out/${TAG}_bench_$w.json ] && cp gpurun_out/${TAG}_bench_$w.json profiles/r05_bench_$w.json
done
python3 tools/rocpd_summary.py gpurun_out/${TAG}_prof/run_results.db 60 > profiles/r05_gp4096_kernel_stats.txt
python3 tools/mfma_busy.py gpurun_out/pmc_${TAG}_gp_mfma/run_results.db > profiles/r05_gp4096_mfma_busy.json
python3 tools/pmc_traffic.py $TAG > profiles/r05_pmc_traffic.json
cp gpurun_out/${TAG}_ubp0.txt profiles/r05_panel_trace_before.txt
cp gpurun_out/${TAG}_ubp1.txt profiles/r05_panel_trace_after.txt
cp gpurun_out/${TAG}_ubt.txt profiles/r05_panel_timeline.txt
grep -E "passed|failed" gpurun_out/${TAG}_pytest.log | tail -1 > profiles/r05_gpu_suite.txt || true
echo collected $TAG
