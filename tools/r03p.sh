set -o pipefail
mkdir -p gpurun_out
bash tools/prof_bench.sh r03p hvp || exit 1
python3 tools/rocpd_summary.py gpurun_out/r03p_prof/run_results.db 30
