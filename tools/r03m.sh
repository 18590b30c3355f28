set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -q -m gpu -k "gemm or chol or gp or mvn or hvp or boundary" --timeout 200 --timeout-method thread > gpurun_out/r03m_t.log 2>&1; rc=$?
tail -2 gpurun_out/r03m_t.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_bench.sh r03m gp || exit 1
python3 tools/phase_sum.py gpurun_out/r03m_prof/run_results.db | head -12
for i in 1 2; do for V in "SMG_INV_SIDE=0 SMG_SPLITK_REDUCE1=1" "SMG_INV_SIDE=1" ; do
  env $V timeout -k 10 300 python bench.py --workload gp --steps 50 --no-cpu-baseline > gpurun_out/r03m.json 2> gpurun_out/r03m.err || { tail gpurun_out/r03m.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03m.json')); print('$V', d['value'], d['ms_per_step'])"
done; done
