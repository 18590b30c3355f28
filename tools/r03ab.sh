set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpp_layer.py tests/test_gpu_kernels.py tests/test_cpp_functors.py -x -q -m gpu -k "gp or cholesky or mvn or hessian or mulchol" --timeout 300 --timeout-method thread > gpurun_out/r03ab_t.log 2>&1; rc=$?
tail -4 gpurun_out/r03ab_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do for V in 1 0; do
  SMG_CHOL_INV_FWD=$V timeout -k 10 300 python bench.py --workload gp --steps 30 --no-cpu-baseline > gpurun_out/r03ab.json 2> gpurun_out/r03ab.err || { tail gpurun_out/r03ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03ab.json')); print('invfwd=$V', round(d['value'],2), round(d['ms_per_step'],3))"
done; done
for W in hvp mulchol; do for V in 1 0; do
  SMG_CHOL_INV_FWD=$V timeout -k 10 300 python bench.py --workload $W --steps 10 --no-cpu-baseline > gpurun_out/r03ab.json 2> gpurun_out/r03ab.err || { tail gpurun_out/r03ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03ab.json')); print('$W invfwd=$V', round(d['value'],2), round(d['ms_per_step'],3))"
done; done
bash tools/prof_bench.sh cb gp
