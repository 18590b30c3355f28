set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpp_layer.py tests/test_gpu_kernels.py -x -q -m gpu -k "gp or cholesky or mvn" --timeout 300 --timeout-method thread > gpurun_out/r03z_t.log 2>&1; rc=$?
tail -4 gpurun_out/r03z_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do for V in 1 0; do
  SMG_CHOL_MVN_ASYNC=$V timeout -k 10 300 python bench.py --workload gp --steps 30 --no-cpu-baseline > gpurun_out/r03z.json 2> gpurun_out/r03z.err || { tail gpurun_out/r03z.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03z.json')); print('async=$V', round(d['value'],2), round(d['ms_per_step'],3))"
done; done
