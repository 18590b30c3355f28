set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cpp_layer.py tests/test_gpu_kernels.py tests/test_cpp_functors.py tests/test_boundary.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03ad_t.log 2>&1; rc=$?
tail -2 gpurun_out/r03ad_t.log; [ $rc -eq 0 ] || exit $rc
for W in gp hvp gp_eigen; do
  timeout -k 10 300 python bench.py --workload $W --steps 20 --no-cpu-baseline > gpurun_out/r03ad_$W.json 2> gpurun_out/r03ad.err || { tail gpurun_out/r03ad.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03ad_$W.json')); print('$W', round(d['value'],2), round(d['ms_per_step'],3))"
done
