set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpp_layer.py -x -q -m gpu -k "gp" --timeout 300 --timeout-method thread > gpurun_out/r03ac_t.log 2>&1; rc=$?
tail -2 gpurun_out/r03ac_t.log; [ $rc -eq 0 ] || exit $rc
SMG_LATE_AT_FWD=1 SMG_SIDE_PRIO=1 timeout -k 10 400 python -u -m pytest tests/test_cpp_layer.py -x -q -m gpu -k "gp" --timeout 300 --timeout-method thread > gpurun_out/r03ac_t2.log 2>&1; rc=$?
tail -2 gpurun_out/r03ac_t2.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for V in "X=0" "SMG_SIDE_PRIO=1" "SMG_LATE_AT_FWD=1" "SMG_LATE_AT_FWD=1 SMG_SIDE_PRIO=1" "SMG_GEMM_TRI=6402" "SMG_GEMM_TRI=128"; do
  env $V timeout -k 10 300 python bench.py --workload gp --steps 30 --no-cpu-baseline > gpurun_out/r03ac.json 2> gpurun_out/r03ac.err || { tail gpurun_out/r03ac.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03ac.json')); print('$V', round(d['value'],2), round(d['ms_per_step'],3))"
done; done
