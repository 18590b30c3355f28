set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -k "hessian or hvp or tangent or mdivide" --timeout 800 --timeout-method thread > gpurun_out/r03o_t.log 2>&1; rc=$?
tail -5 gpurun_out/r03o_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for V in "SMG_CHOL_TANGENT_COMPOSED=1" "SMG_CHOL_TANGENT_COMPOSED=0" ; do
  env $V timeout -k 10 300 python bench.py --workload hvp --steps 10 --no-cpu-baseline > gpurun_out/r03o.json 2> gpurun_out/r03o.err || { tail gpurun_out/r03o.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03o.json')); print('$V', d['value'], d['ms_per_step'])"
done; done
