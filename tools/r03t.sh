set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -k "chol or gp or mvn or boundary or spd or handoff or hessian or mulchol or tape" --timeout 800 --timeout-method thread > gpurun_out/r03t_t.log 2>&1; rc=$?
tail -2 gpurun_out/r03t_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do for V in "SMG_REV_SPLIT=0" "SMG_REV_SPLIT=1"; do for W in gp; do
  env $V timeout -k 10 300 python bench.py --workload $W --steps 40 --no-cpu-baseline > gpurun_out/r03t.json 2> gpurun_out/r03t.err || { tail gpurun_out/r03t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03t.json')); print('$V $W', d['value'], d['ms_per_step'])"
done; done; done
for V in "SMG_REV_SPLIT=0" "SMG_REV_SPLIT=1"; do for W in mulchol hvp; do
  env $V timeout -k 10 300 python bench.py --workload $W --steps 10 --no-cpu-baseline > gpurun_out/r03t.json 2> gpurun_out/r03t.err || { tail gpurun_out/r03t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03t.json')); print('$V $W', d['value'], d['ms_per_step'])"
done; done
