set -o pipefail
mkdir -p gpurun_out
bash tools/prof_bench.sh r03n hvp || exit 1
python3 tools/rocpd_summary.py gpurun_out/r03n_prof/run_results.db 25
for i in 1 2; do for V in "SMG_SPLITK_REDUCE1=1" "SMG_SPLITK_REDUCE1_OFF=1" ; do
  env $V timeout -k 10 300 python bench.py --workload gp --steps 50 --no-cpu-baseline > gpurun_out/r03n.json 2> gpurun_out/r03n.err || { tail gpurun_out/r03n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03n.json')); print('$V', d['value'], d['ms_per_step'])"
done; done
