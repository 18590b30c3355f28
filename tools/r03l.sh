set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03l_gp -o run -- python3 bench.py --workload gp --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03l_gp.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload gp --steps 50 --no-cpu-baseline > gpurun_out/r03l_gp.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --workload hvp --steps 10 --no-cpu-baseline > gpurun_out/r03l_hvp.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --workload mulchol --steps 20 --no-cpu-baseline > gpurun_out/r03l_mc.json 2>/dev/null || exit 1
SMG_BENCH_GLM_RCCL1=1 timeout -k 10 300 python3 bench.py --workload glm --rows 1.25e6 --steps 100 --no-cpu-baseline > gpurun_out/r03l_glm_rccl1.json 2>gpurun_out/r03l_glm_rccl1.err || exit 1
timeout -k 10 300 python3 bench.py --workload glm --rows 1.25e6 --steps 100 --no-cpu-baseline > gpurun_out/r03l_glm.json 2>/dev/null || exit 1
timeout -k 10 300 python -u -m pytest tests -q -m gpu -k "glm or sharding or map_rect" --timeout 120 --timeout-method thread > gpurun_out/r03l_t.log 2>&1; rc=$?; tail -2 gpurun_out/r03l_t.log; exit $rc
