set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for F in 0 1 2 3; do
 SMG_GLM_FIN=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03j_f$F -o run -- python3 bench.py --workload glm --rows 1.25e6 --steps 50 --no-cpu-baseline > gpurun_out/r03j_f$F.log 2>&1 || { tail gpurun_out/r03j_f$F.log; exit 1; }
 SMG_GLM_FIN=$F timeout -k 10 300 python3 bench.py --workload glm --rows 1.25e6 --steps 100 --no-cpu-baseline > gpurun_out/r03j_b$F.json 2>/dev/null || exit 1
done
