#!/bin/bash
# one GPU call (round 6 measurement set): GPU test suite, every bench workload (with
# CPU baselines), the GLM per-rank proxy, the panel kernel's step trace
# (tools/ubench_panel, without and with the resident rows below), the device-clock panel timeline of whole GP
# evaluations (tools/ubench_timeline), the rocprofv3 kernel-trace summary of
# the GP bench, an MFMA-busy PMC pass and the HBM traffic passes (incl.
# k_chol_panel and the last K^{-1} share).  Each step time-limited; the first
# failure ends it.
set -o pipefail
TAG=${1:-r06z}
SKIP_TESTS=${SKIP_TESTS:-0}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
  tail -3 $O/${TAG}_pytest.log
fi
for w in ${WLS:-gp glm mulchol hvp normal gp_eigen}; do
  ST=20; [ $w = normal ] && ST=20000
  timeout -k 10 400 python bench.py --workload $w --steps $ST > $O/${TAG}_bench_$w.json 2> $O/${TAG}_bench_$w.err || { tail $O/${TAG}_bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${TAG}_bench_$w.json'));print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
SMG_BENCH_GLM_RCCL1=1 timeout -k 10 400 python bench.py --workload glm --rows 1.25e6 --steps 100 --no-cpu-baseline > $O/${TAG}_bench_glm_rank.json 2> $O/${TAG}_bench_glm_rank.err || { tail $O/${TAG}_bench_glm_rank.err; exit 1; }
python -c "import json;d=json.load(open('$O/${TAG}_bench_glm_rank.json'));print('glm_rank', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 120 ./tools/ubench_panel > $O/${TAG}_ubp.txt 2>&1 || { tail $O/${TAG}_ubp.txt; exit 1; }
grep -E "panel kernel" $O/${TAG}_ubp.txt
timeout -k 10 60 ./tools/ubench_factor > $O/${TAG}_factor.txt 2>&1 || { tail $O/${TAG}_factor.txt; exit 1; }
timeout -k 10 120 ./tools/ubench_timeline > $O/${TAG}_ubt.txt 2>&1 || { tail $O/${TAG}_ubt.txt; exit 1; }
head -4 $O/${TAG}_ubt.txt
[ "${PROF:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-glm-strong > $O/${TAG}_prof.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${TAG}_gp_mfma -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-glm-strong > $O/pmc_${TAG}_gp_mfma.log 2>&1 || exit 1
bash $GRAFT_REPO_ROOT/tools/pmc_traffic.sh $TAG || exit 1
echo done
