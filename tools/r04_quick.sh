#!/bin/bash
# one GPU call (round 4): selected GPU tests (TESTS, default the boundary suite),
# then the bench workloads in WLS (default gp gp_eigen), each time-limited;
# the first failure ends it.
set -o pipefail
TAG=${1:-r04q}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
TESTS=${TESTS:-tests/test_boundary.py}
if [ "$TESTS" != none ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -q -m gpu -x --timeout 300 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
  tail -3 $O/${TAG}_pytest.log
fi
for w in ${WLS:-gp gp_eigen}; do
  [ $w = none ] && continue
  ST=20; [ $w = normal ] && ST=20000
  timeout -k 10 400 python bench.py --workload $w --steps $ST --no-cpu-baseline > $O/${TAG}_bench_$w.json 2> $O/${TAG}_bench_$w.err || { tail $O/${TAG}_bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${TAG}_bench_$w.json'));print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('eval_phases_ms', ''))"
done
if [ "${UBT:-0}" = 1 ]; then  # device-clock panel timeline of whole GP evaluations (tools/ubench_timeline.cpp)
  timeout -k 10 120 ./tools/ubench_timeline > $O/${TAG}_ubt.txt 2>&1 || { tail $O/${TAG}_ubt.txt; exit 1; }
  cat $O/${TAG}_ubt.txt
fi
if [ "${UBG:-0}" = 1 ]; then  # the GEMM shapes (tools/ubench_gemm.cpp + ubench_shapes.h)
  timeout -k 10 120 ./tools/ubench_gemm > $O/${TAG}_ubg.txt 2>&1 || { tail $O/${TAG}_ubg.txt; exit 1; }
  cat $O/${TAG}_ubg.txt
fi
if [ "${UBH:-0}" = 1 ]; then  # host enqueue vs device time of the factorisation (tools/ubench_host.cpp)
  timeout -k 10 120 ./tools/ubench_host > $O/${TAG}_ubh.txt 2>&1 || { tail $O/${TAG}_ubh.txt; exit 1; }
  cat $O/${TAG}_ubh.txt
fi
if [ "${UBP:-0}" = 1 ]; then  # the panel kernel's chain trace (tools/ubench_panel.hip) + its accuracy vs a host Cholesky
  timeout -k 10 120 ./tools/ubench_panel > $O/${TAG}_ubp.txt 2>&1 || { tail $O/${TAG}_ubp.txt; exit 1; }
  grep -E "panel kernel|potrf_diag" $O/${TAG}_ubp.txt
  if [ -x ./tools/ubench_panel_old ]; then  # the A/B build (UB_OUT=tools/ubench_panel_old)
    timeout -k 10 120 ./tools/ubench_panel_old > $O/${TAG}_ubp_old.txt 2>&1 || { tail $O/${TAG}_ubp_old.txt; exit 1; }
    echo "A/B build:"; grep -E "panel kernel" $O/${TAG}_ubp_old.txt
  fi
fi
if [ "${PROF:-0}" = 1 ]; then  # kernel trace of the GP bench (rocprofv3; the program itself after --)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-glm-strong > $O/${TAG}_prof.log 2>&1 || { tail $O/${TAG}_prof.log; exit 1; }
  echo prof ok
fi
if [ "${UBPH:-0}" = 1 ]; then  # the diagonal factorisation's pieces (tools/ubench_phase.hip)
  timeout -k 10 60 ./tools/ubench_phase > $O/${TAG}_ubph.txt 2>&1 || { tail $O/${TAG}_ubph.txt; exit 1; }
  cat $O/${TAG}_ubph.txt
fi
if [ "${HIPT:-0}" = 1 ]; then  # kernel + HIP API trace of a short GP bench (host enqueue costs)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace -d $O/${TAG}_hipt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-glm-strong > $O/${TAG}_hipt.log 2>&1 || { tail $O/${TAG}_hipt.log; exit 1; }
  echo hipt ok
fi
