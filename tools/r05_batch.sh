#!/bin/bash
# one GPU call (round 5): selected GPU tests ($K), GP env A/B ($CFGS), HVP env
# A/B ($HCFGS), gp_eigen env A/B ($ECFGS), the panel kernel's trace with and without register-resident
# tiles, the device-clock panel timeline.  Each step time-limited; the first
# failure ends it.
set -o pipefail
TAG=${1:-r05b}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "${K:-none}" != none ]; then
  timeout -k 10 700 python -u -m pytest tests -q -m gpu -x -k "$K" --timeout 300 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
  tail -2 $O/${TAG}_pytest.log
fi
if [ -n "$CFGS" ]; then CFGS="$CFGS" REP=${REP:-2} bash tools/r05_env_ab.sh ${TAG}_gp || exit 1; fi
if [ -n "$HCFGS" ]; then CFGS="$HCFGS" WL=hvp REP=${HREP:-2} bash tools/r05_env_ab.sh ${TAG}_hvp || exit 1; fi
if [ -n "$ECFGS" ]; then CFGS="$ECFGS" WL=gp_eigen REP=${EREP:-2} bash tools/r05_env_ab.sh ${TAG}_eig || exit 1; fi
if [ "${UBP:-0}" = 1 ]; then
  for r in 0 1; do
    SMG_PANEL_RESIDENT=$r timeout -k 10 120 ./tools/ubench_panel > $O/${TAG}_ubp$r.txt 2>&1 || { tail $O/${TAG}_ubp$r.txt; exit 1; }
    echo "resident=$r"; grep -E "panel kernel|max" $O/${TAG}_ubp$r.txt | head -5
  done
fi
if [ "${UBT:-0}" = 1 ]; then
  timeout -k 10 120 ./tools/ubench_timeline > $O/${TAG}_ubt.txt 2>&1 || { tail $O/${TAG}_ubt.txt; exit 1; }
  head -6 $O/${TAG}_ubt.txt
fi
echo batch done
