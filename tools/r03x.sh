set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpp_layer.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03x_t.log 2>&1; rc=$?
tail -5 gpurun_out/r03x_t.log; [ $rc -eq 0 ] || exit $rc
STEPS=20 bash tools/ab_lib.sh tri256 gp || exit 1
STEPS=10 bash tools/ab_lib.sh tri256 hvp || exit 1
STEPS=20 bash tools/ab_lib.sh tri256 mulchol || exit 1
