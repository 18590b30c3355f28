mkdir -p gpurun_out
for t in 0 64 6432 12864 12832; do echo "== tile $t"; SMG_GEMM_TILE=$t timeout -k 10 60 tools/ubench_gemm || exit 1; done > gpurun_out/ub_gemm_tiles2.txt 2>&1
