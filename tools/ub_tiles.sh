mkdir -p gpurun_out
for t in 0 128 12864 64 32; do echo "== tile $t"; SMG_GEMM_TILE=$t timeout -k 10 60 tools/ubench_gemm || exit 1; done > gpurun_out/ub_gemm_tiles.txt 2>&1
for t in 128 12864 64; do echo "== tile $t nosplit"; SMG_GEMM_NOSPLIT=1 SMG_GEMM_TILE=$t timeout -k 10 60 tools/ubench_gemm || exit 1; done > gpurun_out/ub_gemm_nosplit.txt 2>&1
