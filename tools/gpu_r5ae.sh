# Prefill GEMM tiles for the residual (O / down) epilogue: 128x128 (v1) vs 256x256 8-wave (v2) vs 4-wave (v3)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5ae; O=gpurun_out/r5ae
timeout -k 10 300 python -u tools/bench_kernels.py gemm --resid --variants 2,1,3 > $O/gemm_resid_tiles.txt 2>&1 || { tail -20 $O/gemm_resid_tiles.txt; exit 1; }
grep -E "^gemm" $O/gemm_resid_tiles.txt
