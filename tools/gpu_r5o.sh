# round 5: decode-attention v2 timeline stamps; residual GEMM epilogue (transposed) vs HEAD in the
# engine's fused form; default dispatch (variant 4) A/B; 28-layer parity on the new prefill numerics
export TMPDIR=/tmp; mkdir -p gpurun_out/r5o; O=gpurun_out/r5o
timeout -k 10 300 python -u tools/a2_stamps.py > $O/a2_stamps.txt 2>&1 || { tail -30 $O/a2_stamps.txt; exit 1; }
grep -v amdgpu.ids $O/a2_stamps.txt
timeout -k 10 600 python -u tools/bench_kernels.py gemm --resid --variants 2 --ref-lib map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so > $O/gemm_resid_ab.txt 2>&1 || { tail -30 $O/gemm_resid_ab.txt; exit 1; }
grep -E "^gemm|^base" $O/gemm_resid_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden28.py tests/test_gpu_parity.py -k "gemm or golden or prefill" -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
