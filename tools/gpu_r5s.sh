# round 5: prefill SwiGLU epilogue with v_rcp_f32 instead of the IEEE division (vs the HEAD build)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5s; O=gpurun_out/r5s
timeout -k 10 600 python -u tools/bench_kernels.py gemm --variants 3,2 --ref-lib map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so > $O/gemm_silu_ab.txt 2>&1 || { tail -30 $O/gemm_silu_ab.txt; exit 1; }
grep -E "^gemm|^base" $O/gemm_silu_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -k "gemm or prefill or decode_attention" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 bash tools/ab3.sh "base||map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so" "new||" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3.txt
