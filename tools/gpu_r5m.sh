# round 5: (a) decode-attention combine, exact preloads + XCD-matched placement (MS_COMBINE_GRP);
# (b) prefill GEMM epilogues on the transposed accumulator (vector stores) vs the HEAD build
export TMPDIR=/tmp; mkdir -p gpurun_out/r5m; O=gpurun_out/r5m
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -k "decode_attention or fused_qkv_attention_bit or decode_tail or gemm or prefill_packing" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/bench_kernels.py gemm --variants 2,3 --ref-lib map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so --torch > $O/gemm_ab.txt 2>&1 || { tail -30 $O/gemm_ab.txt; exit 1; }
grep -v amdgpu.ids $O/gemm_ab.txt
timeout -k 10 900 bash tools/ab3.sh "base|MS_COMBINE_GRP=1|map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so" "grp0|MS_COMBINE_GRP=0|" "grp1|MS_COMBINE_GRP=1|" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3.txt
timeout -k 10 600 bash tools/prof_ab.sh "grp0|MS_COMBINE_GRP=0|" "grp1|MS_COMBINE_GRP=1|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_grp0.txt gpurun_out/prof_grp1.txt $O/
