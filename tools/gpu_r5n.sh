# round 5: transposed-accumulator GEMM epilogues (all EPIs, vector loads/stores, new statistics
# order) vs the HEAD build; gemm variants 0 / 4; combine placement
export TMPDIR=/tmp; mkdir -p gpurun_out/r5n; O=gpurun_out/r5n
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/bench_kernels.py gemm --variants 2,3 --ref-lib map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so --torch > $O/gemm_ab.txt 2>&1 || { tail -30 $O/gemm_ab.txt; exit 1; }
grep -v amdgpu.ids $O/gemm_ab.txt
timeout -k 10 900 bash tools/ab3.sh "base||map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so" "v0grp0|MS_COMBINE_GRP=0|" "v0grp1|MS_COMBINE_GRP=1|" "v4grp1|MS_COMBINE_GRP=1 MS_GEMM_VARIANT=4|" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3.txt
timeout -k 10 600 bash tools/prof_ab.sh "v0grp0|MS_COMBINE_GRP=0|" "v4grp1|MS_COMBINE_GRP=1 MS_GEMM_VARIANT=4|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_v0grp0.txt gpurun_out/prof_v4grp1.txt $O/
