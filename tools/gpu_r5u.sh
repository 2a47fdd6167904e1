# round 5: residual GEMM on the 4-wave tile at K <= 4096 (gemm variant 5) vs the default (4);
# packed-gain epilogue bit-identity (GEMM tests)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5u; O=gpurun_out/r5u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -k "gemm or prefill" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 bash tools/ab3.sh "v4|MS_GEMM_VARIANT=4|" "v5|MS_GEMM_VARIANT=5|" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_v5.txt
timeout -k 10 600 bash tools/prof_ab.sh "v4|MS_GEMM_VARIANT=4|" "v5|MS_GEMM_VARIANT=5|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_v4.txt gpurun_out/prof_v5.txt $O/
