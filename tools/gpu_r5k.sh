# round 5: 4-wave 256x256 GEMM (variant 3) vs the 8-wave one vs torch.matmul; GEMM tests
export TMPDIR=/tmp; mkdir -p gpurun_out/r5k; O=gpurun_out/r5k
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "gemm" -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_gemm.log 2>&1; tail -5 $O/tests_gemm.log
timeout -k 10 600 python -u tools/bench_kernels.py gemm --variants 2,3 --torch > $O/gemm_variants.txt 2>&1 || { tail -30 $O/gemm_variants.txt; exit 1; }
grep -v amdgpu.ids $O/gemm_variants.txt
