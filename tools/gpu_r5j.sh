# round 5: prefill GEMM variants (2: 8-wave 256x256, 3: 4-wave 256x256) against torch.matmul
# (hipBLASLt) on the same operands, same process
export TMPDIR=/tmp; mkdir -p gpurun_out/r5j; O=gpurun_out/r5j
timeout -k 10 600 python -u tools/bench_kernels.py gemm --variants 2,3 --torch > $O/gemm_variants.txt 2>&1 || { tail -30 $O/gemm_variants.txt; exit 1; }
grep -v amdgpu.ids $O/gemm_variants.txt
O=gpurun_out/r5j TAG=q4_k_m KSUB=qgemv timeout -k 10 500 bash tools/gpu_pmc_traffic.sh --weights q4_k_m
O=gpurun_out/r5j TAG=f16 KSUB=gemv_kernel timeout -k 10 500 bash tools/gpu_pmc_traffic.sh
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "gemm" -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_gemm.log 2>&1; tail -5 $O/tests_gemm.log
