# Skinny GEMM vs the weight-streaming GEMV at 8 / 16 rows (bench_kernels dgemm, kh 2 and wn 8)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5ac; O=gpurun_out/r5ac
timeout -k 10 300 python -u tools/bench_kernels.py dgemm --kh 2 > $O/dgemm_kh2.txt 2>&1 || { tail -20 $O/dgemm_kh2.txt; exit 1; }
MS_DGEMM_WN=8 timeout -k 10 300 python -u tools/bench_kernels.py dgemm --kh 1 > $O/dgemm_wn8.txt 2>&1 || { tail -20 $O/dgemm_wn8.txt; exit 1; }
grep -E "M=  8|M= 16" $O/dgemm_kh2.txt $O/dgemm_wn8.txt
