# Skinny-GEMM 128-row blocks (MS_DGEMM_WN=8) over split counts, kh 1
export TMPDIR=/tmp; mkdir -p gpurun_out/r5ab; O=gpurun_out/r5ab
MS_DGEMM_WN=8 timeout -k 10 300 python -u tools/bench_kernels.py dgemm --kh 1 > $O/dgemm_wn8.txt 2>&1 || { tail -20 $O/dgemm_wn8.txt; exit 1; }
cat $O/dgemm_wn8.txt
