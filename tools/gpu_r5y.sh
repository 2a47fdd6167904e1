# Skinny-GEMM block forms kh 2 vs 4 (bench_kernels dgemm)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5y; O=gpurun_out/r5y
for kh in 2 4; do
  timeout -k 10 300 python -u tools/bench_kernels.py dgemm --kh $kh > $O/dgemm_kh$kh.txt 2>&1 || { tail -20 $O/dgemm_kh$kh.txt; exit 1; }
  grep -E "^gu" $O/dgemm_kh$kh.txt
done
