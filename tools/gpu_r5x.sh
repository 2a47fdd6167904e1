# Skinny-GEMM block forms over split counts (bench_kernels dgemm, kh 1 vs 2)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5x; O=gpurun_out/r5x
for kh in 1 2; do
  timeout -k 10 300 python -u tools/bench_kernels.py dgemm --kh $kh > $O/dgemm_kh$kh.txt 2>&1 || { tail -20 $O/dgemm_kh$kh.txt; exit 1; }
  cat $O/dgemm_kh$kh.txt
done
