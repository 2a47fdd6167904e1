export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for v in "1 0" "1 1" "0 0" "0 1"; do set -- $v
  MS_ATTN_SLABS=$1 MS_ATTN_FUSED_COMBINE=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/bench_v$1$2.log 2>&1 || exit 1
done
