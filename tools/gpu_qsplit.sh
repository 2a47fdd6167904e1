# Quantised split-K: new parity tests, then a bench sweep of MS_QSPLIT (0 = the bf16 splits).
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "qgemv or quant" > gpurun_out/qsplit_tests.log 2>&1 || { tail -30 gpurun_out/qsplit_tests.log; exit 1; }
tail -2 gpurun_out/qsplit_tests.log
for v in 1 0 2 3 4; do
  MS_QSPLIT=$v timeout -k 10 200 python bench.py --weights q4_k_m --no-cpu-baseline --steps 2 > gpurun_out/qsplit_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/qsplit_$v.json')); r=d['roofline']; print('QSPLIT=$v', d['value'], d['breakdown']['decode_ms_per_step'], r['achieved'], r['avg_launch_us'])"
done
