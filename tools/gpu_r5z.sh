# k-half gate/up by default: skinny-GEMM tests, the large-engine regime tests, configs[2] bench
export TMPDIR=/tmp; mkdir -p gpurun_out/r5z; O=gpurun_out/r5z
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "dgemm or row_scale" > $O/t_dgemm.log 2>&1 || { tail -30 $O/t_dgemm.log; exit 1; }
tail -2 $O/t_dgemm.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_golden28_regimes.py tests/test_gpu_fullshape.py -s > $O/t_regimes.log 2>&1 || { tail -40 $O/t_regimes.log; exit 1; }
grep -E "PASS|FAIL|worst|agree" $O/t_regimes.log | tail -40
timeout -k 10 400 python -u bench.py --docs 32 --max-batch 128 --steps 3 --warmup 1 --no-cpu-baseline > $O/config2_B128.json 2> $O/config2.err || { tail -20 $O/config2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/config2_B128.json')); print('config2', d.get('value'), d.get('breakdown', {}).get('decode_ms_per_decode_step'), d.get('check'))"
