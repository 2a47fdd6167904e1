# round 5: decode-attention tuning hook bit-identity; decode attention tests
export TMPDIR=/tmp; mkdir -p gpurun_out/r5v; O=gpurun_out/r5v
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullshape.py tests/test_gpu_parity.py -k "attention or decode_tail" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -30
