export TMPDIR=/tmp; mkdir -p gpurun_out/r5a; O=gpurun_out/r5a
timeout -k 10 700 python -u -m pytest tests/test_gpu_golden28_regimes.py tests/test_gpu_fullshape.py tests/test_gpu_parity.py::test_wide_hidden_prefill_takes_the_plain_residual_path -m gpu -x -v -s --timeout 600 --timeout-method thread > $O/new_tests.log 2>&1 || { tail -60 $O/new_tests.log; exit 1; }
grep -E "worst per-layer|teacher-forced|free-running|logits sketch|differ|passed|failed" $O/new_tests.log | tail -80
timeout -k 10 400 python -u bench.py > $O/bench_f16.json 2> $O/bench_f16.err || { tail -30 $O/bench_f16.err; exit 1; }
cat $O/bench_f16.json
