export TMPDIR=/tmp; mkdir -p gpurun_out/r5b; O=gpurun_out/r5b
timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 2 --gen 32 --counts 1,8,64,65,72,128 > $O/diag_q4_l2.txt 2>&1 || { tail -30 $O/diag_q4_l2.txt; exit 1; }
cat $O/diag_q4_l2.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 28 --gen 24 --counts 1,64,65,128 > $O/diag_q4_l28.txt 2>&1 || { tail -30 $O/diag_q4_l28.txt; exit 1; }
cat $O/diag_q4_l28.txt | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1; tail -15 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py > $O/bench_f16.json 2> $O/bench_f16.err || { tail -30 $O/bench_f16.err; exit 1; }
cat $O/bench_f16.json
