# round 5: K-quant row-group fix check, the whole GPU suite, the default bench line
export TMPDIR=/tmp; mkdir -p gpurun_out/r5e; O=gpurun_out/r5e
timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 2 --gen 24 --counts 1,104,128 > $O/diag_q4_fixed.txt 2>&1 || { tail -30 $O/diag_q4_fixed.txt; exit 1; }
grep -v amdgpu.ids $O/diag_q4_fixed.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; tail -12 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py > $O/bench_f16.json 2> $O/bench_f16.err || { tail -30 $O/bench_f16.err; exit 1; }
cat $O/bench_f16.json
