# One short GPU call for the round-end record: the GPU suite, smoke(), the default bench line
# and a kernel-trace profile of the timed workload (no PMC passes; tools/gpu_round.sh has
# those).  Every GPU step has its own limit and the chain stops at the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out; R=/tmp/msfinal; rm -rf $R; mkdir -p $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_f16.json 2> $O/bench_f16.err || { tail -30 $O/bench_f16.err; exit 1; }
cat $O/bench_f16.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --no-cpu-baseline --no-check --no-roofline > $O/prof_bench_f16.json 2> $R/prof.err || { tail -30 $R/prof.err; exit 1; }
cat $O/prof_bench_f16.json
python3 tools/prof_summary.py "$(find $R/prof -name '*kernel_stats.csv' | head -n 1)" > $O/kernel_stats_f16.txt && head -n 14 $O/kernel_stats_f16.txt
echo ALL_OK
