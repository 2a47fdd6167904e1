# round 5 (session 2): rebuilt tree -- whole GPU suite, smoke, default bench line, kernel table
export TMPDIR=/tmp; mkdir -p gpurun_out/r5f; O=gpurun_out/r5f
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -12 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_f16.json 2> $O/bench_f16.err || { tail -30 $O/bench_f16.err; exit 1; }
cat $O/bench_f16.json
R=/tmp/prof_f; rm -rf $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 bench.py --no-cpu-baseline --no-check --no-roofline --steps 1 --warmup 1 > $O/prof.json 2> $R.err || { tail -20 $R.err; exit 1; }
python3 tools/prof_summary.py "$(find $R -name '*kernel_stats.csv' | head -n 1)" > $O/kernel_stats_f16.txt && head -n 24 $O/kernel_stats_f16.txt
