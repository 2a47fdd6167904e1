# One GPU call: parity tests, the default bench line, a kernel-trace profile of the same
# bench, two PMC passes (FETCH_SIZE / WRITE_SIZE cannot share a pass) over a short map
# step with graphs off so every dispatch is attributed, and one MFMA-utilisation pass over
# a prefill-only step.  Every GPU step has its own limit and the chain stops at the first
# failure.  Raw profiler output stays in /tmp on the box; only summaries come back under
# gpurun_out/.
#   usage: bash tools/gpu_round.sh [bench args...]   (e.g. --weights q4_k_m)
export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out; R=/tmp/msprof; rm -rf $R; mkdir -p $R
TAG=${TAG:-f16}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py "$@" > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -30 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
# the profiled run is the timed workload only: no self-check / roofline extra steps (their
# B=1 rerun and event-bracketed step would fold other batch shapes into the averages)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --no-cpu-baseline --no-check --no-roofline "$@" > $O/prof_bench_$TAG.json 2> $R/prof.err || { tail -30 $R/prof.err; exit 1; }
cat $O/prof_bench_$TAG.json
python3 tools/prof_summary.py "$(find $R/prof -name '*kernel_stats.csv' | head -n 1)" > $O/kernel_stats_$TAG.txt && head -n 20 $O/kernel_stats_$TAG.txt
SHORT="bench.py --no-cpu-baseline --no-roofline --no-check --steps 1 --warmup 0 --gen-len 16"
MAPSUM_NO_GRAPHS=1 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/pmc_fetch -o run -- python3 $SHORT "$@" > $R/pmc_fetch.log 2>&1 || { tail -30 $R/pmc_fetch.log; exit 1; }
MAPSUM_NO_GRAPHS=1 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/pmc_write -o run -- python3 $SHORT "$@" > $R/pmc_write.log 2>&1 || { tail -30 $R/pmc_write.log; exit 1; }
FC="$(find $R/pmc_fetch -name '*counter_collection.csv' | head -n 1)"; WC="$(find $R/pmc_write -name '*counter_collection.csv' | head -n 1)"
python3 tools/pmc_summary.py "$FC" > $O/pmc_fetch_$TAG.txt; python3 tools/pmc_summary.py "$WC" > $O/pmc_write_$TAG.txt
python3 tools/traffic_from_pmc.py "$FC" "$WC" "${KSUB:-gemv_kernel}" $O/pmc_traffic_$TAG.json
PRE="bench.py --no-cpu-baseline --no-roofline --no-check --steps 1 --warmup 0 --gen-len 2"
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/pmc_mfma -o run -- python3 $PRE "$@" > $R/pmc_mfma.log 2>&1 || { tail -30 $R/pmc_mfma.log; exit 1; }
python3 tools/mfma_from_pmc.py "$(find $R/pmc_mfma -name '*counter_collection.csv' | head -n 1)" $O/pmc_mfma_$TAG.json
# instruction mix of every kernel (8 SQ counters, one pass) over the short decode step
MAPSUM_NO_GRAPHS=1 timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/pmc_sq -o run -- python3 $SHORT "$@" > $R/pmc_sq.log 2>&1 || { tail -30 $R/pmc_sq.log; exit 1; }
python3 tools/pmc_summary.py "$(find $R/pmc_sq -name '*counter_collection.csv' | head -n 1)" > $O/pmc_sq_$TAG.txt
echo ALL_OK
