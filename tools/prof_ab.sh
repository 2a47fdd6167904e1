# Same-box kernel tables of several (env, library) variants: one rocprofv3 --kernel-trace
# --stats pass each over a short bench (no self-check / roofline extra steps), summarised by
# tools/prof_summary.py into gpurun_out/prof_<tag>.txt.
#   usage: bash tools/prof_ab.sh "TAG|ENV|LIB" ... -- [bench args]
export TMPDIR=/tmp; mkdir -p gpurun_out
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; shift
for v in "${V[@]}"; do
  IFS='|' read -r tag envs lib <<< "$v"
  R=/tmp/profab_$tag; rm -rf $R
  env $envs ${lib:+MAPSUM_LIB=$lib} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 bench.py --no-cpu-baseline --no-roofline --no-check "$@" > $R.json 2> $R.err || { tail -20 $R.err; exit 1; }
  python3 tools/prof_summary.py "$(find $R -name '*kernel_stats.csv' | head -n 1)" > gpurun_out/prof_$tag.txt
  python3 tools/prof_summary.py "$(find $R -name '*kernel_trace.csv' | head -n 1)" > gpurun_out/prof_${tag}_grid.txt
  echo "== $tag"; head -n 16 gpurun_out/prof_${tag}_grid.txt
done
