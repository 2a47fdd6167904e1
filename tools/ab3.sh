# Same-box A/B lines: bench.py over several (env, library) variants, alternating, one JSON
# summary line each.  usage: bash tools/ab3.sh "TAG|ENV|LIB" ... -- [bench args]
mkdir -p gpurun_out; O=gpurun_out/ab3.txt; : > $O
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; shift
for round in 1 2; do
  for v in "${V[@]}"; do
    IFS='|' read -r tag envs lib <<< "$v"
    env $envs ${lib:+MAPSUM_LIB=$lib} timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline "$@" > /tmp/ab3.json 2> /tmp/ab3.err || { tail -20 /tmp/ab3.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/ab3.json')); b=d['breakdown']; print('$tag', d['value'], b['prefill_ms_per_step'], b['decode_ms_per_decode_step'], d['check'])" | tee -a $O
  done
done
