# Same-box A/B of environment variants of one build (box-to-box variance is ~5-20 %, so
# variants are only compared inside one GPU call): alternating short bench lines.
#   usage: VARIANTS="- MS_X=1,MS_Y=2" ROUNDS=2 bash tools/ab_env.sh [bench args...]
mkdir -p gpurun_out; O=gpurun_out/ab_env.txt; : > $O
for r in $(seq ${ROUNDS:-2}); do
  for cfg in ${VARIANTS:--}; do
    (
      if [ "$cfg" != "-" ]; then for kv in $(echo $cfg | tr , ' '); do export "$kv"; done; fi
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps ${STEPS:-2} --warmup 1 "$@" > /tmp/ab.json 2> /tmp/ab.err
    ) || { tail -20 /tmp/ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/ab.json')); b=d['breakdown']; print('%-40s %8.3f chunks/s  prefill %7.2f ms  decode %.4f ms/step  checks %s' % ('$cfg', d['value'], b['prefill_ms_per_step'], b['decode_ms_per_decode_step'], all(d.get('check', {}).values())))" | tee -a $O
  done
done
