# persistent decode step: same-box sweep of the loaders' in-flight depth (MS_PK_DEPTH), bench lines
mkdir -p gpurun_out; O=gpurun_out/pk_depth.txt; : > $O
for d in ${DEPTHS:-12 20 28 36 44}; do
  MS_PERSIST=1 MS_PK_DEPTH=$d timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --steps 2 --warmup 1 > /tmp/pkd.json 2> /tmp/pkd.err || { tail -20 /tmp/pkd.err; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/pkd.json')); b=d['breakdown']; print('depth $d', d['value'], b['decode_ms_per_decode_step'], d['check'])" | tee -a $O
done
