# configs[2] decode attention: v1 (8 pages per wave, default at >16 slots) vs v2 (one page per wave)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5ad; O=gpurun_out/r5ad
for v in 0 1; do
  MS_ATTN_V2=$v timeout -k 10 300 python -u bench.py --docs 32 --max-batch 128 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/config2_v2_$v.json 2> $O/config2_v2_$v.err || { tail -20 $O/config2_v2_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/config2_v2_$v.json')); print('attn_v2=$v', d.get('value'), d.get('breakdown', {}).get('decode_ms_per_decode_step'), d.get('check'))"
done
