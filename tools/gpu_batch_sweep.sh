# Larger per-GPU batches (SURVEY.md §8d config 3 regime: many chunks in flight per GPU)
export TMPDIR=/tmp; mkdir -p gpurun_out
for b in 16 32 64 128; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --chunks-per-gpu $b > gpurun_out/batch_$b.json 2>gpurun_out/batch_$b.err || { tail -5 gpurun_out/batch_$b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/batch_$b.json')); r=d['roofline'] or {}; print('B=$b', d['value'], d['breakdown'], r.get('achieved'))"
done
