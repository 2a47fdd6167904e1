# Decode-chain diagnosis in one GPU call: a kernel-trace profile of the chain, then short
# bench lines for the chain off/on and for split-K choices of the folded projections.
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out; R=/tmp/mschain; rm -rf $R; mkdir -p $R
B="bench.py --no-cpu-baseline --no-roofline --no-check --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 $B > $R/prof.log 2>&1 || { tail -20 $R/prof.log; exit 1; }
python3 tools/prof_summary.py "$(find $R/prof -name '*kernel_stats.csv' | head -n 1)" > $O/chain_kernel_stats.txt && head -n 24 $O/chain_kernel_stats.txt
for cfg in "MS_CHAIN=0" "MS_CHAIN=1" "MS_CHAIN=1 MS_SPLIT_O=2 MS_SPLIT_DOWN=2" "MS_CHAIN=1 MS_SPLIT_O=3 MS_SPLIT_DOWN=4" "MS_CHAIN=1 MS_SPLIT_O=4 MS_SPLIT_DOWN=8" "MS_CHAIN=1 MS_SPLIT_QKV=3"; do
  env $cfg timeout -k 10 120 python3 $B > $R/b.json 2> $R/b.err || { tail -20 $R/b.err; exit 1; }
  echo "$cfg $(python3 -c "import json; d=json.load(open('$R/b.json')); print(d['value'], d['breakdown']['decode_ms_per_decode_step'])")" | tee -a $O/chain_sweep.txt
done
