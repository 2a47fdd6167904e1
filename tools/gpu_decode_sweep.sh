# Decode variants in one GPU call: the GPU parity tests touching decode, a kernel-trace
# profile of the default bench, then short bench lines over the residual-fusion choice.
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out; R=/tmp/msdec; rm -rf $R; mkdir -p $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/dec_tests.log 2>&1 || { tail -30 $O/dec_tests.log; exit 1; }
tail -2 $O/dec_tests.log
B="bench.py --no-cpu-baseline --no-roofline --no-check --steps 2 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 $B > $R/prof.log 2>&1 || { tail -20 $R/prof.log; exit 1; }
python3 tools/prof_summary.py "$(find $R/prof -name '*kernel_stats.csv' | head -n 1)" > $O/dec_kernel_stats.txt && head -n 24 $O/dec_kernel_stats.txt
for cfg in ${SWEEP:-"MS_RESID_FUSED=1" "MS_RESID_FUSED=0"}; do
  env $cfg timeout -k 10 120 python3 $B > $R/b.json 2> $R/b.err || { tail -20 $R/b.err; exit 1; }
  echo "$cfg $(python3 -c "import json; d=json.load(open('$R/b.json')); print(d['value'], d['breakdown']['decode_ms_per_decode_step'])")" | tee -a $O/dec_sweep.txt
done
