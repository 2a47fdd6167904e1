# round 5: K-quant row-group diagnostic; decode attention v2 (one page per wave) -- parity,
# same-box A/B, kernel stats
export TMPDIR=/tmp; mkdir -p gpurun_out/r5c; O=gpurun_out/r5c
timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 2 --gen 32 --counts 1,8,64,65,72,128 > $O/diag_q4_l2.txt 2>&1 || { tail -30 $O/diag_q4_l2.txt; exit 1; }
grep -v amdgpu.ids $O/diag_q4_l2.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "attention_v2 or batch_invariance or attention_variants" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_attn.log 2>&1 || { tail -40 $O/tests_attn.log; exit 1; }
tail -2 $O/tests_attn.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden28.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests_g28.log 2>&1 || { tail -40 $O/tests_g28.log; exit 1; }
tail -2 $O/tests_g28.log
VARIANTS="MS_ATTN_V2=0 MS_ATTN_V2=1 MS_ATTN_V2=1,MS_ATTN_TICKET=1" ROUNDS=2 STEPS=2 timeout -k 10 600 bash tools/ab_env.sh && cp gpurun_out/ab_env.txt $O/ab_attn_v2.txt
for v in 0 1 2; do
  R=/tmp/prof_v$v; rm -rf $R
  MS_ATTN_V2=$((v>0)) MS_ATTN_TICKET=$((v>1)) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 bench.py --no-cpu-baseline --no-check --no-roofline --steps 1 --warmup 1 > $O/prof_v$v.json 2> $R.err || { tail -20 $R.err; exit 1; }
  python3 tools/prof_summary.py "$(find $R -name '*kernel_stats.csv' | head -n 1)" > $O/kernel_stats_attn_v$v.txt && head -n 12 $O/kernel_stats_attn_v$v.txt
done
timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 28 --gen 24 --counts 1,64,65,128 > $O/diag_q4_l28.txt 2>&1 || { tail -30 $O/diag_q4_l28.txt; exit 1; }
grep -v amdgpu.ids $O/diag_q4_l28.txt
