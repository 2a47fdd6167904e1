# One GPU call: the round's bench lines of the other BASELINE configs -- configs[4] (Q4_K_M,
# with its rocprofv3 kernel table), configs[2] (256 chunks through 256 slots, with
# and without a natural-EOS stop set) and configs[3] (ragged hierarchical level).  Each step has
# its own limit and the chain stops at the first failure.
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out; R=/tmp/mscfg; rm -rf $R; mkdir -p $R
timeout -k 10 400 python -u bench.py --weights q4_k_m --no-cpu-baseline > $O/bench_q4_k_m.json 2> $O/bench_q4_k_m.err || { tail -20 $O/bench_q4_k_m.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --weights q4_k_m --no-cpu-baseline --no-check --no-roofline > $O/prof_bench_q4_k_m.json 2> $R/prof.err || { tail -20 $R/prof.err; exit 1; }
python3 tools/prof_summary.py "$(find $R/prof -name '*kernel_stats.csv' | head -n 1)" > $O/kernel_stats_q4_k_m.txt
timeout -k 10 400 python -u bench.py --docs 32 --max-batch 256 --steps 3 --warmup 1 --no-cpu-baseline > $O/config2_B256.json 2> $O/config2.err || { tail -20 $O/config2.err; exit 1; }
timeout -k 10 400 python -u bench.py --docs 32 --max-batch 256 --steps 1 --warmup 1 --no-cpu-baseline --eos 1000 > $O/config2_B256_eos1000.json 2> $O/config2e.err || { tail -20 $O/config2e.err; exit 1; }
timeout -k 10 400 python -u tools/bench_ragged.py > $O/ragged_config3.json 2> $O/ragged.err || { tail -20 $O/ragged.err; exit 1; }
for f in bench_q4_k_m config2_B256 config2_B256_eos1000 ragged_config3; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d.get('value'), d.get('unit'), d.get('breakdown', {}).get('decode_ms_per_decode_step'), d.get('check'))"; done
head -n 16 $O/kernel_stats_q4_k_m.txt
