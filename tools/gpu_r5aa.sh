# Full-tree check after the k-half gate/up GEMM: GPU suite, smoke, default bench, then a
# kernel-trace profile of the configs[2] workload (skinny GEMMs at 128 slots)
bash tools/gpu_final.sh || exit 1
export TMPDIR=/tmp; O=gpurun_out; R=/tmp/mscfg2; rm -rf $R; mkdir -p $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 bench.py --docs 32 --max-batch 128 --steps 1 --warmup 1 --no-cpu-baseline --no-check --no-roofline > $O/prof_config2.json 2> $R/prof.err || { tail -30 $R/prof.err; exit 1; }
python3 tools/prof_summary.py "$(find $R/prof -name '*kernel_stats.csv' | head -n 1)" > $O/kernel_stats_config2.txt && head -n 16 $O/kernel_stats_config2.txt
timeout -k 10 400 python -u bench.py --docs 32 --max-batch 128 --steps 3 --warmup 1 --no-cpu-baseline > $O/config2_B128.json 2> $O/config2.err || { tail -20 $O/config2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/config2_B128.json')); print('config2', d.get('value'), d.get('breakdown', {}).get('decode_ms_per_decode_step'), d.get('check'))"
