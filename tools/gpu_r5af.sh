# HBM traffic of the large-batch skinny GEMMs (configs[2] regime, 128 chunks in 128 slots):
# FETCH_SIZE and WRITE_SIZE passes, per-instantiation bytes per launch
export TMPDIR=/tmp; O=gpurun_out/r5af; mkdir -p $O; R=/tmp/mspmc_dg; rm -rf $R; mkdir -p $R
SHORT="bench.py --no-cpu-baseline --no-roofline --no-check --steps 1 --warmup 0 --gen-len 16 --docs 16 --max-batch 128"
MAPSUM_NO_GRAPHS=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 $SHORT > $R/fetch.log 2>&1 || { tail -30 $R/fetch.log; exit 1; }
MAPSUM_NO_GRAPHS=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -o run -- python3 $SHORT > $R/write.log 2>&1 || { tail -30 $R/write.log; exit 1; }
FC="$(find $R/fetch -name '*counter_collection.csv' | head -n 1)"; WC="$(find $R/write -name '*counter_collection.csv' | head -n 1)"
python3 tools/pmc_summary.py "$FC" > $O/pmc_fetch_dgemm_B128.txt; python3 tools/pmc_summary.py "$WC" > $O/pmc_write_dgemm_B128.txt
python3 tools/traffic_from_pmc.py "$FC" "$WC" dgemm_kernel $O/pmc_traffic_dgemm_B128.json 128 2048 && cat $O/pmc_traffic_dgemm_B128.json
grep -E "dgemm" $O/pmc_fetch_dgemm_B128.txt $O/pmc_write_dgemm_B128.txt | cut -c1-200
