# FETCH_SIZE / WRITE_SIZE passes (separate runs: they cannot share one) over a short map step
# with graphs off, reduced to HBM bytes per decode-GEMV-class launch (tools/traffic_from_pmc.py)
#   usage: TAG=f16 KSUB=gemv_kernel bash tools/gpu_pmc_traffic.sh [bench args]
export TMPDIR=/tmp; O=${O:-gpurun_out}; mkdir -p $O; R=/tmp/mspmc_$TAG; rm -rf $R; mkdir -p $R
SHORT="bench.py --no-cpu-baseline --no-roofline --no-check --steps 1 --warmup 0 --gen-len 16"
MAPSUM_NO_GRAPHS=1 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 $SHORT "$@" > $R/fetch.log 2>&1 || { tail -30 $R/fetch.log; exit 1; }
MAPSUM_NO_GRAPHS=1 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -o run -- python3 $SHORT "$@" > $R/write.log 2>&1 || { tail -30 $R/write.log; exit 1; }
FC="$(find $R/fetch -name '*counter_collection.csv' | head -n 1)"; WC="$(find $R/write -name '*counter_collection.csv' | head -n 1)"
python3 tools/pmc_summary.py "$FC" > $O/pmc_fetch_$TAG.txt; python3 tools/pmc_summary.py "$WC" > $O/pmc_write_$TAG.txt
python3 tools/traffic_from_pmc.py "$FC" "$WC" "${KSUB:-gemv_kernel}" $O/pmc_traffic_$TAG.json && cat $O/pmc_traffic_$TAG.json
