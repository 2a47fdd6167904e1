# HBM traffic of the large-batch K-quant skinny GEMM (k_qdgemm.hip) against its algorithmic bytes,
# per decode-GEMM shape at M rows: FETCH_SIZE and WRITE_SIZE passes (one counter block each) over
# tools/bench_kernels.py qdgemm, whose > 512 MB weight rotations keep every launch cold.
#   bash tools/qdgemm_traffic.sh [rows]        -> gpurun_out/qdgemm_traffic_M<rows>.json
export TMPDIR=/tmp; mkdir -p gpurun_out; R=/tmp/qdtraffic; rm -rf $R; mkdir -p $R
MS=${1:-128}
for SH in gu qkv o down down6 lm_head6; do
  PRE="tools/bench_kernels.py qdgemm --ms $MS --only $SH"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $R/$SH.$C -o run -- python3 $PRE > $R/$SH.$C.log 2>&1 || { tail -30 $R/$SH.$C.log; exit 1; }
  done
  grep -v "^[EWI]2026" $R/$SH.FETCH_SIZE.log | tail -2
done
mkdir -p gpurun_out/qdt_csv && for d in $R/*_SIZE; do cp $d/run_counter_collection.csv gpurun_out/qdt_csv/$(basename $d).csv; done
python3 tools/qdgemm_traffic.py $R $MS > gpurun_out/qdgemm_traffic_M$MS.json && cat gpurun_out/qdgemm_traffic_M$MS.json
