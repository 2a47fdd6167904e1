# SQ counters of the large-batch skinny GEMMs (k_qdgemm.hip / k_dgemm.hip) on one shape:
#   bash tools/qdgemm_pmc.sh [shape] [rows]      (tools/bench_kernels.py qdgemm names; default gu 128)
export TMPDIR=/tmp; mkdir -p gpurun_out; R=/tmp/qdpmc; rm -rf $R
SH=${1:-gu}; MS=${2:-128}
PRE="tools/bench_kernels.py qdgemm --ms $MS --only $SH"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $R/a -o run -- python3 $PRE > $R.a.log 2>&1 || { tail -30 $R.a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/b -o run -- python3 $PRE > $R.b.log 2>&1 || { tail -30 $R.b.log; exit 1; }
for p in a b; do f="$(find $R/$p -name '*counter_collection.csv' 2>/dev/null | head -n 1)"; [ -n "$f" ] && python3 tools/pmc_summary.py "$f" | grep -E "kernel|dgemm" > gpurun_out/qdgemm_pmc_$p.txt; done
cat gpurun_out/qdgemm_pmc_*.txt
