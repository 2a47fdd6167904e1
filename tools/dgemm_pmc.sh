export TMPDIR=/tmp; mkdir -p gpurun_out; R=/tmp/dgpmc; rm -rf $R
PRE="bench.py --no-cpu-baseline --no-roofline --no-check --docs 32 --max-batch 128 --steps 1 --warmup 0 --gen-len 8"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $R/a -o run -- python3 $PRE > $R.a.log 2>&1 || { tail -30 $R.a.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/b -o run -- python3 $PRE > $R.b.log 2>&1 || { tail -30 $R.b.log; exit 1; }
for p in a b; do python3 tools/pmc_summary.py "$(find $R/$p -name '*counter_collection.csv' | head -n 1)" | grep -E "kernel|dgemm|attn_decode" > gpurun_out/dgemm_pmc_$p.txt; done
cat gpurun_out/dgemm_pmc_a.txt gpurun_out/dgemm_pmc_b.txt
