# SQ PMC passes over the Q4_K_M decode Q-GEMVs (configs[4], B = 8): where the Q6_K down and
# Q4_K gate/up launches spend their cycles beyond the bytes / 6.25 TB/s line
export TMPDIR=/tmp; mkdir -p gpurun_out/r5ag; O=gpurun_out/r5ag; R=/tmp/qpmc; rm -rf $R
PRE="bench.py --weights q4_k_m --no-cpu-baseline --no-roofline --no-check --steps 1 --warmup 0 --gen-len 16"
MAPSUM_NO_GRAPHS=1 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $R/a -o run -- python3 $PRE > $R.a.log 2>&1 || { tail -30 $R.a.log; exit 1; }
MAPSUM_NO_GRAPHS=1 timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/b -o run -- python3 $PRE > $R.b.log 2>&1 || { tail -30 $R.b.log; exit 1; }
for p in a b; do python3 tools/pmc_summary.py "$(find $R/$p -name '*counter_collection.csv' | head -n 1)" | grep -E "kernel|qgemv" > $O/qgemv_pmc_$p.txt; done
cat $O/qgemv_pmc_a.txt $O/qgemv_pmc_b.txt | cut -c1-220
