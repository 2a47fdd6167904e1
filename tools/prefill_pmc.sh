# Prefill kernels' counters (attention and the 256x256 GEMM), two --pmc passes over a
# prefill-dominated bench (2 generated tokens), each its own run (counter limits per block).
#   usage: TAG=r04 bash tools/prefill_pmc.sh [bench args]
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out; R=/tmp/ppmc_$$; rm -rf $R; mkdir -p $R
PRE="bench.py --no-cpu-baseline --no-roofline --no-check --steps 1 --warmup 0 --gen-len 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $R/a -o run -- python3 $PRE "$@" > $R/a.log 2>&1 || { tail -30 $R/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/b -o run -- python3 $PRE "$@" > $R/b.log 2>&1 || { tail -30 $R/b.log; exit 1; }
for p in a b; do python3 tools/pmc_summary.py "$(find $R/$p -name '*counter_collection.csv' | head -n 1)" | grep -E "kernel|attn_prefill|gemm256|gemm4w" > $O/prefill_pmc_${TAG:-x}_$p.txt; done
python3 tools/mfma_from_pmc.py "$(find $R/b -name '*counter_collection.csv' | head -n 1)" $O/prefill_pmc_${TAG:-x}_mfma.json
cat $O/prefill_pmc_${TAG:-x}_a.txt $O/prefill_pmc_${TAG:-x}_b.txt $O/prefill_pmc_${TAG:-x}_mfma.json
