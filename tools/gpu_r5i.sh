# round 5: fused QKV + attention timeline stamps per page-load placement; hipBLASLt kernel names
export TMPDIR=/tmp; mkdir -p gpurun_out/r5i; O=gpurun_out/r5i
for o in 0 1 2; do
  MS_QA_ORDER=$o timeout -k 10 300 python -u tools/qa_stamps.py > $O/stamps_o$o.txt 2>&1 || { tail -30 $O/stamps_o$o.txt; exit 1; }
  echo "== order $o"; grep -v amdgpu.ids $O/stamps_o$o.txt
done
R=/tmp/prof_t; rm -rf $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R -o run -- python3 tools/gemm_ref_torch.py > $O/gemm_ref.txt 2>&1 || { tail -20 $O/gemm_ref.txt; exit 1; }
python3 tools/prof_summary.py "$(find $R -name '*kernel_stats.csv' | head -n 1)" > $O/gemm_ref_kernels.txt; head -n 12 $O/gemm_ref_kernels.txt
python3 - "$(find $R -name '*kernel_stats.csv' | head -n 1)" > $O/gemm_ref_names.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r.get("Name", r.get("KernelName", "")), r.get("Calls", ""), r.get("AverageNs", ""))
PY
cat $O/gemm_ref_names.txt
