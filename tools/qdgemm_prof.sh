# Kernel table of a 128-slot Q4_K_M map step with the K-quant skinny GEMM (k_qdgemm.hip) and with
# the fp16 copies through k_dgemm.hip (MS_QDGEMM=0): bash tools/qdgemm_prof.sh
export TMPDIR=/tmp; mkdir -p gpurun_out; R=/tmp/qdprof; rm -rf $R
B="bench.py --weights q4_k_m --docs 16 --max-batch 128 --steps 1 --warmup 0 --no-cpu-baseline --no-roofline --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/q -o q -- python3 $B > $R.q.log 2>&1 || { tail -20 $R.q.log; exit 1; }
MS_QDGEMM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/f -o f -- python3 $B > $R.f.log 2>&1 || { tail -20 $R.f.log; exit 1; }
for v in q f; do
  f="$(find $R/$v -name '*kernel_stats.csv' | head -n 1)"
  python3 - "$f" > gpurun_out/qdprof_$v.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:110]}')
PY
done
tail -n 3 $R.q.log; tail -n 3 $R.f.log
cat gpurun_out/qdprof_q.txt; echo; cat gpurun_out/qdprof_f.txt
