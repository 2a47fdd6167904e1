# Decode-attention variants, one GPU call: for each config (comma-separated VAR=value
# list, "-" for the defaults) a kernel-trace profile of a short bench, printing the decode
# attention kernel's average duration and the decode step time.
#   usage: SWEEP="- MS_ATTN_PPW=1 ..." ARGS="bench args" bash tools/attn_sweep.sh
export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out/attn_sweep.txt; : > $O
B="bench.py --no-cpu-baseline --no-roofline --no-check --steps 1 --warmup 0 ${ARGS}"
for cfg in ${SWEEP:--}; do
  R=/tmp/as_$$; rm -rf $R; mkdir -p $R
  (
    if [ "$cfg" != "-" ]; then for kv in $(echo $cfg | tr , ' '); do export "$kv"; done; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/prof -o run -- python3 $B > $R/b.json 2> $R/b.err
  ) || { tail -20 $R/b.err; exit 1; }
  S="$(find $R/prof -name '*kernel_stats.csv' | head -n 1)"
  python3 - "$cfg" "$S" "$R/b.json" <<'PY' | tee -a $O
import csv, json, sys
cfg, stats, bj = sys.argv[1:4]
att = [r for r in csv.DictReader(open(stats)) if "attn_decode_kernel" in r["Name"]]
comb = [r for r in csv.DictReader(open(stats)) if "attn_decode_combine" in r["Name"]]
d = json.load(open(bj))
us = lambda rs: sum(float(r["TotalDurationNs"]) for r in rs) / max(1, sum(int(r["Calls"]) for r in rs)) / 1e3
print(f"{cfg:40s} attn {us(att):7.2f} us  combine {us(comb):5.2f} us  step {d['breakdown']['decode_ms_per_decode_step']:.4f} ms  {d['value']:.3f} chunks/s")
PY
done
