# Same-box A/B of two builds of libmapsum (box-to-box variance is ~5-20 %, so variants are
# only ever compared inside one GPU call): alternating short bench lines, an optional
# large-batch line (LARGE="bench args"), then the kernel micro-benchmarks of each.
#   usage: bash tools/ab.sh LIB_A LIB_B [bench args...]
A=$1; B=$2; shift 2
mkdir -p gpurun_out; O=gpurun_out/ab.txt; : > $O
run() {  # run <lib> <tag> <bench args...>
  L=$1; v=$2; shift 2
  MAPSUM_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline "$@" > /tmp/ab.json 2> /tmp/ab.err || { tail -20 /tmp/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('/tmp/ab.json')); b=d['breakdown']; print('$v', d['value'], b['prefill_ms_per_step'], b['decode_ms_per_decode_step'])" | tee -a $O
}
for v in A B A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  run $L $v --steps 3 --warmup 1 "$@"
done
if [ -n "$LARGE" ]; then
  for v in A B; do
    if [ $v = A ]; then L=$A; else L=$B; fi
    run $L "$v large" $LARGE
  done
fi
for v in A B; do
  if [ $v = A ]; then L=$A; else L=$B; fi
  echo "== $v ${KERNELS:-qgemv split}" | tee -a $O
  for k in ${KERNELS:-qgemv split}; do
    MAPSUM_LIB=$L timeout -k 10 200 python3 tools/bench_kernels.py $k --m 8 >> $O 2>&1 || exit 1
  done
done
cat $O
