# Skinny-GEMM k-half form (MS_DGEMM_KH=2): kernel check + timing, then configs[2] A/B
export TMPDIR=/tmp; mkdir -p gpurun_out/r5w; O=gpurun_out/r5w
timeout -k 10 240 python -u tools/dgemm_kh.py > $O/dgemm_kh.txt 2>&1 || { tail -20 $O/dgemm_kh.txt; exit 1; }
cat $O/dgemm_kh.txt
for kh in 1 2; do
  MS_DGEMM_KH=$kh timeout -k 10 300 python -u bench.py --docs 32 --max-batch 128 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $O/config2_kh$kh.json 2> $O/config2_kh$kh.err || { tail -20 $O/config2_kh$kh.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/config2_kh$kh.json')); print('kh$kh', d.get('value'), d.get('breakdown', {}).get('decode_ms_per_decode_step'), d.get('check'))"
done
