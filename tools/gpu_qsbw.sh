# Q4 GEMV super-blocks-per-wave sweep (MS_QSBW; 0 = heuristic) x split (MS_QSPLIT)
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "0 0" "2 0" "1 0" "2 1" "0 1"; do set -- $v
  MS_QSBW=$1 MS_QSPLIT=$2 timeout -k 10 200 python bench.py --weights q4_k_m --no-cpu-baseline --steps 2 > gpurun_out/qsbw_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/qsbw_$1_$2.json')); r=d['roofline']; print('QSBW=$1 QSPLIT=$2', d['value'], d['breakdown']['decode_ms_per_step'], r['achieved'], r['avg_launch_us'])"
done
