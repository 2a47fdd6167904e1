# bf16 decode split-K sweep (MS_SPLIT_QKV / MS_SPLIT_O / MS_SPLIT_DOWN), short bench runs
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "6 6 4" "4 4 4" "8 8 4" "6 6 8" "4 6 2" "3 3 4" "6 4 4"; do set -- $v
  MS_SPLIT_QKV=$1 MS_SPLIT_O=$2 MS_SPLIT_DOWN=$3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 2 > gpurun_out/split_$1_$2_$3.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/split_$1_$2_$3.json')); print('split $1 $2 $3', d['value'], d['breakdown']['decode_ms_per_step'])"
done
