# round 5: decode-attention v2 prologue timing (stamps) under the three issue orders
export TMPDIR=/tmp; mkdir -p gpurun_out/r5q; O=gpurun_out/r5q
for o in 0 2; do
  MS_A2_ORDER=$o timeout -k 10 300 python -u tools/a2_stamps.py > $O/a2_stamps_order$o.txt 2>&1 || { tail -30 $O/a2_stamps_order$o.txt; exit 1; }
  echo "== order $o"; grep -v amdgpu.ids $O/a2_stamps_order$o.txt | head -16
done
