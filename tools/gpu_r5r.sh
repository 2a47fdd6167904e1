# round 5: decode attention v2 with a dedicated prologue wave (MS_A2_ORDER=3) -- tests, stamps,
# same-box A/B against the all-waves prologue (order 0)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5r; O=gpurun_out/r5r
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -k "decode_attention or fused_qkv or decode_tail or batch_invariance or decode_b32 or config2" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
MS_A2_ORDER=3 timeout -k 10 300 python -u tools/a2_stamps.py > $O/a2_stamps_order3.txt 2>&1 || { tail -30 $O/a2_stamps_order3.txt; exit 1; }
grep -v amdgpu.ids $O/a2_stamps_order3.txt | head -16
timeout -k 10 900 bash tools/ab3.sh "ord0|MS_A2_ORDER=0|" "ord3|MS_A2_ORDER=3|" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_order.txt
timeout -k 10 600 bash tools/prof_ab.sh "ord0|MS_A2_ORDER=0|" "ord3|MS_A2_ORDER=3|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_ord0.txt gpurun_out/prof_ord3.txt $O/
