# round 5: decode-attention v2 with every wave's prologue loads queued ahead of the pages
# (MS_A2_ORDER=1) -- stamps, tests, same-box A/B against the order-0 form
export TMPDIR=/tmp; mkdir -p gpurun_out/r5p; O=gpurun_out/r5p
timeout -k 10 300 python -u tools/a2_stamps.py > $O/a2_stamps_order1.txt 2>&1 || { tail -30 $O/a2_stamps_order1.txt; exit 1; }
grep -v amdgpu.ids $O/a2_stamps_order1.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -k "decode_attention or fused_qkv or decode_tail or batch_invariance" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 bash tools/ab3.sh "ord0|MS_A2_ORDER=0|" "ord1|MS_A2_ORDER=1|" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_order.txt
timeout -k 10 600 bash tools/prof_ab.sh "ord0|MS_A2_ORDER=0|" "ord1|MS_A2_ORDER=1|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_ord0.txt gpurun_out/prof_ord1.txt $O/
