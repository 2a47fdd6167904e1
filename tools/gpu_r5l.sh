# round 5: decode-attention combine with exact preloads and XCD-matched placement (MS_COMBINE_GRP)
export TMPDIR=/tmp; mkdir -p gpurun_out/r5l; O=gpurun_out/r5l
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullshape.py -k "decode_attention or fused_qkv_attention_bit or decode_tail" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_combine.log 2>&1 || { tail -40 $O/tests_combine.log; exit 1; }
tail -1 $O/tests_combine.log
timeout -k 10 900 bash tools/ab3.sh "grp0|MS_COMBINE_GRP=0|" "grp1|MS_COMBINE_GRP=1|" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_combine.txt
timeout -k 10 600 bash tools/prof_ab.sh "grp0|MS_COMBINE_GRP=0|" "grp1|MS_COMBINE_GRP=1|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_grp0.txt gpurun_out/prof_grp1.txt $O/
