# round 5: fused QKV projection + decode attention (k_qkvattn.hip) -- bit-exactness, timeout
# recovery, 28-layer fixtures through it, same-box A/B, kernel table
export TMPDIR=/tmp; mkdir -p gpurun_out/r5g; O=gpurun_out/r5g
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullshape.py -k "fused_qkv" -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/tests_qa.log 2>&1 || { tail -60 $O/tests_qa.log; exit 1; }
grep -E "passed|failed|PASSED|FAILED" $O/tests_qa.log | tail -8
timeout -k 10 900 bash tools/ab3.sh "plain|MS_QKV_ATTN=0|" "fused|MS_QKV_ATTN=1|" -- --steps 2 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_qkv_attn.txt
timeout -k 10 600 bash tools/prof_ab.sh "fused|MS_QKV_ATTN=1|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_fused.txt $O/
head -n 14 $O/prof_fused.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_golden28.py -m gpu -x -q --timeout 800 --timeout-method thread -p no:cacheprovider > $O/tests_g28.log 2>&1 || { tail -40 $O/tests_g28.log; exit 1; }
tail -2 $O/tests_g28.log
