# round 5: fused QKV + attention page-load placement A/B (MS_QA_ORDER 0/1/2), kernel tables;
# torch.matmul reference rates at the prefill GEMM shapes
export TMPDIR=/tmp; mkdir -p gpurun_out/r5h; O=gpurun_out/r5h
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullshape.py -k "fused_qkv_attention_bit_exact or ragged" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests_qa.log 2>&1 || { tail -40 $O/tests_qa.log; exit 1; }
tail -1 $O/tests_qa.log
timeout -k 10 900 bash tools/ab3.sh "plain|MS_QKV_ATTN=0|" "o0|MS_QA_ORDER=0|" "o1|MS_QA_ORDER=1|" "o2|MS_QA_ORDER=2|" -- --steps 2 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_order.txt
timeout -k 10 600 bash tools/prof_ab.sh "o1|MS_QA_ORDER=1|" "o2|MS_QA_ORDER=2|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_o1.txt gpurun_out/prof_o2.txt $O/
timeout -k 10 300 python -u tools/gemm_ref_torch.py > $O/gemm_ref_torch.txt 2>&1; cat $O/gemm_ref_torch.txt
