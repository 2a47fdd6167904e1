# round 5: K-quant row-group bisect; attention v2 in-launch merge (sc1 hand-off); nt weights A/B
export TMPDIR=/tmp; mkdir -p gpurun_out/r5d; O=gpurun_out/r5d
timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 2 --gen 16 --counts 1,96,97,104 > $O/diag_q4_a.txt 2>&1 || { tail -30 $O/diag_q4_a.txt; exit 1; }
grep -v amdgpu.ids $O/diag_q4_a.txt
MS_QSPLIT=1 timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 2 --gen 16 --counts 1,104 > $O/diag_q4_qsplit1.txt 2>&1 || { tail -30 $O/diag_q4_qsplit1.txt; exit 1; }
grep -v amdgpu.ids $O/diag_q4_qsplit1.txt
MS_QGEMV_GS=0 timeout -k 10 300 python -u tools/diag_q4_rowgroups.py --layers 2 --gen 16 --counts 1,104 > $O/diag_q4_gs0.txt 2>&1 || { tail -30 $O/diag_q4_gs0.txt; exit 1; }
grep -v amdgpu.ids $O/diag_q4_gs0.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "attention_v2" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_attn.log 2>&1 || { tail -40 $O/tests_attn.log; exit 1; }
tail -2 $O/tests_attn.log
L=map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum
timeout -k 10 900 bash tools/ab3.sh "v1|MS_ATTN_V2=0|" "v2|MS_ATTN_V2=1|" "v2t|MS_ATTN_V2=1 MS_ATTN_TICKET=1|" "v2nt|MS_ATTN_V2=1|$PWD/$L/libmapsum_nt.so" -- --steps 2 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_attn_nt.txt
timeout -k 10 600 bash tools/prof_ab.sh "v2t|MS_ATTN_V2=1 MS_ATTN_TICKET=1|" "v2nt|MS_ATTN_V2=1|$PWD/$L/libmapsum_nt.so" -- --steps 1 --warmup 1 && cp gpurun_out/prof_v2t.txt gpurun_out/prof_v2nt.txt $O/
