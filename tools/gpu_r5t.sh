# round 5: one weight arena (MS_ARENA=1) / physically contiguous weights and K/V pools (2) vs
# one allocation per matrix (0): translation reach for the decode weight stream
export TMPDIR=/tmp; mkdir -p gpurun_out/r5t; O=gpurun_out/r5t
MS_ARENA=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_fullshape.py -k "batch_invariance or host" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 1200 bash tools/ab3.sh "ar0|MS_ARENA=0|" "ar1|MS_ARENA=1|" "ar2|MS_ARENA=2|" -- --steps 3 --warmup 1 && cp gpurun_out/ab3.txt $O/ab3_arena.txt
timeout -k 10 600 bash tools/prof_ab.sh "ar0|MS_ARENA=0|" "ar2|MS_ARENA=2|" -- --steps 1 --warmup 1 && cp gpurun_out/prof_ar0.txt gpurun_out/prof_ar2.txt $O/
