# One GPU call: the GPU suite, then same-box A/B bench lines of the working tree against the
# HEAD build (tools/build_base.sh).  A test FAILURE (rc 1) still runs the A/B; a crash, abort
# or time limit (any other rc) ends the call there.
#   usage: bash tools/gpu_check_ab.sh [pytest selection...]
export TMPDIR=/tmp; mkdir -p gpurun_out
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
BASE=map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so
bash tools/ab3.sh "base||$PWD/$BASE" "new||" -- --steps 3 --warmup 1 || exit 1
exit $rc
