"""The engine's host side under AddressSanitizer + UBSan (SURVEY.md §5 'race / memory
detection'): the scheduler, the KV page and slot allocator, the request queue, result
hand-back and the C-ABI error paths, driven by a standalone native program
(tests/native/engine_host_sanitize.cpp) built with -fsanitize on the host compilation only --
device code and the HIP runtime are not instrumented (GPU sanitizers are not available on
this pool).  Leaks are checked too, with the ROCm runtime's process-lifetime allocations
suppressed (tests/native/lsan.supp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "native", "engine_host_sanitize")
SUPP = os.path.join(ROOT, "tests", "native", "lsan.supp")


@pytest.mark.gpu
def test_engine_host_side_under_asan_ubsan():
    assert os.path.exists(BIN), ("not built: make -C map-reduced-approach-for-vietnamese-long-document-summarization_amd"
                                 "/csrc sanitize (__graft_entry__.build() runs it)")
    env = dict(os.environ,
               ASAN_OPTIONS="verify_asan_link_order=0:halt_on_error=1:detect_leaks=1:exitcode=23",
               LSAN_OPTIONS=f"suppressions={SUPP}:exitcode=24",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=25")
    r = subprocess.run([BIN], env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout[-3000:])
    print(r.stderr[-6000:])
    assert r.returncode == 0, f"exit {r.returncode} (23 ASan, 24 LSan, 25 UBSan, 1 a failed check)"
    assert "HOST_SANITIZE_OK" in r.stdout
