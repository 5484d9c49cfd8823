"""CPU, no GPU: the sanitizer leg of SURVEY §5.  The kernel's CPU twin (oracle/scvx_cpu.cpp) and the FOH
restatement (oracle/foh_ref.c) -- the checkers every QP GPU test and the CPU baseline rest on -- built with
-fsanitize=address,undefined and no recovery (`make -C oracle asan`), run cold and warm-started on every
problem family of the tests (tools/asan_twin.py); any sanitizer report aborts the run.  The sanitized
outputs must equal the regular -O3 build's (same statuses, objective 1e-8 relative)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_twin_and_foh_are_sanitizer_clean():
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import asan_twin
    assert asan_twin.main() == 0
