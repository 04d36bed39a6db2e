"""CPU sanitizer builds (ASan on the CPU twin; host C++):

* oracle/lib/sanitize_check -- the C twin (sampler_ref.c) under ASan+UBSan,
  every entry point on small inputs;
* _build/san/plan_check -- libqba's host-side C++ (resource planning:
  gate validation, permutation mask, union-find registers, alias tables,
  closed-form classification, stage tables, program image; the error
  channel) under ASan+UBSan, without a GPU (hipcc, -Xarch_host sanitizers:
  device code is not instrumented).

Both are built by __graft_entry__.build(); a test builds them if missing."""
import os
import subprocess

import pytest

from conftest import ROOT, PKG_NAME

CHECKS = [
    (ROOT / "oracle", "sanitize", ROOT / "oracle" / "lib" / "sanitize_check"),
    (ROOT / PKG_NAME / "csrc", "sanitize", ROOT / PKG_NAME / "_build" / "san" / "plan_check"),
]


@pytest.mark.parametrize("src,target,binary", CHECKS, ids=["c_twin", "host_cpp"])
def test_sanitized_build_runs_clean(src, target, binary):
    if not binary.exists():
        subprocess.run(["make", "-C", str(src), target], check=True, capture_output=True, timeout=600)
    env = dict(os.environ, OMP_NUM_THREADS="2", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    out = subprocess.run([str(binary)], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    assert "all" in out.stdout and "passed" in out.stdout
