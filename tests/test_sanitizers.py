"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer:
the oracle's restatement (oracle/cpu_ref.cpp) and the FASTA parser
(dbindex_amd/csrc/dbi_fasta.cpp) built from their sources with
tools/sanitize/Makefile and driven by tools/sanitize/harness.cpp (edge cases,
multi-threaded paths).  Any memory error, leak or UB aborts the harness."""
from __future__ import annotations

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "sanitize")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", SAN], check=True)
    # (verify_asan_link_order=0: the ASan runtime need not be the first library a
    # process environment may preload)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(SAN, "build", "harness")], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
    assert "ok" in r.stdout
