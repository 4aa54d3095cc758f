"""Host AddressSanitizer + UndefinedBehaviorSanitizer runs (race
detection / sanitizers): the C oracle (oracle/san_check.c drives every
exported routine, 1 and 4 OpenMP threads) and the host-side C++ of the
product library (tools/host_san_check.cpp over host_ec.hpp / host_pairing.hpp:
MSM tails, Straus s*pi_A + r*B1, the verifier's pairing).  Device code cannot
run under a sanitizer on this pool; these are host builds with g++ / gcc."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-C", ORACLE, "san"], check=True, capture_output=True, timeout=300)


@pytest.mark.parametrize("prog,marker", [("san_check", "oracle sanitizer check ok"),
                                         ("host_san_check", "host sanitizer check ok")])
def test_sanitized_run(san_build, prog, marker):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="4")
    res = subprocess.run([os.path.join(ORACLE, "_san", prog)], env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-4000:]
    assert marker in res.stdout
    assert "runtime error" not in res.stderr and "ERROR: AddressSanitizer" not in res.stderr
