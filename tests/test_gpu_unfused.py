"""The unfused quotient path (ZK_NTT_FUSE=0: iNTT, separate n^-1 g^i scale,
NTT) stays bit-exact: it is the fallback the fused tile kernel replaced and
no other test runs it (the switch is read once per process, so a child
process runs it).  Sizes cover 1 NTT pass (2^0 .. 2^11), 2 passes (2^12) and
3 passes (2^21)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.timeout(300)
def test_unfused_quotient_matches_oracle():
    env = dict(os.environ, ZK_NTT_FUSE="0")
    res = subprocess.run([sys.executable, os.path.join(HERE, "unfused_quotient_check.py"), "0", "1", "11", "12", "21"],
                         env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert res.stdout.count(" ok") == 5
