"""Non-default prover paths stay bit-exact, each in a child process (the
switches are read once per process).  The unfused quotient path (ZK_NTT_FUSE=0: iNTT, separate n^-1 g^i scale,
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
    res = subprocess.run([sys.executable, os.path.join(HERE, "unfused_quotient_check.py"), "ZK_NTT_FUSE=0", "0", "1", "11",
                          "12", "21"],
                         env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert res.stdout.count(" ok") == 5


@pytest.mark.timeout(300)
def test_large_domain_quotient_path_matches_oracle():
    """ZK_NTT_FUSE=0 ZK_H_NATURAL=1: the quotient path the library picks from
    2^23 constraints up (separate iNTT / bit-reversed-table coset scale / NTT,
    and the final coset iNTT in natural order through ntt_natural), forced
    at 1-, 2- and 3-pass sizes including the size-1 domain."""
    env = dict(os.environ, ZK_NTT_FUSE="0", ZK_H_NATURAL="1")
    res = subprocess.run([sys.executable, os.path.join(HERE, "unfused_quotient_check.py"), "ZK_H_NATURAL=1", "0", "1",
                          "11", "12", "21"], env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert res.stdout.count(" ok") == 5


@pytest.mark.timeout(300)
def test_natural_final_with_fused_shift_matches_oracle():
    """ZK_H_NATURAL=1 with the fused coset shift (the two switches combine)."""
    env = dict(os.environ, ZK_H_NATURAL="1")
    res = subprocess.run([sys.executable, os.path.join(HERE, "unfused_quotient_check.py"), "ZK_H_NATURAL=1", "2",
                          "13"], env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert res.stdout.count(" ok") == 2


@pytest.mark.timeout(300)
def test_lazy_accumulate_matches_oracle():
    """ZK_LAZY_ACCUM=1: the G1 bucket accumulate in csrc/lazy.hpp's redundant
    signed-limb Fq form (an opt-in experiment) against the oracle."""
    env = dict(os.environ, ZK_LAZY_ACCUM="1")
    res = subprocess.run([sys.executable, os.path.join(HERE, "unfused_quotient_check.py"), "ZK_LAZY_ACCUM=1", "2", "10",
                          "16"], env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert res.stdout.count(" ok") == 3


@pytest.mark.timeout(300)
def test_packed_bases_match_oracle():
    """ZK_BASE_PAD=0: the proving key's window copies stay packed (96-byte G1,
    192-byte G2 points) instead of line-padded -- the accumulate's base
    stride is a launch parameter, so both layouts must prove the same bytes."""
    env = dict(os.environ, ZK_BASE_PAD="0")
    res = subprocess.run([sys.executable, os.path.join(HERE, "unfused_quotient_check.py"), "ZK_BASE_PAD=0", "3", "10",
                          "14"], env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert res.stdout.count(" ok") == 3


@pytest.mark.timeout(300)
def test_three_window_plan_matches_oracle():
    """ZK_PROVE_WIN_C=22: the 3-window / 2^21-bucket plan the library picks
    from 2^24 constraints up, forced at small sizes (the batch keys reach
    23 bits, so the radix sort, merge and bucket reduction see 2^21-bucket
    segments)."""
    env = dict(os.environ, ZK_PROVE_WIN_C="22")
    res = subprocess.run([sys.executable, os.path.join(HERE, "unfused_quotient_check.py"), "ZK_PROVE_WIN_C=22", "4",
                          "12"], env=env, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    assert res.stdout.count(" ok") == 2
