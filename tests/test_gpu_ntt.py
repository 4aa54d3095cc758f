"""GPU radix-2 NTT parity vs the oracle and golden vectors (bit-exact)."""
import numpy as np
import pytest

from helpers import fr_rows, golden

pytestmark = pytest.mark.gpu
G = golden()


@pytest.mark.parametrize("vec", G["ntt"], ids=lambda v: "n%d" % v["n"])
def test_ntt_golden(ctx, oracle, vec):
    x = fr_rows(vec["in"])
    assert oracle.fr_ints(ctx.ntt(x)) == [int(a, 16) for a in vec["fft"]]
    assert oracle.fr_ints(ctx.ntt(x, inverse=True)) == [int(a, 16) for a in vec["ifft"]]
    assert oracle.fr_ints(ctx.ntt(x, coset=7)) == [int(a, 16) for a in vec["coset_fft_g7"]]


@pytest.mark.parametrize("log_n", [1, 2, 3, 5, 9, 10, 11, 12, 13, 14, 16, 18, 20, 21, 22])
def test_ntt_vs_oracle(ctx, oracle, log_n):
    x = oracle.random_fr(1 << log_n, 40 + log_n)
    assert np.array_equal(ctx.ntt(x), oracle.fft(x))
    assert np.array_equal(ctx.ntt(x, inverse=True), oracle.fft(x, inverse=True))


@pytest.mark.parametrize("log_n", [0, 1, 4, 9, 10, 11, 15, 21])
@pytest.mark.parametrize("g", [7, 5, 0x1234567890ABCDEF1234])
def test_ntt_coset_vs_oracle(ctx, oracle, log_n, g):
    """Radix2EvaluationDomain::coset_fft / coset_ifft with an arbitrary shift:
    the first pass's fused g^i load factor and the bit reversal's n^-1 g^-i."""
    x = oracle.random_fr(1 << log_n, 70 + log_n)
    assert np.array_equal(ctx.ntt(x, coset=g), oracle.coset_fft(x, g))
    assert np.array_equal(ctx.ntt(x, inverse=True, coset=g), oracle.coset_fft(x, g, inverse=True))


def test_ntt_rejects_bad_coset(ctx, zkp, oracle):
    x = oracle.random_fr(16, 3)
    with pytest.raises(ValueError):
        ctx.ntt(x, coset=0, inverse=True)


def test_ntt_coset_roundtrip(ctx, oracle):
    x = oracle.random_fr(1 << 12, 99)
    y = ctx.ntt(x, coset=7)
    assert np.array_equal(ctx.ntt(y, inverse=True, coset=7), x)


@pytest.mark.parametrize("log_n", [20, 22, 23])
def test_ntt_roundtrip_large(ctx, oracle, log_n):
    """2^23: three DIT passes (11 gathered + 6 + 6 stages) on the natural-order path."""
    x = oracle.random_fr(1 << log_n, 7)
    y = ctx.ntt(x)
    assert np.array_equal(ctx.ntt(y, inverse=True), x)
    # X_0 = sum_j x_j
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    assert oracle.fr_ints(y[:1])[0] == sum(oracle.fr_ints(x)) % R
