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
    """2^23: three DIT passes (10 gathered + 7 + 6 stages) on the natural-order path."""
    x = oracle.random_fr(1 << log_n, 7)
    y = ctx.ntt(x)
    assert np.array_equal(ctx.ntt(y, inverse=True), x)
    # X_0 = sum_j x_j
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    assert oracle.fr_ints(y[:1])[0] == sum(oracle.fr_ints(x)) % R


@pytest.mark.parametrize("log_n", [0, 1, 10, 13])
@pytest.mark.parametrize("where", ["first", "last"])
def test_ntt_rejects_non_canonical_input(ctx, zkp, oracle, log_n, where):
    """An element >= r (here = r, and all-ones limbs) is ZK_ERR_ARG on both
    entry points -- checked in the first pass's load -- like every other
    Fr input of the ABI; a valid transform after it still matches."""
    import ctypes as C
    import torch
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    n = 1 << log_n
    for bad in ([(R >> (64 * i)) & (2 ** 64 - 1) for i in range(4)], [2 ** 64 - 1] * 4):
        x = oracle.random_fr(n, 5 + log_n)
        x[0 if where == "first" else n - 1] = bad
        for inverse in (False, True):
            with pytest.raises(ValueError):
                ctx.ntt(x, inverse=inverse)
        d = torch.from_numpy(x.view(np.int64).copy()).cuda()
        rc = zkp.lib().zk_ntt_fr_dev(C.c_void_p(ctx._h), C.c_void_p(d.data_ptr()), C.c_uint32(log_n), C.c_int(1),
                                    None)
        assert rc == zkp.ZK_ERR_ARG
    x = oracle.random_fr(n, 6 + log_n)
    assert np.array_equal(ctx.ntt(x), oracle.fft(x))


@pytest.mark.parametrize("log_n", [4, 11, 12, 17, 22])
@pytest.mark.parametrize("kind", ["max", "alt", "two"])
def test_ntt_extreme_inputs(ctx, oracle, log_n, kind):
    """Inputs at the top of the field (r - 1 everywhere, r - 1 / 0 alternating,
    r - 1 / r - 2) push the passes' [0, 2r) tile values (ntt.hip fr_*_lz:
    products without final subtraction, sums mod 2r with a carry out of 2^256)
    to their bounds; forward, inverse and coset must still equal the oracle."""
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    n = 1 << log_n
    lim = lambda v: [(v >> (64 * i)) & (2 ** 64 - 1) for i in range(4)]
    x = np.zeros((n, 4), dtype=np.uint64)
    x[:] = lim(R - 1)
    if kind == "alt":
        x[1::2] = 0
    elif kind == "two":
        x[1::2] = lim(R - 2)
    assert np.array_equal(ctx.ntt(x), oracle.fft(x))
    assert np.array_equal(ctx.ntt(x, inverse=True), oracle.fft(x, inverse=True))
    if log_n <= 17:
        assert np.array_equal(ctx.ntt(x, coset=7), oracle.coset_fft(x, 7))
