"""GPU MSM parity (libzkp_amd.so through the C ABI) vs the oracle and the
golden vectors.  Bit-exact: MSM outputs are unique affine group elements."""
import numpy as np
import pytest

from helpers import fr_rows, g1_words, g2_words, golden

pytestmark = pytest.mark.gpu
G = golden()


@pytest.mark.parametrize("vec", G["msm"], ids=lambda v: v["name"])
def test_msm_golden(ctx, vec):
    sc = fr_rows(vec["scalars"])
    bits = 64 if vec["name"].endswith("_64") else 255
    if vec["group"] == 1:
        bases = np.array([g1_words(p) for p in vec["bases"]], dtype=np.uint64)
        assert list(ctx.msm_g1(bases, sc, bits)) == g1_words(vec["out"])
    else:
        bases = np.array([g2_words(p) for p in vec["bases"]], dtype=np.uint64)
        assert list(ctx.msm_g2(bases, sc, bits)) == g2_words(vec["out"])


def _g1_bases(oracle, n, seed):
    g = oracle.g1_generator()
    ks = oracle.random_fr(n, seed)
    return np.array([oracle.g1_mul(g, k) for k in oracle.fr_ints(ks)])


def _g2_bases(oracle, n, seed):
    g = oracle.g2_generator()
    ks = oracle.random_fr(n, seed)
    return np.array([oracle.g2_mul(g, k & ((1 << 64) - 1)) for k in oracle.fr_ints(ks)])


@pytest.fixture(scope="module")
def g1_pool(oracle):
    return _g1_bases(oracle, 2048, 11)


@pytest.mark.parametrize("n", [1, 2, 31, 100, 1000, 2048])
@pytest.mark.parametrize("bits", [64, 255])
def test_msm_g1_random_vs_oracle(ctx, oracle, g1_pool, n, bits):
    bases = g1_pool[:n].copy()
    sc = oracle.random_fr(n, 1000 + n)
    if bits == 64:
        sc[:, 1:] = 0
    if n > 4:
        bases[3] = 0
        bases[3, 12] = 1            # infinity base
        sc[4] = 0                    # zero scalar
    assert np.array_equal(ctx.msm_g1(bases, sc, bits), oracle.msm_g1(bases, sc))


def test_msm_g1_degenerate_buckets(ctx, oracle, g1_pool):
    """Equal points in one bucket (doubling branch), P and -P (cancellation),
    and one huge bucket spanning many accumulate threads (all scalars 1)."""
    n = 3000
    bases = np.repeat(g1_pool[:3], n // 3, axis=0)
    sc = np.zeros((n, 4), dtype=np.uint64)
    sc[:, 0] = 1
    assert np.array_equal(ctx.msm_g1(bases, sc, 64), oracle.msm_g1(bases, sc))
    # P, -P with equal scalars -> identity
    p = g1_pool[5].copy()
    q = oracle.g1_mul(p, oracle.lib and (0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001 - 1))
    out = ctx.msm_g1(np.array([p, q]), np.array([[7, 0, 0, 0], [7, 0, 0, 0]], dtype=np.uint64), 64)
    assert out[12] == 1
    # duplicates with mixed scalars
    sc = oracle.random_fr(n, 77)
    sc[:, 1:] = 0
    sc[:, 0] &= 0xFF                 # few distinct digits: long runs per bucket
    assert np.array_equal(ctx.msm_g1(bases, sc, 64), oracle.msm_g1(bases, sc))


def test_msm_empty_and_len_error(ctx, zkp, g1_pool):
    out = ctx.msm_g1(np.zeros((0, 13), dtype=np.uint64), np.zeros((0, 4), dtype=np.uint64))
    assert out[12] == 1
    with pytest.raises(zkp.MSMError):
        ctx.msm_g1(g1_pool[:3], np.zeros((2, 4), dtype=np.uint64))


@pytest.mark.parametrize("n", [1, 7, 200])
@pytest.mark.parametrize("bits", [64, 255])
def test_msm_g2_random_vs_oracle(ctx, oracle, n, bits):
    bases = _g2_bases(oracle, n, 21 + n)
    sc = oracle.random_fr(n, 3000 + n)
    if bits == 64:
        sc[:, 1:] = 0
    if n > 4:
        bases[2] = 0
        bases[2, 24] = 1
    assert np.array_equal(ctx.msm_g2(bases, sc, bits), oracle.msm_g2(bases, sc))


R_MOD = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
LIN_A, LIN_B = 0xDEADBEEF, 0xC0FFEE


@pytest.fixture(scope="module")
def lin_bases(oracle):
    """2^16 bases (a + i b) G, built incrementally."""
    n = 1 << 16
    g = oracle.g1_generator()
    step = oracle.g1_mul(g, LIN_B)
    bases = np.empty((n, 13), dtype=np.uint64)
    bases[0] = oracle.g1_mul(g, LIN_A)
    for i in range(1, n):
        bases[i] = oracle.g1_add(bases[i - 1], step)
    return bases


def _closed_form(oracle, sc):
    s = oracle.fr_ints(sc)
    k = (LIN_A * sum(s) + LIN_B * sum(i * x for i, x in enumerate(s))) % R_MOD
    return oracle.g1_mul(oracle.g1_generator(), k)


def test_msm_g1_linearity_large(ctx, oracle, lin_bases):
    """Size-independent property at 2^16: bases (a + i b) G give
    G * (a sum s_i + b sum i s_i)."""
    sc = oracle.random_fr(len(lin_bases), 0x5EED0001)
    assert np.array_equal(ctx.msm_g1(lin_bases, sc, 255), _closed_form(oracle, sc))


@pytest.mark.parametrize("pattern", ["ones", "bits", "two_bits", "one_value", "sparse_big"])
@pytest.mark.parametrize("bits", [64, 255])
def test_msm_g1_skewed_scalars(ctx, oracle, lin_bases, pattern, bits):
    """Witness-like scalar distributions: most scalars 0/1 put 2^16 entries
    into one bucket, which the segmented merge must finish at log depth."""
    n = len(lin_bases)
    rng = np.random.default_rng(5)
    sc = np.zeros((n, 4), dtype=np.uint64)
    if pattern == "ones":
        sc[:, 0] = 1
    elif pattern == "bits":
        sc[:, 0] = rng.integers(0, 2, n, dtype=np.uint64)
    elif pattern == "two_bits":
        sc[:, 0] = rng.integers(0, 4, n, dtype=np.uint64)
    elif pattern == "one_value":
        sc[:] = oracle.random_fr(1, 9)[0]
        if bits == 64:
            sc[:, 1:] = 0
    else:
        sc[:, 0] = rng.integers(0, 2, n, dtype=np.uint64)
        idx = rng.choice(n, 64, replace=False)
        big = oracle.random_fr(64, 10)
        if bits == 64:
            big[:, 1:] = 0
        sc[idx] = big
    assert np.array_equal(ctx.msm_g1(lin_bases, sc, bits), _closed_form(oracle, sc))


@pytest.mark.parametrize("pattern", ["ones", "two_bits"])
def test_msm_g2_skewed_scalars(ctx, oracle, pattern):
    n = 4096
    bases = np.repeat(_g2_bases(oracle, 16, 99), n // 16, axis=0)
    sc = np.zeros((n, 4), dtype=np.uint64)
    sc[:, 0] = 1 if pattern == "ones" else np.random.default_rng(3).integers(0, 4, n, dtype=np.uint64)
    assert np.array_equal(ctx.msm_g2(bases, sc, 64), oracle.msm_g2(bases, sc))


def _msm_uploaded(zkp, ctx, bases, sc, bits, windows):
    """zk_msm_g1_upload(_windows) + zk_msm_g1_dev with scalars in HBM."""
    import ctypes as C
    import torch
    L = zkp.lib()
    hb = C.c_void_p()
    n = len(bases)
    if windows is None:
        zkp._check(L.zk_msm_g1_upload(C.c_void_p(ctx._h), zkp._p(bases), C.c_size_t(n), C.byref(hb)), ctx)
    else:
        zkp._check(L.zk_msm_g1_upload_windows(C.c_void_p(ctx._h), zkp._p(bases), C.c_size_t(n),
                                              C.c_uint32(windows), C.byref(hb)), ctx)
    d = torch.from_numpy(np.ascontiguousarray(sc, dtype=np.uint64).view(np.int64)).cuda()
    out = np.zeros(13, dtype=np.uint64)
    try:
        zkp._check(L.zk_msm_g1_dev(C.c_void_p(ctx._h), hb, C.c_void_p(d.data_ptr()), C.c_size_t(n),
                                   C.c_uint32(bits), zkp._p(out)), ctx)
    finally:
        L.zk_msm_bases_free(hb)
    return out


@pytest.mark.parametrize("windows", [64, 255, 0])
@pytest.mark.parametrize("bits", [64, 255])
@pytest.mark.parametrize("pattern", ["uniform", "ones", "sparse_big"])
def test_msm_g1_window_upload(ctx, zkp, oracle, lin_bases, windows, bits, pattern):
    """Bases uploaded with their window-shifted copies (one shared bucket set)
    give the same point as the plain upload and the closed form; scalars
    wider than the upload's window bits fall back to per-window buckets."""
    n = 1 << 14
    bases = lin_bases[:n].copy()
    rng = np.random.default_rng(17)
    if pattern == "uniform":
        sc = oracle.random_fr(n, 23)
    else:
        sc = np.zeros((n, 4), dtype=np.uint64)
        sc[:, 0] = 1 if pattern == "ones" else rng.integers(0, 2, n, dtype=np.uint64)
        if pattern == "sparse_big":
            idx = rng.choice(n, 32, replace=False)
            sc[idx] = oracle.random_fr(32, 24)
    if bits == 64:
        sc[:, 1:] = 0
    bases[5] = 0
    bases[5, 12] = 1                       # an infinity base
    want = _closed_form(oracle, np.where(np.arange(n)[:, None] == 5, 0, sc).astype(np.uint64))
    got = _msm_uploaded(zkp, ctx, bases, sc, bits, windows)
    assert np.array_equal(got, want)
    assert np.array_equal(got, _msm_uploaded(zkp, ctx, bases, sc, bits, None))
