"""CPU tests of the oracle (oracle/zk_oracle.c via oracle/binding.py) against
the reference's own KATs, mathematical KATs and the golden fixtures made by
the independent pure-Python restatement (tests/golden/gen_golden.py).
Parity status: partially pinned -- see oracle/zk_oracle.h."""
import numpy as np
import pytest

from helpers import constraints_of, fr_rows, g1_words, g2_words, golden, proof_words

G = golden()
R = int(G["consts"]["r"], 16)


def test_constants(oracle, pyref):
    assert oracle.fr_root_of_unity(32) == int(G["consts"]["root_of_unity_2_32"], 16)
    assert oracle.fr_root_of_unity(32) == 0x16A2A19EDFE81F20D09B681922C813B4B63683508C2280B93829971F439F0D2B
    w = oracle.fr_root_of_unity(32)
    assert pow(w, 1 << 32, R) == 1 and pow(w, 1 << 31, R) != 1
    # omega_2^20 as tabulated in SURVEY.md 8(a)-a5
    assert oracle.fr_root_of_unity(20) == 0x03E1C54BCB947035A57A6E07CB98DE4A2F69E02D265E09D9FECE7E0E39898D4B
    # ... and at the other config sizes (2^21 the reference FFT at configs[3], 2^22 configs[2], 2^24 configs[4])
    assert oracle.fr_root_of_unity(21) == 0x47C8B5817018AF4FC70D0874B0691D4E46B3105F04DB5844CD3979122D3EA03A
    assert oracle.fr_root_of_unity(22) == 0x0ABE6A5E5ABCAA32F2D38F10FBB8D1BBE08FEC7C86389BEEC6E7A6FFB08E3363
    assert oracle.fr_root_of_unity(24) == 0x291CF6D68823E6876E0BCD91EE76273072CF6A8029B7D7BC92CF4DEB77BD779C
    g1, g2 = oracle.g1_generator(), oracle.g2_generator()
    assert oracle.g1_on_curve(g1) and oracle.g2_on_curve(g2)
    assert oracle.g1_mul(g1, R)[12] == 1 and oracle.g2_mul(g2, R)[24] == 1     # r * G = O
    # zcash / ark-bls12-381 compressed generator encoding
    assert oracle.g1_compress(g1).hex() == G["consts"]["g1_generator_compressed"]
    assert oracle.g1_compress(g1).hex().startswith("97f1d3a73197d7942695638c4fa9ac0f")
    assert oracle.g2_compress(g2).hex() == G["consts"]["g2_generator_compressed"]


def test_reference_field_kats(oracle):
    """crates/groth16-field/src/lib.rs:180-234"""
    L = oracle.lib()
    import ctypes as C
    a = np.array([5, 0, 0, 0], dtype=np.uint64)
    b = np.array([3, 0, 0, 0], dtype=np.uint64)
    out = np.zeros(4, dtype=np.uint64)
    p = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    L.or_fr_add(p(out), p(a), p(b)); assert out[0] == 8
    L.or_fr_mul(p(out), p(a), p(b)); assert out[0] == 15
    L.or_fr_sub(p(out), p(a), p(b)); assert out[0] == 2
    inv = np.zeros(4, dtype=np.uint64)
    L.or_fr_inv(p(inv), p(a)); L.or_fr_mul(p(out), p(a), p(inv))
    assert list(out) == [1, 0, 0, 0]


def test_qap_kats(oracle):
    """crates/groth16-qap/src/lib.rs:334-448: x*y=z, [1,3,4,12] ok, [1,3,4,13] rejected."""
    csr = oracle.CSR.from_constraints([({1: 1}, {2: 1}, {3: 1})], 4)
    assert oracle.domain_size(1) == 1 and csr.num_variables == 4
    ok = oracle.fr_array([1, 3, 4, 12])
    bad = oracle.fr_array([1, 3, 4, 13])
    assert oracle.validate(csr, ok) == oracle.OR_OK
    assert oracle.quotient(csr, ok)[0] == oracle.OR_OK
    assert oracle.quotient(csr, bad)[0] == oracle.OR_ERR_QAP_DIVISION
    assert oracle.validate(csr, bad) == oracle.OR_ERR_INVALID_WITNESS


@pytest.mark.parametrize("case", G["prove"], ids=lambda c: c["name"])
def test_oracle_vs_golden_prove(oracle, case):
    V = case["num_variables"]
    csr = oracle.CSR.from_constraints(constraints_of(case), V)
    params = [int(x, 16) for x in case["params"]]
    rc, pk, vk = oracle.setup(csr, params, case["num_public"])
    assert rc == oracle.OR_OK
    gp = case["pk"]
    for name in ("a_g1", "b_g1", "ic_g1", "h_g1"):
        want = np.array([g1_words(p) for p in gp[name]], dtype=np.uint64).reshape(-1, 13)
        got = getattr(pk, name)[:len(want)]
        assert np.array_equal(got, want), name
    assert np.array_equal(pk.b_g2, np.array([g2_words(p) for p in gp["b_g2"]], dtype=np.uint64))
    for name in ("alpha_g1", "beta_g1", "delta_g1"):
        assert list(pk.field(name)) == g1_words(gp[name])
    for name in ("beta_g2", "delta_g2"):
        assert list(pk.field(name)) == g2_words(gp[name])
    assert list(vk.field("gamma_g2")) == g2_words(case["vk"]["gamma_g2"])
    assert np.array_equal(vk.ic_g1, np.array([g1_words(p) for p in case["vk"]["ic_g1"]], dtype=np.uint64))
    z = fr_rows(case["z"])
    rc, proof = oracle.prove(pk, csr, z, case["num_public"], int(case["r"], 16), int(case["s"], 16))
    if case["error"] is None:
        assert rc == oracle.OR_OK
        assert list(proof) == proof_words(case)
        assert oracle.proof_compress(proof).hex() == case["proof_compressed"]
    else:
        assert rc in (oracle.OR_ERR_INVALID_WITNESS, oracle.OR_ERR_QAP_DIVISION)
        want = oracle.OR_ERR_QAP_DIVISION if "QAP" in case["error"] else oracle.OR_ERR_INVALID_WITNESS
        assert rc == want


@pytest.mark.parametrize("case", G["prove"], ids=lambda c: c["name"])
def test_oracle_quotient_vs_golden(oracle, case):
    V = case["num_variables"]
    csr = oracle.CSR.from_constraints(constraints_of(case), V)
    z = fr_rows(case["z"])
    rc, h = oracle.quotient(csr, z)
    rcd, hd = oracle.quotient(csr, z, dense=True)
    assert rc == rcd
    if case["h"] is None:
        assert rc == oracle.OR_ERR_QAP_DIVISION
        return
    assert rc == oracle.OR_OK and np.array_equal(h, hd)
    want = [int(x, 16) for x in case["h"]]
    got = oracle.fr_ints(h)
    assert got[:len(want)] == want and not any(got[len(want):])


@pytest.mark.parametrize("vec", G["msm"], ids=lambda v: v["name"])
def test_oracle_msm_golden(oracle, vec):
    sc = fr_rows(vec["scalars"])
    if vec["group"] == 1:
        bases = np.array([g1_words(p) for p in vec["bases"]], dtype=np.uint64)
        assert list(oracle.msm_g1(bases, sc)) == g1_words(vec["out"])
    else:
        bases = np.array([g2_words(p) for p in vec["bases"]], dtype=np.uint64)
        assert list(oracle.msm_g2(bases, sc)) == g2_words(vec["out"])


@pytest.mark.parametrize("vec", G["ntt"], ids=lambda v: "n%d" % v["n"])
def test_oracle_ntt_golden(oracle, vec):
    x = fr_rows(vec["in"])
    assert oracle.fr_ints(oracle.fft(x)) == [int(a, 16) for a in vec["fft"]]
    assert oracle.fr_ints(oracle.fft(x, inverse=True)) == [int(a, 16) for a in vec["ifft"]]


@pytest.mark.parametrize("log_n", [5, 7, 10])
def test_oracle_sparse_vs_dense_quotient(oracle, log_n):
    """The O(n log n) quotient restatement equals the literal dense reference
    algorithm (qap:95-187 + qap:225-271) on the synthetic circuit."""
    n = 1 << log_n
    csr = oracle.CSR.synthetic(n)
    z = oracle.synthetic_witness(n, 5 + log_n)
    rc, h = oracle.quotient(csr, z)
    rcd, hd = oracle.quotient(csr, z, dense=True)
    assert rc == rcd == oracle.OR_OK and np.array_equal(h, hd)


def test_oracle_msm_linearity(oracle):
    """MSM with bases (a + i b) G equals G * (a sum s_i + b sum i s_i)."""
    n, a, b = 300, 0x1234567, 0x89ABCDEF
    g = oracle.g1_generator()
    sc = oracle.random_fr(n, 0x5EED0001)
    step = oracle.g1_mul(g, b)
    bases = [oracle.g1_mul(g, a)]
    for _ in range(n - 1):
        bases.append(oracle.g1_add(bases[-1], step))
    s = oracle.fr_ints(sc)
    k = (a * sum(s) + b * sum(i * x for i, x in enumerate(s))) % R
    assert np.array_equal(oracle.msm_g1(np.array(bases), sc), oracle.g1_mul(g, k))


def test_oracle_threads_do_not_change_results(oracle, pyref):
    """The chunked multi-thread oracle (MSM chunks, FFT butterflies, parallel
    point loads) gives the single-thread restatement's outputs bit for bit:
    MSM over G1 and G2, the FFT, the 2^13 prove, and the chunked (a + i b) G1
    bases against the incremental chain."""
    saved = oracle.get_threads()
    try:
        n = 1 << 13
        csr = oracle.CSR.synthetic(n)
        rng = pyref.SplitMix64(0x7E)
        params = [rng.fr() for _ in range(5)]
        r, s = rng.fr(), rng.fr()
        rc, pk, _ = oracle.setup(csr, params, 1, nthreads=8)
        z = oracle.synthetic_witness(n, 0x7F)
        bases = oracle.g1_lin_bases(0xABC, 0xDEF, 1 << 14)
        sc = oracle.random_fr(1 << 14, 0x80)
        x = oracle.random_fr(1 << 14, 0x81)
        out = {}
        for t in (1, 8):
            oracle.set_threads(t)
            out[t] = (oracle.prove(pk, csr, z, 1, r, s), oracle.msm_g1(bases, sc),
                      oracle.msm_g2(pk.b_g2[:9000], sc[:9000]), oracle.fft(x), oracle.g1_lin_bases(0xABC, 0xDEF, 1 << 14))
        assert out[1][0][0] == out[8][0][0] == oracle.OR_OK
        assert np.array_equal(out[1][0][1], out[8][0][1])
        for k in range(1, 5):
            assert np.array_equal(out[1][k], out[8][k])
        g = oracle.g1_generator()
        step, p = oracle.g1_mul(g, 0xDEF), oracle.g1_mul(g, 0xABC)
        for i in range(1, 6000):
            p = oracle.g1_add(p, step)
            if i in (1, 4095, 4096, 5999):
                assert np.array_equal(bases[i], p)
    finally:
        oracle.set_threads(saved)


def test_setup_sample_equals_full_setup(oracle):
    """or_setup_sample (sampled key entries, used to check the sharded 2^24
    GPU setup) gives exactly or_setup's entries."""
    import numpy as np
    import pyref
    n = 1 << 8
    csr = oracle.CSR.synthetic(n)
    rng = pyref.SplitMix64(99)
    params = [rng.fr() for _ in range(5)]
    rc, pk, vk = oracle.setup(csr, params, 1, nthreads=4)
    assert rc == 0
    vars_ = np.array([0, 1, 2, 3, 5, 100, 3 * n], dtype=np.uint64)
    hidx = np.array([0, 1, 7, n - 1], dtype=np.uint64)
    rc, smp = oracle.setup_sample(csr, params, 1, vars_, hidx)
    assert rc == 0
    assert np.array_equal(smp["a_g1"], pk.a_g1[vars_])
    assert np.array_equal(smp["b_g1"], pk.b_g1[vars_])
    assert np.array_equal(smp["b_g2"], pk.b_g2[vars_])
    assert np.array_equal(smp["h_g1"], pk.h_g1[hidx])
    for k, v in enumerate(vars_):
        want = pk.ic_g1[v - 2] if v > 1 else vk.ic_g1[v]
        assert np.array_equal(smp["ic"][k], want), v
