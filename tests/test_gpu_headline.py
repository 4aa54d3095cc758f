"""Bit-exact parity at the headline sizes of BASELINE.json:

  configs[1]  G1 MSM, 2^20 bases, full-width scalars -- against the closed
              form  sum_i s_i (a + i b) G1 = (a sum s_i + b sum i s_i) G1
              (SURVEY 8(c)3 / 8(d)), plain and window-shifted uploads;
  configs[3]  Groth16 prove, 2^20-constraint synthetic circuit
              (crates/groth16-cli/src/lib.rs:57-70) -- GPU setup -> GPU prove
              against the C oracle's prove() on the same pk / z / r / s
              (crates/groth16-core/src/lib.rs:139-300);
  2^22        the same prove at 4x the size (the MSM plan -- window, chunk
              count, merge depth, batch keys -- changes with n).

The oracle runs on every host core here (oracle/binding.py default_threads):
its chunked Pippenger gives the same group elements as the single-thread
restatement (tests/test_oracle.py::test_oracle_threads_do_not_change_results).
"""
import ctypes as C

import numpy as np
import pytest

import gpu_util as U

pytestmark = pytest.mark.gpu

R_MOD = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
LIN_A, LIN_B = 0x1234567890ABCDEF1122334455667788, 0x0F1E2D3C4B5A6978
N20 = 1 << 20


@pytest.fixture(scope="module")
def lin_bases_2p20(oracle):
    return oracle.g1_lin_bases(LIN_A, LIN_B, N20)


def _closed_form(oracle, sc):
    s = oracle.fr_ints(sc)
    k = (LIN_A * sum(s) + LIN_B * sum(i * x for i, x in enumerate(s))) % R_MOD
    return oracle.g1_mul(oracle.g1_generator(), k)


def _msm_uploaded(zkp, ctx, bases, sc, bits, windows):
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


@pytest.mark.parametrize("bits", [255, 64])
def test_msm_g1_2p20_closed_form(ctx, zkp, oracle, lin_bases_2p20, bits):
    """configs[1] at its size: seed 0x5eed0001 uniform scalars,
    through the host entry point (zk_msm_g1), a plain device upload and the
    window-shifted upload the bench uses."""
    sc = oracle.random_fr(N20, 0x5EED0001)
    if bits == 64:
        sc[:, 1:] = 0
    want = _closed_form(oracle, sc)
    assert np.array_equal(ctx.msm_g1(lin_bases_2p20, sc, bits), want)
    assert np.array_equal(_msm_uploaded(zkp, ctx, lin_bases_2p20, sc, bits, None), want)
    assert np.array_equal(_msm_uploaded(zkp, ctx, lin_bases_2p20, sc, bits, bits), want)


def _prove_vs_oracle(ctx, zkp, oracle, log_n, seed):
    import torch
    n = 1 << log_n
    rng = __import__("pyref").SplitMix64(seed)
    params = [rng.fr() for _ in range(5)]
    r, s = rng.fr(), rng.fr()
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)   # GPU setup, host key
    z = oracle.synthetic_witness(n, seed + 1)
    opk = U.oracle_pk_from(oracle, crs.pk)
    rc, oproof = oracle.prove(opk, oracle.CSR.synthetic(n), z, 1, r, s)
    assert rc == 0
    del opk
    # host key uploaded, host witness (the drop-in zk_groth16_prove path)
    dpk = crs.pk.upload(ctx)
    proof = zkp.Prover.prove(dpk, zkp.Witness(z, 1), r=r, s=s)
    dpk.free()
    assert np.array_equal(proof.words, oproof)
    del crs
    # setup straight into HBM + witness in HBM (the bench's timed path)
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    dz = torch.from_numpy(z.view(np.int64).copy()).cuda()
    proof2 = zkp.Prover.prove_device(dpk, dz.data_ptr(), len(z), 1, r, s)
    dpk.free()
    assert np.array_equal(proof2.words, oproof)


@pytest.mark.timeout(300)
def test_prove_2p20_vs_oracle(ctx, zkp, oracle):
    """configs[3]: the full 2^20-constraint prove, bit-exact vs the oracle."""
    _prove_vs_oracle(ctx, zkp, oracle, 20, 0x20)


@pytest.mark.timeout(600)
def test_prove_2p22_vs_oracle(ctx, zkp, oracle):
    """The same at 2^22 (the MSM plan at 4x the points)."""
    _prove_vs_oracle(ctx, zkp, oracle, 22, 0x22)
