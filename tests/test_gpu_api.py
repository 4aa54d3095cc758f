"""The reference's QAP / witness API mirrored on the GPU, the boundary's
input checks, the prove schedules and the synthetic witness generator.

  QAP::evaluate_at / verify_evaluation   crates/groth16-qap/src/lib.rs:190-220, 274-282
  utils::batch_evaluate                  crates/groth16-qap/src/lib.rs:315-322
  Witness::public_inputs / private_inputs crates/groth16-core/src/lib.rs:101-109
"""
import numpy as np
import pytest

import gpu_util as U

pytestmark = pytest.mark.gpu
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _xyz_qap(zkp):
    cs = zkp.R1CS(0)
    x, y, z = (cs.allocate_variable() for _ in range(3))
    cs.enforce_multiplication(zkp.LinearCombination.from_variable(x), zkp.LinearCombination.from_variable(y),
                              zkp.LinearCombination.from_variable(z))
    return zkp.QAP.from_r1cs(cs)


def test_reference_qap_evaluation(ctx, zkp):
    """test_qap_evaluation / test_invalid_assignment (qap:356-383, 423-448):
    [1,3,4,12] satisfies x*y=z at the domain generator, [1,3,4,13] does not."""
    qap = _xyz_qap(zkp)
    w = 1   # omega of the size-1 domain
    ev = qap.evaluate_at(w, [1, 3, 4, 12], ctx)
    assert (ev.a_val, ev.b_val, ev.c_val, ev.z_val) == (3, 4, 12, 0)
    assert qap.verify_evaluation(ev)
    assert not qap.verify_evaluation(qap.evaluate_at(w, [1, 3, 4, 13], ctx))
    with pytest.raises(zkp.DimensionMismatch):
        qap.evaluate_at(w, [1, 3, 4], ctx)


@pytest.mark.parametrize("log_n", [3, 8])
def test_evaluate_at_vs_oracle(ctx, zkp, oracle, log_n):
    """A(t) = sum_i z_i A_i(t) against the oracle's per-variable A_i(t), at a
    random point and at domain points; Z(t) = t^n - 1."""
    n = 1 << log_n
    nc = n - 3                                # the last domain rows are padding
    z = oracle.synthetic_witness(n, 0x55 + log_n)
    rp = np.arange(nc + 1, dtype=np.uint64)
    j = np.arange(nc, dtype=np.uint32)
    qap = zkp.QAP(zkp.CSRMatrices(nc, 3 * n + 1, [(rp, 1 + 3 * j, None), (rp, 2 + 3 * j, None), (rp, 3 + 3 * j, None)]))
    csr_o = oracle.CSR(nc, 3 * n + 1, [(rp, (1 + 3 * j).astype(np.uint32), None), (rp, (2 + 3 * j).astype(np.uint32), None),
                                       (rp, (3 + 3 * j).astype(np.uint32), None)])
    zi = oracle.fr_ints(z)
    w = oracle.fr_root_of_unity(log_n)
    for t in (0x1234567890ABCDEF, w, pow(w, 5, R), 0):
        V = 3 * n + 1
        av, bv, cv = (np.zeros((V, 4), dtype=np.uint64) for _ in range(3))
        import ctypes as C
        oracle.lib().or_qap_eval_at(C.byref(csr_o.s), oracle._p(np.array(oracle.int_to_limbs(t, 4), dtype=np.uint64)),
                                    oracle._p(av), oracle._p(bv), oracle._p(cv))
        want = [sum(a * b for a, b in zip(zi, oracle.fr_ints(m))) % R for m in (av, bv, cv)]
        ev = qap.evaluate_at(t, z, ctx)
        assert [ev.a_val, ev.b_val, ev.c_val] == want
        assert ev.z_val == (pow(t, n, R) - 1) % R
    # Witness::validate semantics: satisfied at a domain point of a real row
    assert qap.verify_evaluation(qap.evaluate_at(w, z, ctx))


def test_batch_evaluate(ctx, zkp, oracle):
    rng = np.random.default_rng(3)
    polys = [oracle.fr_ints(oracle.random_fr(int(k), 40 + i)) for i, k in enumerate([0, 1, 5, 64, 65, 1000, 4097])]
    t = 0xDEADBEEF12345
    want = [sum(c * pow(t, e, R) for e, c in enumerate(p)) % R for p in polys]
    assert zkp.batch_evaluate(polys, t, ctx) == want
    assert zkp.batch_evaluate([], t, ctx) == []
    del rng


def test_witness_inputs(zkp):
    w = zkp.Witness([1, 7, 8, 9, 10], 2)
    assert [int(x[0]) for x in w.public_inputs()] == [7, 8]
    assert [int(x[0]) for x in w.private_inputs()] == [9, 10]
    bad = np.zeros((4, 4), dtype=np.uint64)
    bad[0, 0] = 1
    bad[2] = [(R >> (64 * i)) & (2 ** 64 - 1) for i in range(4)]     # == r
    with pytest.raises(ValueError):
        zkp.Witness(bad, 1)


def test_synthetic_witness_generator(ctx, zkp, oracle):
    """zk_synthetic_witness_dev: z = [1, x, y, x y mod r, ...], canonical,
    deterministic in the seed, and a valid witness of the synthetic circuit."""
    n = 1 << 12
    z = ctx.synthetic_witness(n, 77).cpu().numpy().view(np.uint64)
    assert np.array_equal(z, ctx.synthetic_witness(n, 77).cpu().numpy().view(np.uint64))
    assert not np.array_equal(z, ctx.synthetic_witness(n, 78).cpu().numpy().view(np.uint64))
    zi = oracle.fr_ints(z)
    assert zi[0] == 1 and all(v < R for v in zi)
    for j in list(range(0, n, 97)) + [n - 1]:
        assert zi[3 + 3 * j] == zi[1 + 3 * j] * zi[2 + 3 * j] % R
    assert oracle.quotient(oracle.CSR.synthetic(n), z)[0] == oracle.OR_OK


def _rows_r():
    return [(R >> (64 * i)) & (2 ** 64 - 1) for i in range(4)]


def test_prove_rejects_non_canonical(ctx, zkp, oracle):
    """z_i >= r, r >= r or s >= r: ZK_ERR_ARG (ValueError), on the host- and
    device-witness paths -- never a silently different proof."""
    import torch
    n = 1 << 8
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    rng = __import__("pyref").SplitMix64(99)
    params = [rng.fr() for _ in range(5)]
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    z = oracle.synthetic_witness(n, 5)
    good = zkp.Prover.prove(dpk, zkp.Witness(z, 1), r=3, s=4)
    zb = z.copy()
    zb[7] = _rows_r()
    zb[7, 0] += 5                         # r + 5: same lo64 residue class, not canonical
    dz = torch.from_numpy(zb.view(np.int64).copy()).cuda()
    with pytest.raises(ValueError):
        zkp.Prover.prove_device(dpk, dz.data_ptr(), len(zb), 1, 3, 4)
    import ctypes as C
    out = zkp._Proof()
    r_ok, s_ok = zkp._fr(3), zkp._fr(4)
    # the host-witness path checks each uploaded part: a bad entry in the
    # first half (7) and in the second (3n)
    for bad in (7, 3 * n):
        zh = z.copy()
        zh[bad] = _rows_r()
        zh[bad, 0] += 5
        rc = zkp.lib().zk_groth16_prove(C.c_void_p(ctx._h), C.c_void_p(dpk._h), zkp._p(zh), C.c_size_t(len(zh)),
                                        C.c_size_t(1), C.byref(r_ok), C.byref(s_ok), C.byref(out))
        assert rc == zkp.ZK_ERR_ARG, bad
    for rr, ss in ((R, 4), (3, R + 1)):
        r_fr, s_fr = zkp._Fr(), zkp._Fr()
        for i, x in enumerate(zkp.to_limbs(rr)):
            r_fr.l[i] = x
        for i, x in enumerate(zkp.to_limbs(ss)):
            s_fr.l[i] = x
        rc = zkp.lib().zk_groth16_prove(C.c_void_p(ctx._h), C.c_void_p(dpk._h), zkp._p(z), C.c_size_t(len(z)),
                                        C.c_size_t(1), C.byref(r_fr), C.byref(s_fr), C.byref(out))
        assert rc == zkp.ZK_ERR_ARG
    # still proves the good witness afterwards
    assert zkp.Prover.prove(dpk, zkp.Witness(z, 1), r=3, s=4) == good
    dpk.free()


def test_msm_rejects_bad_scalars(ctx, zkp, oracle):
    g = oracle.g1_generator()
    bases = np.array([g, oracle.g1_mul(g, 5)])
    sc = np.zeros((2, 4), dtype=np.uint64)
    sc[0] = _rows_r()                                        # == r
    with pytest.raises(ValueError):
        ctx.msm_g1(bases, sc, 255)
    sc[0] = [0, 1, 0, 0]                                     # 2^64 with scalar_bits = 64
    with pytest.raises(ValueError):
        ctx.msm_g1(bases, sc, 64)
    assert ctx.msm_g1(bases, sc, 255)[12] == 0               # fine at 255 bits
    # device scalars (zk_msm_g1_dev) through the device flag
    import ctypes as C
    import torch
    L = zkp.lib()
    hb = C.c_void_p()
    zkp._check(L.zk_msm_g1_upload(C.c_void_p(ctx._h), zkp._p(bases), C.c_size_t(2), C.byref(hb)), ctx)
    try:
        out = np.zeros(13, dtype=np.uint64)
        for bad, bits in ((_rows_r(), 255), ([0, 1, 0, 0], 64)):
            s2 = np.zeros((2, 4), dtype=np.uint64)
            s2[1] = bad
            d = torch.from_numpy(s2.view(np.int64)).cuda()
            rc = L.zk_msm_g1_dev(C.c_void_p(ctx._h), hb, C.c_void_p(d.data_ptr()), C.c_size_t(2), C.c_uint32(bits),
                                 zkp._p(out))
            assert rc == zkp.ZK_ERR_ARG
        s2 = np.zeros((2, 4), dtype=np.uint64)
        s2[1, 0] = 3
        d = torch.from_numpy(s2.view(np.int64)).cuda()
        zkp._check(L.zk_msm_g1_dev(C.c_void_p(ctx._h), hb, C.c_void_p(d.data_ptr()), C.c_size_t(2), C.c_uint32(64),
                                   zkp._p(out)), ctx)
        assert np.array_equal(out, oracle.g1_mul(g, 15))
    finally:
        L.zk_msm_bases_free(hb)


@pytest.mark.parametrize("log_n", [10, 13])
def test_schedules_give_the_same_proof(ctx, zkp, oracle, log_n):
    """zk_ctx_set_schedule (overlapped, serial) changes only the stream
    order: the oracle's proof every time."""
    import torch
    n = 1 << log_n
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    rng = __import__("pyref").SplitMix64(log_n)
    params = [rng.fr() for _ in range(5)]
    r, s = rng.fr(), rng.fr()
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)
    z = ctx.synthetic_witness(n, 9)
    zh = z.cpu().numpy().view(np.uint64)
    rc, oproof = oracle.prove(U.oracle_pk_from(oracle, crs.pk), oracle.CSR.synthetic(n), zh, 1, r, s)
    assert rc == 0
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    try:
        for sched in (0, 3, -1):
            ctx.set_schedule(sched)
            p = zkp.Prover.prove_device(dpk, z.data_ptr(), len(zh), 1, r, s)
            torch.cuda.synchronize()
            assert np.array_equal(p.words, oproof), sched
            # the host-witness prove: z uploaded in two parts, the first
            # part's MSMs overlapping the second part's copy
            ph = zkp.Prover.prove(dpk, zkp.Witness(zh, 1), r=r, s=s)
            assert np.array_equal(ph.words, oproof), ("host", sched)
    finally:
        ctx.set_schedule(-1)
        dpk.free()
