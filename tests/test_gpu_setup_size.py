"""GPU setup (CRS::generate_from_qap, crates/groth16-setup/src/lib.rs:141-268)
against the oracle's own or_setup at the configs' sizes -- not only the GPU
key fed to both provers:

  * the host-returned key (zk_groth16_setup) equals or_setup's entry for
    entry at 2^16 and 2^20 constraints (every base vector, the five points,
    the vk);
  * a 2^20 proof from the ORACLE's key (uploaded with zk_pk_upload) equals
    the oracle's proof from the same key;
  * the device-resident keys the bench and the sharded prover use
    (zk_groth16_setup_dev[_shard], read back through the test library's
    zk_test_pk_bases) hold exactly or_setup's non-identity bases, each once
    across 1 or 4 shards, the extras (alpha_1, 2^(64k) delta, beta), and
    window copies equal to 2^(c w) times the base.

The 2^24 sharded setup is checked by sampled indices in test_gpu_2p24.py."""
import numpy as np
import pytest

import gpu_util as U

pytestmark = pytest.mark.gpu

SLOTS = ((0, "a_g1"), (1, "b_g2"), (2, "b_g1"), (3, "ic_g1"), (4, "h_g1"))


def _case(zkp, oracle, log_n, seed):
    import pyref
    n = 1 << log_n
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    csr_o = oracle.CSR.synthetic(n)
    rng = pyref.SplitMix64(seed)
    params = [rng.fr() for _ in range(5)]
    r, s = rng.fr(), rng.fr()
    return qap, csr_o, params, r, s


@pytest.fixture(scope="module")
def key_2p20(zkp, oracle):
    qap, csr_o, params, r, s = _case(zkp, oracle, 20, 0x5E70)
    rc, opk, ovk = oracle.setup(csr_o, params, 1, nthreads=oracle.default_threads())
    assert rc == 0
    return qap, csr_o, params, r, s, opk, ovk


def _compare_host(zkp, ctx, qap, params, opk, ovk):
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)
    for nm in ("a_g1", "b_g1", "b_g2", "h_g1"):
        assert np.array_equal(getattr(crs.pk, nm), getattr(opk, nm)), nm
    assert np.array_equal(crs.pk.ic_g1, opk.ic_g1[:len(crs.pk.ic_g1)])
    for nm in ("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"):
        assert np.array_equal(crs.pk.point(nm), opk.field(nm)), nm
    assert np.array_equal(crs.vk.ic_g1, ovk.ic_g1)
    for nm in ("alpha_g1", "beta_g2", "gamma_g2", "delta_g2"):
        assert np.array_equal(crs.vk.point(nm), ovk.field(nm)), nm


@pytest.mark.timeout(600)
def test_host_setup_equals_oracle_setup_2p16(ctx, zkp, oracle):
    qap, csr_o, params, r, s = _case(zkp, oracle, 16, 0x5E16)
    rc, opk, ovk = oracle.setup(csr_o, params, 1, nthreads=oracle.default_threads())
    assert rc == 0
    _compare_host(zkp, ctx, qap, params, opk, ovk)


@pytest.mark.timeout(600)
def test_host_setup_equals_oracle_setup_2p20(ctx, zkp, key_2p20):
    qap, _, params, _, _, opk, ovk = key_2p20
    _compare_host(zkp, ctx, qap, params, opk, ovk)


@pytest.mark.timeout(600)
def test_prove_on_oracle_key_2p20(ctx, zkp, oracle, key_2p20):
    """GPU prove from the oracle's key (not a GPU-made one) = oracle prove."""
    qap, csr_o, params, r, s, opk, _ = key_2p20
    z = oracle.synthetic_witness(1 << 20, 0x5E71)
    rc, oproof = oracle.prove(opk, csr_o, z, 1, r, s)
    assert rc == 0
    dpk = U.pk_from_oracle(zkp, opk, qap, 1).upload(ctx)
    try:
        proof = zkp.Prover.prove(dpk, zkp.Witness(z, 1), r=r, s=s)
    finally:
        dpk.free()
    assert np.array_equal(proof.words, oproof)


def _ref_rows(opk, slot, idx):
    if slot == 3:
        return opk.ic_g1[idx.astype(np.int64) - 2]   # ic_g1[k] <-> variable k + num_public + 1
    return getattr(opk, dict(SLOTS)[slot])[idx]


def _is_identity(words):
    return words[:, -1] == 1


def check_extras(oracle, opk, slot, words, count, nex):
    """shard 0's extras: alpha_1 + 2^(64k) delta_1 (pi_A), beta_2 + 2^(64k)
    delta_2 (pi_B), beta_1 (B_1)."""
    ex = words[count:count + nex]
    if slot == 0:
        want = [opk.field("alpha_g1")] + [oracle.g1_mul(opk.field("delta_g1"), 1 << (64 * k)) for k in range(4)]
    elif slot == 1:
        want = [opk.field("beta_g2")] + [oracle.g2_mul(opk.field("delta_g2"), 1 << (64 * k)) for k in range(4)]
    elif slot == 2:
        want = [opk.field("beta_g1")]
    else:
        want = []
    assert len(ex) == len(want), (slot, len(ex))
    for a, b in zip(ex, want):
        assert np.array_equal(a, b), slot


def check_windows(oracle, dpk, slot, base_words, rng, samples=6):
    """window copy w of base k = 2^(c w) * base k."""
    win, win_c, _, _ = dpk.test_info()
    mul = oracle.g2_mul if slot == 1 else oracle.g1_mul
    for w in range(1, win):
        _, ww, _ = dpk.test_bases(slot, w)
        for k in rng.choice(len(base_words), size=min(samples, len(base_words)), replace=False):
            assert np.array_equal(ww[k], mul(base_words[k], 1 << (win_c * w))), (slot, w, k)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("nshards", [1, 4])
def test_device_key_equals_oracle_setup_2p20(ctx, zkp, oracle, key_2p20, nshards):
    qap, _, params, _, _, opk, _ = key_2p20
    n = 1 << 20
    rng = np.random.default_rng(nshards)
    seen = {slot: [] for slot, _ in SLOTS}
    for shard in range(nshards):
        dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1, shard=shard, nshards=nshards)
        try:
            assert dpk.test_info()[2:] == (shard, nshards)
            for slot, _ in SLOTS:
                idx, words, nex = dpk.test_bases(slot)
                assert np.array_equal(words[:len(idx)], _ref_rows(opk, slot, idx)), (slot, shard)
                if slot == 4:
                    assert (idx % nshards == shard).all()   # H bases i = shard mod N
                assert nex == (0 if shard or slot in (3, 4) else (5 if slot in (0, 1) else 1))
                if nex:
                    check_extras(oracle, opk, slot, words, len(idx), nex)
                if shard == 0:
                    check_windows(oracle, dpk, slot, words[:len(idx)], rng)
                seen[slot].append(idx)
        finally:
            dpk.free()
    # every non-identity base of the oracle's key is held by exactly one shard
    for slot, nm in SLOTS:
        allidx = np.sort(np.concatenate(seen[slot]).astype(np.int64))
        ref = getattr(opk, nm)[:n if slot == 4 else len(getattr(opk, nm))]
        if slot == 3:
            ref = opk.ic_g1[:3 * n - 1]
            want = np.nonzero(~_is_identity(ref))[0] + 2
        else:
            want = np.nonzero(~_is_identity(ref))[0]
        assert np.array_equal(allidx, want), nm
