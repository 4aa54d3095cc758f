"""The MSM bucket grouping (csrc/group.hip: stable LSD counting sort, no
vendor sort): deterministic bytes, and exact proofs / MSMs under the skewed
digit distributions that make one bucket hold most entries.

The reference's MSM is ark's VariableBaseMSM (crates/groth16-core/src/lib.rs:
275-300); its result is a unique group element, so the checks are against the
oracle's group elements.  What the grouping adds is reproducibility: the
XYZZ partials zk_groth16_prove_partial returns are projective (not unique),
so they are only reproducible if the order inside every bucket is."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _circuit(zkp, oracle, log_n, seed):
    n = 1 << log_n
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    csr_o = oracle.CSR.synthetic(n)
    rng = __import__("pyref").SplitMix64(seed)
    params = [rng.fr() for _ in range(5)]
    r, s = rng.fr(), rng.fr()
    return n, qap, csr_o, params, r, s


def _skewed_witness(n, kind, seed):
    """x_i, y_i drawn from a tiny set, z_i = x_i y_i (the synthetic circuit's
    rows hold for any x, y): most digits of the lo64 scalars then fall in a
    handful of buckets."""
    rng = np.random.default_rng(seed)
    if kind == "bits":
        x, y = rng.integers(0, 2, n), rng.integers(0, 2, n)
    elif kind == "small":
        x, y = rng.integers(0, 4, n), rng.integers(0, 4, n)
    else:   # "ones": every x, y, z equal to 1
        x, y = np.ones(n, dtype=np.int64), np.ones(n, dtype=np.int64)
    z = np.zeros((3 * n + 1, 4), dtype=np.uint64)
    z[0, 0] = 1
    z[1::3, 0] = x.astype(np.uint64)
    z[2::3, 0] = y.astype(np.uint64)
    z[3::3, 0] = (x * y).astype(np.uint64)
    return z


@pytest.mark.parametrize("kind", ["bits", "small", "ones"])
def test_skewed_witness_prove_vs_oracle(ctx, zkp, oracle, kind):
    n, qap, csr_o, params, r, s = _circuit(zkp, oracle, 12, 4242)
    z = _skewed_witness(n, kind, 7)
    rc, opk, _ = oracle.setup(csr_o, params, 1, nthreads=8)
    assert rc == 0
    rc, oproof = oracle.prove(opk, csr_o, z, 1, r, s)
    assert rc == 0
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    proof = zkp.Prover.prove(dpk, zkp.Witness(z, 1), r=r, s=s)
    dpk.free()
    assert np.array_equal(proof.words, oproof)


@pytest.mark.parametrize("schedule", [0, 3])
def test_prove_partial_bytes_reproducible(ctx, zkp, oracle, schedule):
    """Two consecutive zk_groth16_prove_partial calls on the same key and
    witness return the same bytes (the XYZZ partials, not just the same
    points), with random and with skewed scalars."""
    import torch
    n, qap, csr_o, params, r, s = _circuit(zkp, oracle, 12, 99)
    for z in (oracle.synthetic_witness(n, 100), _skewed_witness(n, "bits", 3)):
        dz = torch.from_numpy(z.view(np.int64).copy()).cuda()
        parts = []
        ctx.set_schedule(schedule)
        try:
            for k in range(2):
                dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1, shard=k, nshards=2)
                a = zkp.Prover.prove_partial(dpk, dz.data_ptr(), len(z), 1, r, s)
                b = zkp.Prover.prove_partial(dpk, dz.data_ptr(), len(z), 1, r, s)
                dpk.free()
                assert a == b, f"shard {k}: partial bytes differ between two runs"
                parts.append(a)
        finally:
            ctx.set_schedule(0)
        rc, opk, _ = oracle.setup(csr_o, params, 1, nthreads=8)
        rc, oproof = oracle.prove(opk, csr_o, z, 1, r, s)
        assert np.array_equal(zkp.Prover.combine(parts, r, s).words, oproof)


@pytest.mark.parametrize("bits", [64, 255])
def test_msm_repeat_identical_and_vs_oracle(ctx, oracle, bits):
    """zk_msm_g1 (per-window bucket plan: the grouping's four-word scalar path
    at 255 bits, one-word at 64) twice on the same 8192 pairs: equal to the
    oracle's Pippenger and to itself."""
    n = 8192
    g = oracle.g1_generator()
    bases = np.array([oracle.g1_mul(g, k) for k in oracle.fr_ints(oracle.random_fr(n, 5))])
    sc = oracle.random_fr(n, 6)
    if bits == 64:
        sc[:, 1:] = 0
    sc[: n // 2, :] = sc[0]          # half the scalars equal: one bucket per window holds them
    want = oracle.msm_g1(bases, sc)
    a = ctx.msm_g1(bases, sc, bits)
    b = ctx.msm_g1(bases, sc, bits)
    assert np.array_equal(a, b) and np.array_equal(a, want)
