"""configs[4] at size: the 2^24-constraint synthetic circuit
(crates/groth16-cli/src/lib.rs:55-70, num_public = 1) proved three ways on
ONE GPU, each bit for bit against the C oracle's prove() on the same
pk / z / r / s (crates/groth16-core/src/lib.rs:139-272):

  (a) the single-GPU proof: GPU setup straight into HBM, the c = 22
      three-window plan and the large-domain quotient the library picks at
      this size;
  (b) 8 virtual shards (zk_test_prove_virtual_shards): the 8-GPU layout --
      per-shard keys of 2^21 constraints (c = 16), the distributed quotient
      at m = 2^21 with its real index maps, the three all-to-alls as device
      copies, the MSM bases sharded by quotient-row ownership;
  (c) the same 8 shard keys through zk_groth16_prove_partial (each rank
      computing the whole quotient, no exchange) and zk_groth16_prove_combine.

Seeds are bench.py's (setup params 0x5EED0001, witness 0x5EED0002), so the
oracle's proof also equals the one recorded in profiles/r02_check_2p24_quot.json
(bench.ORACLE_2P24: the oracle is deterministic across rounds).  Each key is
freed before the next is made.  Host memory: ~55 GB (the host key and the
oracle's copy of it); GPU: ~70 GB for the 8 shard keys."""
import os
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOG_N = 24


def _bench():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    return bench


@pytest.fixture(scope="module")
def case_2p24(ctx, zkp, oracle):
    """(qap, params, r, s, device witness, oracle proof words) at 2^24."""
    bench = _bench()
    n = 1 << LOG_N
    params, r, s = bench.setup_params(0x5EED0001)
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    z = ctx.synthetic_witness(n, 0x5EED0002)
    t = time.perf_counter()
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)   # host key for the checker
    opk = bench.oracle_pk(oracle, crs.pk)
    del crs
    zh = z.cpu().numpy().view(np.uint64)
    rc, oproof = oracle.prove(opk, oracle.CSR.synthetic(n), zh, 1, r, s)
    del opk
    assert rc == 0
    print(f"\n[2^24] oracle proof on {oracle.default_threads()} threads: {time.perf_counter() - t:.1f} s", flush=True)
    assert oracle.proof_compress(oproof).hex() == bench.ORACLE_2P24   # the bytes bench.py's anchor is checked against
    return qap, params, r, s, z, oproof


def sample_key(dpk, rng, per_slot=48):
    """(slot -> (indices, canonical words)) of per_slot random compacted bases
    of a device key (test library readback, window 0)."""
    out = {}
    for slot in range(5):
        idx, words, _ = dpk.test_bases(slot)
        pick = rng.choice(len(idx), size=min(per_slot, len(idx)), replace=False)
        out[slot] = (idx[pick].astype(np.uint64), words[pick])
    return out


def check_samples(oracle, csr_o, params, samples):
    """The sampled device-key bases against or_setup_sample (the oracle's
    setup arithmetic at the sampled indices; crates/groth16-setup/src/lib.rs:141-268)."""
    vars_ = np.unique(np.concatenate([samples[k][0] for k in (0, 1, 2, 3)]))
    hidx = np.unique(samples[4][0])
    rc, ref = oracle.setup_sample(csr_o, params, 1, vars_, hidx)
    assert rc == 0
    pos = {int(v): i for i, v in enumerate(vars_)}
    hpos = {int(v): i for i, v in enumerate(hidx)}
    for slot, nm in ((0, "a_g1"), (1, "b_g2"), (2, "b_g1"), (3, "ic")):
        idx, words = samples[slot]
        want = ref[nm][[pos[int(v)] for v in idx]]
        assert np.array_equal(words, want), nm
    idx, words = samples[4]
    assert np.array_equal(words, ref["h_g1"][[hpos[int(v)] for v in idx]]), "h_g1"
    return len(vars_) + len(hidx)


@pytest.mark.timeout(900)
def test_2p24_single_gpu_prove(ctx, zkp, case_2p24):
    qap, params, r, s, z, oproof = case_2p24
    n = 1 << LOG_N
    t = time.perf_counter()
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    t_setup = time.perf_counter() - t
    try:
        zkp.Prover.prove_device(dpk, z.data_ptr(), 3 * n + 1, 1, r, s)
        t = time.perf_counter()
        proof = zkp.Prover.prove_device(dpk, z.data_ptr(), 3 * n + 1, 1, r, s)
        dt = time.perf_counter() - t
        samples = sample_key(dpk, np.random.default_rng(24))
    finally:
        dpk.free()
    print(f"[2^24] GPU setup {t_setup:.2f} s, prove {dt * 1e3:.1f} ms; build {zkp.build_id()}", flush=True)
    assert np.array_equal(proof.words, oproof)
    # the key itself, not only the proof: sampled bases vs the oracle's setup
    import binding as oracle
    k = check_samples(oracle, oracle.CSR.synthetic(n), params, samples)
    print(f"[2^24] single-GPU key: {k} sampled entries equal or_setup's", flush=True)


@pytest.mark.timeout(900)
def test_2p24_eight_shards_virtual_and_partial(ctx, zkp, case_2p24):
    qap, params, r, s, z, oproof = case_2p24
    n, N = 1 << LOG_N, 8
    t = time.perf_counter()
    dpks = [zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1, shard=k, nshards=N) for k in range(N)]
    t_setup = time.perf_counter() - t
    try:
        t = time.perf_counter()
        proof_v = zkp.Prover.prove_virtual_shards(dpks, z.data_ptr(), 3 * n + 1, 1, r, s)
        t_v = time.perf_counter() - t
        assert np.array_equal(proof_v.words, oproof), "8 virtual shards (distributed quotient)"
        t = time.perf_counter()
        parts = [zkp.Prover.prove_partial(d, z.data_ptr(), 3 * n + 1, 1, r, s) for d in dpks]
        t_p = time.perf_counter() - t
        proof_p = zkp.Prover.combine(parts, r, s)
        assert np.array_equal(proof_p.words, oproof), "8 shards' prove_partial + combine"
        rng = np.random.default_rng(8)
        shard_samples = [sample_key(d, rng, per_slot=24) for d in dpks]
    finally:
        for d in dpks:
            d.free()
    print(f"[2^24 x 8 shards] GPU setup {t_setup:.2f} s, virtual-rank proof {t_v * 1e3:.0f} ms, "
          f"8 partials (replicated quotient) {t_p * 1e3:.0f} ms", flush=True)
    # the sharded setup's bases themselves, sampled on every shard, against
    # the oracle's setup arithmetic at those indices
    import binding as oracle
    merged = {slot: (np.concatenate([sm[slot][0] for sm in shard_samples]),
                     np.concatenate([sm[slot][1] for sm in shard_samples])) for slot in range(5)}
    for k, sm in enumerate(shard_samples):
        assert (sm[4][0] % N == k).all()
    cnt = check_samples(oracle, oracle.CSR.synthetic(n), params, merged)
    print(f"[2^24 x 8 shards] {cnt} sampled key entries equal or_setup's", flush=True)


@pytest.mark.timeout(600)
def test_bench_anchor_matches_pinned_oracle_proof(ctx, zkp, case_2p24):
    """bench.py's N = 1 strong-scaling anchor (configs[4] on one GPU) checks
    its proof against bench.ORACLE_2P24; the fixture above pinned those bytes
    to a fresh oracle run."""
    bench = _bench()
    params, r, s = bench.setup_params(bench.DEFAULT_SEED)
    rec = bench.anchor_bench(zkp, ctx, LOG_N, params, r, s, bench.DEFAULT_SEED, 1, 0)
    assert rec["bit_exact_vs_oracle"] is True
    assert rec["msm_only"]["ms_per_step"] > 0 and rec["roofline"]["avg_launch_ms"] > 0
    print(f"[2^24 anchor] {rec['ms_per_step']} ms, MSM kernels {rec['msm_only']['ms_per_step']} ms", flush=True)
