"""The prover paths the library picks by size, each forced at small sizes
through zk_ctx_set_option (explicit ctx options; the library reads no
environment variables) and checked bit for bit against the C oracle:

  ZK_OPT_QUOTIENT_PATH = 1  the large-domain quotient (separate iNTT /
                            bit-reversed-table coset scale / NTT passes, and
                            the final coset iNTT in natural order through
                            ntt_natural) that the library takes from 2^23
                            constraints, at 1-, 2- and 3-pass sizes
                            including the size-1 domain;
  ZK_OPT_PROVE_WIN_C = 22   the 3-window / 2^21-bucket prove plan taken from
                            2^24 constraints per key shard (the batch keys
                            reach 23 bits, so the radix sort, merge and
                            bucket reduction see 2^21-bucket segments).
The defaults themselves run at 2^24 in tests/test_gpu_2p24.py."""
import numpy as np
import pytest

import gpu_util as U

pytestmark = pytest.mark.gpu


def _prove_vs_oracle(ctx, zkp, oracle, log_n):
    import pyref
    n = 1 << log_n
    rng = pyref.SplitMix64(900 + log_n)
    params = [rng.fr() for _ in range(5)]
    r, s = rng.fr(), rng.fr()
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)
    z = oracle.synthetic_witness(n, 901 + log_n)
    rc, want = oracle.prove(U.oracle_pk_from(oracle, crs.pk), oracle.CSR.synthetic(n), z, 1, r, s)
    assert rc == 0
    dpk = crs.pk.upload(ctx)
    got = zkp.Prover.prove(dpk, zkp.Witness(z, 1), r=r, s=s)
    dpk.free()
    assert np.array_equal(got.words, want), f"2^{log_n}"


@pytest.mark.parametrize("log_n", [0, 1, 11, 12, 21])
def test_large_domain_quotient_path_matches_oracle(zkp, oracle, log_n):
    with zkp.Context(0) as ctx:
        ctx.set_option(zkp.ZK_OPT_QUOTIENT_PATH, 1)
        _prove_vs_oracle(ctx, zkp, oracle, log_n)


@pytest.mark.parametrize("log_n", [0, 13])
def test_small_domain_quotient_path_forced_matches_oracle(zkp, oracle, log_n):
    with zkp.Context(0) as ctx:
        ctx.set_option(zkp.ZK_OPT_QUOTIENT_PATH, 0)
        _prove_vs_oracle(ctx, zkp, oracle, log_n)


@pytest.mark.parametrize("log_n", [4, 12])
def test_three_window_plan_matches_oracle(zkp, oracle, log_n):
    with zkp.Context(0) as ctx:
        ctx.set_option(zkp.ZK_OPT_PROVE_WIN_C, 22)
        _prove_vs_oracle(ctx, zkp, oracle, log_n)


def test_options_reject_unknown_values(zkp):
    with zkp.Context(0) as ctx:
        # 4: the old fault-injection option, now only in libzkp_amd_test.so
        for opt, val in ((zkp.ZK_OPT_QUOTIENT_PATH, 2), (zkp.ZK_OPT_PROVE_WIN_C, 17), (zkp.ZK_OPT_DIST_QUOTIENT, 1),
                         (zkp.ZK_OPT_EXCHANGE_FIRST, 2), (zkp.ZK_OPT_EXCHANGE_FIRST, -1),
                         (4, 2), (99, 0)):
            with pytest.raises(ValueError):
                ctx.set_option(opt, val)
        for sched in (1, 4, 9):
            with pytest.raises(ValueError):
                ctx.set_schedule(sched)
