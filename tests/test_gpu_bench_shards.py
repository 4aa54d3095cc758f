"""bench.py's one-GPU shard measurement (strong_scaling_anchor.shard8_msm_only)
at a small size: every key shard of the anchor's circuit set up and proved on
this GPU, the folded partials equal to the anchor's proof, per-shard MSM times
as medians over the proofs."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu


def _bench():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    return bench


@pytest.mark.parametrize("nshards", [2, 4])
def test_shard_msm_bench_folds_to_the_anchor_proof(ctx, zkp, nshards):
    bench = _bench()
    log_n = 12
    params, r, s = bench.setup_params(bench.DEFAULT_SEED)
    anc = bench.anchor_bench(zkp, ctx, log_n, params, r, s, bench.DEFAULT_SEED, 2, 1)
    assert anc["msm_only"]["ms_per_step"] > 0 and anc["msm_only"]["mean_ms"] > 0
    sh = bench.shard_msm_bench(zkp, ctx, log_n, nshards, params, r, s, bench.DEFAULT_SEED, 3,
                               anc["msm_only"]["ms_per_step"], anc["proof_compressed"])
    assert sh["folded_proof_bit_exact_vs_anchor"] is True
    assert sh["partials_reproducible"] is True
    assert len(sh["per_shard_ms"]) == nshards and min(sh["per_shard_ms"]) > 0
    assert sh["ms_per_step"] == max(sh["per_shard_ms"])
    assert sh["msm_scaling_projected"] > 0
    for k, (first, second) in sh["remeasured"].items():
        assert sh["per_shard_ms"][k] == min(first, second)
