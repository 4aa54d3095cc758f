"""N virtual ranks of one sharded key on one GPU (test library's
zk_test_prove_virtual_shards: the distributed quotient's stages rank by rank,
all-to-alls as device copies, then each rank's MSMs), timed; for rocprofv3
kernel traces of the distributed-quotient kernels at configs[4] size.

  python tools/virtual_shards.py [log_n] [nshards] [steps]"""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    ctx = zkp.Context(0)
    n = 1 << log_n
    params, r, s = bench.setup_params(bench.DEFAULT_SEED)
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    dpks = [zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1, shard=k, nshards=N) for k in range(N)]
    z = ctx.synthetic_witness(n, bench.DEFAULT_SEED + 1)
    p = zkp.Prover.prove_virtual_shards(dpks, z.data_ptr(), 3 * n + 1, 1, r, s)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        p = zkp.Prover.prove_virtual_shards(dpks, z.data_ptr(), 3 * n + 1, 1, r, s)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / steps * 1e3
    ok = log_n == 24 and p.serialize_compressed().hex() == bench.ORACLE_2P24
    print(f"{N} virtual shards of 2^{log_n}: {ms:.1f} ms per proof (all ranks serial on one GPU); "
          f"pinned oracle proof: {ok}", flush=True)


if __name__ == "__main__":
    main()
