"""One-off parity check at configs[4]'s size on ONE GPU: the 2^24-constraint
synthetic prove (GPU setup straight into HBM, witness in HBM) against the C
oracle (all host cores) proving from the same key / witness / r / s.
Prints timings and the verdict as one JSON line (profiles/r02_check_2p24.json).

  python tools/check_2p24.py [log_n]
"""
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402


def main():
    import torch
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    gpu_only = len(sys.argv) > 2 and sys.argv[2] == "gpu"
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    import binding as oracle
    n = 1 << log_n
    ctx = zkp.Context(0)
    params, r, s = bench.setup_params(0x5EED0001)
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    t = time.perf_counter()
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    t_setup = time.perf_counter() - t
    z = ctx.synthetic_witness(n, 0x5EED0002)
    zlen = 3 * n + 1
    for _ in range(2):
        zkp.Prover.prove_device(dpk, z.data_ptr(), zlen, 1, r, s)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        proof = zkp.Prover.prove_device(dpk, z.data_ptr(), zlen, 1, r, s)
    torch.cuda.synchronize()
    t_prove = (time.perf_counter() - t) / 5
    print(f"[2^{log_n}] setup {t_setup:.2f} s, prove {t_prove * 1e3:.2f} ms", flush=True)
    dpk.free()
    if gpu_only:
        print(json.dumps({"log_n": log_n, "gpu_ms_per_prove": round(t_prove * 1e3, 2),
                          "proof_compressed": proof.serialize_compressed().hex(),
                          "env": {k: v for k, v in os.environ.items() if k.startswith("ZK_")}}), flush=True)
        return
    t = time.perf_counter()
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)
    opk = bench.oracle_pk(oracle, crs.pk)
    del crs
    t_hostkey = time.perf_counter() - t
    zh = z.cpu().numpy().view(np.uint64)
    print(f"[2^{log_n}] host key for the oracle {t_hostkey:.1f} s; oracle prove on {oracle.default_threads()} threads",
          flush=True)
    t = time.perf_counter()
    rc, oproof = oracle.prove(opk, oracle.CSR.synthetic(n), zh, 1, r, s)
    t_oracle = time.perf_counter() - t
    exact = rc == 0 and bool(np.array_equal(proof.words, oproof))
    ocomp = oracle.proof_compress(oproof).hex() if rc == 0 else None
    rec = {"log_n": log_n, "constraints": n, "gpu_setup_s": round(t_setup, 2), "gpu_ms_per_prove": round(t_prove * 1e3, 2),
           "gpu_constraints_per_s": round(n / t_prove, 1), "oracle_threads": oracle.default_threads(),
           "oracle_s": round(t_oracle, 1), "oracle_constraints_per_s": round(n / t_oracle, 1),
           "bit_exact_vs_oracle": exact, "proof_compressed": proof.serialize_compressed().hex(),
           "oracle_proof_compressed": ocomp,
           "components_equal": {"a": bool(np.array_equal(proof.words[:13], oproof[:13])),
                                "b": bool(np.array_equal(proof.words[13:38], oproof[13:38])),
                                "c": bool(np.array_equal(proof.words[38:], oproof[38:]))},
           "ntt_fuse": os.environ.get("ZK_NTT_FUSE", "auto (fused below 2^23)"), "build_id": zkp.build_id()}
    print(json.dumps(rec), flush=True)
    if not exact:
        sys.exit(1)


if __name__ == "__main__":
    main()
