"""Host-witness (drop-in zk_groth16_prove) vs device-witness prove time at
2^log_n, alternating library variants (ZK_AMD_LIB paths given as arguments,
'base' = the default build).  A/B tooling, not the bench."""
import importlib
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(log_n):
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    import bench
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    ctx = zkp.Context(0)
    n = 1 << log_n
    params, r, s = bench.setup_params(bench.DEFAULT_SEED)
    dpk = zkp.CRS.generate_device(ctx, zkp.QAP(zkp.CSRMatrices.synthetic(n)), zkp.SetupParams(*params), 1)
    d_z = ctx.synthetic_witness(n, bench.DEFAULT_SEED + 1)
    zh = d_z.cpu().numpy().view(np.uint64)
    w = zkp.Witness(zh, 1)
    res = {}
    for name, fn in (("dev", lambda: zkp.Prover.prove_device(dpk, d_z.data_ptr(), 3 * n + 1, 1, r, s)),
                     ("host", lambda: zkp.Prover.prove(dpk, w, r=r, s=s))):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(8):
            p = fn()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t) / 8 * 1e3
        res[name + "_proof"] = p
    assert res["dev_proof"] == res["host_proof"]
    print(f"{res['dev']:.3f} {res['host']:.3f}", flush=True)


def main():
    if sys.argv[1] == "--child":
        child(int(sys.argv[2]))
        return
    rounds, variants = int(sys.argv[1]), sys.argv[2:]
    out = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            env = dict(os.environ)
            if v != "base":
                env["ZK_AMD_LIB"] = os.path.join(ROOT, "zero-knowledge-proofs_amd", f"var_{v}", "libzkp_amd.so")
            r = subprocess.run([sys.executable, __file__, "--child", "20"], env=env, capture_output=True, text=True,
                               timeout=300)
            if r.returncode:
                print(v, "FAILED", r.stderr[-2000:], flush=True)
                continue
            dev, host = map(float, r.stdout.split()[-2:])
            out[v].append((dev, host))
            print(v, dev, host, flush=True)
    for v, xs in out.items():
        if xs:
            print(f"{v:10s} dev median {statistics.median(x[0] for x in xs):.3f}  host median "
                  f"{statistics.median(x[1] for x in xs):.3f}  extra {statistics.median(x[1] - x[0] for x in xs):.3f} ms")


if __name__ == "__main__":
    main()
