"""Stream timeline of proves (tuning): HIP events of the live profiler,
offsets from each prove's first event (zk_ctx_profile(ctx, 2) +
zk_ctx_timeline_read).

  python tools/timeline_live.py [log_n] [schedule] [host]
host: the drop-in zk_groth16_prove from a host witness (the split upload)
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    sched = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    ctx = zkp.Context(0)
    ctx.set_schedule(sched)
    n = 1 << log_n
    params, r, s = bench.setup_params(1)
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    z = ctx.synthetic_witness(n, 2)
    host = len(sys.argv) > 3 and sys.argv[3] == "host"
    if host:
        import numpy as np
        w = zkp.Witness(z.cpu().numpy().view(np.uint64), 1)

    def one():
        if host:
            zkp.Prover.prove(dpk, w, r=r, s=s)
        else:
            zkp.Prover.prove_device(dpk, z.data_ptr(), 3 * n + 1, 1, r, s)
    for _ in range(3):
        one()
    torch.cuda.synchronize()
    ctx.profile(2)
    for _ in range(4):
        one()
    text = ctx.timeline_read()
    ctx.profile(False)
    blocks = [b for b in text.strip().split("--") if b.strip()]
    for bi, blk in enumerate(blocks[-2:]):
        lines = [ln.split() for ln in blk.strip().splitlines() if ln.strip()]
        streams = {}
        for name, st, a, b in lines:
            streams.setdefault(st, []).append((float(a), float(b), name))
        print(f"== prove {bi}: span {max(float(l[3]) for l in lines):.3f} ms")
        for k, (st, ev) in enumerate(sorted(streams.items(), key=lambda kv: min(e[0] for e in kv[1]))):
            print(f"  stream {k}")
            for a, b, name in sorted(ev):
                print(f"    {name:28s} {a:7.3f} -> {b:7.3f}  ({b - a:.3f})")
    ctx.close()


if __name__ == "__main__":
    main()
