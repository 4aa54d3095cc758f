"""Isolated per-phase timings of the hot kernels (one at a time, no stream
overlap), for kernel tuning.  Not part of the bench contract.

  python tools/phase_bench.py [--log-n 20] [--steps 5]
"""
import argparse
import ctypes as C
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (random_fr, setup_params)


def timed(ctx, fn, steps, warmup):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e3
    prof = ctx.profile_read()
    ctx.profile(False)
    return {"wall_ms": round(dt, 3),
            **{k: round(v["ms"] / steps, 3) for k, v in sorted(prof.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--ntt-log-n", type=int, default=22)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-ntt", action="store_true")
    args = ap.parse_args()
    import torch
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    L = zkp.lib()
    ctx = zkp.Context(0)
    h = C.c_void_p(ctx._h)
    n = 1 << args.log_n
    rp = np.arange(n + 1, dtype=np.uint64)
    col = np.arange(1, n + 1, dtype=np.uint32)
    csr = zkp.CSRMatrices(n, n + 1, [(rp, col, None), (rp, col, None), (rp, col, None)])
    params, _, _ = bench.setup_params(1)
    crs = zkp.CRS.generate_from_qap(ctx, zkp.QAP(csr), zkp.SetupParams(*params), 0)
    hb1, hb2 = C.c_void_p(), C.c_void_p()
    zkp._check(L.zk_msm_g1_upload(h, zkp._p(crs.pk.h_g1), C.c_size_t(n), C.byref(hb1)), ctx)
    zkp._check(L.zk_msm_g2_upload(h, zkp._p(crs.pk.b_g2), C.c_size_t(n), C.byref(hb2)), ctx)
    rng = np.random.default_rng(7)
    sc255 = torch.from_numpy(bench.random_fr(rng, n).view(np.int64)).cuda()
    s64 = np.zeros((n, 4), dtype=np.uint64)
    s64[:, 0] = rng.integers(0, 2 ** 64, size=n, dtype=np.uint64)
    sc64 = torch.from_numpy(s64.view(np.int64)).cuda()
    o1 = np.zeros(13, dtype=np.uint64)
    o2 = np.zeros(25, dtype=np.uint64)
    res = {}
    for nm, fn in [
        ("g1_255", lambda: L.zk_msm_g1_dev(h, hb1, C.c_void_p(sc255.data_ptr()), C.c_size_t(n), 255, zkp._p(o1))),
        ("g1_64", lambda: L.zk_msm_g1_dev(h, hb1, C.c_void_p(sc64.data_ptr()), C.c_size_t(n), 64, zkp._p(o1))),
        ("g2_64", lambda: L.zk_msm_g2_dev(h, hb2, C.c_void_p(sc64.data_ptr()), C.c_size_t(n), 64, zkp._p(o2))),
    ]:
        res[f"msm_{nm}_2^{args.log_n}"] = timed(ctx, lambda: zkp._check(fn(), ctx, nm), args.steps, args.warmup)
        print(nm, res[f"msm_{nm}_2^{args.log_n}"], file=sys.stderr, flush=True)
    for ln in ([] if args.no_ntt else sorted({args.log_n, args.ntt_log_n})):
        d = torch.from_numpy(bench.random_fr(rng, 1 << ln).view(np.int64)).cuda()
        res[f"ntt_fwd_2^{ln}"] = timed(
            ctx, lambda: zkp._check(L.zk_ntt_fr_dev(h, C.c_void_p(d.data_ptr()), ln, 1, None), ctx), args.steps,
            args.warmup)
        print(ln, res[f"ntt_fwd_2^{ln}"], file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
