"""The configs[2] NTT alone (zk_ntt_fr_dev, 2^log_n forward + inverse), for
kernel profiling: rocprofv3 ... -- python3 tools/ntt_only.py [log_n] [steps] [fwd]"""
import ctypes as C
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    fwd_only = len(sys.argv) > 3 and sys.argv[3] == "fwd"
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    ctx = zkp.Context(0)
    n = 1 << log_n
    x = bench.random_fr(np.random.default_rng(1), n)
    d = torch.from_numpy(x.view(np.int64).copy()).cuda()
    L = zkp.lib()
    if fwd_only:   # PMC runs: exactly `steps` forward transforms, nothing else on the GPU
        for _ in range(steps):
            zkp._check(L.zk_ntt_fr_dev(C.c_void_p(ctx._h), C.c_void_p(d.data_ptr()), C.c_uint32(log_n), C.c_int(1),
                                       None), ctx)
        torch.cuda.synchronize()
        print(f"ntt 2^{log_n}: {steps} forward transforms", flush=True)
        ctx.close()
        return
    for direction in (1, -1) * steps:
        zkp._check(L.zk_ntt_fr_dev(C.c_void_p(ctx._h), C.c_void_p(d.data_ptr()), C.c_uint32(log_n),
                                   C.c_int(direction), None), ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        zkp._check(L.zk_ntt_fr_dev(C.c_void_p(ctx._h), C.c_void_p(d.data_ptr()), C.c_uint32(log_n), C.c_int(1),
                                   None), ctx)
    torch.cuda.synchronize()
    print(f"ntt 2^{log_n}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms host-timed", flush=True)
    ok = True
    for _ in range(steps):
        zkp._check(L.zk_ntt_fr_dev(C.c_void_p(ctx._h), C.c_void_p(d.data_ptr()), C.c_uint32(log_n), C.c_int(-1),
                                   None), ctx)
    ok = np.array_equal(d.cpu().numpy().view(np.uint64).reshape(-1, 4), x)
    print("roundtrip", ok)
    ctx.close()


if __name__ == "__main__":
    main()
