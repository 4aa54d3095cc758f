"""The configs[1] G1 MSM alone (zk_msm_g1_dev over window-shifted bases,
2^log_n uniform 255-bit scalars in HBM), for kernel profiling:

  rocprofv3 ... -- python3 tools/msm_only.py [log_n] [steps]

Bases: h_g1 of a GPU setup on an n-constraint diagonal circuit, as bench.py's
msm_g1_bench builds them."""
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
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    ctx = zkp.Context(0)
    n = 1 << log_n
    rp = np.arange(n + 1, dtype=np.uint64)
    col = np.arange(1, n + 1, dtype=np.uint32)
    csr = zkp.CSRMatrices(n, n + 1, [(rp, col, None), (rp, col, None), (rp, col, None)])
    params, _, _ = bench.setup_params(0x5EED0001)
    bases = zkp.CRS.generate_from_qap(ctx, zkp.QAP(csr), zkp.SetupParams(*params), 0).pk.h_g1
    sc = bench.random_fr(np.random.default_rng(0x5EED0001 + 7), n)
    d = torch.from_numpy(sc.view(np.int64)).cuda()
    L = zkp.lib()
    hb = C.c_void_p()
    zkp._check(L.zk_msm_g1_upload_windows(C.c_void_p(ctx._h), zkp._p(bases), C.c_size_t(n), C.c_uint32(255),
                                          C.byref(hb)), ctx, "upload")
    out = np.zeros(13, dtype=np.uint64)

    def run():
        zkp._check(L.zk_msm_g1_dev(C.c_void_p(ctx._h), hb, C.c_void_p(d.data_ptr()), C.c_size_t(n), C.c_uint32(255),
                                   zkp._p(out)), ctx, "zk_msm_g1_dev")
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    print(f"msm g1 2^{log_n}: {(time.perf_counter() - t0) / steps * 1e3:.3f} ms host-timed, {steps + 1} calls",
          flush=True)
    L.zk_msm_bases_free(hb)
    ctx.close()


if __name__ == "__main__":
    main()
