"""Per-proof wall time of the 2^20 device-witness prove with the phase
profiler off vs on (HIP events around every phase, collected after each
proof), alternating blocks on one box; and the wall time against the GPU span
the profiler reports.  python tools/overhead_ab.py [log_n] [steps] [rounds]"""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    ctx = zkp.Context(0)
    n = 1 << log_n
    params, r, s = bench.setup_params(bench.DEFAULT_SEED)
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    z = ctx.synthetic_witness(n, bench.DEFAULT_SEED + 1)
    zlen = 3 * n + 1

    def block(prof):
        ctx.profile(prof)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            p = zkp.Prover.prove_device(dpk, z.data_ptr(), zlen, 1, r, s)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        span = None
        if prof:
            ph = ctx.profile_read()
            span = ph["prove_gpu_span"]["ms"] / steps if "prove_gpu_span" in ph else None
            if "host_prove_total" in ph:
                print(f"  host: prove_partial {ph['host_prove_total']['ms'] / steps:.3f} ms, launch "
                      f"{ph['host_launch']['ms'] / steps:.3f}, finish {ph['host_finish']['ms'] / steps:.3f}, "
                      f"after last {ph['host_tail_after_last']['ms'] / steps:.3f} ms per proof", flush=True)
            ctx.profile(False)
        return ms, span, p

    for _ in range(3):
        zkp.Prover.prove_device(dpk, z.data_ptr(), zlen, 1, r, s)
    off, on = [], []
    ref = None
    for k in range(rounds):
        for prof in ((False, True) if k % 2 == 0 else (True, False)):
            ms, span, p = block(prof)
            ref = ref or p
            assert p == ref
            (on if prof else off).append((ms, span))
            print(f"round {k} profile {'on ' if prof else 'off'}: {ms:.3f} ms per proof"
                  + (f" (GPU span {span:.3f} ms)" if span else ""), flush=True)
    med = lambda v: sorted(v)[len(v) // 2]
    print(f"median off {med([m for m, _ in off]):.3f} ms, on {med([m for m, _ in on]):.3f} ms, "
          f"GPU span {med([s for _, s in on]):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
