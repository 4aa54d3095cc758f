"""Host-to-device copy rates for a prove-sized witness (3n+1 Fr, 2^20: 100 MB):
pageable vs pinned source, one stream vs several concurrent copies.  Informs
the drop-in host-witness path (zk_groth16_prove).  Not part of the bench."""
import sys
import time

import numpy as np
import torch


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return nbytes / dt / 1e9, dt * 1e3


def main():
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    nbytes = (3 * (1 << log_n) + 1) * 32
    host = np.random.default_rng(1).integers(0, 2 ** 63, size=nbytes // 8, dtype=np.int64)
    src = torch.from_numpy(host)
    pinned = src.pin_memory()
    dst = torch.empty_like(src, device="cuda")
    out = {}
    out["pageable_1"] = rate(lambda: dst.copy_(src, non_blocking=False), nbytes)
    out["pinned_1"] = rate(lambda: dst.copy_(pinned, non_blocking=True), nbytes)
    for k in (2, 4):
        streams = [torch.cuda.Stream() for _ in range(k)]
        ch = nbytes // 8 // k

        def go():
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    dst[i * ch:(i + 1) * ch].copy_(pinned[i * ch:(i + 1) * ch], non_blocking=True)
        out[f"pinned_{k}streams"] = rate(go, nbytes)
    t = time.perf_counter()
    for _ in range(5):
        np.copyto(pinned.numpy(), host)
    out["host_memcpy_to_pinned"] = (nbytes / ((time.perf_counter() - t) / 5) / 1e9, (time.perf_counter() - t) / 5 * 1e3)
    for k, (gbs, ms) in out.items():
        print(f"{k:24s} {gbs:7.1f} GB/s  {ms:7.3f} ms for {nbytes / 1e6:.0f} MB")


if __name__ == "__main__":
    main()
