"""Benchmark: Groth16 prove constraints/s on the synthetic 2^20-constraint
R1CS (BASELINE.json configs[3]; circuit of crates/groth16-cli/src/lib.rs:57-70),
plus G1 MSM scalar-point pairs/s at 2^20 (configs[1]) on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--log-n 20]
  torchrun --nproc-per-node N bench.py --gpus N ...

A step = one full prove (quotient NTTs + 5 MSMs + host tail) with the proving
key and witness already resident in HBM.  N > 1: weak scaling -- the circuit
has N * 2^log_n constraints, every rank holds 1/N of every base vector
(GPU setup of its shard), computes its 1/N of the quotient
(four-step transforms with three RCCL all-to-alls inside the library, H
coefficients i = rank mod N), runs its MSM shard, and the 1.5 KB partial
accumulators meet in ONE all-gather over RCCL (the torch.distributed "nccl"
backend) before the fold.  Rank 0 prints one JSON
line.  The CPU baseline leg times the C restatement (oracle/, single thread)
on a bounded sample of the same workload.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
G1_PAIR_BYTES = 32 + 96        # scalar + affine base
G2_PAIR_BYTES = 32 + 192
METRIC = "Groth16 prove constraints/sec at 2^20 R1CS; G1 MSM throughput (scalar-point/s)"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def random_fr(rng, n):
    """n uniform canonical Fr (rejection on the top limb), (n, 4) uint64."""
    out = np.empty((n, 4), dtype=np.uint64)
    filled = 0
    rbytes = R.to_bytes(32, "little")
    top = int.from_bytes(rbytes[24:], "little")
    while filled < n:
        m = int((n - filled) * 1.1) + 16
        w = rng.integers(0, 2 ** 64, size=(m, 4), dtype=np.uint64)
        w[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
        ok = w[:, 3] < np.uint64(top)          # strictly below r's top limb: always < r
        w = w[ok][: n - filled]
        out[filled:filled + len(w)] = w
        filled += len(w)
    return out


def synthetic_witness(n, seed):
    """z = [1, x_0, y_0, x_0 y_0, ...] with uniform x, y (numpy + Python ints for x*y)."""
    rng = np.random.default_rng(seed)
    xy = random_fr(rng, 2 * n)
    ints = [int.from_bytes(row.tobytes(), "little") for row in xy]
    z = np.zeros((3 * n + 1, 4), dtype=np.uint64)
    z[0, 0] = 1
    z[1::3] = xy[0::2]
    z[2::3] = xy[1::2]
    prod = [(ints[2 * j] * ints[2 * j + 1]) % R for j in range(n)]
    z[3::3] = np.frombuffer(b"".join(p.to_bytes(32, "little") for p in prod), dtype=np.uint64).reshape(-1, 4)
    return z


def setup_params(seed):
    rng = np.random.default_rng(seed)
    vals = [int.from_bytes(r.tobytes(), "little") for r in random_fr(rng, 7)]
    return vals[:5], vals[5], vals[6]


def phase_table(prof):
    return {k: {"ms": round(v["ms"], 3), "launches": v["launches"], "units": v["units"]} for k, v in prof.items()}


# VALU view of the same kernel: every mixed add (madd-2008-s) in the prove's
# G1 MSMs is 8 Fq products of 14 x 14 radix-2^28 limb products (196 v_mad
# each; Y3 = R(Q-X3) - Y1 PPP counts two), 2 squarings (105 each) and 9
# Montgomery reductions of 196 (Y3's two products share one) = 3542
# v_mad_u64_u32; a prove MSM has 4 digit windows (64-bit scalars, c = 16).
# Peak: tools/mulbench.hip, best radix-2^28 variant, 72.2 G Fq-mul/s x 392 =
# 28.3 T v_mad_u64_u32/s.
MADS_PER_MADD = 8 * 196 + 2 * 105 + 9 * 196
PROVE_WINDOWS = 4
VALU_PEAK_TMADS = 28.3


def roofline_from(prof):
    """Dominant kernel: k_msm_accum<G1> (bucket accumulation of the four G1
    MSMs), priced at SURVEY 8(d)'s 128 B per scalar-point pair."""
    g1 = prof.get("msm_accum_g1", {"ms": 0.0, "launches": 0, "units": 0})
    ms, launches, units = g1["ms"], g1["launches"], g1["units"]
    if ms <= 0 or launches == 0:
        return None
    algo_bytes = G1_PAIR_BYTES * units
    achieved = algo_bytes / (ms / 1e3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get("msm_accum_g1_bytes_per_launch")
        except Exception:
            traffic = None
    tmads = units * PROVE_WINDOWS * MADS_PER_MADD / (ms / 1e3) / 1e12
    return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
            "kernel": "k_msm_accum<G1>",
            "algorithmic_bytes_per_launch": int(algo_bytes / launches),
            "avg_launch_ms": round(ms / launches, 4),
            "valu": {"achieved_tmad_per_s": round(tmads, 2), "peak_tmad_per_s": VALU_PEAK_TMADS,
                     "frac": round(tmads / VALU_PEAK_TMADS, 4)},
            "note": "integer-VALU bound (381-bit Montgomery products), not HBM; see DESIGN.md"}


def cpu_baseline(zkp, ctx, log_n, seed):
    """Oracle (C restatement, single thread) prove on a 2^log_n sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding as oracle   # cpu_baseline leg only
    n = 1 << log_n
    params, r, s = setup_params(seed)
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)   # pk built on GPU (not timed)
    opk = oracle.PK(qap.num_variables, n, 1)
    for nm in ("a_g1", "b_g1", "b_g2", "h_g1"):
        getattr(opk, nm)[:] = getattr(crs.pk, nm)
    opk.ic_g1[:len(crs.pk.ic_g1)] = crs.pk.ic_g1
    for nm in ("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"):
        w = crs.pk.point(nm)
        arr = getattr(opk.s, nm)
        for i, x in enumerate(w):
            arr[i] = int(x)
    opk.s.a_len = opk.s.b_len = opk.s.b2_len = qap.num_variables
    opk.s.ic_len, opk.s.h_len, opk.s.num_public = len(crs.pk.ic_g1), n, 1
    csr = oracle.CSR.synthetic(n)
    z = synthetic_witness(n, seed + 1)
    t0 = time.perf_counter()
    rc, proof = oracle.prove(opk, csr, z, 1, r, s)
    dt = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(f"oracle prove failed: {rc}")
    # same pk / z / r / s on the GPU must give the same bytes
    dpk = crs.pk.upload(ctx)
    gproof = zkp.Prover.prove(dpk, zkp.Witness(z, 1), r=r, s=s)
    dpk.free()
    return {"value": round(n / dt, 2), "unit": "constraints/s", "cores": 1, "kind": "port",
            "sample": f"oracle/zk_oracle.c prove() of the 2^{log_n}-constraint synthetic circuit, "
                      f"single thread (reference arkworks build has no `parallel`), {dt:.2f} s",
            "bit_exact_vs_gpu": bool(np.array_equal(gproof.words, proof))}


def msm_g1_bench(zkp, ctx, log_n, steps, warmup, seed):
    """configs[1]: G1 MSM, 2^log_n bases, uniform full-width scalars, inputs in HBM."""
    import torch
    n = 1 << log_n
    # 2^log_n distinct bases: h_g1 of a GPU setup on an n-constraint circuit
    # (row j uses variable j + 1 only)
    rp = np.arange(n + 1, dtype=np.uint64)
    col = np.arange(1, n + 1, dtype=np.uint32)
    csr = zkp.CSRMatrices(n, n + 1, [(rp, col, None), (rp, col, None), (rp, col, None)])
    params, _, _ = setup_params(seed)
    crs = zkp.CRS.generate_from_qap(ctx, zkp.QAP(csr), zkp.SetupParams(*params), 0)
    bases = crs.pk.h_g1
    import ctypes as C
    sc = random_fr(np.random.default_rng(seed + 7), n)
    d_sc = torch.from_numpy(sc.view(np.int64)).to(f"cuda:{ctx.device}")

    def measure(windows):
        """windows: bases uploaded with their 16 window-shifted copies
        (zk_msm_g1_upload_windows: one bucket set), else plain."""
        hb = C.c_void_p()
        up = zkp.lib().zk_msm_g1_upload_windows if windows else zkp.lib().zk_msm_g1_upload
        args = (C.c_void_p(ctx._h), zkp._p(bases), C.c_size_t(n)) + ((C.c_uint32(255),) if windows else ())
        t_up = time.perf_counter()
        zkp._check(up(*args, C.byref(hb)), ctx, "upload")
        t_up = time.perf_counter() - t_up
        out = np.zeros(13, dtype=np.uint64)

        def run():
            zkp._check(zkp.lib().zk_msm_g1_dev(C.c_void_p(ctx._h), hb, C.c_void_p(d_sc.data_ptr()), C.c_size_t(n),
                                                C.c_uint32(255), zkp._p(out)), ctx, "zk_msm_g1_dev")
        for _ in range(warmup):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        zkp.lib().zk_msm_bases_free(hb)
        return dt, t_up, out.copy()

    dt, t_up, r1 = measure(True)
    dt_plain, _, r2 = measure(False)
    if not np.array_equal(r1, r2):
        raise SystemExit("windowed and plain MSM disagree")
    return {"pairs_per_s": round(n / dt, 1), "n": n, "scalar_bits": 255, "ms_per_msm": round(dt * 1e3, 3),
            "bases": "uploaded once with 16 window-shifted copies (zk_msm_g1_upload_windows, %.0f ms)" % (t_up * 1e3),
            "plain": {"pairs_per_s": round(n / dt_plain, 1), "ms_per_msm": round(dt_plain * 1e3, 3),
                      "bases": "uploaded once, one copy (zk_msm_g1_upload)"}}


def ntt_bench(zkp, ctx, log_n, steps, warmup, seed):
    """configs[2]: forward radix-2 NTT over Fr, 2^log_n points in HBM, plus a
    round-trip check (inverse of the forward is the identity)."""
    import ctypes as C
    import torch
    n = 1 << log_n
    x = random_fr(np.random.default_rng(seed), n)
    d = torch.from_numpy(x.view(np.int64).copy()).to(f"cuda:{ctx.device}")
    L = zkp.lib()
    h = C.c_void_p(ctx._h)

    def run(direction):
        zkp._check(L.zk_ntt_fr_dev(h, C.c_void_p(d.data_ptr()), C.c_uint32(log_n), C.c_int(direction), None),
                   ctx, "zk_ntt_fr_dev")
    for _ in range(warmup):
        run(1)
        run(-1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run(1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    for _ in range(steps):
        run(-1)
    ok = bool(np.array_equal(d.cpu().numpy().view(np.uint64).reshape(-1, 4), x))
    return {"log_n": log_n, "ms_per_ntt": round(dt * 1e3, 3), "elements_per_s": round(n / dt, 1),
            "roundtrip_identity": ok}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-n", type=int, default=20, help="log2 constraints per GPU")
    ap.add_argument("--cpu-log-n", type=int, default=17, help="CPU baseline sample size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-msm", action="store_true")
    ap.add_argument("--seed", type=int, default=0x5EED0001)
    args = ap.parse_args()

    import torch
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # Rehearsal knobs (not the bench contract): ZK_BENCH_DIST_BACKEND=gloo and
    # ZK_BENCH_DEVICE=0 run N ranks on one GPU with CPU-side collectives and
    # no RCCL communicator (each rank then recomputes the whole quotient).
    backend = os.environ.get("ZK_BENCH_DIST_BACKEND", "nccl")
    local = int(os.environ.get("ZK_BENCH_DEVICE", local))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    coll_dev = f"cuda:{local}" if backend == "nccl" else "cpu"

    ctx = zkp.Context(local)
    if dist and backend == "nccl":
        # one RCCL communicator inside the library for the distributed
        # quotient (three all-to-alls per proof over xGMI); the unique id
        # travels over the torch process group
        obj = [zkp.Context.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        try:
            ctx.attach_rccl(obj[0], rank, world)
        except zkp.GrothError as e:   # every rank then recomputes the whole quotient
            log(f"[bench] RCCL attach failed ({e}); quotient replicated per rank")
    n = (1 << args.log_n) * world
    log_n_total = n.bit_length() - 1
    params, r, s = setup_params(args.seed)
    log(f"[bench] rank0: setup 2^{log_n_total}-constraint synthetic circuit on GPU (shard {rank}/{world})")
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    t0 = time.perf_counter()
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1, shard=rank, nshards=world)
    t_setup = time.perf_counter() - t0
    z = synthetic_witness(n, args.seed + 1)
    d_z = torch.from_numpy(z.view(np.int64)).to(f"cuda:{local}")
    zlen = len(z)
    log(f"[bench] setup {t_setup:.2f}s; witness ready ({zlen} vars)")

    def step():
        if world == 1:
            return zkp.Prover.prove_device(dpk, d_z.data_ptr(), zlen, 1, r, s)
        part = zkp.Prover.prove_partial(dpk, d_z.data_ptr(), zlen, 1, r, s)
        mine = torch.frombuffer(bytearray(part), dtype=torch.uint8).to(coll_dev)
        bufs = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(bufs, mine)                      # the one RCCL exchange
        return zkp.Prover.combine([b.cpu().numpy().tobytes() for b in bufs], r, s)

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        proof = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed / args.steps * 1e3
    value = n / (elapsed / args.steps)

    extra = {}
    if rank == 0 and world == 1:
        # PCIe-inclusive rate: the witness crosses from host memory each proof
        w = zkp.Witness(z, 1)
        zkp.Prover.prove(dpk, w, r=r, s=s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            zkp.Prover.prove(dpk, w, r=r, s=s)
        torch.cuda.synchronize()
        t_pc = (time.perf_counter() - t0) / 3
        extra["pcie_inclusive"] = {"ms_per_step": round(t_pc * 1e3, 3), "value": round(n / t_pc, 1),
                                   "note": "zk_groth16_prove with the witness in host memory"}
        dpk.free()
        if not args.no_msm:
            log("[bench] G1 MSM 2^20 (configs[1])")
            extra["msm_g1"] = msm_g1_bench(zkp, ctx, 20, args.steps, args.warmup, args.seed + 11)
            log("[bench] NTT 2^22 (configs[2])")
            extra["ntt"] = ntt_bench(zkp, ctx, 22, args.steps, args.warmup, args.seed + 31)
        if not args.no_cpu_baseline:
            log(f"[bench] CPU baseline: oracle prove at 2^{args.cpu_log_n}, 1 thread")
            extra["cpu_baseline"] = cpu_baseline(zkp, ctx, args.cpu_log_n, args.seed + 21)
    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 1), "unit": "constraints/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32", "data": "synthetic",
            "config": {"workload": "groth16_prove", "circuit": "n x (x*y=z) (groth16-cli generate_crs)",
                       "field": "BLS12-381 Fq/Fr Montgomery, 32x32->64-bit limb products (radix 2^28)",
                       "constraints": n, "constraints_per_gpu": 1 << args.log_n, "num_public": 1,
                       "parallelism": f"msm-shard{world}+quotient-a2a" if world > 1 else "single-gpu",
                       "setup_s": round(t_setup, 2)},
            "roofline": roofline_from(prof),
            "phases_ms_total": phase_table(prof),
            "proof_compressed_prefix": proof.serialize_compressed().hex()[:32],
        }
        rec.update(extra)
        rec.setdefault("cpu_baseline", None)
        print(json.dumps(rec), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
