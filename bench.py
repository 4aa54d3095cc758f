"""Benchmark: Groth16 prove constraints/s on the synthetic R1CS of
crates/groth16-cli/src/lib.rs:57-70 (BASELINE.json configs[3] at one GPU,
configs[4] on N > 1), plus G1 MSM scalar-point pairs/s at 2^20 (configs[1])
and the 2^22 Fr NTT (configs[2]) on rank 0 of a one-GPU run.

  python bench.py [--gpus 1] [--steps K] [--warmup W]
  python bench.py --gpus N ...          (starts its own N rank processes)
  torchrun --nproc-per-node N bench.py --gpus N ...

A step = one full prove (quotient NTTs + 5 MSMs + host tail) with the proving
key and the witness already resident in HBM.

  N = 1  the 2^20-constraint prove (configs[3]); its own timed proof is
         checked bit for bit against the C oracle (oracle/, all host cores)
         proving from the same key, witness, r and s.  The line also carries
         `strong_scaling_anchor`: configs[4]'s 2^24 circuit -- the workload
         the N > 1 lines shard -- proved on this one GPU (proof checked
         against the oracle's pinned bytes, MSM kernel time from a
         serial-schedule pass), the N = 1 point of the strong-scaling curve.
  N > 1  strong scaling (default): ONE 2^24-constraint circuit (configs[4],
         --total-log-n) sharded over the N ranks -- every rank holds 1/N of
         every base vector (GPU setup of its shard), computes its 1/N of the
         quotient (four-step transforms with three RCCL all-to-alls inside the
         library; H coefficients i = rank mod N) and its MSM shard; the 1.5 KB
         partial accumulators meet in ONE all-gather over RCCL before the
         fold.  Beside the timed value: `msm_only` (max over ranks of the MSM
         kernels' time per proof, serial schedule), `roofline` (rank 0's
         accumulate), `quotient_replicated` (same keys, every rank computing
         the whole quotient, no all-to-all), `exchange_first` (the MSMs
         waiting for the distributed quotient) and `cpu_baseline` (the oracle on
         a bounded sample, rank 0).  --scaling weak keeps 2^log_n constraints
         per GPU instead.

Without a launcher (`--gpus N`, no WORLD_SIZE in the environment) the
parent process starts the N ranks itself as fresh child processes (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set), before
importing torch or the package: it never touches a GPU, the children share
its stdout (rank 0's JSON line), and it exits non-zero if any rank fails.

The ranks' control plane (barriers, the max-over-ranks timing, agreements) is
a gloo group; the library's RCCL communicator (the distributed quotient's
all-to-alls) and a torch RCCL group (the partials' all-gather) are attached
after it.  If either fails on any rank -- or the first distributed proof
does -- every rank carries on without it, labelled in the line ("quotient":
"replicated (rccl: ...)", "partials_gather": "gloo (rccl: ...)"), so the
MSM-scaling curve still comes out.

Rank 0 prints one JSON line.  The CPU baseline leg times the C restatement
(oracle/, test infrastructure) single-threaded on a bounded sample and on all
host cores at the full 2^20 size (N = 1), or on all host cores at a bounded
sample size (N > 1).
"""
import argparse
import glob
import importlib
import json
import statistics
import os
import platform
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
# The C oracle's compressed proof of the 2^24-constraint synthetic circuit at
# the default seeds (setup params 0x5EED0001, witness 0x5EED0002): the oracle
# is deterministic, so the one-GPU 2^24 anchor of the N = 1 line is checked
# against these bytes without a 45-s oracle run (tests/test_gpu_2p24.py
# reruns the oracle and pins it to the same bytes).
DEFAULT_SEED = 0x5EED0001
ORACLE_2P24 = ("975ca696ac5acaa2c7690b9d89ab763ee435fdae4fa76daf9d90e40e6c4cef0407dec0cf4b602165b475c26696cbec3e"
               "a7ab7a7b36fda6704c05a6dedbb181099f278a050b96ebd2862da2a29bb0b436efb8cb355c2bb4c889dd0089e68a7d45"
               "13db14b6f7322595e922f20c068400f5a044f3a4ce7311fec64d1f7e76ea24d68c1dd5328373c7369b56bd414eb6dea3"
               "9583f11348f3813b597738ee46c4145abb606199f147e04bf4786b7fbe29b7e9646516e5f7dedf4535783d11ece4d9ce")


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def random_fr(rng, n):
    """n uniform canonical Fr (rejection on the top limb), (n, 4) uint64."""
    out = np.empty((n, 4), dtype=np.uint64)
    filled = 0
    top = R >> 192
    while filled < n:
        m = int((n - filled) * 1.1) + 16
        w = rng.integers(0, 2 ** 64, size=(m, 4), dtype=np.uint64)
        w[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
        ok = w[:, 3] < np.uint64(top)          # strictly below r's top limb: always < r
        w = w[ok][: n - filled]
        out[filled:filled + len(w)] = w
        filled += len(w)
    return out


def setup_params(seed):
    rng = np.random.default_rng(seed)
    vals = [int.from_bytes(r.tobytes(), "little") for r in random_fr(rng, 7)]
    return vals[:5], vals[5], vals[6]


def prove_msm_pairs(n):
    """Scalar-point pairs of the reference's five MSMs for the synthetic
    circuit (V = 3n+1, num_public = 1; core:164-265): G1 = pi_A (V+2) + B_1
    (V+1) + H (n-1: coefficient n-1 is 0) + pi_C (V-2 ic terms + 3) = 10n+6,
    G2 = pi_B (V+2) = 3n+3."""
    return 10 * n + 6, 3 * n + 3


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
VALU_PEAK_TMADS = 28.3


def prove_windows(constraints_per_shard):
    """Digit windows of the prove MSMs' 64-bit scalars: the library's rule
    (prove.hip prove_win_c) -- c = 16 (4 windows), c = 22 (3 windows) from
    2^24 constraints per key shard."""
    c = 22 if constraints_per_shard >= 1 << 24 else 16
    return -(-64 // c)


def traffic_for(log_n):
    """HBM bytes per k_msm_accum<G1> launch from the FETCH/WRITE passes at
    THIS size (profiles/pmc_traffic_2p<log_n>.json), else None."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_2p{log_n}.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        return d.get("msm_accum_g1_bytes_per_launch"), os.path.relpath(path, ROOT)
    except Exception:
        return None, None


def msm_kernel_ms(prof):
    """Device ms of the MSM kernels (sort, accumulate, merge, bucket sums) in
    a profile; serial runs tag phases per MSM pipeline ("AB/msm_accum_g1")."""
    return sum(v["ms"] for k, v in prof.items() if k.split("/")[-1].startswith("msm_"))


def roofline_from(prof, log_n, overlapped=None, nshards=1):
    """Dominant kernel: k_msm_accum<G1> (bucket accumulation of the G1 MSMs:
    the A+B1 batch and the IC+H MSM), priced at SURVEY 8(d)'s 128 B per
    scalar-point pair.  `prof` comes from proves run with every kernel in order on one
    stream (zk_ctx_set_schedule 3), so a launch's HIP-event span is the
    kernel's own duration; `overlapped` (a profiled pass of the default
    four-stream schedule, after the timed region) is reported beside it."""
    def accum(pr):   # serial runs tag phases per MSM pipeline ("AB/msm_accum_g1", "ICH/msm_accum_g1")
        ms = launches = units = 0
        for k, v in pr.items():
            if k.split("/")[-1] == "msm_accum_g1":
                ms, launches, units = ms + v["ms"], launches + v["launches"], units + v["units"]
        return ms, launches, units
    ms, launches, units = accum(prof)
    if ms <= 0 or launches == 0:
        return None
    algo_bytes = G1_PAIR_BYTES * units
    achieved = algo_bytes / (ms / 1e3) / 1e9
    traffic, tsrc = traffic_for(log_n if nshards == 1 else f"{log_n}_shard{nshards}")
    tmads = units * prove_windows((1 << log_n) // nshards) * MADS_PER_MADD / (ms / 1e3) / 1e12
    out = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
           "traffic_source": tsrc, "kernel": "k_msm_accum<G1>",
           "algorithmic_bytes_per_launch": int(algo_bytes / launches),
           "avg_launch_ms": round(ms / launches, 4), "launches": launches,
           "schedule": "serial (zk_ctx_set_schedule 3): one stream, kernels in order",
           "valu": {"achieved_tmad_per_s": round(tmads, 2), "peak_tmad_per_s": VALU_PEAK_TMADS,
                    "frac": round(tmads / VALU_PEAK_TMADS, 4)},
           "note": "integer-VALU bound (381-bit Montgomery products), not HBM; see DESIGN.md"}
    issue = os.path.join(ROOT, "profiles", "r03_accum_valu_issue.json")
    if os.path.exists(issue):
        # SQ_INSTS_VALU pass + measured per-instruction issue costs: how close
        # the kernel is to the VALU issue limit of its own instruction mix
        d = json.load(open(issue))
        out["valu"]["issue"] = {"valu_instr_per_mixed_add": d["valu_wave_instructions_per_mixed_add"],
                                "v_mad_per_mixed_add": d["v_mad_per_mixed_add"],
                                "simd_cycles_per_valu_instr": d["simd_cycles_per_valu_instruction"]["no_counters"],
                                "source": os.path.relpath(issue, ROOT)}
    if overlapped:
        oms, ola, _ = accum(overlapped)
        if ola:
            out["overlapped_avg_launch_ms"] = round(oms / ola, 4)
    return out


def host_threads_label(nt):
    """Which host cores a CPU leg used: OMP threads against the lease's
    affinity set and the CPUs the OS shows (a GPU box lease sees far more
    CPUs than it may use)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    what = "all cores of this lease" if nt == aff else f"{nt} of the lease's {aff} affinity CPUs (OMP_NUM_THREADS)"
    return {"threads": nt, "affinity_cpus": aff, "host_cpus_visible": os.cpu_count(), "label": what}


def oracle_threads():
    """The oracle's default OpenMP thread count (oracle/binding.py)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding as oracle   # cpu_baseline legs only
    return oracle.default_threads()


def oracle_leg(fn, threads):
    """Time fn() with the oracle on `threads` OpenMP threads."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding as oracle   # cpu_baseline legs only
    prev = oracle.get_threads()
    oracle.set_threads(threads)
    try:
        t0 = time.perf_counter()
        out = fn(oracle)
        return out, time.perf_counter() - t0
    finally:
        oracle.set_threads(prev)


CORES_NOTE = ("the lease's CPU share: the GPU box shows every CPU of the shared host in its affinity set and sets "
              "OMP_NUM_THREADS to one GPU's share, which this leg keeps (the box rules forbid sizing worker pools "
              "beyond it); `all_affinity_cpus_projection` scales the measured 1-thread rate to every affinity CPU")


def affinity_projection(v1, v_nt, nt):
    """The oracle on EVERY CPU of the affinity set, projected linearly from
    its measured 1-thread rate: an upper bound (the measured nt-thread rate
    shows the real efficiency), so GPU / projection is a lower bound on the
    GPU's lead over this host."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"cpus": aff, "value": round(v1 * aff, 1), "basis": "1-thread rate x affinity CPUs (linear upper bound)",
            "measured_efficiency_at_lease_threads": round(v_nt / (v1 * nt), 3) if nt > 1 else None}


def host_cpu():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def oracle_pk(oracle, pk):
    V, n = pk.qap.num_variables, pk.qap.domain_size
    opk = oracle.PK(V, n, pk.num_public)
    for nm in ("a_g1", "b_g1", "b_g2", "h_g1"):
        getattr(opk, nm)[:] = getattr(pk, nm)
    opk.ic_g1[:len(pk.ic_g1)] = pk.ic_g1
    for nm in ("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"):
        arr = getattr(opk.s, nm)
        for i, x in enumerate(pk.point(nm)):
            arr[i] = int(x)
    opk.s.a_len, opk.s.b_len, opk.s.b2_len = len(pk.a_g1), len(pk.b_g1), len(pk.b_g2)
    opk.s.ic_len, opk.s.h_len, opk.s.num_public = len(pk.ic_g1), len(pk.h_g1), pk.num_public
    return opk


def cpu_baseline(zkp, ctx, n, params, r, s, z_host, gpu_proof, log_n_1t, seed):
    """The oracle (C restatement of the reference prover, test infrastructure)
    timed on this box's host cores:
      all cores  the full 2^20 prove on the bench's own key / witness / r / s,
                 which also checks the bench's timed proof bit for bit;
      1 thread   the reference's arkworks build has no `parallel` feature
                 (Cargo.lock:101-113,161-170): a bounded 2^log_n_1t sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding as oracle   # cpu_baseline leg only
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)   # same key, host copy (not timed)
    opk = oracle_pk(oracle, crs.pk)
    del crs
    csr = oracle.CSR.synthetic(n)
    nt = oracle.default_threads()
    oracle.set_threads(nt)
    t0 = time.perf_counter()
    rc, proof = oracle.prove(opk, csr, z_host, 1, r, s)
    dt_all = time.perf_counter() - t0
    del opk
    if rc != 0:
        raise RuntimeError(f"oracle prove failed: {rc}")
    exact = bool(np.array_equal(gpu_proof.words, proof))
    # single thread, bounded sample of the same workload
    n1 = 1 << log_n_1t
    qap1 = zkp.QAP(zkp.CSRMatrices.synthetic(n1))
    crs1 = zkp.CRS.generate_from_qap(ctx, qap1, zkp.SetupParams(*params), 1)
    opk1 = oracle_pk(oracle, crs1.pk)
    z1 = ctx.synthetic_witness(n1, seed).cpu().numpy().view(np.uint64)
    oracle.set_threads(1)
    t0 = time.perf_counter()
    rc, proof1 = oracle.prove(opk1, oracle.CSR.synthetic(n1), z1, 1, r, s)
    dt_1 = time.perf_counter() - t0
    oracle.set_threads(nt)
    dpk1 = crs1.pk.upload(ctx)
    g1 = zkp.Prover.prove(dpk1, zkp.Witness(z1, 1), r=r, s=s)
    dpk1.free()
    cpu = host_cpu()
    lab = host_threads_label(nt)
    v1 = n1 / dt_1
    return {"value": round(n / dt_all, 2), "unit": "constraints/s", "cores": nt, "kind": "port",
            "cores_note": CORES_NOTE,
            "all_affinity_cpus_projection": affinity_projection(v1, n / dt_all, nt),
            "sample": f"oracle/zk_oracle.c prove() of the full 2^{n.bit_length() - 1}-constraint circuit on "
                      f"{lab['label']} (OpenMP: MSM point chunks, FFT butterflies), {dt_all:.2f} s, same pk/z/r/s "
                      f"as the GPU's timed proof",
            "cpu_model": cpu, "host_cpus_visible": os.cpu_count(), "affinity_cpus": lab["affinity_cpus"],
            "bit_exact_vs_gpu": exact,
            "single_thread": {"value": round(n1 / dt_1, 2), "unit": "constraints/s", "cores": 1,
                              "sample": f"2^{log_n_1t}-constraint prove, 1 thread (the reference's build), "
                                        f"{dt_1:.2f} s",
                              "bit_exact_vs_gpu": bool(np.array_equal(g1.words, proof1))}}


def cpu_sample_baseline(zkp, ctx, log_n, params, r, s, seed):
    """N > 1 lines (rank 0, after the timed region): the oracle on all its
    OpenMP threads, proving a bounded 2^log_n sample of the same circuit
    family from a GPU-made key, checked bit for bit against this GPU's
    one-GPU proof of the same sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import binding as oracle   # cpu_baseline leg only
    n = 1 << log_n
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    crs = zkp.CRS.generate_from_qap(ctx, qap, zkp.SetupParams(*params), 1)
    opk = oracle_pk(oracle, crs.pk)
    d_z = ctx.synthetic_witness(n, seed)
    z_host = d_z.cpu().numpy().view(np.uint64)
    dpk = crs.pk.upload(ctx)
    del crs
    gpu = zkp.Prover.prove_device(dpk, d_z.data_ptr(), 3 * n + 1, 1, r, s)
    dpk.free()
    nt = oracle.default_threads()
    oracle.set_threads(nt)
    t0 = time.perf_counter()
    rc, proof = oracle.prove(opk, oracle.CSR.synthetic(n), z_host, 1, r, s)
    dt = time.perf_counter() - t0
    del opk
    if rc != 0:
        raise RuntimeError(f"oracle prove failed: {rc}")
    lab = host_threads_label(nt)
    # the 1-thread rate on a 2^15 sample for the all-CPU projection
    n1 = 1 << 15
    csr1 = oracle.CSR.synthetic(n1)
    crs1 = zkp.CRS.generate_from_qap(ctx, zkp.QAP(zkp.CSRMatrices.synthetic(n1)), zkp.SetupParams(*params), 1)
    opk1 = oracle_pk(oracle, crs1.pk)
    z1 = ctx.synthetic_witness(n1, seed).cpu().numpy().view(np.uint64)
    oracle.set_threads(1)
    t0 = time.perf_counter()
    oracle.prove(opk1, csr1, z1, 1, r, s)
    v1 = n1 / (time.perf_counter() - t0)
    oracle.set_threads(nt)
    return {"value": round(n / dt, 2), "unit": "constraints/s", "cores": nt, "kind": "port",
            "cores_note": CORES_NOTE, "all_affinity_cpus_projection": affinity_projection(v1, n / dt, nt),
            "sample": f"oracle/zk_oracle.c prove() of a 2^{log_n}-constraint sample of the same synthetic circuit "
                      f"family on {lab['label']} (rank 0, after the timed region), {dt:.2f} s; the oracle's "
                      f"constraints/s barely depends on size (2^20 vs 2^24 within 10 %, DESIGN.md 4)",
            "cpu_model": host_cpu(), "host_cpus_visible": os.cpu_count(), "affinity_cpus": lab["affinity_cpus"],
            "bit_exact_vs_gpu": bool(np.array_equal(gpu.words, proof))}


def anchor_bench(zkp, ctx, log_n, params, r, s, seed, steps, warmup, win_c=0):
    """The N = 1 line's strong-scaling anchor: the SAME workload the N > 1
    lines shard (configs[4], 2^log_n constraints) proved on this one GPU,
    overlapped schedule timed like the headline, plus a serial-schedule pass
    for the MSM kernels' own time.  Its compressed proof is checked against
    the oracle's pinned bytes (ORACLE_2P24) at the default seeds."""
    import torch
    n = 1 << log_n
    zlen = 3 * n + 1
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    t0 = time.perf_counter()
    ctx.set_option(zkp.ZK_OPT_PROVE_WIN_C, win_c)   # 0: the library's choice by size
    try:
        dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    finally:
        ctx.set_option(zkp.ZK_OPT_PROVE_WIN_C, 0)
    t_setup = time.perf_counter() - t0
    d_z = ctx.synthetic_witness(n, seed + 1)
    try:
        def run():
            return zkp.Prover.prove_device(dpk, d_z.data_ptr(), zlen, 1, r, s)
        for _ in range(warmup):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            proof = run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        ctx.set_schedule(3)
        ctx.profile(True)
        ks = max(2, steps // 2)
        t0 = time.perf_counter()
        msm_each, p3, prof = per_proof_msm_ms(ctx, run, ks)
        torch.cuda.synchronize()
        t_ser = (time.perf_counter() - t0) / ks
        ctx.profile(False)
        ctx.set_schedule(0)
    finally:
        dpk.free()
        del d_z
    if p3 != proof:
        raise SystemExit("anchor: serial-schedule proof differs from the overlapped one")
    hexp = proof.serialize_compressed().hex()
    pinned = ORACLE_2P24 if (log_n == 24 and seed == DEFAULT_SEED) else None
    msm_ms = statistics.median(msm_each)
    g1, g2 = prove_msm_pairs(n)
    return {"workload": f"groth16_prove_2^{log_n}", "constraints": n, "n_gpus": 1, "steps": steps,
            "ms_per_step": round(dt * 1e3, 3), "value": round(n / dt, 1), "unit": "constraints/s",
            "setup_s": round(t_setup, 2),
            "msm_only": {"ms_per_step": round(msm_ms, 3), "pairs_per_s": round((g1 + g2) / (msm_ms / 1e3), 1),
                         "g1_pairs": g1, "g2_pairs": g2, "mean_ms": round(sum(msm_each) / ks, 3),
                         "timing": "HIP events around every MSM kernel (sort, accumulate, merge, bucket sums) of "
                                   "serial-schedule proves (zk_ctx_set_schedule 3), median over the proofs"},
            "serial_schedule": {"ms_per_step": round(t_ser * 1e3, 3), "steps": ks,
                                "phases_ms_total": phase_table(prof),
                                "note": "every kernel in order on one stream, HIP events per phase; totals over "
                                        "`steps` proofs"},
            "window_bits": win_c or (22 if n >= 1 << 24 else 16),
            "roofline": roofline_from(prof, log_n) if not win_c else None,
            "proof_compressed": hexp,
            "bit_exact_vs_oracle": (hexp == pinned) if pinned else None,
            "oracle_reference": "bench.ORACLE_2P24 (pinned oracle proof; tests/test_gpu_2p24.py reruns the oracle)"
                                if pinned else "no pinned oracle proof at these seeds/size",
            "note": "the same circuit, key parameters, witness and r, s as the N > 1 lines (configs[4]); "
                    "strong-scaling speedup at N = value_N / this value, MSM scaling = this msm_only.ms_per_step "
                    "/ msm_only.ms_per_step of the N line (DESIGN.md 5)"}


def per_proof_msm_ms(ctx, run, ks):
    """ks proofs with the phase profile on: the MSM kernels' ms of each proof
    (differences of the cumulative profile, which every proof collects before
    it returns), the last proof and the cumulative profile."""
    times, prev, out = [], 0.0, None
    for _ in range(ks):
        out = run()
        cum = msm_kernel_ms(ctx.profile_read())
        times.append(cum - prev)
        prev = cum
    return times, out, ctx.profile_read()


def msm_phase_split(prof, steps):
    """Per-proof ms of the MSM phases of a serial-schedule profile, summed
    over the MSMs: sort (grouping), accumulate (G1 / G2), merge (fixups),
    bucket sums (row/column sums + quantities)."""
    out = {"sort": 0.0, "accum_g1": 0.0, "accum_g2": 0.0, "merge": 0.0, "bucket_sum": 0.0}
    for k, v in prof.items():
        ph = k.split("/")[-1]
        key = {"msm_sort": "sort", "msm_accum_g1": "accum_g1", "msm_accum_g2": "accum_g2", "msm_merge": "merge",
               "msm_bucket_sum": "bucket_sum"}.get(ph)
        if key:
            out[key] += v["ms"] / steps
    return {k: round(v, 3) for k, v in out.items()}


def shard_msm_bench(zkp, ctx, log_n, nshards, params, r, s, seed, ks, anchor_msm_ms, anchor_hex):
    """One GPU, one shard at a time: the N = nshards lines' key shards of the
    2^log_n circuit (GPU setup of shard k of nshards, the same witness, r, s
    as the anchor), each proved with every kernel in order on one stream
    (zk_ctx_set_schedule 3) and the MSM kernels' HIP-event time taken per
    proof -- the per-rank MSM work of the N = nshards run, measured here.
    The shards' partials are folded (zk_groth16_prove_combine) and the proof
    checked against the anchor's (= the pinned oracle proof).  No exchange is
    attached, so each shard computes the whole quotient locally; only MSM
    kernels are counted."""
    import torch
    n = 1 << log_n
    zlen = 3 * n + 1
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    d_z = ctx.synthetic_witness(n, seed + 1)
    def measure(k):
        dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1, shard=k, nshards=nshards)
        try:
            ctx.set_schedule(3)
            part = zkp.Prover.prove_partial(dpk, d_z.data_ptr(), zlen, 1, r, s)   # warm-up, and the partial
            torch.cuda.synchronize()
            ctx.profile(True)

            def run():
                p = zkp.Prover.prove_partial(dpk, d_z.data_ptr(), zlen, 1, r, s)
                if p != part:
                    raise SystemExit(f"shard {k}: partials of consecutive proofs differ")
                return p
            each, _, prof = per_proof_msm_ms(ctx, run, ks)
        finally:
            ctx.profile(False)
            ctx.set_schedule(0)
            dpk.free()
        return round(statistics.median(each), 3), msm_phase_split(prof, ks), part

    per, parts, phases = [], [], []
    t0 = time.perf_counter()
    for k in range(nshards):
        ms, ph, part = measure(k)
        per.append(ms)
        phases.append(ph)
        parts.append(part)
    # the shards are the same work up to the key's variable split: a shard
    # more than 10 % above the median of the shards is measured once more (a
    # slow spell of the box spans whole shards, not single proofs) and keeps
    # the lower median; both values are reported
    remeasured = {}
    mid = statistics.median(per)
    for k in range(nshards):
        if per[k] > 1.1 * mid:
            ms, ph, _ = measure(k)
            remeasured[k] = [per[k], ms]
            if ms < per[k]:
                per[k], phases[k] = ms, ph
    del d_z
    proof = zkp.Prover.combine(parts, r, s)
    worst = max(range(nshards), key=lambda k: per[k])
    return {"shards": nshards, "constraints_per_shard": n // nshards, "steps": ks,
            "ms_per_step": per[worst], "shard0_ms": per[0], "slowest_shard": worst, "per_shard_ms": per,
            "phases_ms_slowest": phases[worst],
            "msm_scaling_projected": round(anchor_msm_ms / per[worst], 3),
            "folded_proof_bit_exact_vs_anchor": proof.serialize_compressed().hex() == anchor_hex,
            "partials_reproducible": True, "remeasured": remeasured,
            "timing": "median over the shard's proofs of the MSM kernels' HIP-event ms per proof",
            "wall_s": round(time.perf_counter() - t0, 1)}


FR_MUL_MADS = 9 * 9 * 2   # radix-2^29 Fr product: 81 limb products + 81 in the reduction (ff.hpp)


def traffic_file(name):
    """HBM bytes per launch of a kernel from a committed rocprofv3 FETCH/WRITE
    pass (profiles/<name>), else (None, None)."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None, None
    try:
        return json.load(open(path)).get("bytes_per_launch"), os.path.relpath(path, ROOT)
    except Exception:
        return None, None


def latest_profile(suffix):
    """profiles/rNN_<suffix> of the latest round that has one (None if none)."""
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r[0-9][0-9]_{suffix}")))
    return os.path.basename(found[-1]) if found else suffix


def kernel_stats_file(name, prefix):
    """(calls, total ms) of the kernels whose name starts with `prefix` in a
    committed rocprofv3 --stats summary (profiles/<name>, the markdown table
    tools/prof_summary.py writes), else None."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    calls, total = 0, 0.0
    for ln in open(path).read().splitlines()[2:]:
        c = [x.strip() for x in ln.strip().strip("|").split("|")]
        if len(c) >= 3 and c[0].startswith(prefix):
            calls += int(c[1])
            total += float(c[2])
    return (calls, total, os.path.relpath(path, ROOT)) if calls else None


NTT_TILE_LOG = 10   # ntt.hip: 2^10-element tiles


def ntt_passes(log_n):
    """Passes of one 2^log_n API transform (ntt.hip pass_plan: the contiguous
    pass takes up to NTT_TILE_LOG stages, the rest is split into passes of
    <= NTT_TILE_LOG)."""
    t = NTT_TILE_LOG
    return 1 + (max(log_n - t, 0) + t - 1) // t


def msm_g1_bench(zkp, ctx, log_n, steps, warmup, seed, cpu=True):
    """configs[1]: G1 MSM, 2^log_n bases, uniform full-width scalars, inputs in HBM."""
    import ctypes as C
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
    sc = random_fr(np.random.default_rng(seed + 7), n)
    d_sc = torch.from_numpy(sc.view(np.int64)).to(f"cuda:{ctx.device}")
    sc64 = np.zeros_like(sc)                 # also the prove path's 64-bit scalars
    sc64[:, 0] = sc[:, 0]
    d_sc64 = torch.from_numpy(sc64.view(np.int64)).to(f"cuda:{ctx.device}")
    phases = {}

    def measure(windows, bits=255, profile=False):
        """windows: bases uploaded with their window-shifted copies (13 at c = 20 for 255-bit scalars,
        4 at c = 16 for 64-bit ones; zk_msm_g1_upload_windows: one bucket set), else plain."""
        hb = C.c_void_p()
        up = zkp.lib().zk_msm_g1_upload_windows if windows else zkp.lib().zk_msm_g1_upload
        args = (C.c_void_p(ctx._h), zkp._p(bases), C.c_size_t(n)) + ((C.c_uint32(bits),) if windows else ())
        t_up = time.perf_counter()
        zkp._check(up(*args, C.byref(hb)), ctx, "upload")
        t_up = time.perf_counter() - t_up
        out = np.zeros(13, dtype=np.uint64)
        d = d_sc if bits > 64 else d_sc64

        def run():
            zkp._check(zkp.lib().zk_msm_g1_dev(C.c_void_p(ctx._h), hb, C.c_void_p(d.data_ptr()), C.c_size_t(n),
                                                C.c_uint32(bits), zkp._p(out)), ctx, "zk_msm_g1_dev")
        for _ in range(warmup):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        if profile:   # per-phase kernel time from live HIP events, untimed loop
            ctx.profile(True)
            for _ in range(steps):
                run()
            phases.update(ctx.profile_read())
            ctx.profile(False)
        zkp.lib().zk_msm_bases_free(hb)
        return dt, t_up, out.copy()

    dt, t_up, r1 = measure(True, profile=True)
    dt_plain, _, r2 = measure(False)
    if not np.array_equal(r1, r2):
        raise SystemExit("windowed and plain MSM disagree")
    dt64, _, r3 = measure(True, 64)
    dt64_plain, _, r4 = measure(False, 64)
    if not np.array_equal(r3, r4):
        raise SystemExit("windowed and plain 64-bit MSM disagree")
    # roofline: the whole MSM and its dominant kernel (the bucket accumulate),
    # 128 B per pair; VALU at 3542 v_mad per mixed add, one add
    # per (point, digit window): 13 windows of 20 bits for 255-bit scalars
    nwin = -(-255 // 20)
    ph = {k: v["ms"] / steps for k, v in phases.items() if k.startswith("msm_")}
    tot = sum(ph.values()) or float("nan")
    acc_ms = ph.get("msm_accum_g1", float("nan"))
    algo = G1_PAIR_BYTES * n
    tmads = n * nwin * MADS_PER_MADD / (acc_ms / 1e3) / 1e12
    traffic, tsrc = traffic_file(f"pmc_msm_2p{log_n}.json")
    roof = {"bound": "hbm", "achieved": round(algo / dt / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(algo / dt / 1e9 / HBM_PEAK_GBS, 6), "traffic": traffic, "traffic_source": tsrc,
            "algorithmic_bytes": algo, "kernel": "k_msm_accum<G1>", "kernel_ms": round(acc_ms, 4),
            "kernel_frac": round(algo / (acc_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 6),
            "valu": {"achieved_tmad_per_s": round(tmads, 2), "peak_tmad_per_s": VALU_PEAK_TMADS,
                     "frac": round(tmads / VALU_PEAK_TMADS, 4),
                     "count": f"{nwin} windows x n mixed adds x {MADS_PER_MADD} v_mad_u64_u32, accumulate kernel"},
            "phase_ms": {k: round(v, 4) for k, v in ph.items()},
            "sort_and_reduction_share": round(1 - acc_ms / tot, 4),
            "note": "integer-VALU bound (381-bit Montgomery products); HBM frac reported as north_star asks"}
    rec = {"pairs_per_s": round(n / dt, 1), "n": n, "scalar_bits": 255, "ms_per_msm": round(dt * 1e3, 3),
           "bases": "uploaded once with 13 window-shifted copies (c = 20; zk_msm_g1_upload_windows, %.0f ms)" % (t_up * 1e3),
           "plain": {"pairs_per_s": round(n / dt_plain, 1), "ms_per_msm": round(dt_plain * 1e3, 3),
                     "bases": "uploaded once, one copy (zk_msm_g1_upload)"},
           "bits64": {"pairs_per_s": round(n / dt64, 1), "ms_per_msm": round(dt64 * 1e3, 3),
                      "plain_ms_per_msm": round(dt64_plain * 1e3, 3),
                      "note": "the same bases with the low 64 bits of the scalars (the prove path's lo64 "
                              "distribution): 4 window copies at c = 16; checked equal to the plain upload"},
           "roofline": roof,
           "parity": "tests/test_gpu_headline.py::test_msm_g1_2p20_closed_form (same sizes, closed form)"}
    if cpu:
        # the oracle's ark-style signed-digit Pippenger on the same bases and
        # scalars: all OMP threads on the full size (checked equal to the GPU
        # result), one thread on a 2^16 prefix
        nt = oracle_threads()
        res, dt_n = oracle_leg(lambda o: o.msm_g1(bases, sc), nt)
        n1 = min(n, 1 << 16)
        _, dt_1 = oracle_leg(lambda o: o.msm_g1(bases[:n1], sc[:n1]), 1)
        lab = host_threads_label(nt)
        rec["cpu_baseline"] = {"value": round(n / dt_n, 1), "unit": "pairs/s", "cores": nt, "kind": "port",
                               "sample": f"oracle/zk_oracle.c or_msm_g1 (ark-style signed-digit Pippenger), the "
                                         f"same 2^{log_n} bases and scalars on {lab['label']}, {dt_n:.2f} s",
                               "bit_exact_vs_gpu": bool(np.array_equal(res, r1)), **{k: lab[k] for k in
                                                                                       ("affinity_cpus", "host_cpus_visible")},
                               "single_thread": {"value": round(n1 / dt_1, 1), "unit": "pairs/s", "cores": 1,
                                                 "sample": f"2^{n1.bit_length() - 1}-pair prefix, 1 thread, {dt_1:.2f} s"}}
    return rec


def ntt_bench(zkp, ctx, log_n, steps, warmup, seed, cpu=True):
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
    for _ in range(max(warmup, 10)):   # ~12 ms of warmup: the clocks ramp up
        run(1)
        run(-1)
    torch.cuda.synchronize()
    steps = max(steps, 20)
    t0 = time.perf_counter()
    for _ in range(steps):
        run(1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    for _ in range(steps):
        run(-1)
    ok = bool(np.array_equal(d.cpu().numpy().view(np.uint64).reshape(-1, 4), x))
    # kernel time of the forward transform alone: HIP events around its
    # passes on the launching stream, over the same number of forward calls
    ctx.profile(True)
    for _ in range(steps):
        run(1)
    torch.cuda.synchronize()
    k = ctx.profile_read().get("ntt", {"ms": 0.0, "launches": 0})
    ctx.profile(False)
    y = d.cpu().numpy().view(np.uint64).reshape(-1, 4).copy()   # = NTT^steps(x): only the roofline run's state
    ems = k["ms"] / max(k["launches"], 1)
    # kernel time per transform from the committed rocprofv3 kernel trace of
    # tools/ntt_only.py at this size (the pass kernels' total over the
    # transforms it ran); the live events above bracket whole calls and
    # include the gaps between the passes' launches
    ks = kernel_stats_file(latest_profile(f"ntt_2p{log_n}_kernel_stats.md"), "k_ntt_pass")
    if ks:
        kms = ks[1] / (ks[0] / ntt_passes(log_n))
        ksrc = f"rocprofv3 --kernel-trace --stats of tools/ntt_only.py {log_n} ({ks[2]}): {ks[0]} pass launches"
    else:
        kms = ems
        ksrc = "HIP events around whole transform calls (no rocprof summary at this size)"
    algo = 2 * 32 * n
    bfly = (n // 2) * log_n
    tmads = bfly * FR_MUL_MADS / (kms / 1e3) / 1e12
    traffic, tsrc = traffic_file(f"pmc_ntt_2p{log_n}.json")
    rec = {"log_n": log_n, "ms_per_ntt": round(dt * 1e3, 3), "elements_per_s": round(n / dt, 1),
           "kernel_ms_per_ntt": round(kms, 4),
           "kernel_timing": ksrc,
           "event_ms_per_ntt": round(ems, 4),
           "event_timing": "HIP events around each forward call on the library's stream, %d calls: the passes plus "
                           "the launch gaps between them" % steps,
           "api": "zk_ntt_fr_dev (natural order in and out, data in HBM, one stream sync per call)",
           "roundtrip_identity": ok,
           "roofline": {"bound": "hbm", "achieved": round(algo / (kms / 1e3) / 1e9, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(algo / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 6),
                        "traffic": traffic, "traffic_source": tsrc, "algorithmic_bytes": algo,
                        "valu": {"achieved_tmad_per_s": round(tmads, 2), "peak_tmad_per_s": VALU_PEAK_TMADS,
                                 "frac": round(tmads / VALU_PEAK_TMADS, 4),
                                 "count": f"(n/2) log n butterflies x {FR_MUL_MADS} v_mad (one Fr product each)"},
                        "note": "latency-bound inside the butterfly chains (DESIGN.md 7.3)"}}
    if cpu:
        # the oracle's radix-2 FFT (ark-poly Radix2EvaluationDomain semantics)
        # on the same input, all OMP threads, then one thread; both checked
        # against a GPU forward transform of the same input
        d.copy_(torch.from_numpy(x.view(np.int64).copy()).to(d.device))
        run(1)
        gpu_y = d.cpu().numpy().view(np.uint64).reshape(-1, 4).copy()
        nt = oracle_threads()
        yn, dt_n = oracle_leg(lambda o: o.fft(x), nt)
        y1, dt_1 = oracle_leg(lambda o: o.fft(x), 1)
        lab = host_threads_label(nt)
        rec["cpu_baseline"] = {"value": round(n / dt_n, 1), "unit": "elements/s", "cores": nt, "kind": "port",
                               "sample": f"oracle/zk_oracle.c or_fft (iterative radix-2, ark-poly semantics), the same "
                                         f"2^{log_n} input on {lab['label']}, {dt_n:.2f} s",
                               "bit_exact_vs_gpu": bool(np.array_equal(yn, gpu_y) and np.array_equal(y1, gpu_y)),
                               "affinity_cpus": lab["affinity_cpus"], "host_cpus_visible": lab["host_cpus_visible"],
                               "single_thread": {"value": round(n / dt_1, 1), "unit": "elements/s", "cores": 1,
                                                 "sample": f"the full 2^{log_n} transform, 1 thread, {dt_1:.2f} s"}}
    del y
    return rec


# The driver keeps only the last ~8 KB of stdout, so the JSON line stays
# under LINE_BUDGET bytes: the full record (phase tables, notes, long sample
# descriptions) goes to a file named in the line (`details`), and the line
# keeps every number (values, rooflines, CPU legs, anchor and shard timings,
# bit-exactness flags).
LINE_BUDGET = 6000
VERBOSE_KEYS = ("phases_ms_total", "note", "timing", "cores_note", "kernel_timing", "event_timing", "api",
                "schedule", "oracle_reference", "label", "basis", "count", "parity", "bases", "phase_ms",
                "per_shard_ms")


def compact_line(rec, details_path):
    """Write the full record to details_path and return the compact line."""
    try:
        os.makedirs(os.path.dirname(details_path), exist_ok=True)
        with open(details_path, "w") as f:
            json.dump(rec, f, indent=1)
        where = os.path.relpath(details_path, ROOT)
    except OSError as e:
        where = f"(not written: {e})"

    def strip(o, depth=0):
        if isinstance(o, dict):
            return {k: strip(v, depth + 1) for k, v in o.items()
                    if k not in VERBOSE_KEYS and not (k == "sample" and isinstance(v, str) and len(v) > 90)}
        return o
    line = strip(rec)
    line["details"] = where
    # last resort: drop the least important sub-records (all still in the
    # details file) until the line fits
    for path in (("strong_scaling_anchor", "same_plan_c16", "serial_schedule"),
                 ("strong_scaling_anchor", "serial_schedule"), ("serial_schedule",),
                 ("strong_scaling_anchor", "roofline"), ("msm_g1", "plain"), ("msm_g1", "bits64"),
                 ("strong_scaling_anchor", "same_plan_c16"), ("ntt", "cpu_baseline"),
                 ("msm_g1", "cpu_baseline")):
        if len(json.dumps(line)) <= LINE_BUDGET:
            break
        holder = line
        for k in path[:-1]:
            holder = holder.get(k) if isinstance(holder, dict) else None
        if isinstance(holder, dict):
            holder.pop(path[-1], None)
    return line


def spawn_ranks(n):
    """`--gpus N` without torchrun: start the N ranks as fresh child processes
    (this process has not imported torch or the package and never touches a
    GPU), wait for them, and return the job's exit code -- the first non-zero
    rank code; ranks still running 60 s after a rank failed are killed (by
    their own PIDs)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for rank in range(n):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def forward(sig, _frame):
        for pr in procs:
            if pr.poll() is None:
                pr.send_signal(sig)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    t_fail = None
    while True:
        codes = [pr.poll() for pr in procs]
        if all(c is not None for c in codes):
            break
        if t_fail is None and any(c not in (None, 0) for c in codes):
            t_fail = time.time()
            log(f"[bench] a rank failed (exit codes {codes}); waiting 60 s for the others")
        if t_fail is not None and time.time() - t_fail > 60:
            for pr in procs:
                if pr.poll() is None:
                    pr.kill()
        time.sleep(0.2)
    bad = [c for c in codes if c != 0]
    if not bad:
        return 0
    return bad[0] if bad[0] > 0 else 128 - bad[0]


def probe(dist, fn):
    """Run fn() on every rank and agree on the outcome over the (gloo) control
    group: (result, None) if it succeeded everywhere, else (result or None,
    "rank k: <error>") of the first failing rank -- the same on every rank."""
    try:
        out, err = fn(), None
    except Exception as e:   # noqa: BLE001 -- reported, and every rank follows the same branch
        out, err = None, f"{type(e).__name__}: {e}"[:300]
    errs = [None] * dist.get_world_size()
    dist.all_gather_object(errs, err)
    bad = [(k, e) for k, e in enumerate(errs) if e]
    return out, (f"rank {bad[0][0]}: {bad[0][1]}" if bad else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="N > 1: strong = one 2^total-log-n circuit sharded (configs[4]); weak = 2^log-n per GPU")
    ap.add_argument("--total-log-n", type=int, default=24, help="N > 1 strong scaling: log2 constraints in total")
    ap.add_argument("--log-n", type=int, default=20, help="log2 constraints (N = 1), per GPU (N > 1 weak)")
    ap.add_argument("--cpu-log-n", type=int, default=17, help="single-thread CPU baseline sample size")
    ap.add_argument("--cpu-sample-log-n", type=int, default=22,
                    help="N > 1: size of the all-threads oracle sample on rank 0")
    ap.add_argument("--anchor-log-n", type=int, default=24,
                    help="N = 1: the strong-scaling anchor (the N > 1 lines' circuit on one GPU); 0 = skip")
    ap.add_argument("--shard-scaling", type=int, default=8,
                    help="N = 1: measure the anchor key's N shards one by one on this GPU (MSM scaling); <2 = skip")
    ap.add_argument("--details", default=os.path.join(ROOT, "profiles", "bench_details_last.json"),
                    help="rank 0 writes the full record (phase tables, notes) here; stdout gets the compact line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-msm", action="store_true", help="skip the configs[1] MSM and configs[2] NTT lines")
    ap.add_argument("--no-serial", action="store_true", help="skip the serial-schedule roofline proves")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the host-witness leg (profiling runs: only full-size prove launches)")
    ap.add_argument("--seed", type=int, default=DEFAULT_SEED)
    ap.add_argument("--schedule", type=int, choices=(0, 3), default=0,
                    help="prove stream schedule of the timed region (3: every kernel serial, for profilers)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if os.environ.get("ZK_BENCH_LAUNCH_ECHO"):   # CPU test of the launcher: no torch, no GPU
        sys.stdout.write(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                                      "MASTER_ADDR")}) + "\n")
        sys.stdout.flush()
        sys.exit(int(os.environ["ZK_BENCH_LAUNCH_ECHO"]) if os.environ.get("RANK") == "1" else 0)

    import torch
    zkp = importlib.import_module("zero-knowledge-proofs_amd")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # Rehearsal knobs (not the bench contract): ZK_BENCH_DIST_BACKEND=gloo and
    # ZK_BENCH_DEVICE=0 run N ranks on one GPU with CPU-side collectives only:
    # the distributed quotient's all-to-alls then go through the library's
    # host-staged exchange over the gloo group ("quotient":
    # "distributed-host") instead of RCCL.  ZK_BENCH_FAIL_RCCL=k makes rank
    # k's RCCL attach fail (tests of the fallback below).
    backend = os.environ.get("ZK_BENCH_DIST_BACKEND", "nccl")
    local = int(os.environ.get("ZK_BENCH_DEVICE", local))
    fail_rccl = int(os.environ.get("ZK_BENCH_FAIL_RCCL", "-1"))
    torch.cuda.set_device(local)
    dist = None
    coll_dev = "cpu"   # control-plane tensors (gloo)
    if world > 1:
        import torch.distributed as dist
        from datetime import timedelta
        dist.init_process_group("gloo", timeout=timedelta(seconds=900))

    ctx = zkp.Context(local)
    quotient_mode = "local"
    data_group, gather_mode = None, None
    if dist:
        quotient_mode, gather_mode = "replicated", "gloo"
        if backend == "nccl" or fail_rccl >= 0:
            # one RCCL communicator inside the library for the distributed
            # quotient (three all-to-alls per proof over xGMI); the unique id
            # travels over the control group.  If the attach fails on any
            # rank, every rank detaches and proves with the replicated
            # quotient, labelled as such.
            def attach():
                uid, err = None, None
                if rank == 0:
                    try:
                        uid = zkp.Context.rccl_unique_id()
                    except Exception as e:   # noqa: BLE001 -- broadcast, then raised on every rank
                        err = str(e)
                obj = [(uid, err)]
                dist.broadcast_object_list(obj, src=0)
                if obj[0][1]:
                    raise zkp.ExchangeError(f"rank 0 rccl_unique_id: {obj[0][1]}")
                if fail_rccl >= 0:   # rehearsal: rank fail_rccl fails, the others skip the attach
                    if rank == fail_rccl:
                        raise zkp.ExchangeError("ZK_BENCH_FAIL_RCCL: attach failure injected")
                    return
                ctx.attach_rccl(obj[0][0], rank, world)
            _, err = probe(dist, attach)
            if err:
                probe(dist, ctx.detach_exchange)   # every rank drops it, agreed on the control group
                quotient_mode = f"replicated (rccl: {err})"
                log(f"[bench] RCCL attach failed ({err}): replicated quotient")
            else:
                quotient_mode = "distributed-rccl"
        else:
            # the host-staged exchange gets a gloo group of its own: its abort
            # (a rank failing mid-quotient) destroys that group, never the
            # control group the fallback below is agreed on
            # (bounded timeout: a peer whose exchange aborted leaves this
            # rank's pending all-to-all to fail within it, not after the
            # control group's 900 s)
            ctx.attach_exchange(zkp.TorchExchange(dist.new_group(backend="gloo", timeout=timedelta(seconds=60))),
                                rank, world)
            quotient_mode = "distributed-host"
        if backend == "nccl":
            # the partials' all-gather over RCCL (a torch nccl group beside
            # the gloo control plane), gloo if that group does not come up
            def rccl_group():
                g = dist.new_group(backend="nccl")
                t = torch.zeros(world, dtype=torch.int64, device=f"cuda:{local}")
                dist.all_gather_into_tensor(t, torch.full((1,), rank, dtype=torch.int64, device=t.device), group=g)
                if t.cpu().tolist() != list(range(world)):
                    raise RuntimeError(f"rccl all-gather check failed: {t.cpu().tolist()}")
                return g
            data_group, err = probe(dist, rccl_group)
            if err:
                data_group, gather_mode = None, f"gloo (rccl: {err})"
                log(f"[bench] RCCL group failed ({err}): partials over gloo")
            else:
                gather_mode = "rccl"
    strong = world > 1 and args.scaling == "strong"
    if world == 1:
        n = 1 << args.log_n
    elif strong:
        n = 1 << args.total_log_n
    else:
        n = (1 << args.log_n) * world
    log_n_total = n.bit_length() - 1
    params, r, s = setup_params(args.seed)
    extra = {}
    if world == 1 and not args.no_msm:
        # configs[2] first, on a fresh context (after the prove's multi-GB key
        # allocations the same transform measured ~20 % slower)
        log("[bench] NTT 2^22 (configs[2])")
        extra["ntt"] = ntt_bench(zkp, ctx, 22, args.steps, args.warmup, args.seed + 31,
                                 cpu=not args.no_cpu_baseline)
    log(f"[bench] setup 2^{log_n_total}-constraint synthetic circuit on GPU (shard {rank}/{world})")
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    t0 = time.perf_counter()
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1, shard=rank, nshards=world)
    t_setup = time.perf_counter() - t0
    d_z = ctx.synthetic_witness(n, args.seed + 1)      # identical on every rank (same seed)
    zlen = 3 * n + 1
    log(f"[bench] setup {t_setup:.2f}s; witness ready ({zlen} vars)")

    def gather(part):
        """The ONE exchange of the MSM shards: every rank's 1.5 KB partials,
        all-gathered (RCCL when its group came up, else gloo)."""
        if data_group is not None:
            mine = torch.frombuffer(bytearray(part), dtype=torch.uint8).to(f"cuda:{local}")
            allp = torch.empty(world * len(part), dtype=torch.uint8, device=mine.device)
            dist.all_gather_into_tensor(allp, mine, group=data_group)
        else:
            mine = torch.frombuffer(bytearray(part), dtype=torch.uint8)
            allp = torch.empty(world * len(part), dtype=torch.uint8)
            dist.all_gather_into_tensor(allp, mine)
        b = allp.cpu().numpy().tobytes()
        return [b[k * len(part):(k + 1) * len(part)] for k in range(world)]

    def step():
        if world == 1:
            return zkp.Prover.prove_device(dpk, d_z.data_ptr(), zlen, 1, r, s)
        part = zkp.Prover.prove_partial(dpk, d_z.data_ptr(), zlen, 1, r, s)
        return zkp.Prover.combine(gather(part), r, s)

    if dist:
        # the first sharded proof, agreed: a distributed quotient that fails
        # on any rank (RCCL between real peers) -> every rank detaches and
        # carries on with the replicated quotient, labelled.
        # ZK_BENCH_FAIL_FIRST_PROOF=k (rehearsal): rank k's first distributed
        # proof fails after its 2nd all-to-all (test library fault hook)
        fail_first = int(os.environ.get("ZK_BENCH_FAIL_FIRST_PROOF", "-1"))
        if fail_first == rank and quotient_mode.startswith("distributed"):
            ctx.test_fault_after_exchange(2)
        _, err = probe(dist, lambda: zkp.Prover.prove_partial(dpk, d_z.data_ptr(), zlen, 1, r, s))
        if err and quotient_mode.startswith("distributed"):
            probe(dist, ctx.detach_exchange)
            quotient_mode = f"replicated ({quotient_mode.split('-')[1]}: first distributed proof failed: {err})"
            log(f"[bench] first distributed proof failed ({err}): replicated quotient")
            _, err = probe(dist, lambda: zkp.Prover.prove_partial(dpk, d_z.data_ptr(), zlen, 1, r, s))
        if err:
            raise SystemExit(f"sharded prove failed: {err}")
        if data_group is not None:
            _, err = probe(dist, lambda: gather(b"\0" * zkp.PARTIAL_BYTES))
            if err:
                data_group, gather_mode = None, f"gloo (rccl all-gather failed: {err})"

    ctx.set_schedule(args.schedule)
    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed region runs the product path as shipped: the phase profiler
    # (HIP events around every phase, ~0.07 ms per 2^20 proof:
    # profiles/r04_profiler_overhead.txt) is off here and on in the short
    # pass below, which supplies phases_ms_total
    t0 = time.perf_counter()
    for _ in range(args.steps):
        proof = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.profile(True)
    prof_steps = max(2, min(args.steps, 5))
    for _ in range(prof_steps):
        if step() != proof:
            raise SystemExit("profiled proof differs from the timed one")
    torch.cuda.synchronize()
    prof = ctx.profile_read()
    ctx.profile(False)
    if dist:
        dist.barrier()
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_step = elapsed / args.steps * 1e3
    value = n / (elapsed / args.steps)
    g1_pairs, g2_pairs = prove_msm_pairs(n)
    roofline = None

    if world > 1:
        # PCIe-inclusive sharded proof: every rank gets only ITS witness slice
        # (zk_groth16_witness_ranges) from host memory, the drop-in
        # prove(pk, witness) split across the ranks
        z_host = d_z.cpu().numpy().view(np.uint64)
        z_slice = dpk.witness_slice(z_host)

        def step_host():
            part = zkp.Prover.prove_partial_host(dpk, z_slice, zlen, 1, r, s)
            return zkp.Prover.combine(gather(part), r, s)
        step_host()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(3):
            ph = step_host()
        dist.barrier()
        t_pc = torch.tensor([(time.perf_counter() - t0) / 3, float(z_slice.nbytes)], dtype=torch.float64,
                            device=coll_dev)
        dist.all_reduce(t_pc, op=dist.ReduceOp.MAX)
        if ph != proof:
            raise SystemExit("host-slice sharded proof differs from the device-witness one")
        extra["pcie_inclusive"] = {"ms_per_step": round(float(t_pc[0]) * 1e3, 3),
                                   "value": round(n / float(t_pc[0]), 1), "unit": "constraints/s",
                                   "max_rank_witness_bytes": int(t_pc[1]), "witness_bytes": int(z_host.nbytes),
                                   "note": "zk_groth16_prove_partial_host: each rank uploads only its witness "
                                           "slice from host memory every proof"}
        # MSM kernels' own time per proof on every rank (serial schedule:
        # every kernel in order on one stream), max over ranks -> the MSM
        # throughput of this N apart from the quotient's all-to-alls; rank
        # 0's profile also gives the roofline of the dominant kernel
        if not args.no_serial:
            ctx.set_schedule(3)
            torch.cuda.synchronize()
            dist.barrier()
            ctx.profile(True)
            ks = max(2, args.steps // 2)
            t0 = time.perf_counter()
            for _ in range(ks):
                p3 = step()
            torch.cuda.synchronize()
            t_ser = (time.perf_counter() - t0) / ks
            serial_prof = ctx.profile_read()
            ctx.profile(False)
            ctx.set_schedule(args.schedule)
            if p3 != proof:
                raise SystemExit("serial-schedule sharded proof differs from the overlapped one")
            mx = torch.tensor([msm_kernel_ms(serial_prof) / ks, t_ser], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            msm_ms = float(mx[0])
            extra["msm_only"] = {"ms_per_step": round(msm_ms, 3),
                                 "pairs_per_s": round((g1_pairs + g2_pairs) / (msm_ms / 1e3), 1),
                                 "g1_pairs": g1_pairs, "g2_pairs": g2_pairs,
                                 "timing": "max over ranks of the HIP-event time of every MSM kernel (sort, "
                                           "accumulate, merge, bucket sums) per serial-schedule proof: the MSMs "
                                           "without the quotient and its all-to-alls"}
            extra["serial_schedule"] = {"ms_per_step": round(float(mx[1]) * 1e3, 3), "steps": ks}
            if rank == 0:
                roofline = roofline_from(serial_prof, log_n_total, overlapped=prof, nshards=world)
        def timed_alternative(option, value, default):
            """ms per step (max over ranks) of the same proof with one ctx
            option changed; the proof must not change"""
            ctx.set_option(option, value)
            step()
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                pa = step()
            torch.cuda.synchronize()
            dist.barrier()
            t_alt = torch.tensor([(time.perf_counter() - t0) / args.steps], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t_alt, op=dist.ReduceOp.MAX)
            ctx.set_option(option, default)
            if pa != proof:
                raise SystemExit(f"proof with option {option} = {value} differs from the default one")
            return {"ms_per_step": round(float(t_alt[0]) * 1e3, 3), "value": round(n / float(t_alt[0]), 1),
                    "unit": "constraints/s"}
        if quotient_mode.startswith("distributed"):
            # the replicated alternative on the same keys: every rank computes
            # the whole quotient (ZK_OPT_DIST_QUOTIENT 0), no all-to-all
            extra["quotient_replicated"] = dict(
                timed_alternative(zkp.ZK_OPT_DIST_QUOTIENT, 0, -1),
                note="same keys and witness, every rank computing the whole 2^%d quotient "
                     "(zk_ctx_set_option ZK_OPT_DIST_QUOTIENT 0) instead of the three all-to-alls; "
                     "the line's value is the distributed mode" % log_n_total)
            # the other order: the quotient and its all-to-alls first, the G2
            # and A+B1+IC MSMs after them (ZK_OPT_EXCHANGE_FIRST 1)
            extra["exchange_first"] = dict(
                timed_alternative(zkp.ZK_OPT_EXCHANGE_FIRST, 1, 0),
                note="same keys and witness, the G2 and A+B1+IC MSMs waiting for the distributed quotient "
                     "(zk_ctx_set_option ZK_OPT_EXCHANGE_FIRST 1) so that its all-to-alls never queue behind "
                     "a full-occupancy accumulate; the line's value is the default order (MSMs start with "
                     "the witness)")
        if not args.no_cpu_baseline:
            if rank == 0:
                log(f"[bench] CPU baseline: oracle 2^{args.cpu_sample_log_n} sample on rank 0")
                extra["cpu_baseline"] = cpu_sample_baseline(zkp, ctx, args.cpu_sample_log_n, params, r, s,
                                                            args.seed + 21)
            dist.barrier()

    if rank == 0 and world == 1:
        # the dominant kernel's own duration: the same proves, every kernel in
        # order on one stream (overlap would stretch its HIP-event span)
        serial_prof = None
        if not args.no_serial:
            ctx.set_schedule(3)
            torch.cuda.synchronize()
            ctx.profile(True)
            t0 = time.perf_counter()
            ks = max(3, args.steps // 2)
            for _ in range(ks):
                p3 = zkp.Prover.prove_device(dpk, d_z.data_ptr(), zlen, 1, r, s)
            torch.cuda.synchronize()
            t_ser = (time.perf_counter() - t0) / ks
            serial_prof = ctx.profile_read()
            ctx.profile(False)
            ctx.set_schedule(args.schedule)
            if p3 != proof:
                raise SystemExit("serial-schedule proof differs from the overlapped one")
            extra["serial_schedule"] = {"ms_per_step": round(t_ser * 1e3, 3), "steps": ks,
                                        "phases_ms_total": phase_table(serial_prof)}
        roofline = roofline_from(serial_prof or prof, log_n_total, overlapped=prof)
        # PCIe-inclusive rate (the drop-in zk_groth16_prove: witness crosses from host memory each proof)
        z_host = d_z.cpu().numpy().view(np.uint64)
        if not args.no_pcie:
            w = zkp.Witness(z_host, 1)
            zkp.Prover.prove(dpk, w, r=r, s=s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                pp = zkp.Prover.prove(dpk, w, r=r, s=s)
            torch.cuda.synchronize()
            t_pc = (time.perf_counter() - t0) / 3
            if pp != proof:
                raise SystemExit("host-witness proof differs from the device-witness one")
            extra["pcie_inclusive"] = {"ms_per_step": round(t_pc * 1e3, 3), "value": round(n / t_pc, 1),
                                       "unit": "constraints/s", "over_resident_ms": round(t_pc * 1e3 - ms_step, 3),
                                       "note": "zk_groth16_prove (the drop-in prove(pk, witness)): the 3n+1-element "
                                               "witness crosses PCIe from host memory every proof, in two parts, the "
                                               "first part's MSMs running while the second is copied (DESIGN.md 4.2)"}
        dpk.free()
        if not args.no_msm:
            log("[bench] G1 MSM 2^20 (configs[1])")
            extra["msm_g1"] = msm_g1_bench(zkp, ctx, 20, args.steps, args.warmup, args.seed + 11,
                                           cpu=not args.no_cpu_baseline)
        if not args.no_cpu_baseline:
            log(f"[bench] CPU baseline: oracle prove at 2^{log_n_total} on "
                f"{host_threads_label(oracle_threads())['label']}"
                f", 2^{args.cpu_log_n} on 1 thread")
            extra["cpu_baseline"] = cpu_baseline(zkp, ctx, n, params, r, s, z_host, proof, args.cpu_log_n,
                                                 args.seed + 21)
            extra["bit_exact_vs_oracle"] = extra["cpu_baseline"]["bit_exact_vs_gpu"]
        if args.anchor_log_n:
            log(f"[bench] strong-scaling anchor: 2^{args.anchor_log_n} prove on this GPU")
            torch.cuda.empty_cache()
            anc = anchor_bench(zkp, ctx, args.anchor_log_n, params, r, s, args.seed, args.steps, args.warmup)
            if args.anchor_log_n >= 24:
                # the same circuit with the N > 1 shards' window plan (c = 16,
                # 4 windows): MSM scaling at an equal plan
                torch.cuda.empty_cache()
                c16 = anchor_bench(zkp, ctx, args.anchor_log_n, params, r, s, args.seed, max(2, args.steps // 2),
                                   1, win_c=16)
                anc["same_plan_c16"] = {k: c16[k] for k in ("ms_per_step", "value", "msm_only", "window_bits",
                                                            "bit_exact_vs_oracle", "serial_schedule")}
            if args.shard_scaling > 1:
                # the N = shard_scaling run's per-rank MSM work, measured on
                # this GPU shard by shard (north_star's >= 6x MSM scaling)
                log(f"[bench] the 2^{args.anchor_log_n} key's {args.shard_scaling} shards, one at a time")
                torch.cuda.empty_cache()
                sh = shard_msm_bench(zkp, ctx, args.anchor_log_n, args.shard_scaling, params, r, s, args.seed,
                                     max(2, args.steps // 4), anc["msm_only"]["ms_per_step"], anc["proof_compressed"])
                anc[f"shard{args.shard_scaling}_msm_only"] = sh
                anc[f"msm_scaling_projected_{args.shard_scaling}"] = sh["msm_scaling_projected"]
                if "same_plan_c16" in anc:
                    # the same ratio at an equal window plan (c = 16 on both
                    # sides): what sharding itself costs, without the one-GPU
                    # anchor's c = 22 saving (3 windows instead of 4)
                    anc[f"msm_scaling_projected_{args.shard_scaling}_same_plan"] = round(
                        anc["same_plan_c16"]["msm_only"]["ms_per_step"] / sh["ms_per_step"], 3)
            extra["strong_scaling_anchor"] = anc
    if rank == 0:
        if world == 1:
            workload = f"groth16_prove_2^{log_n_total}"
        elif strong:
            workload = f"groth16_prove_2^{log_n_total}_sharded_{world}gpu"
        else:
            workload = f"groth16_prove_2^{args.log_n}_per_gpu"
        rec = {
            "metric": METRIC, "workload_metric": f"Groth16 prove constraints/sec at 2^{log_n_total} R1CS",
            "value": round(value, 1), "unit": "constraints/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": "u32", "data": "synthetic",
            "config": {"workload": workload, "circuit": "n x (x*y=z) (groth16-cli generate_crs)",
                       "field": "BLS12-381 Fq/Fr Montgomery, 32x32->64-bit limb products (radix 2^28/2^29)",
                       "constraints": n, "constraints_per_gpu": n // world, "num_public": 1,
                       "parallelism": (f"msm-shard{world}+quotient-a2a" if quotient_mode == "distributed-rccl"
                                       else f"msm-shard{world}" if world > 1 else "single-gpu"),
                       "quotient": quotient_mode, "setup_s": round(t_setup, 2),
                       **({"partials_gather": gather_mode,
                           "launcher": "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ else "bench.py"}
                          if world > 1 else {})},
            "msm_pairs_per_s": {"g1": round(g1_pairs / (ms_step / 1e3), 1), "g2": round(g2_pairs / (ms_step / 1e3), 1),
                                "total": round((g1_pairs + g2_pairs) / (ms_step / 1e3), 1),
                                "note": "scalar-point pairs of the reference's 5 MSMs per proof (G1 10n+6, G2 3n+3) "
                                        "/ whole-job time per proof"},
            "roofline": roofline,
            "phases_ms_total": phase_table(prof), "phases_proofs": prof_steps,
            "proof_compressed": proof.serialize_compressed().hex(),
            "build_id": zkp.build_id(),
        }
        rec.update(extra)
        rec.setdefault("cpu_baseline", None)
        proj = (rec["cpu_baseline"] or {}).get("all_affinity_cpus_projection")
        if proj:
            proj["gpu_over_projection"] = round(rec["value"] / proj["value"], 2)
        if world > 1 and log_n_total == 24 and args.seed == DEFAULT_SEED:
            rec["bit_exact_vs_oracle"] = rec["proof_compressed"] == ORACLE_2P24   # the pinned oracle proof
        line = compact_line(rec, args.details)
        sys.stdout.write(json.dumps(line) + "\n")   # one write: ranks share the launcher's stdout
        sys.stdout.flush()
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
