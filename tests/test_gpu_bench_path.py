"""bench.py's N > 1 path (the configs[4] strong-scaling line) rehearsed on ONE
GPU: two ranks on device 0 -- started by torchrun, or by bench.py itself
when no launcher set WORLD_SIZE -- with gloo collectives
(ZK_BENCH_DIST_BACKEND=gloo ZK_BENCH_DEVICE=0).  RCCL refuses two ranks on
one device, so the distributed quotient's three all-to-alls run through the
library's host-staged exchange over the gloo group ("quotient":
"distributed-host") -- the same stages and index maps as over RCCL.  The
folded proof of the sharded run must equal the single-GPU proof of the same
circuit, key parameters, witness and r, s byte for byte, and the
PCIe-inclusive leg must send each rank only its ~1/N witness slice.  A
forced RCCL attach failure on one rank must still give a line, with the
replicated quotient and the same proof."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


LOG_N, SEED = 12, 0x5EED0001
ARGS = ["--gpus", "2", "--steps", "1", "--warmup", "0", "--total-log-n", str(LOG_N), "--seed", str(SEED),
        "--cpu-sample-log-n", "10"]


def _run(launcher, **env_extra):
    env = dict(os.environ, ZK_BENCH_DIST_BACKEND="gloo", ZK_BENCH_DEVICE="0", **env_extra)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py")]
    else:   # bench.py starts its own two rank processes
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")]
    res = subprocess.run(cmd + ARGS, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-3000:]      # rank 0 only
    return json.loads(lines[0])


def _single_gpu_proof(ctx, zkp):
    sys.path.insert(0, ROOT)
    import bench
    params, r, s = bench.setup_params(SEED)
    n = 1 << LOG_N
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    z = ctx.synthetic_witness(n, SEED + 1)
    proof = zkp.Prover.prove_device(dpk, z.data_ptr(), 3 * n + 1, 1, r, s)
    dpk.free()
    return proof.serialize_compressed().hex()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("launcher", ["torchrun", "bench.py"])
def test_bench_two_rank_path_matches_single_gpu(ctx, zkp, launcher):
    log_n = LOG_N
    rec = _run(launcher)
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong"
    assert rec["config"]["constraints"] == 1 << log_n and rec["config"]["quotient"] == "distributed-host"
    assert rec["config"]["launcher"] == launcher and rec["config"]["partials_gather"] == "gloo"
    pc = rec["pcie_inclusive"]
    assert pc["max_rank_witness_bytes"] <= pc["witness_bytes"] // 2 + 64
    # the fields that make the driver's 1 -> 8 GPU run readable as a curve
    # (DESIGN.md 5): the MSMs' own time, the dominant kernel's roofline, the
    # replicated-quotient alternative on the same keys, a CPU baseline
    mo = rec["msm_only"]
    assert 0 < mo["ms_per_step"] <= rec["serial_schedule"]["ms_per_step"]
    assert mo["pairs_per_s"] > 0 and mo["g1_pairs"] == 10 * (1 << log_n) + 6
    roof = rec["roofline"]
    assert roof["kernel"] == "k_msm_accum<G1>" and 0 < roof["frac"] < 1 and roof["avg_launch_ms"] > 0
    assert rec["quotient_replicated"]["ms_per_step"] > 0
    assert rec["exchange_first"]["ms_per_step"] > 0
    cb = rec["cpu_baseline"]
    assert cb["value"] > 0 and cb["bit_exact_vs_gpu"] and cb["cores"] >= 1
    proj = cb["all_affinity_cpus_projection"]
    assert proj["cpus"] >= 1 and proj["value"] > 0 and proj["gpu_over_projection"] > 0
    assert rec["proof_compressed"] == _single_gpu_proof(ctx, zkp)


@pytest.mark.timeout(300)
def test_bench_rccl_attach_failure_falls_back_to_replicated(ctx, zkp):
    """ZK_BENCH_FAIL_RCCL=1: rank 1's RCCL attach fails.  Every rank learns
    it through the control-group agreement, detaches, and the line still
    comes out -- labelled "replicated (rccl: ...)", with the same proof."""
    rec = _run("bench.py", ZK_BENCH_FAIL_RCCL="1")
    q = rec["config"]["quotient"]
    assert q.startswith("replicated (rccl: rank 1: ExchangeError") and "injected" in q, q
    assert rec["config"]["parallelism"] == "msm-shard2"
    assert "quotient_replicated" not in rec and rec["msm_only"]["ms_per_step"] > 0
    assert rec["proof_compressed"] == _single_gpu_proof(ctx, zkp)


@pytest.mark.timeout(300)
def test_bench_first_distributed_proof_failure_falls_back(ctx, zkp):
    """ZK_BENCH_FAIL_FIRST_PROOF=1 (gloo, host-staged exchange): rank 1's
    first distributed proof fails after its 2nd all-to-all, and its abort
    tears down the exchange's OWN gloo group.  The control group survives,
    so every rank agrees, detaches (without calling the abort hook again)
    and carries on with the replicated quotient: the line still comes out,
    labelled, with the same proof."""
    rec = _run("bench.py", ZK_BENCH_FAIL_FIRST_PROOF="1")
    q = rec["config"]["quotient"]
    assert q.startswith("replicated (host: first distributed proof failed: rank"), q
    assert "quotient_replicated" not in rec and rec["msm_only"]["ms_per_step"] > 0
    assert rec["proof_compressed"] == _single_gpu_proof(ctx, zkp)
