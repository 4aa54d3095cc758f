"""bench.py's N > 1 path (the configs[4] strong-scaling line) rehearsed on ONE
GPU: two torchrun ranks on device 0 with gloo collectives
(ZK_BENCH_DIST_BACKEND=gloo ZK_BENCH_DEVICE=0).  RCCL refuses two ranks on
one device, so the distributed quotient's three all-to-alls run through the
library's host-staged exchange over the gloo group ("quotient":
"distributed-host") -- the same stages and index maps as over RCCL.  The
folded proof of the sharded run must equal the single-GPU proof of the same
circuit, key parameters, witness and r, s byte for byte, and the
PCIe-inclusive leg must send each rank only its ~1/N witness slice."""
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


@pytest.mark.timeout(300)
def test_bench_two_rank_path_matches_single_gpu(ctx, zkp):
    log_n, seed = 12, 0x5EED0001
    env = dict(os.environ, ZK_BENCH_DIST_BACKEND="gloo", ZK_BENCH_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--total-log-n", str(log_n), "--seed", str(seed), "--cpu-sample-log-n", "10"]
    res = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert res.returncode == 0, res.stderr[-3000:]
    line = [ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong"
    assert rec["config"]["constraints"] == 1 << log_n and rec["config"]["quotient"] == "distributed-host"
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
    sys.path.insert(0, ROOT)
    import bench
    params, r, s = bench.setup_params(seed)
    n = 1 << log_n
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(n))
    dpk = zkp.CRS.generate_device(ctx, qap, zkp.SetupParams(*params), 1)
    z = ctx.synthetic_witness(n, seed + 1)
    proof = zkp.Prover.prove_device(dpk, z.data_ptr(), 3 * n + 1, 1, r, s)
    dpk.free()
    assert rec["proof_compressed"] == proof.serialize_compressed().hex()
