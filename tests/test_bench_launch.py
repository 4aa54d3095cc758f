"""bench.py's N > 1 plumbing on CPU (no GPU, no torch in the launcher):

  * `python bench.py --gpus N` without torchrun starts N fresh rank processes
    itself, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR set
    (ZK_BENCH_LAUNCH_ECHO: the ranks print their environment and stop before
    importing torch), and the job's exit code is the failing rank's;
  * `probe` (the agreement behind the RCCL fallback) gives every rank of a
    gloo world-2 group the same verdict when one rank fails."""
import json
import os
import socket
import subprocess
import sys

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(n, echo):
    env = dict(os.environ, ZK_BENCH_LAUNCH_ECHO=str(echo))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)], env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=120)


def test_bench_starts_its_own_ranks():
    res = _launch(4, 0)
    assert res.returncode == 0, res.stderr[-2000:]
    recs = sorted((json.loads(ln) for ln in res.stdout.splitlines() if ln.startswith("{")), key=lambda d: d["RANK"])
    assert [d["RANK"] for d in recs] == ["0", "1", "2", "3"]
    assert all(d["WORLD_SIZE"] == "4" and d["LOCAL_RANK"] == d["RANK"] and d["MASTER_ADDR"] == "127.0.0.1"
               for d in recs)


def test_bench_launcher_returns_a_failing_rank_code():
    res = _launch(2, 7)          # rank 1 exits 7
    assert res.returncode == 7, (res.returncode, res.stderr[-2000:])


def _probe_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def fn():
        if rank == 1:
            raise RuntimeError("attach refused")
        return rank * 10
    val, err = bench.probe(dist, fn)
    ok_val, ok_err = bench.probe(dist, lambda: rank)
    with open(os.path.join(out, f"{rank}.json"), "w") as f:
        json.dump({"val": val, "err": err, "ok_val": ok_val, "ok_err": ok_err}, f)
    dist.destroy_process_group()


def test_probe_agrees_on_one_rank_failing(tmp_path):
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    mp.spawn(_probe_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (json.load(open(tmp_path / f"{k}.json")) for k in range(2))
    assert r0["err"] == r1["err"] == "rank 1: RuntimeError: attach refused"
    assert r0["val"] == 0 and r1["val"] is None
    assert r0["ok_err"] is None and r1["ok_err"] is None and (r0["ok_val"], r1["ok_val"]) == (0, 1)
