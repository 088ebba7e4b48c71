"""bench.py's multi-GPU bookkeeping on CPU: a world-size-2 gloo job checks the
rank environment, the max-over-ranks timing and the whole-job value; the
`--gpus N --dry-run` launcher runs the N > 1 line's data-parallel protocol
(skge_amd.dp.dp_epoch with the NumPy rank compute over gloo) and must print ONE
line shaped like the one-model DP line (parallelism dpN, strong scaling,
identical replicas).  The protocol's numerics: tests/test_dp_protocol.py."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", init_method="env://")
    w, r, lr = bench.dist_env()
    elapsed = 1.0 + rank   # rank 1 is the slow replica
    mx = bench.max_over_ranks(elapsed, w, "cpu")
    val = bench.replica_value(1000, w, mx)
    dist.barrier()
    dist.destroy_process_group()
    out.put((r, w, lr, mx, val))


def test_replica_bookkeeping_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r, w, lr) for r, w, lr, _, _ in res] == [(0, 2, 0), (1, 2, 1)]
    for _, _, _, mx, val in res:
        assert mx == 2.0                      # the slowest replica's time on every rank
        assert val == pytest.approx(1000.0)   # 2 ranks x 1000 positives / 2 s


def test_single_process_defaults(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert bench.dist_env() == (1, 0, 0)
    assert bench.max_over_ranks(3.5, 1) == 3.5
    assert bench.replica_value(10, 1, 2.0) == 5.0


def _bench_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    """`bench.py --gpus N` outside torchrun starts N ranks itself (CPU dry mode:
    gloo, no GPU) and rank 0 alone prints one line with n_gpus == N."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--dry-run", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _bench_lines(r.stdout)
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == n and line["dry_run"] is True
    assert sorted(line["detail"]["ranks"]) == list(range(n))
    assert line["steps"] == 3 and line["value"] > 0
    # the N > 1 line is ONE model trained data parallel, not N replicas
    assert line["config"]["parallelism"] == "dp%d" % n
    assert line["scaling"] == "strong" and line["cpu_baseline"] is None
    assert line["detail"]["dp"]["replicas_identical"] is True
    assert "ONE TransE-L1" in line["config"]["workload"]


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--dry-run"], capture_output=True, text=True, timeout=120, env=env,
                       cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
