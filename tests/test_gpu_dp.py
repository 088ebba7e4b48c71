"""Data-parallel TransE-L1 (skge_amd.dp: one model over G ranks; SURVEY.md
8(e) configs 1-4) on the GPU.

Every rank scores its slice of each union batch, the records are
all-gathered, and every rank scatters + applies the whole batch, so the
replicas must equal -- BIT FOR BIT -- one GPU training on the union batches
(the two-launch device runner, and hence the pipelined runner, which equals it
bitwise; test_gpu_device_loop):
  * one process, no group (G = 1);
  * two ranks on one GPU over gloo (the all-gather staged through the host):
    both replicas, after 2 epochs, against the one-GPU run;
  * one rank under "nccl" (RCCL): the epoch, all-gathers included, captured
    in a CUDA graph and replayed.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(n_ent, n_rel, d, seed=11):
    import skge_amd as S
    np.random.seed(seed)
    m = S.TransE((n_ent, n_ent, n_rel), d)
    m.add_hyperparam("margin", 2.0)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
    return m, upd


def _result(m, upd, nviol):
    return {"E": m.E.data.cpu().numpy().copy(), "R": m.R.data.cpu().numpy().copy(),
            "pE": upd["E"].p2.cpu().numpy().copy(), "pR": upd["R"].p2.cpu().numpy().copy(),
            "nviol": int(nviol)}


def _one_gpu(trip, n_ent, n_rel, d, nb, epochs, seed, pipelined=False):
    from skge_amd.device import DeviceKG, EpochRunner
    m, upd = _model(n_ent, n_rel, d)
    r = EpochRunner(m, upd, DeviceKG(trip, m.device), nbatches=nb, seed=seed, pipelined=pipelined)
    r.run(epochs)
    r.synchronize()
    return _result(m, upd, r.nviol_total.item())


def _dp(trip, n_ent, n_rel, d, nb, epochs, seed, group=None, capture=None):
    from skge_amd.device import DeviceKG
    from skge_amd.dp import DataParallelRunner
    m, upd = _model(n_ent, n_rel, d)
    r = DataParallelRunner(m, upd, DeviceKG(trip, m.device), nb, seed=seed, group=group,
                           capture=capture)
    r.run(epochs)
    r.synchronize()
    for acc in (r.accE, r.accR):
        assert int(acc.cnt.abs().sum().item()) == 0
    out = _result(m, upd, r.total_violations())
    out["graph"] = r.graph is not None
    return out


def _same(a, b):
    assert a["nviol"] == b["nviol"] > 0
    for k in ("E", "R", "pE", "pR"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb", [
    (500, 7, 3001, 200, 7),         # ragged remainder batch
    (40, 3, 1200, 52, 4),           # tiny graph: rows shared by most positives
    (2000, 11, 8000, 512, 20),      # config-5 width
    (40943, 18, 141442, 200, 50),   # WN18, 2 x 1414 positives per union batch
])
def test_dp_one_process_bitwise_equals_one_gpu_runner(n_ent, n_rel, T, d, nb):
    from test_gpu_device_loop import make_kg
    trip, _ = make_kg(n_ent, n_rel, T)
    want = _one_gpu(trip, n_ent, n_rel, d, nb, 2, 5)
    got = _dp(trip, n_ent, n_rel, d, nb, 2, 5)
    assert got["graph"]                      # captured epoch (no process group)
    _same(got, want)
    pipe = _one_gpu(trip, n_ent, n_rel, d, nb, 2, 5, pipelined=True)
    _same(pipe, want)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb", [
    (500, 7, 3001, 50, 7),          # the reference's d = 50 (BASELINE configs[0])
    (300, 5, 2000, 13, 5),          # odd width
])
def test_dp_padded_width_bitwise_equals_padded_pipelined(n_ent, n_rel, T, d, nb):
    """d % 4 != 0: the data-parallel runner works on zero-padded tables like
    the one-GPU pipelined runner, so the two train bit for bit alike."""
    from test_gpu_device_loop import make_kg
    trip, _ = make_kg(n_ent, n_rel, T)
    want = _one_gpu(trip, n_ent, n_rel, d, nb, 2, 5, pipelined=True)
    got = _dp(trip, n_ent, n_rel, d, nb, 2, 5)
    assert got["E"].shape[1] == d
    _same(got, want)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, backend, args, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank))
    for p in (ROOT, os.path.join(ROOT, "scikit-kge_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from test_gpu_device_loop import make_kg
    torch.cuda.set_device(0)
    dist.init_process_group(backend, init_method="env://")
    n_ent, n_rel, T, d, nb, epochs, seed = args
    trip, _ = make_kg(n_ent, n_rel, T)
    res = _dp(trip, n_ent, n_rel, d, nb, epochs, seed)
    dist.barrier()
    dist.destroy_process_group()
    out.put((rank, res))


def _spawn(world, backend, args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, args, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=150) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [r[1] for r in res]


@pytest.mark.parametrize("world,args", [(2, (500, 7, 3001, 200, 7, 2, 5)),      # ragged: last slice short
                                        (2, (40943, 18, 14140, 200, 5, 2, 9)),  # WN18 rows, 2828 / batch
                                        (3, (500, 7, 3001, 200, 7, 2, 5)),      # slices of unequal size
                                        (4, (40943, 18, 14140, 200, 5, 2, 9))])
def test_dp_ranks_on_one_gpu_gloo_bitwise(world, args):
    """world ranks (processes) sharing one GPU, the exchange over gloo: every
    rank's tables bit for bit the one-GPU pipelined runner's (the N > 1
    protocol -- slices, in-place record gather, remote scatter -- rehearsed
    where only one GPU is available)."""
    from test_gpu_device_loop import make_kg
    n_ent, n_rel, T, d, nb, epochs, seed = args
    got = _spawn(world, "gloo", args)
    trip, _ = make_kg(n_ent, n_rel, T)
    want = _one_gpu(trip, n_ent, n_rel, d, nb, epochs, seed)
    assert not any(g["graph"] for g in got)     # gloo: eager
    for g in got:
        _same(g, want)


def test_dp_one_rank_nccl_captured_all_gather():
    from test_gpu_device_loop import make_kg
    args = (500, 7, 3001, 200, 7, 3, 5)
    got = _spawn(1, "nccl", args)[0]
    assert got["graph"]
    n_ent, n_rel, T, d, nb, epochs, seed = args
    trip, _ = make_kg(n_ent, n_rel, T)
    _same(got, _one_gpu(trip, n_ent, n_rel, d, nb, epochs, seed))
