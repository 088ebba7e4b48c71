"""Row-sharded TransE-L1 step on the GPU (skge_amd.shard, csrc/skge_shard.hip).

* the HIP routing equals the NumPy layout of tests/shard_numpy.py exactly;
* one rank (G = 1): the sharded runner trains, bit for bit, like the
  two-launch device runner (same epoch draws, exact packed sums, same apply);
* one sharded batch against the oracle replaying its recorded pairs (1e-5);
* two ranks on one GPU over gloo: the assembled entity table after a batch is
  the oracle's union-batch step (1e-5) and the relation replicas agree bit
  for bit.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import parity_util
from oracle import skge_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("G,count,start", [(1, 37, 0), (2, 1000, 3), (3, 257, 10), (8, 4096, 0),
                                           (5, 1, 0), (2, 0, 0)])
def test_route_matches_numpy_layout(G, count, start):
    from skge_amd import _lib as L
    from shard_numpy import random_records, route
    rec, rec_n1 = random_records(np.random.RandomState(G + count), 5000, 997, 9, skip=0.2)
    dev = torch.device("cuda", 0)
    r = torch.as_tensor(rec, device=dev)
    r1 = torch.as_tensor(rec_n1, device=dev)
    n = max(4 * count, 1)
    ids = torch.full((n,), -9, dtype=torch.int32, device=dev)
    pos = torch.full((n,), -9, dtype=torch.int32, device=dev)
    counts = torch.full((G,), -9, dtype=torch.int64, device=dev)
    wsb = int(L.lib().skge_shard_route_workspace_bytes(count, G))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    L.check(L.lib().skge_shard_route(L.stream_ptr(), L.ptr(r), L.ptr(r1), start, count, G,
                                     L.ptr(ids), L.ptr(pos), L.ptr(counts), L.ptr(ws), wsb))
    want_ids, want_pos, want_counts = route(rec, rec_n1, start, count, G)
    c = counts.cpu().numpy()
    assert c.tolist() == want_counts.tolist()
    nsend = int(c.sum())
    assert np.array_equal(ids.cpu().numpy()[:nsend], want_ids)
    assert np.array_equal(pos.cpu().numpy()[:4 * count], want_pos)


@pytest.mark.parametrize("G,count,start,C", [(1, 37, 0, 148), (2, 1000, 3, 2100), (3, 257, 10, 400),
                                             (8, 4096, 0, 2200), (2, 0, 0, 8)])
def test_route_cap_matches_numpy_layout(G, count, start, C):
    from skge_amd import _lib as L
    from shard_numpy import random_records, route_cap
    rec, rec_n1 = random_records(np.random.RandomState(G + count), 5000, 997, 9, skip=0.2)
    dev = torch.device("cuda", 0)
    r = torch.as_tensor(rec, device=dev)
    r1 = torch.as_tensor(rec_n1, device=dev)
    ids = torch.full((G * C,), -9, dtype=torch.int32, device=dev)
    pos = torch.full((max(4 * count, 1),), -9, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    wsb = int(L.lib().skge_shard_route_workspace_bytes(count, G))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    L.check(L.lib().skge_shard_route_cap(L.stream_ptr(), L.ptr(r), L.ptr(r1), start, count, G, C,
                                         L.ptr(ids), L.ptr(pos), L.ptr(ws), wsb, L.ptr(err)))
    want_ids, want_pos = route_cap(rec, rec_n1, start, count, G, C)
    assert int(err.item()) == 0
    assert np.array_equal(ids.cpu().numpy(), want_ids)
    assert np.array_equal(pos.cpu().numpy()[:4 * count], want_pos)


def test_sharded_runner_captured_epochs_equal_eager():
    """The fixed-capacity epoch captured in one graph (no host read per batch)
    trains bit for bit like the same epochs issued eagerly."""
    from skge_amd.shard import ShardedRunner
    from test_gpu_device_loop import make_kg
    n_ent, n_rel, d = 700, 6, 128
    trip, _ = make_kg(n_ent, n_rel, 4000)
    E, R = _init_tables(n_ent, n_rel, d, 3)
    out = []
    for cap in (True, False):
        dev = torch.device("cuda", 0)
        r = ShardedRunner(n_ent, torch.as_tensor(E, device=dev), torch.as_tensor(R, device=dev),
                          torch.as_tensor(trip, device=dev), 9, seed=4, capture=cap)
        r.run(3)
        r.synchronize()
        assert (r.graph is not None) == cap
        out.append((int(r.nviol_total.item()), r.E.data.cpu().numpy(), r.R.data.cpu().numpy()))
    assert out[0][0] == out[1][0] > 0
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


def test_sharded_bucket_overflow_is_reported():
    from skge_amd import _lib as L
    from skge_amd.shard import ShardedRunner
    from test_gpu_device_loop import make_kg
    trip, _ = make_kg(300, 5, 2000)
    E, R = _init_tables(300, 5, 32, 1)
    dev = torch.device("cuda", 0)
    r = ShardedRunner(300, torch.as_tensor(E, device=dev), torch.as_tensor(R, device=dev),
                      torch.as_tensor(trip, device=dev), 8, seed=5, capacity=64)
    # the contribution records live inside a guarded allocation: a record
    # written for a dropped request (slot -1) would land in the front guard
    C = r.bufs["contrib"]
    guard = 4096
    big = torch.full((C.numel() + 2 * guard,), 0xA5, dtype=torch.uint8, device=dev)
    r.bufs["contrib"] = big[guard:guard + C.numel()].view(C.shape)
    r.run(1)
    with pytest.raises(L.SkgeError, match="overflowed"):
        r.synchronize()
    torch.cuda.synchronize()
    g = big.cpu().numpy()
    assert (g[:guard] == 0xA5).all() and (g[-guard:] == 0xA5).all()
    # a skipped positive adds nothing anywhere: tables finite, sums drained
    assert torch.isfinite(r.E.data).all() and torch.isfinite(r.R.data).all()
    for acc in (r.accE, r.accR):
        assert int(acc.cnt.abs().sum().item()) == 0


def _init_tables(n_ent, n_rel, d, seed):
    rs = np.random.RandomState(seed)
    E = rs.uniform(-0.3, 0.3, size=(n_ent, d))
    E /= np.sqrt((E ** 2).sum(axis=1))[:, None]
    R = rs.uniform(-0.3, 0.3, size=(n_rel, d))
    return E.astype(np.float32), R.astype(np.float32)


@pytest.mark.parametrize("n_ent,n_rel,T,d,nb", [
    (500, 7, 3001, 200, 7),     # ragged remainder batch
    (40, 3, 1200, 52, 4),       # tiny graph: every row in every batch
    (2000, 11, 8000, 512, 20),  # config-5 width
])
def test_single_rank_bitwise_equals_device_runner(n_ent, n_rel, T, d, nb):
    from test_gpu_device_loop import _runner_result
    from skge_amd.shard import ShardedRunner
    a, trip = _runner_result(n_ent, n_rel, T, d, nb, pipelined=False, seed=11)
    import skge_amd as S
    np.random.seed(11)
    m = S.TransE((n_ent, n_ent, n_rel), d)   # the same initial tables as _runner_result
    dev = m.device
    r = ShardedRunner(n_ent, m.E.data.clone(), m.R.data.clone(), torch.as_tensor(trip, device=dev),
                      nb, lr=0.1, margin=2.0, seed=11)
    r.run(2)
    r.synchronize()
    assert int(r.epoch_key.item()) == 2
    assert int(r.nviol_total.item()) == a["nviol"] > 0
    assert np.array_equal(r.E.data.cpu().numpy(), a["E"])
    assert np.array_equal(r.R.data.cpu().numpy(), a["R"])
    assert np.array_equal(r.updE.p2.cpu().numpy(), a["pE"])
    assert np.array_equal(r.updR.p2.cpu().numpy(), a["pR"])
    for acc in (r.accE, r.accR):
        assert int(acc.cnt.abs().sum().item()) == 0
        assert float(acc.sum.abs().sum().item()) == 0.0


def _oracle_union(E, R, recs, batches, lr=0.1, margin=2.0):
    from shard_numpy import union_pairs
    params = {"E": E.astype(np.float64), "R": R.astype(np.float64)}
    state = {k: np.zeros_like(v) for k, v in params.items()}
    nv = 0
    for start, count in batches:
        pos, neg = union_pairs([(rec, rec_n1, start, count) for rec, rec_n1 in recs])
        nv += O.pairwise_step("transe", params, state, pos, neg, lr, margin, "adagrad", l1=True)[2]
    return params, state, nv


@pytest.mark.parametrize("d", [200, 512])      # 512: the config-5 width
def test_single_rank_batches_match_oracle(d):
    from skge_amd.shard import ShardedRunner
    from test_gpu_device_loop import make_kg
    n_ent, n_rel = 300, 5
    trip, _ = make_kg(n_ent, n_rel, 2000)
    E, R = _init_tables(n_ent, n_rel, d, 1)
    dev = torch.device("cuda", 0)
    r = ShardedRunner(n_ent, torch.as_tensor(E, device=dev), torch.as_tensor(R, device=dev),
                      torch.as_tensor(trip, device=dev), 8, seed=5)
    r.sample_epoch()
    batches = [(0, 250), (250, 250)]
    for b in batches:
        r.step(*b)
    r.fold_violations()
    r.synchronize()
    params, state, nv = _oracle_union(E, R, [(r.rec.cpu().numpy(), r.rec_n1.cpu().numpy())],
                                      batches)
    assert int(r.nviol_total.item()) == nv > 0
    parity_util.check(r.E.data, params["E"], "shard d%d E" % d, lr=0.1, p2=state["E"])
    parity_util.check(r.R.data, params["R"], "shard d%d R" % d, lr=0.1, p2=state["R"])
    parity_util.check(r.updE.p2, state["E"], "shard d%d p2 E" % d)
    parity_util.check(r.updR.p2, state["R"], "shard d%d p2 R" % d)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


N2, M2, T2 = 400, 6, 3000
BATCHES2 = [(0, 300), (300, 300)]


def _two_rank_worker(rank, world, port, out, D2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank))
    for p in (ROOT, os.path.join(ROOT, "scikit-kge_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from skge_amd.shard import ShardedRunner
    from test_gpu_device_loop import make_kg
    dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    trip, _ = make_kg(N2, M2, T2, seed=4)
    E, R = _init_tables(N2, M2, D2, 2)
    r = ShardedRunner(N2, torch.as_tensor(E[rank::world], device=dev),
                      torch.as_tensor(R, device=dev),
                      torch.as_tensor(trip[rank::world], device=dev), 5, seed=20 + rank)
    r.sample_epoch()
    for b in BATCHES2:
        r.step(*b)
    r.fold_violations()
    r.synchronize()
    full = r.gather_full_E().cpu().numpy()
    out.put((rank, r.rec.cpu().numpy(), r.rec_n1.cpu().numpy(), full,
             r.R.data.cpu().numpy(), int(r.nviol_total.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("D2", [128, 512])     # 512: the config-5 width
def test_two_ranks_on_one_gpu_match_union_oracle(D2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, q, D2)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=100) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    E, R = _init_tables(N2, M2, D2, 2)
    params, state, nv = _oracle_union(E, R, [(x[1], x[2]) for x in res], BATCHES2)
    assert res[0][5] + res[1][5] == nv > 0
    assert np.array_equal(res[0][3], res[1][3])          # both ranks assembled the same table
    assert np.array_equal(res[0][4], res[1][4])          # relation replicas identical
    parity_util.check(res[0][3], params["E"], "shard 2 ranks d%d E" % D2, lr=0.1, p2=state["E"])
    parity_util.check(res[0][4], params["R"], "shard 2 ranks d%d R" % D2, lr=0.1, p2=state["R"])


def test_config5_rows_past_2_31_elements_match_oracle():
    """Config 5's row range (|E| = 50M at d = 512 puts row r at element offset
    r * 512, past 2^31 from row 4,194,304 on): a d = 512 table of 4.3M rows
    (8.8 GB, and as much again for its AdaGrad state) whose positives use only
    rows >= 4,194,304 as s and o (the corruptions are uniform over all rows).
    Two batches of 4096 positives through the sharded step at G = 1, compared
    on every touched row and its AdaGrad state with oracle.pairwise_step on
    the gathered sub-table; the single-GPU device runners (pipelined and
    two-launch) must reproduce the sharded step bit for bit on the whole
    table (the G = 1 identity test_single_rank_bitwise_equals_device_runner
    checks at small sizes)."""
    import skge_amd as S
    from skge_amd.shard import ShardedRunner
    from skge_amd.device import DeviceKG, EpochRunner
    from shard_numpy import union_pairs
    N, M, d, B = 4_300_000, 16, 512, 4096
    LO = 1 << 22                     # first row whose element offset r * 512 reaches 2^31
    assert LO * d == 1 << 31 and N > LO
    dev = torch.device("cuda", 0)
    rs = np.random.RandomState(17)
    keys = set()
    while len(keys) < 2 * B:
        s, o, p = (int(x) for x in (rs.randint(LO, N), rs.randint(LO, N), rs.randint(M)))
        keys.add((s, o, p))
    trip = np.array(sorted(keys), dtype=np.int32)
    rs.shuffle(trip)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    E0 = torch.empty((N, d), dtype=torch.float32, device=dev)
    E0.uniform_(-0.08, 0.08, generator=g)
    for r0 in range(0, N, 1 << 20):
        blk = E0[r0:r0 + (1 << 20)]
        blk.div_(blk.norm(dim=1, keepdim=True))
    R0 = torch.empty((M, d), dtype=torch.float32, device=dev)
    R0.uniform_(-0.1, 0.1, generator=g)
    seed = 23
    # ---- the sharded step at G = 1, two batches, replayed by the oracle ----
    r = ShardedRunner(N, E0.clone(), R0.clone(), torch.as_tensor(trip, device=dev), 2, seed=seed)
    r.sample_epoch()
    torch.cuda.synchronize()
    rec, rec_n1 = r.rec.cpu().numpy(), r.rec_n1.cpu().numpy()
    ids = np.concatenate([rec[:, 0], rec[:, 1], rec[:, 3], rec_n1])
    rows = np.unique(ids[ids >= 0])
    assert rows[-1] >= LO and (rec[:, :2] >= LO).all()
    for b in range(2):
        r.step(b * B, B)
    r.fold_violations()
    r.synchronize()
    sub = torch.as_tensor(rows, device=dev, dtype=torch.int64)
    E_sh, p2_sh = r.E.data[sub].cpu().numpy(), r.updE.p2[sub].cpu().numpy()
    R_sh, pR_sh = r.R.data.cpu().numpy(), r.updR.p2.cpu().numpy()
    nv_sh = int(r.nviol_total.item())
    full_sh = (r.E.data.clone(), r.updE.p2.clone())
    del r
    remap = lambda x: np.where(x[:, :2] >= 0, np.searchsorted(rows, x[:, :2]), x[:, :2])
    params = {"E": E0[sub].cpu().numpy().astype(np.float64), "R": R0.cpu().numpy().astype(np.float64)}
    state = {k: np.zeros_like(v) for k, v in params.items()}
    nv = 0
    for b in range(2):
        pos, neg = union_pairs([(rec, rec_n1, b * B, B)])
        pos[:, :2], neg[:, :2] = remap(pos), remap(neg)
        nv += O.pairwise_step("transe", params, state, pos, neg, 0.1, 2.0, "adagrad", l1=True)[2]
    assert nv_sh == nv > 0
    parity_util.check(E_sh, params["E"], "c5 rows>2^31 E", lr=0.1, p2=state["E"])
    parity_util.check(p2_sh, state["E"], "c5 rows>2^31 p2 E")
    parity_util.check(R_sh, params["R"], "c5 rows>2^31 R", lr=0.1, p2=state["R"])
    parity_util.check(pR_sh, state["R"], "c5 rows>2^31 p2 R")
    # ---- the single-GPU device runners: one epoch = the same two batches ----
    kg = DeviceKG(trip, dev)
    for pipelined in (None, False):
        m = S.TransE((N, N, M), d, init="device_nunif")
        m.add_hyperparam("margin", 2.0)
        m.E.data.copy_(E0)
        m.R.data.copy_(R0)
        upd = {pid: S.AdaGrad(p, 0.1) for pid, p in m.params.items()}
        er = EpochRunner(m, upd, kg, nbatches=2, seed=seed, pipelined=pipelined)
        er.run(1)
        er.synchronize()
        torch.cuda.synchronize()
        assert int(er.nviol_total.item()) == nv, (pipelined, er.pipelined)
        assert torch.equal(m.E.data, full_sh[0]), (pipelined, er.pipelined)
        assert torch.equal(upd["E"].p2, full_sh[1]), (pipelined, er.pipelined)
        assert np.array_equal(m.R.data.cpu().numpy(), R_sh)
        del er, m, upd
        torch.cuda.empty_cache()
