"""The data-parallel epoch's protocol (skge_amd.dp.dp_epoch: per union batch
one launch applies the previous batch and scores this rank's slice, adding
its contributions locally; the slices' records are all-gathered and the
other ranks' positives added; the flush applies the last batch) over
world-size 2 and 3 gloo jobs
on CPU, with the NumPy rank compute of tests/dp_numpy.py.  After every batch
each rank's replica must equal ONE process's reference step
(oracle.pairwise_step: skge/transe.py:48-165 + AdaGrad + normalize) over the
union batch, and the replicas must be identical.  A 30-entity graph makes
rows shared across the ranks' slices; ragged batches leave the last rank's
slice short or empty."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_ENT, N_REL, D, T = 30, 4, 8, 40
MARGIN, LR = 2.0, 0.1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _problem():
    rs = np.random.RandomState(11)
    E = rs.uniform(-0.5, 0.5, size=(N_ENT, D))
    E /= np.sqrt((E ** 2).sum(axis=1))[:, None]
    R = rs.uniform(-0.5, 0.5, size=(N_REL, D))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from shard_numpy import random_records
    rec, rec_n1 = random_records(np.random.RandomState(5), T, N_ENT, N_REL)
    return E, R, rec, rec_n1


def _worker(rank, world, port, batches, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank))
    for p in (ROOT, os.path.join(ROOT, "scikit-kge_amd"), os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from skge_amd.dp import DPExchange, dp_epoch
    from dp_numpy import NumpyDPOps
    dist.init_process_group("gloo", init_method="env://")
    E, R, rec, rec_n1 = _problem()
    ops = NumpyDPOps(rec, rec_n1, E, R, MARGIN, LR)
    ex = DPExchange()
    dp_epoch(ops, ex, batches)
    snaps = ops.snaps               # the tables after every union batch's apply
    dist.barrier()
    dist.destroy_process_group()
    out.put((rank, snaps, ops.nviol))


def _run(world, batches):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batches, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,batches", [(2, [(0, 40)]), (2, [(0, 13), (13, 13), (26, 13), (39, 1)]),
                                           (3, [(0, 20), (20, 20)]), (3, [(0, 2), (2, 38)])])
def test_dp_protocol_matches_union_batch(world, batches):
    from oracle import skge_oracle as O
    from shard_numpy import union_pairs
    res = _run(world, batches)
    assert all(len(r[1]) == len(batches) for r in res)
    E, R, rec, rec_n1 = _problem()
    params = {"E": E.copy(), "R": R.copy()}
    state = {k: np.zeros_like(v) for k, v in params.items()}
    nviol = 0
    for b, (start, count) in enumerate(batches):
        pos, neg = union_pairs([(rec, rec_n1, start, count)])
        nviol += O.pairwise_step("transe", params, state, pos, neg, LR, MARGIN, "adagrad",
                                 l1=True)[2]
        for rank, snaps, _ in res:
            np.testing.assert_allclose(snaps[b][0], params["E"], rtol=0, atol=1e-12)
            np.testing.assert_allclose(snaps[b][1], params["R"], rtol=0, atol=1e-12)
            np.testing.assert_allclose(snaps[b][2], state["E"], rtol=0, atol=1e-12)
            # identical replicas on every rank
            assert np.array_equal(snaps[b][0], res[0][1][b][0])
            assert np.array_equal(snaps[b][1], res[0][1][b][1])
    assert nviol > 0
    assert sum(r[2] for r in res) == nviol     # every pair scored by exactly one rank


def test_slices_partition_every_batch():
    from skge_amd.dp import slice_of
    for count in (0, 1, 2, 7, 1414, 11312):
        for G in (1, 2, 3, 8):
            got = [slice_of(count, G, g)[1:] for g in range(G)]
            covered = [w for lo, hi in got for w in range(lo, hi)]
            assert covered == list(range(count))
            share = slice_of(count, G, 0)[0]
            assert all(lo == min(g * share, count) for g, (lo, _) in enumerate(got))
