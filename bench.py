#!/usr/bin/env python3
"""Throughput benchmark: WN18-shaped TransE-L1 d=200 PairwiseStochasticTrainer
+ AdaGrad on MI355X (BASELINE.json configs[1]).

One STEP = one training epoch over the synthetic WN18-shaped KG
(|E|=40943, |R|=18, T=141,442 unique uniform triples, RandomState(0)) at the
reference's geometry nb=100 (100 batches of 1,414 positives + one of 42),
each positive with its two RandomModeSampler negatives (mode 0 corrupts s,
mode 1 corrupts o), margin 2.0, lr 0.1 -- run by the native hipGraph epoch
runner (device permutation, device sampler, fused score+scatter, fused
mean+AdaGrad+normalize).  value = positive triples fully processed per second.

Multi-GPU: one process per GPU.  `--gpus N` without a torchrun environment
starts the N ranks itself (torch.distributed.run as a child process, before
anything touches a GPU); under torchrun it checks WORLD_SIZE == N.  Configs
1-2 at N > 1 (default `--mode auto` = dp): the line is ONE TransE model
trained data parallel over the N GPUs on the same KG (skge_amd.dp: every rank
scores its slice of each union batch of the reference's 1414 positives, RCCL
all-gather of the records, replicated scatter + apply; strong scaling).  At
this batch the per-batch all-gather and the replicated apply bound it, so it
is expected at or below one GPU and reported as such.
The union batch N x 1414 (with the one-GPU runner at that batch) and N
independent replicas ("independent jobs": N models on N KGs, no exchange)
are measured into `detail` only.  `--mode replicas` prints the independent
jobs as the line, named so in the metric.  Config 5 at N > 1: the
row-sharded table (`--shard`, RCCL all-to-all + reduce-scatter of
contributions).  Any multi-rank measurement that raises or does not finish
within SKGE_BENCH_DP_TIMEOUT seconds ends the job with a non-zero status
(after rank 0 has printed its line, the failure marked in it).
`--dry-run`: the launcher, rendezvous, the data-parallel protocol
(skge_amd.dp.dp_epoch with a NumPy rank compute, gloo) and the
max-over-ranks bookkeeping on CPU, no GPU (tests/test_bench_dist.py).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--nb 100]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "scikit-kge_amd"))
sys.path.insert(0, ROOT)

N_ENT, N_REL, N_TRIPLES = 40943, 18, 141442
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def make_wn18_kg(n_ent=N_ENT, n_rel=N_REL, n_triples=N_TRIPLES, seed=0):
    """Unique uniform (s, o, p) triples, RandomState(seed)."""
    rs = np.random.RandomState(seed)
    out = np.empty((0, 3), dtype=np.int64)
    while len(out) < n_triples:
        m = (n_triples - len(out)) * 2 + 1024
        cand = np.stack([rs.randint(n_ent, size=m), rs.randint(n_ent, size=m),
                         rs.randint(n_rel, size=m)], axis=1)
        allt = np.concatenate([out, cand])
        key = (allt[:, 0] * n_ent + allt[:, 1]) * n_rel + allt[:, 2]
        _, first = np.unique(key, return_index=True)
        out = allt[np.sort(first)][:n_triples]
    return out.astype(np.int32)


def make_zipf_kg(n_ent=N_ENT, n_rel=N_REL, n_triples=N_TRIPLES, alpha=1.1, seed=0):
    """SURVEY 8(d)'s skew variant: entity ids Zipf(alpha) - 1, truncated to
    [0, n_ent) by redrawing (clipping would pile ~1/3 of the draws onto one
    id), relations uniform; unique (s, o, p), RandomState(seed).  At WN18's N
    and alpha 1.1 entity 0 is ~14% of the s / o draws: hot rows, duplicate
    slots and pending-row hand-offs in nearly every scoring wave."""
    rs = np.random.RandomState(seed)

    def ids(m):
        x = np.empty(0, dtype=np.int64)
        while len(x) < m:
            z = rs.zipf(alpha, size=2 * (m - len(x)) + 64) - 1
            x = np.concatenate([x, z[z < n_ent]])
        return x[:m]
    out = np.empty((0, 3), dtype=np.int64)
    while len(out) < n_triples:
        m = (n_triples - len(out)) * 2 + 1024
        cand = np.stack([ids(m), ids(m), rs.randint(n_rel, size=m)], axis=1)
        allt = np.concatenate([out, cand])
        key = (allt[:, 0] * n_ent + allt[:, 1]) * n_rel + allt[:, 2]
        _, first = np.unique(key, return_index=True)
        out = allt[np.sort(first)][:n_triples]
    return out.astype(np.int32)


def bench_kg(args, seed):
    """The WN18-shaped KG of configs 1-4: uniform, or Zipf-skewed (--skew zipf)."""
    if getattr(args, "skew", "none") == "zipf":
        return make_zipf_kg(seed=seed)
    return make_wn18_kg(seed=seed)


def kg_label(args, seed_txt):
    if getattr(args, "skew", "none") == "zipf":
        return ("synthetic WN18-shaped KG (|E|=40943 |R|=18 T=141442, entity ids Zipf(1.1) "
                "truncated, %s)" % seed_txt)
    return "synthetic WN18-shaped KG (|E|=40943 |R|=18 T=141442 uniform, %s)" % seed_txt


# The round whose committed PMC summaries a line may quote: only the same
# round's (a line never cites an older kernel's traffic; without this round's
# summary, traffic is null)
PMC_ROUND = "r06"


def _round_files(fname):
    f = os.path.join(ROOT, "profiles", PMC_ROUND, fname)
    return [f] if os.path.exists(f) else []


def pmc_traffic(kernel_substr, fname="pmc.json"):
    """Per-launch HBM-side traffic of a kernel from this round's committed
    rocprofv3 PMC summary (profiles/<PMC_ROUND>/<fname>, made by
    `tools/gpu_run.sh pmc` + tools/pmc_summary.py; pmc.json for the default
    line, pmc_c<k>.json for config k): 2*FETCH_SIZE + WRITE_SIZE per the
    gfx950 correction in MI355X_MICROARCH.md "HBM"."""
    for f in _round_files(fname):
        data = json.load(open(f))
        for name, e in data.items():
            if kernel_substr in name and "traffic_bytes_per_launch" in e:
                grids = [g for g in e.get("by_grid", {}).values()
                         if "traffic_bytes_per_launch" in g]
                if grids:   # the geometry launched most (the timed epochs, not the detail lines)
                    g = max(grids, key=lambda x: x["calls"])
                    return g["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
                return e["traffic_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def pmc_traffic_epochs(kernel_substr, fname, first, count):
    """Config 5: a kernel's per-launch traffic averaged over the SAME epochs
    the line times (first .. first+count-1; epoch 0 = the warm-up), from the
    round's committed per-epoch PMC summary (tools/pmc_epochs.py)."""
    for f in _round_files(fname):
        data = json.load(open(f))
        for name, eps in data.items():
            if kernel_substr in name:
                sel = [e for e in eps if first <= e["epoch"] < first + count]
                if len(sel) == count:
                    return (sum(e["traffic_bytes_per_launch"] for e in sel) / count,
                            "%s epochs %d..%d" % (os.path.relpath(f, ROOT), first, first + count - 1))
    return None, None


def dist_env():
    """(world, rank, local_rank) from the torchrun environment (1, 0, 0 alone)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def free_port():
    import socket
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` outside torchrun: run this script as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) in a
    CHILD process -- this parent never touches a GPU (no exec from a process
    that has) -- forward its output and return its exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def acc_label(acc):
    """Encoding of an accumulator's sums."""
    from skge_amd import _lib as L
    return {L.SKGE_ACC_F32: "fp32", L.SKGE_ACC_I16X4: "int16x4 exact",
            L.SKGE_ACC_I32X2: "int32x2 exact", L.SKGE_ACC_FX64: "fixed-point int64 exact",
            L.SKGE_ACC_I8X4: "int8x4 exact"}[int(acc.mode)]


def run_dry(args):
    """--dry-run: the multi-rank bookkeeping without a GPU -- rendezvous over
    gloo, the data-parallel protocol of the N > 1 line (skge_amd.dp.dp_epoch:
    apply + slice scoring, all-gather, remote scatter) with the float64 NumPy rank
    compute of tests/dp_numpy.py on a small KG, barrier-bracketed timing, max
    over ranks and ONE line from rank 0 with the DP line's shape (not a
    measurement: "dry_run": true)."""
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from dp_numpy import NumpyDPOps
    from shard_numpy import random_records
    from skge_amd.dp import DPExchange, dp_epoch
    world, rank, _ = dist_env()
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    n_ent, n_rel, d, T, nb = 200, 6, 8, 400, 4
    rs = np.random.RandomState(0)          # ONE model: the same problem on every rank
    E = rs.uniform(-0.5, 0.5, size=(n_ent, d))
    E /= np.sqrt((E ** 2).sum(axis=1))[:, None]
    R = rs.uniform(-0.5, 0.5, size=(n_rel, d))
    rec, rec_n1 = random_records(np.random.RandomState(5), T, n_ent, n_rel)
    ops = NumpyDPOps(rec, rec_n1, E, R, 2.0, 0.1)
    ex = DPExchange()
    bs = T // nb
    batches = [(s0, min(bs, T - s0)) for s0 in range(0, T, bs)]
    for _ in range(args.warmup):
        dp_epoch(ops, ex, batches)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dp_epoch(ops, ex, batches)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, world)
    ranks, cks = [rank], [float(ops.E.sum())]
    if world > 1:
        out = [None] * world
        dist.all_gather_object(out, (rank, float(ops.E.sum())))
        ranks, cks = [r for r, _ in out], [c for _, c in out]
    if rank == 0:
        m = {"value": round(T * args.steps / elapsed, 1),
             "ms_per_step": round(1000.0 * elapsed / args.steps, 4), "union_batch": bs, "nb": nb,
             "per_gpu_batch": -(-bs // world), "replicas_identical": len(set(cks)) == 1}
        line = dp_line(args, world, m, None, d=d, nb=nb, workload_kg="dry-run KG (|E|=%d |R|=%d "
                       "T=%d), float64 NumPy rank compute (tests/dp_numpy.py)" % (n_ent, n_rel, T))
        line.update(metric="dry-run (launcher and DP-protocol bookkeeping, no GPU)", dry_run=True,
                    unit="triples/s")
        line["detail"] = {"ranks": ranks, "dp": m, "backend": "gloo"}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def setup_ranks():
    """(world, rank, local, device) of this process: the process group
    (RCCL, i.e. "nccl"; SKGE_BENCH_BACKEND=gloo for a rehearsal) and its GPU.
    SKGE_BENCH_ONE_GPU=1 puts every rank on GPU 0 (a multi-rank rehearsal on a
    one-GPU box; RCCL refuses two ranks on one GPU, so pair it with gloo)."""
    import torch
    import torch.distributed as dist
    world, rank, local = dist_env()
    if world > 1:
        dist.init_process_group(os.environ.get("SKGE_BENCH_BACKEND", "nccl"),
                                init_method="env://")
    if os.environ.get("SKGE_BENCH_ONE_GPU") == "1":
        local = 0
    torch.cuda.set_device(local)
    return world, rank, local, torch.device("cuda", local)


def rank_setup_info(world, local):
    """What the job ran on, for the line: the backend, the number of distinct
    GPUs the ranks used (max over ranks of local index + 1 on one node) and
    whether it is a one-GPU rehearsal (SKGE_BENCH_ONE_GPU=1: every rank on GPU
    0, so its numbers are not a scaling point)."""
    import torch.distributed as dist
    backend = dist.get_backend() if world > 1 else None
    devices = int(max_over_ranks(local + 1, world, coll_device("cuda"))) if world > 1 else 1
    return {"backend": backend, "distinct_gpus": devices,
            "rehearsal_one_gpu": os.environ.get("SKGE_BENCH_ONE_GPU") == "1"}


def parallelism_label(base, info):
    """base (e.g. 'dp2'), marked when every rank shared one GPU."""
    return base + ("-on-1gpu-rehearsal" if info.get("rehearsal_one_gpu") else "")


def coll_device(device):
    """Where a bookkeeping collective's tensor lives: the GPU under RCCL, the
    host under gloo."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "gloo":
        return "cpu"
    return device


def max_over_ranks(x, world, device="cpu"):
    """The maximum of a per-rank float over all ranks (the timed region's
    wall clock: the job is done when the slowest replica is)."""
    if world <= 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def replica_value(positives_per_rank, world, elapsed_max):
    """Whole-job throughput of N independent replicas (weak scaling): every
    rank's positives over the slowest rank's time."""
    return world * positives_per_rank / elapsed_max


def handoff_probe(dev, rounds=2000, reps=3):
    """skge_handoff_probe: the pipelined runner's publish / wait hand-off (16-B
    write-through payload, drain, write-through flag; sc1 poll + re-read)
    ping-ponged between two workgroups.  Reported in the line's detail so a
    slow box's hand-off chain is visible in the record itself (the headline
    launch is a chain of such hops).  Best of `reps` runs, us per hop."""
    import torch
    from skge_amd import _lib as L
    lib = L.lib()
    buf = torch.zeros(256, dtype=torch.int32, device=dev)
    out = torch.zeros(3, dtype=torch.int64, device=dev)
    best, bad, gave_up = None, 0, 0
    for _ in range(reps):
        L.check(lib.skge_handoff_probe(L.stream_ptr(), L.ptr(buf), rounds, L.ptr(out)),
                "handoff probe")
        torch.cuda.synchronize()
        ticks, b, g = (int(x) for x in out.tolist())
        us_hop = ticks * 0.01 / (2 * rounds)
        best = us_hop if best is None else min(best, us_hop)
        bad += b
        gave_up |= g
    return {"us_per_hop": round(best, 4), "us_per_round_trip": round(2 * best, 4),
            "rounds": rounds, "payload_mismatches": bad, "wait_gave_up": bool(gave_up),
            "form": "16-B sc1 payload + vmcnt(0) + sc1 flag; sc1 poll + s_sleep(2), sc1 re-read; "
                    "blocks 0/1 (round-robin: different XCDs), idle chip, best of %d" % reps}


def algorithmic_bytes(d, B, P, U_E, U_R, opt_k=12):
    """BYTES(batch) = 4d(3B + P) + k d (U_E + U_R) + 20B."""
    return 4 * d * (3 * B + P) + opt_k * d * (U_E + U_R) + 20 * B


# The reference's own pure-NumPy path, measured in the survey container
# (BASELINE.md table "CPU reference, measured in the survey container":
# positive triples/s, 8-vCPU Xeon, effectively one thread); it cannot travel to
# the GPU box, so lines carry it beside their own timed oracle sample
REFERENCE_CPU = {
    ("transe", 200, "adagrad"): (21600.0, "score+grad+update only (BASELINE.md config 2)"),
    ("transe", 50, "sgd"): (44300.0, "end-to-end incl. the Python sampler; no score-only "
                                     "figure (BASELINE.md config 1)"),
    ("transe", 50, "adagrad"): (36500.0, "end-to-end incl. the Python sampler (BASELINE.md "
                                         "config 1')"),
    ("hole", 200, "adagrad"): (6300.0, "score+grad+update only (BASELINE.md config 3)"),
    ("rescal", 200, "adagrad"): (6490.0, "score+grad+update only, 5 batches (BASELINE.md "
                                         "config 4)"),
    ("transe", 512, "adagrad"): (5600.0, "score+grad+update only, |E|=1M scaled-down table "
                                         "(BASELINE.md config 5)"),
}


def reference_cpu(model, d, opt):
    """The reference's own figure for this workload (None if the survey did
    not measure one)."""
    v = REFERENCE_CPU.get((model, d, opt))
    if v is None:
        return None
    return {"value": v[0], "unit": "triples/s", "cores": 1, "kind": "reference",
            "measured": "survey container (8-vCPU Xeon, numpy 2.2.6), not this box: the "
                        "reference cannot travel to the GPU box",
            "what": v[1], "source": "BASELINE.md"}


def cpu_baseline(trip, d, nb, seconds=12.0, model="transe", margin=2.0, opt="adagrad"):
    """The oracle (fp64 NumPy restatement, oracle/skge_oracle.py) on a bounded
    sample of the same workload: consecutive nb=100 batches of epoch 1,
    negatives from the reference-semantics host sampler (not timed)."""
    from oracle import skge_oracle as O
    rs = np.random.RandomState(42)
    np.random.seed(42)

    def nunif(rows, cols):
        bnd = np.sqrt(6) / np.sqrt(rows + cols)
        return rs.uniform(-bnd, bnd, size=(rows, cols))

    if model == "transe":
        params = {"E": O.normalize(nunif(N_ENT, d), None), "R": nunif(N_REL, d)}
    elif model == "hole":
        params = {"E": O.normless1(nunif(N_ENT, d), None), "R": nunif(N_REL, d)}
    else:
        params = {"E": nunif(N_ENT, d), "W": np.array([nunif(d, d) for _ in range(N_REL)])}
    state = {k: np.zeros_like(v) for k, v in params.items()}
    tset = set(map(tuple, trip.tolist()))
    idx = np.arange(len(trip))
    np.random.shuffle(idx)
    bounds = O.batch_bounds(len(trip), nb)
    t_step = 0.0
    t_all = 0.0
    npos = 0
    nb_done = 0
    for (a, b) in bounds:
        t0 = time.perf_counter()
        pairs = O.random_mode_sample(trip[idx[a:b]], tset, (N_ENT, N_ENT, N_REL))
        pos = np.array([p for p, _ in pairs])
        neg = np.array([n for _, n in pairs])
        t1 = time.perf_counter()
        O.pairwise_step(model, params, state, pos, neg, 0.1, margin, opt, l1=True)
        t2 = time.perf_counter()
        t_step += t2 - t1
        t_all += t2 - t0
        npos += b - a
        nb_done += 1
        if t_all > seconds:
            break
    return {"value": npos / t_step, "unit": "triples/s", "cores": 1, "kind": "port",
            "sample": "%d nb=%d batches (%d positives) of epoch 1, WN18-shaped KG, %s "
                      "d=%d %s margin %g; oracle/skge_oracle.py fp64 NumPy, 1 thread; "
                      "score+grad+update only (host sampler untimed)"
                      % (nb_done, nb, npos, {"transe": "TransE-L1", "hole": "HolE",
                                             "rescal": "RESCAL"}[model], d,
                         {"adagrad": "AdaGrad", "sgd": "SGD"}[opt], margin),
            "e2e_value": npos / t_all,
            "reference": reference_cpu(model, d, opt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed epochs")
    ap.add_argument("--warmup", type=int, default=3, help="untimed epochs")
    ap.add_argument("--nb", type=int, default=100, help="nbatches (reference geometry)")
    ap.add_argument("--d", type=int, default=200)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--skew", choices=("none", "zipf"), default="none",
                    help="configs 1-4: entity ids Zipf(1.1) instead of uniform (SURVEY 8(d)'s "
                         "skew variant: hot rows, duplicate slots)")
    ap.add_argument("--opt", choices=["adagrad", "sgd"], default=None,
                    help="updater (default: AdaGrad; config 1: SGD)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--acc", choices=["auto", "f32"], default="auto",
                    help="accumulator encoding (auto: exact packed int16x4 for TransE-L1)")
    ap.add_argument("--reps", type=int, default=1, help="relation accumulator copies")
    ap.add_argument("--large-nb", type=int, default=2,
                    help="also time this nbatches (large-batch detail line); 0 = skip")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="1: WN18 TransE d=50 SGD (BASELINE configs[0], the reference CLI's "
                         "run_transe.py shape); "
                         "2: WN18 TransE d=200 (the headline); 3: WN18 HolE d=200; 4: WN18 "
                         "RESCAL d=200 (pairwise, device pair loop); 5: synthetic |E|=50M "
                         "|R|=10k d=512, B=131072 per GPU (BASELINE.json configs[4])")
    ap.add_argument("--c5-scale", type=float, default=1.0,
                    help="config 5 only: scale |E| and T (quick rehearsals)")
    ap.add_argument("--c5-no-counter-split", action="store_true",
                    help="config 5 only: skip the extra epoch that prices the update counters")
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the measured gather roofline (skge_roofline_gather)")
    ap.add_argument("--runner", default="auto", choices=["auto", "pairs", "hole_pipe"],
                    help="configs 3/4: device runner (auto: HolE pipelined where it applies)")
    ap.add_argument("--mode", choices=["auto", "replicas", "dp"], default="auto",
                    help="configs 1/2 on N > 1 GPUs: 'dp' (= auto, the default: the line is ONE "
                         "model trained data parallel; independent replicas in detail) or "
                         "'replicas' (the line is N independent jobs, named so in the metric)")
    ap.add_argument("--dp-batch", choices=["per-gpu", "global"], default="global",
                    help="--mode dp: 'global' (default) keeps the union batch at the reference's "
                         "1414 (1414 / N per GPU: strong scaling); 'per-gpu' keeps 1414 per GPU "
                         "(union batch N x 1414, nb = nb / N: a larger batch, weak scaling)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: the multi-rank launcher and bookkeeping over gloo")
    ap.add_argument("--shard", action="store_true",
                    help="config 5 only: row-shard E and its AdaGrad state over the ranks "
                         "(skge_amd.shard; RCCL all-to-all row fetch + contribution "
                         "reduce-scatter, relation sums all-reduced) instead of replicas")
    args = ap.parse_args()
    if args.config == 1:
        # BASELINE configs[0]: TransE on WN18, ncomp=50, nb=100, margin 2.0, SGD
        # (run_transe_wn18.sh:3-5 / run_transe.py; the reference CLI itself
        # passes no param_update, i.e. AdaGrad: --opt adagrad times that)
        args.d = 50
        if args.opt is None:
            args.opt = "sgd"
    if args.opt is None:
        args.opt = "adagrad"
    world = dist_env()[0]
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (launch N ranks with --gpus N)"
                         % (args.gpus, world))
    if args.dry_run:
        return run_dry(args)
    if args.config == 5 and (args.shard or (world > 1 and args.mode != "replicas")):
        return run_config5_sharded(args)     # N > 1: one model, the table row-sharded
    if args.config == 5:
        return run_config5(args)
    if args.config in (3, 4):
        return run_config34(args)
    if world > 1 and args.mode != "replicas":
        return run_dp(args)                  # N > 1: one model, data parallel

    import torch
    import torch.distributed as dist
    world, rank, local, dev = setup_ranks()
    info = rank_setup_info(world, local)

    import skge_amd as S
    from skge_amd import _lib as L
    from skge_amd.device import DeviceKG, EpochRunner

    d, nb = args.d, args.nb
    trip = bench_kg(args, rank)           # replica r trains on its own KG
    np.random.seed(42 + rank)
    model = S.TransE((N_ENT, N_ENT, N_REL), d, l1=True)
    model.add_hyperparam("margin", 2.0)
    Upd = S.SGD if args.opt == "sgd" else S.AdaGrad
    upd = {pid: Upd(p, 0.1) for pid, p in model.params.items()}
    kg = DeviceKG(trip, dev)
    runner = EpochRunner(model, upd, kg, nbatches=nb, seed=1234 + rank,
                         force_f32=args.acc == "f32", replicas=args.reps)
    st = runner.stream
    init = {pid: p.data.clone() for pid, p in model.params.items()}

    # warmup (graph replays), then restore the initial parameters so the timed
    # epochs are epochs 1..K of a fresh training run (the busiest: most violations)
    runner.run(args.warmup)
    runner.synchronize()
    for pid, p in model.params.items():
        p.data.copy_(init[pid])
        upd[pid].reset()
    runner.nviol_total.zero_()
    torch.cuda.synchronize()

    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(st)
    runner.run(args.steps)
    ev1.record(st)
    runner.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    gpu_ms = ev0.elapsed_time(ev1)
    elapsed = max_over_ranks(elapsed, world, dev)
    nviol = int(runner.nviol_total.item())
    positives = N_TRIPLES * args.steps
    value = replica_value(positives, world, elapsed)
    rank_value = positives / (t1 - t0)      # this replica alone

    # ---- per-kernel timing (HIP events on the runner stream, eager launches of
    # one more epoch, outside the timed region) for the roofline.  The tables
    # are rolled back to the initial state first, so the profiled epoch does
    # the same work as the timed region's first epoch ----
    for pid, p in model.params.items():
        p.data.copy_(init[pid])
        upd[pid].reset()
    torch.cuda.synchronize()
    opt_k = 4 if args.opt == "sgd" else 12     # k = 4 (SGD) / 12 (AdaGrad)
    prof = pipe_profile(runner, kg, nb, d, epochs=args.steps,
                        gpu_ms_per_epoch=gpu_ms / args.steps, opt_k=opt_k) if runner.pipelined else \
        kernel_profile(model, upd, kg, nb, d, st, runner, opt_k=opt_k)
    meas = None
    if runner.pipelined and not args.no_roofline:
        # the same per-launch row traffic without the path's
        # dependencies, and the streaming random-row gather rate of the table
        geo = prof["geometry"]
        npos = int(round(geo["positives"]))
        # d % 4 != 0: the runner moves its zero-padded rows (quad layout)
        dr = runner.d_pad if getattr(runner, "_pad", False) else d
        m_us, m_b, m_gbs = measured_roofline(dev, N_ENT, dr, npos, 5,
                                             int(round(geo["atomic_rows"] / max(npos, 1))),
                                             int(round(geo["applied_rows"])))
        s_us, s_b, s_gbs = measured_roofline(dev, N_ENT, dr, 262144, 5, 0, 0, launches=10, reps=3)
        h_us, h_b, h_gbs = measured_roofline(dev, 5_000_000, dr, 262144, 5, 0, 0, launches=10,
                                             reps=3)
        sg = s_gbs
        meas = {"kernel": "k_roofline (skge_roofline_gather)",
                "frac_of_streaming_gather": round(prof["dominant"]["achieved_gbs"] / sg, 4),
                "geometry": "per launch: %d waves x 5 random %d-B row gathers + %d atomic rows "
                            "each, %d rows read+written (20d B), WN18 table"
                            % (npos, 4 * dr, int(round(geo["atomic_rows"] / max(npos, 1))),
                               int(round(geo["applied_rows"]))),
                "avg_launch_us": round(m_us, 3), "bytes_per_launch": round(m_b),
                "GB_s": round(m_gbs, 1),
                "frac_of_same_geometry_kernel":
                    round(prof["dominant"].get("impl_gbs", prof["dominant"]["achieved_gbs"])
                          / m_gbs, 4),
                "frac_note": "implementation bytes / the same bytes moved by a same-geometry "
                             "kernel without dependencies (itself latency-bound: not a roofline)",
                "streaming_gather_GB_s": {"wn18_table_33MB": round(s_gbs, 1),
                                          "table_4GB": round(h_gbs, 1)}}

    # ---- detail: the same path at a large batch ("throughput at
    # nb=100 and at a stated larger batch"), not the headline value ----
    large = None
    if args.large_nb and args.large_nb != nb and world == 1:
        for pid, p in model.params.items():
            p.data.copy_(init[pid])
            upd[pid].reset()
        r2 = EpochRunner(model, upd, kg, nbatches=args.large_nb, seed=4321,
                         force_f32=args.acc == "f32", replicas=args.reps)
        r2.run(1)
        r2.synchronize()
        # the headline's protocol: epochs 1..K of a fresh run (K = --steps; the
        # work per epoch falls as training proceeds, so the first-5 figure of
        # rounds 3-4 is kept beside it, from the same timed epochs)
        e2 = max(5, args.steps)
        for pid, p in model.params.items():   # the timed and profiled epochs start fresh
            p.data.copy_(init[pid])
            upd[pid].reset()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        f0, f5, f1 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        f0.record(r2.stream)
        r2.run(5)
        f5.record(r2.stream)
        r2.run(e2 - 5)
        f1.record(r2.stream)
        r2.synchronize()
        t2 = time.perf_counter() - t2
        for pid, p in model.params.items():
            p.data.copy_(init[pid])
            upd[pid].reset()
        torch.cuda.synchronize()
        p2 = pipe_profile(r2, kg, args.large_nb, d, epochs=e2,
                          gpu_ms_per_epoch=f0.elapsed_time(f1) / e2, opt_k=opt_k) if r2.pipelined \
            else kernel_profile(model, upd, kg, args.large_nb, d, r2.stream, r2, opt_k=opt_k)
        k2 = p2["dominant"]
        sgl = meas["streaming_gather_GB_s"]["wn18_table_33MB"] if meas else None
        large = {"nbatches": args.large_nb, "batch": N_TRIPLES // args.large_nb,
                 "frac_of_streaming_gather": round(k2["achieved_gbs"] / sgl, 4) if sgl else None,
                 "epoch_GB_s_8d": round(p2["epoch_bytes"] / (t2 / e2) / 1e9, 1),
                 "value": round(N_TRIPLES * e2 / t2, 1), "unit": "triples/s",
                 "ms_per_epoch": round(1000.0 * t2 / e2, 4),
                 "kernel": k2["name"], "achieved_GB_s": round(k2["achieved_gbs"], 1),
                 "frac_of_peak": round(k2["achieved_gbs"] / HBM_PEAK_GBS, 4),
                 "avg_launch_us": round(k2["avg_us"], 3),
                 "epochs": "1..%d of a fresh run (as the headline)" % e2,
                 "first5_ms_per_epoch": round(f0.elapsed_time(f5) / 5, 4),
                 "runner": "pipelined" if r2.pipelined else "two-launch"}
        del r2

    probe = handoff_probe(dev) if runner.pipelined else None
    pipelined, nlaunches = runner.pipelined, runner.nlaunches
    hot_rows = getattr(runner, "hot_rows", 0)
    acc_names = {"entity": acc_label(runner.accE), "relation": acc_label(runner.accR)}
    launch_us_max = max_over_ranks(prof["dominant"]["avg_us"], world, dev)
    line = None
    if rank == 0:
        # the CPU baseline on rank 0 at N = 1 only (the bench contract)
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline(trip, d, nb, args.cpu_seconds,
                                                                   opt=args.opt)
        k = prof["dominant"]
        kname = {"transe_sample_grad": "sample_grad", "accum_apply": "k_apply",
                 "pipe_batch": "k_pipe_batch", "pipe_fused": "k_pipe_fused"}[k["name"]]
        # config 1's own PMC pass (pmc_c1.json: d=50 padded to 64, SGD), not config 2's
        traffic, traffic_src = pmc_traffic(kname, "pmc.json" if args.config == 2 else
                                           "pmc_c%d.json" % args.config)
        line = {
            "metric": ("triples/sec (score+grad+update), WN18 TransE d=200, 1/2/4/8 MI355X"
                       if args.config == 2 else
                       "triples/sec (score+grad+update), WN18 TransE d=%d %s (BASELINE configs[0])"
                       % (d, args.opt)) +
                      ("" if world == 1 else " -- %d independent replicas (weak; not one model)"
                       % world),
            "value": round(value, 1),
            "unit": "triples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True,
            # --mode replicas at N > 1: one replica per GPU, one epoch of its own
            # KG per step: per-GPU work fixed as N grows (the default N > 1 line
            # is the one-model data-parallel run, run_dp)
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": kg_label(args, "RandomState(0)") + "; random-init params (nunif, seed 42)",
            "config": {"workload": "TransE-L1 d=%d PairwiseStochasticTrainer+%s, WN18 shape, "
                                   "nb=%d (B=%d), margin 2.0, lr 0.1, device RandomModeSampler(1,[0,1]); "
                                   "step = 1 epoch" % (d, {"sgd": "SGD", "adagrad": "AdaGrad"}[args.opt],
                                                       nb, N_TRIPLES // nb) +
                                   ("" if world == 1 else
                                    "; %d independent replicas (one per GPU, each its own KG "
                                    "and model; no exchange: the 33 MB table is replicated, "
                                    "north_star)" % world),
                       "global_batch": N_TRIPLES // nb,
                       "parallelism": parallelism_label("replicas%d" % world, info)
                       if world > 1 else "1gpu"},
            "roofline": {"bound": "hbm", "kernel": k["name"],
                         "achieved": round(k["achieved_gbs"], 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(k["achieved_gbs"] / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src,
                         "bytes_per_launch": round(k["bytes_per_launch"]),
                         "bytes_formula": prof.get("formula"),
                         "impl_bytes_per_launch": round(k.get("impl_bytes_per_launch",
                                                              k["bytes_per_launch"])),
                         "avg_launch_us": round(k["avg_us"], 3),
                         "avg_launch_source": "timed-region HIP events (graph replays) minus "
                                              "the draw/advance launches, per batch launch",
                         "eager_avg_launch_us": round(k.get("eager_avg_us", k["avg_us"]), 3),
                         "avg_launch_us_max_over_ranks": round(launch_us_max, 3),
                         "measured": meas},
            "cpu_baseline": cpu,
            "detail": {
                "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
                # 2 pairs per positive (RandomModeSampler modes [0, 1]; on
                # this sparse KG a negative is always found), the positive re-scored
                # per pair (base.py:1411-1427): 4 scored triples per positive
                "pairs_per_s": round(2.0 * value, 1),
                "scored_triples_per_s": round(4.0 * value, 1),
                "violations_per_pair": round(nviol / (2.0 * positives), 4),
                "kernels": {n: {"avg_us": round(v["avg_us"], 3), "launches": v["launches"],
                                "GB_s": round(v["achieved_gbs"], 1)}
                            for n, v in prof["kernels"].items()},
                "step_algorithmic_GB_s": round(prof["epoch_bytes"] / (elapsed / args.steps) / 1e9, 1),
                "launches_per_step": nlaunches,
                "runner": "pipelined (1 launch/batch)" if pipelined else "two-launch",
                "accumulator": acc_names,
                "hot_rows": hot_rows,   # entity rows with replicated sums (skewed KGs)
                "handoff_probe": probe,
                "per_replica_value": round(rank_value, 1),
                "large_batch": large,
                "rank_setup": info,
            },
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


WATCHDOG_EXIT = 3   # a multi-rank measurement raised or hung: the job failed


def mark_failure(line, key, msg):
    """Record a failed measurement in rank 0's line: key None = the line's own
    value (set to null), else detail[key]."""
    if line is None:
        return
    err = msg if isinstance(msg, dict) else {"error": msg}
    if key is None:
        line["value"] = None
        line.update(err)
    else:
        line.setdefault("detail", {})[key] = err


def run_with_watchdog(fn, line, limit, key=None):
    """fn() with a time limit.  Returns fn's result, or {"error": ...} if it
    raised (the caller then prints the line and ends with WATCHDOG_EXIT).  If
    fn has not returned after `limit` seconds (a collective that never
    completes), a watchdog thread marks the failure in `line` (rank 0's bench
    line; None on other ranks) under `key` (see mark_failure), prints it once
    and ends this rank's process with status WATCHDOG_EXIT -- never 0: a hung
    GPU collective must not look like a successful run."""
    import threading
    done = threading.Event()
    state = {"printed": False}
    lock = threading.Lock()

    def watchdog():
        if done.wait(limit):
            return
        with lock:
            if line is not None and not state["printed"]:
                mark_failure(line, key, "did not finish within %g s (multi-rank collective); "
                                        "not measured" % limit)
                print(json.dumps(line), flush=True)
                state["printed"] = True
        os._exit(WATCHDOG_EXIT)
    threading.Thread(target=watchdog, daemon=True).start()
    try:
        out = fn()
    except Exception as e:
        import traceback
        where = traceback.extract_tb(e.__traceback__)[-3:]
        out = {"error": "%s: %s" % (type(e).__name__, e),
               "where": ["%s:%d %s" % (os.path.basename(f.filename), f.lineno, f.name)
                         for f in where]}
    with lock:
        done.set()
        if state["printed"]:
            os._exit(WATCHDOG_EXIT)
    return out


def failed(x):
    return isinstance(x, dict) and "error" in x


def measure_dp(args, dev, nb, warmup, steps, profile=True):
    """ONE TransE-L1 model trained data parallel over the ranks
    (skge_amd.dp.DataParallelRunner; reference semantics
    skge/base.py:1394-1427, 1306-1316): every rank holds the whole WN18 model;
    per union batch ONE pipelined launch applies the previous batch and scores
    the rank's slice, the slices' records are all-gathered over RCCL and the
    other ranks' positives added, so all replicas equal one GPU's run on the
    union batches bit for bit.  Timed epochs start from the initial tables;
    max over ranks.  profile: one more eager epoch with HIP events between
    the phases of every union batch (launch / all-gather / scatter on the
    runner stream), for the per-rank roofline."""
    import torch
    import torch.distributed as dist
    import skge_amd as S
    from skge_amd.device import DeviceKG
    from skge_amd.dp import DataParallelRunner
    world = dist.get_world_size()
    d = args.d
    trip = bench_kg(args, 0)              # ONE model: the same KG on every rank
    np.random.seed(42)
    model = S.TransE((N_ENT, N_ENT, N_REL), d, l1=True)
    model.add_hyperparam("margin", 2.0)
    Upd = S.SGD if args.opt == "sgd" else S.AdaGrad
    upd = {pid: Upd(p, 0.1) for pid, p in model.params.items()}
    kg = DeviceKG(trip, dev)
    runner = DataParallelRunner(model, upd, kg, nb, seed=1234)
    init = {pid: p.data.clone() for pid, p in model.params.items()}

    def rollback():
        for pid, p in model.params.items():
            p.data.copy_(init[pid])
            upd[pid].reset()
        runner.nviol_total.zero_()
        torch.cuda.synchronize()

    runner.run(max(warmup, 1))               # the first epoch also captures the graph
    runner.synchronize()
    rollback()
    dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(runner.stream)
    runner.run(steps)
    ev1.record(runner.stream)
    runner.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    dist.barrier()
    elapsed = max_over_ranks(elapsed, world, dev)
    gpu_ms = ev0.elapsed_time(ev1)
    nviol = runner.total_violations()
    # replicas identical: every rank's tables must agree
    ck = torch.tensor([float(model.E.data.double().sum().item()),
                       float(model.R.data.double().sum().item())], dtype=torch.float64,
                      device=coll_device(dev))
    cks = [torch.zeros_like(ck) for _ in range(world)]
    dist.all_gather(cks, ck)
    same = all(torch.equal(c, cks[0]) for c in cks)
    bs = N_TRIPLES // nb
    out = {"union_batch": bs, "nb": nb, "per_gpu_batch": -(-bs // world),
           "value": round(N_TRIPLES * steps / elapsed, 1), "unit": "triples/s",
           "ms_per_step": round(1000.0 * elapsed / steps, 4),
           "gpu_event_ms_per_step": round(gpu_ms / steps, 4),
           "us_per_union_batch": round(1e6 * elapsed / steps / len(runner.batches), 2),
           "violations_per_pair": round(nviol / (2.0 * N_TRIPLES * steps), 4),
           "replicas_identical": bool(same), "captured_graph": runner.graph is not None,
           "record_bytes_per_positive": runner.rec_bytes}
    if profile:
        rollback()
        out["phases"] = dp_profile(runner, args, world)
    del runner
    return out


def dp_profile(runner, args, world):
    """Per-rank phases of one eager data-parallel epoch (HIP events on the
    runner stream; the all-gather's time is the RCCL collective's, incl. its
    wait for the slowest rank) and their algorithmic bytes (per
    rank): launch = ONE k_pipe_batch in its data-parallel form (union batch
    b-1's rows applied, k d U, while the rank's slice of batch b is scored,
    4d x 5 rows + 20 B per positive, and its records written); all_gather =
    G x share records received; scatter = the other ranks' records read (none
    at G = 1; their packed atomics are implementation bytes, not 8(d)'s).  U
    is counted on the even batches (their accumulator copy is the caller's
    table) and averaged."""
    import torch
    d, k = runner.d, (4 if args.opt == "sgd" else 12)
    rb = runner.rec_bytes
    ops, ex, st = runner.ops, runner.ex, runner.stream
    from skge_amd.dp import slice_of
    names = ("launch", "all_gather", "scatter")
    ms = dict.fromkeys(names, 0.0)
    by = dict.fromkeys(names, 0.0)
    Us = []
    runner._pad_in()
    nbat = len(runner.batches)
    grouped = ex.backend is not None
    with torch.cuda.stream(st):
        ops.begin()
        for b, (start, count) in enumerate(runner.batches):
            share, lo, hi = slice_of(count, ex.G, ex.rank)
            remote = grouped and ex.G > 1
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record(st)
            send = ops.batch(b, start, count, lo, hi, share, fold=not remote)
            ev[1].record(st)
            recs = ops.gathered(ex, send, share) if grouped else send
            ev[2].record(st)
            if remote:
                ops.scatter(b, start, count, recs, lo, hi)
            ev[3].record(st)
            st.synchronize()
            if b % 2 == 0:   # batch b's rows, pending for launch b + 1
                Us.append(int((runner.accE.cnt != 0).sum().item()))
            for i, n in enumerate(names):
                ms[n] += ev[i].elapsed_time(ev[i + 1])
            by["launch"] += (hi - lo) * (4.0 * d * 5 + 20 + rb)
            by["all_gather"] += ex.G * share * rb if grouped else 0.0
            by["scatter"] += (count - (hi - lo)) * rb if remote else 0.0
        ops.flush(nbat)
        ops.end()
    st.synchronize()
    runner._pad_out()
    U = float(np.mean(Us)) if Us else 0.0
    by["launch"] += k * d * (U + N_REL) * nbat      # each launch applies the previous batch
    ph = {}
    for n in names:
        us = 1000.0 * ms[n] / nbat
        b = by[n] / nbat
        ph[n] = {"us_per_batch": round(us, 3), "bytes_per_batch": round(b),
                 "GB_s": round(b / (us * 1e-6) / 1e9, 1) if us > 0 else None}
    ph["launch"]["applied_rows_per_batch"] = round(U, 1)
    return ph


def dp_line(args, world, m, ph, d=None, nb=None, workload_kg=None, info=None):
    """The N > 1 line of configs 1-2: ONE TransE-L1 model trained data parallel
    (measure_dp's result m; ph: its per-rank phases, the roofline's source)."""
    d = d or args.d
    nb = nb or args.nb
    bs = m["union_batch"]
    opt = {"sgd": "SGD", "adagrad": "AdaGrad"}[args.opt]
    line = {
        "metric": "triples/sec (score+grad+update), WN18 TransE d=200, 1/2/4/8 MI355X"
                  if args.config == 2 else
                  "triples/sec (score+grad+update), WN18 TransE d=%d %s (BASELINE configs[0])"
                  % (d, args.opt),
        "value": m["value"], "unit": "triples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": m["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong" if args.dp_batch == "global" else "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": (workload_kg or "synthetic WN18-shaped KG (|E|=40943 |R|=18 T=141442 uniform, "
                 "RandomState(0))") + ", the same on every rank; random-init params (nunif, seed 42)",
        "config": {"workload": "ONE TransE-L1 d=%d model, PairwiseStochasticTrainer+%s, union "
                               "batch %d positives (nb=%d; ~%d per GPU), margin 2.0, lr 0.1, "
                               "device RandomModeSampler(1,[0,1]); data parallel over %d GPUs: "
                               "one pipelined launch per union batch (apply + slice scoring), "
                               "all-gather of the records, the other ranks' positives added; "
                               "step = 1 epoch" % (d, opt, bs, nb, m["per_gpu_batch"], world),
                   "global_batch": bs,
                   "parallelism": parallelism_label("dp%d" % world, info or {})},
        "roofline": None,
        "cpu_baseline": None,        # the bench contract: rank 0 at N = 1 only
        "detail": {"runner": "DataParallelRunner (skge_amd.dp)", "dp": m,
                   "rank_setup": info},
    }
    if ph:
        dom = max(("launch", "scatter"), key=lambda n: ph[n]["us_per_batch"])
        line["roofline"] = {
            "bound": "hbm", "kernel": "dp_" + dom, "achieved": ph[dom]["GB_s"],
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ph[dom]["GB_s"] / HBM_PEAK_GBS, 4) if ph[dom]["GB_s"] else None,
            "traffic": None, "bytes_per_launch": ph[dom]["bytes_per_batch"],
            "avg_launch_us": ph[dom]["us_per_batch"], "phases_per_rank": ph,
            "note": "rank 0, per union batch, eager epoch with HIP events between phases "
                    "(bench.dp_profile); all_gather = RCCL over xGMI"}
    return line


def run_dp(args):
    """Configs 1-2 on N > 1 GPUs (the default): the line is ONE model trained
    data parallel (measure_dp).  --dp-batch global (default): union batch =
    the reference's 1414 (strong scaling); per-gpu: 1414 per GPU (union batch
    N x 1414, weak).  detail: the other union batch with the one-GPU
    pipelined runner at that batch beside it, one GPU alone at the line's
    batch (vs_one_gpu), and N independent jobs (N models on N KGs, no
    exchange) -- never the value.  Every multi-rank measurement runs under
    run_with_watchdog: a failure or hang ends the job with WATCHDOG_EXIT."""
    import torch
    import torch.distributed as dist
    world, rank, local, dev = setup_ranks()
    info = rank_setup_info(world, local)
    limit = float(os.environ.get("SKGE_BENCH_DP_TIMEOUT", "300"))
    nb = max(1, args.nb // world) if args.dp_batch == "per-gpu" else args.nb
    bs = N_TRIPLES // nb
    skel = None
    if rank == 0:
        skel = dp_line(args, world, {"value": None, "ms_per_step": None, "union_batch": bs,
                                     "per_gpu_batch": -(-bs // world)}, None, nb=nb, info=info)
    m = run_with_watchdog(lambda: measure_dp(args, dev, nb, args.warmup, args.steps), skel, limit)
    if failed(m):
        if rank == 0:
            mark_failure(skel, None, m)
            print(json.dumps(skel), flush=True)
        os._exit(WATCHDOG_EXIT)     # ranks may be out of step in a failed collective
    line = dp_line(args, world, m, m.get("phases"), nb=nb, info=info) if rank == 0 else None
    torch.cuda.synchronize()

    def details():
        out = {}
        one = one_gpu_value(args, dev, nb)
        out["one_gpu_same_batch"] = dict(one, vs=None)
        out["vs_one_gpu"] = round(m["value"] / one["value"], 4)
        nb2 = args.nb if args.dp_batch == "per-gpu" else max(1, args.nb // world)
        w = measure_dp(args, dev, nb2, args.warmup, args.steps, profile=False)
        same = one_gpu_value(args, dev, nb2)
        out["other_union_batch"] = dict(
            w, scaling="strong" if nb2 == args.nb else "weak (union batch grows with N)",
            one_gpu_same_geometry=same,
            vs_one_gpu_same_geometry=round(w["value"] / same["value"], 4))
        ind = one_gpu_value(args, dev, args.nb, kg_seed=rank, seed=1234 + rank)
        el = max_over_ranks(ind["elapsed_s"], world, dev)
        out["independent_jobs"] = {
            "what": "%d independent models, one per GPU, each on its own KG, no exchange (job "
                    "throughput, not one model trained faster)" % world,
            "value": round(replica_value(N_TRIPLES * ind["epochs"], world, el), 1),
            "nb": args.nb, "ms_per_step": round(1000.0 * el / ind["epochs"], 4)}
        return out
    det = run_with_watchdog(details, line, limit, key="details")
    if rank == 0:
        if failed(det):
            mark_failure(line, "details", det)
        else:
            line["detail"].update(det)
        print(json.dumps(line), flush=True)
    if failed(det):
        os._exit(WATCHDOG_EXIT)
    dist.destroy_process_group()


def one_gpu_value(args, dev, nb, epochs=None, kg_seed=0, seed=1234):
    """The one-GPU pipelined runner (this rank's GPU alone, no collective) on
    the same KG, model and union batch as a data-parallel run: what the
    batch size alone buys, so a scaling curve does not credit it to the GPUs
    (kg_seed = rank: an independent job on its own KG)."""
    import torch
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner
    epochs = epochs or args.steps
    trip = bench_kg(args, kg_seed)
    np.random.seed(42 + kg_seed)
    model = S.TransE((N_ENT, N_ENT, N_REL), args.d, l1=True)
    model.add_hyperparam("margin", 2.0)
    Upd = S.SGD if args.opt == "sgd" else S.AdaGrad
    upd = {pid: Upd(p, 0.1) for pid, p in model.params.items()}
    r = EpochRunner(model, upd, DeviceKG(trip, dev), nbatches=nb, seed=seed)
    init = {pid: p.data.clone() for pid, p in model.params.items()}
    r.run(max(args.warmup, 1))
    r.synchronize()
    for pid, p in model.params.items():     # timed epochs start from the initial tables
        p.data.copy_(init[pid])
        upd[pid].reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.run(epochs)
    r.synchronize()
    el = time.perf_counter() - t0
    out = {"nb": nb, "union_batch": N_TRIPLES // nb, "value": round(N_TRIPLES * epochs / el, 1),
           "ms_per_step": round(1000.0 * el / epochs, 4), "elapsed_s": el, "epochs": epochs,
           "runner": "pipelined" if r.pipelined else "two-launch"}
    del r
    return out


def _score_bytes(d, cnt, V, packed=True, hole=False):
    """Scoring part of a batch: gathers of s, o, p + 2
    corrupted rows, 20 B of index/hash traffic per positive, and the atomic row
    adds of the violating positives (<= 5 rows each; 2 B per element with the
    exact int16x4 sums, 4 B with fp32).  HolE (fp32): a violating positive adds
    3 + (its violating pairs) rows, at least 2.5 V rows for V violating pairs
    (the lower bound is used)."""
    ab = 2 * d if packed else 4 * d
    rows = 2.5 * V if hole else min(5 * cnt, 2 * V + 3 * cnt)
    return 4 * d * (3 * cnt + 2 * cnt) + 20 * cnt + ab * rows


def _apply_bytes(d, rows, packed=True):
    """Per applied row: read param + AdaGrad state, write both (16d), read the
    sums and write them back zeroed (4d packed, 8d fp32)."""
    return (16 * d + (4 * d if packed else 8 * d)) * rows


def pipe_profile(runner, kg, nb, d, epochs=1, gpu_ms_per_epoch=None, hole=False, opt_k=12):
    """Pipelined runner: `epochs` eager epochs with HIP events around every
    launch and the kernel's own per-launch counters (skge_pipe_runner_profile,
    on the runner's stream), started from the same state as the timed region.
    Launch i >= 1 scores batch i-1 and applies batch i-2: its algorithmic
    bytes are the scoring bytes of its batch plus 20 B/element for each row it
    applied (read sum, param, state; write param, state, zero sum), with the
    applied-row and violation counts the kernel itself recorded.

    avg_us: with gpu_ms_per_epoch (the timed region's HIP-event time per
    epoch, graph replays) the batch launches' share of it -- the epoch minus
    the draw and key-advance launches, over the batch launches; else the
    eager per-launch event times (which include per-launch event overhead)."""
    T = kg.T
    bs = T // nb
    counts = [min(bs, T - s) for s in range(0, T, bs)] + [0]   # + the flush launch
    n = len(counts)
    b_pipe, t_pipe, total, t_other = 0.0, 0.0, 0.0, 0.0
    geo = np.zeros(4)   # positives, atomic rows, applied rows, launches
    us0 = 0.0
    for _ in range(epochs):
        us, stats = runner.profile()
        us0 += float(us[0])
        t_other += float(us[0]) + float(us[n + 1])
        for i, cnt in enumerate(counts, start=1):
            UE, UR, V = (int(x) for x in stats[i])
            b = _score_bytes(d, cnt, V, packed=not hole, hole=hole) + \
                _apply_bytes(d, UE + UR, packed=not hole)
            b_pipe += b
            t_pipe += float(us[i])
            if cnt:
                total += algorithmic_bytes(d, cnt, 2 * cnt, 0, 0)
            total += opt_k * d * (UE + UR)
            geo += (cnt, 2.5 * V if hole else min(5 * cnt, 2 * V + 3 * cnt), UE + UR, 1)
    eager_us = t_pipe / (n * epochs)
    avg_us = eager_us
    if gpu_ms_per_epoch is not None:
        avg_us = (1000.0 * gpu_ms_per_epoch - t_other / epochs) / n
    bpl = b_pipe / (n * epochs)       # implementation bytes (packed sums, atomics)
    apl = total / (n * epochs)        # SURVEY 8(d) algorithmic bytes
    # the batch kernel the runner launches (k_pipe_batch / k_pipe_fused / k_hole_pipe)
    kn = "hole_pipe" if hole else getattr(runner, "kernel", "k_pipe_batch")[2:]
    kern = {kn: {
                           "name": kn, "avg_us": avg_us,
                           "launches": n,
                           "eager_avg_us": eager_us, "bytes_per_launch": apl,
                           "achieved_gbs": apl / (avg_us * 1e-6) / 1e9,
                           "impl_bytes_per_launch": bpl,
                           "impl_gbs": bpl / (avg_us * 1e-6) / 1e9},
            # per positive: triple 12 B, two filter words 8 B, record 20 B
            "epoch_sample": {"name": "epoch_sample", "avg_us": us0 / epochs, "launches": 1,
                             "bytes_per_launch": 40.0 * T,
                             "achieved_gbs": 40.0 * T / (us0 / epochs * 1e-6) / 1e9}}
    g = geo / geo[3]
    return {"kernels": kern, "dominant": kern[kn],
            "source": ("timed-region epoch time (graph replays) minus the draw / key-advance "
                       "launches, per batch launch" if gpu_ms_per_epoch is not None else
                       "eager epoch, HIP events around every launch"),
            "epoch_bytes": total / epochs,
            "geometry": {"positives": g[0], "atomic_rows": g[1], "applied_rows": g[2]},
            # the 8(d) formula's inputs per launch (averaged over the profiled
            # epochs' n launches): B positives scored, P = 2B pairs, U rows applied
            "formula": {"launches": n, "B": g[0], "P": 2.0 * g[0], "U": g[2], "d": d,
                        "k": opt_k, "bytes_per_launch": apl,
                        "expr": "4d(3B+P) + k d U + 20B"}}


def measured_roofline(dev, rows, d, n_gather, rows_per_wave, atom_rows, n_rmw, launches=101,
                      reps=5):
    """skge_roofline_gather (csrc/skge_roofline.hip): the same row traffic as
    one training launch without its dependencies, `launches` launches
    captured in one graph like an epoch; returns (us per launch, bytes per
    launch, GB/s).  Scratch tables of the training table's shape."""
    import torch
    from skge_amd import _lib as L
    P = torch.rand((rows, d), dtype=torch.float32, device=dev)
    A = torch.rand((rows, d), dtype=torch.float32, device=dev)
    S = torch.zeros(rows * d // 4, dtype=torch.int64, device=dev)
    out = torch.empty(max(n_gather, 1), dtype=torch.float32, device=dev)
    lib = L.lib()

    def launch_all():
        for i in range(launches):
            L.check(lib.skge_roofline_gather(L.stream_ptr(), L.ptr(P), L.ptr(A), L.ptr(S), rows, d,
                                             n_gather, rows_per_wave, atom_rows, n_rmw,
                                             (i * 7919 + 13) & 0xFFFFFFFF, L.ptr(out)), "roofline")

    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        launch_all()                      # warm (eager)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        launch_all()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    with torch.cuda.stream(st):
        for _ in range(reps):
            g.replay()
    e1.record(st)
    torch.cuda.synchronize()
    us = 1000.0 * e0.elapsed_time(e1) / (reps * launches)
    b = n_gather * (rows_per_wave * 4.0 * d + atom_rows * 2.0 * d) + n_rmw * 20.0 * d
    del P, A, S, out, g
    return us, b, b / (us * 1e-6) / 1e9


N5, M5, D5, T5, B5 = 50_000_000, 10_000, 512, 100_000_000, 131072


def cpu_baseline_config5(seconds=10.0, n_ent=1_000_000, n_rel=10_000, d=512, batch=10_000):
    """The oracle on the config-5 model at SURVEY 6's scaled-down shape (the
    full 50M x 512 fp64 table and its state, 205 GB, are not a CPU sample):
    TransE-L1 d=512 AdaGrad margin 2.0, |E|=1M |R|=10k, batches of 10k
    positives with their RandomModeSampler negatives (untimed), consecutive
    batches until `seconds` of score+grad+update time."""
    from oracle import skge_oracle as O
    rs = np.random.RandomState(5)
    T = 6 * batch
    trip = np.stack([rs.randint(n_ent, size=T), rs.randint(n_ent, size=T),
                     rs.randint(n_rel, size=T)], axis=1)
    tset = set(map(tuple, trip.tolist()))
    bnd = np.sqrt(6) / np.sqrt(n_ent + d)
    E = rs.uniform(-bnd, bnd, size=(n_ent, d))
    E /= np.sqrt((E ** 2).sum(axis=1))[:, None]
    bnd = np.sqrt(6) / np.sqrt(n_rel + d)
    params = {"E": E, "R": rs.uniform(-bnd, bnd, size=(n_rel, d))}
    state = {k: np.zeros_like(v) for k, v in params.items()}
    np.random.seed(42)
    t_step, npos, nbat = 0.0, 0, 0
    for a in range(0, T, batch):
        pairs = O.random_mode_sample(trip[a:a + batch], tset, (n_ent, n_ent, n_rel))
        pos = np.array([p for p, _ in pairs])
        neg = np.array([q for _, q in pairs])
        t0 = time.perf_counter()
        O.pairwise_step("transe", params, state, pos, neg, 0.1, 2.0, "adagrad", l1=True)
        t_step += time.perf_counter() - t0
        npos += min(batch, T - a)
        nbat += 1
        if t_step > seconds:
            break
    return {"value": npos / t_step, "unit": "triples/s", "cores": 1, "kind": "port",
            "sample": "%d batches of %d positives, TransE-L1 d=%d AdaGrad margin 2.0 at the "
                      "SURVEY 6 scaled-down config-5 shape (|E|=%d |R|=%d; the 50M-row fp64 "
                      "table and state do not make a CPU sample); oracle/skge_oracle.py fp64 "
                      "NumPy, 1 thread; score+grad+update only (host sampler untimed)"
                      % (nbat, batch, d, n_ent, n_rel),
            "reference": reference_cpu("transe", 512, "adagrad")}


def make_config5_kg(n_ent, n_rel, n_triples, dev, seed):
    """Unique uniform (s, o, p) triples drawn on the device (torch generator)."""
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    out = None
    while out is None or out.shape[0] < n_triples:
        need = n_triples - (0 if out is None else out.shape[0])
        m = need + need // 64 + 1024
        cand = torch.stack([torch.randint(n_ent, (m,), device=dev, generator=g, dtype=torch.int32),
                            torch.randint(n_ent, (m,), device=dev, generator=g, dtype=torch.int32),
                            torch.randint(n_rel, (m,), device=dev, generator=g, dtype=torch.int32)],
                           dim=1)
        allt = cand if out is None else torch.cat([out, cand])
        out = torch.unique(allt, dim=0)   # sorted order; the runner permutes per epoch
        del cand, allt
    out = out[:n_triples].contiguous()
    torch.cuda.empty_cache()
    return out


# kernel_profile's names -> the HIP kernel names rocprofv3 reports
PMC_KERNEL = {"transe_sample_grad": "k_transe_l1_sample_grad", "accum_apply": "k_apply",
              "pipe_batch": "k_pipe_batch", "pipe_fused": "k_pipe_fused"}


def run_config5(args):
    """BASELINE.json configs[4] on one GPU per rank: TransE-L1 d=512, |E|=50M,
    |R|=10k, T=100M synthetic triples, B=131072 positives per batch, AdaGrad.
    The tables (E 102 GB + AdaGrad state 102 GB + packed sums 51 GB) fit one
    MI355X, so N GPUs run replicas (north_star: shard only past 288 GB)."""
    import torch
    import torch.distributed as dist
    world, rank, local, dev = setup_ranks()
    import skge_amd as S
    from skge_amd.device import DeviceKG, EpochRunner
    n_ent, T = int(N5 * args.c5_scale), int(T5 * args.c5_scale)
    d, n_rel = D5, M5
    t_build = time.perf_counter()
    trip = make_config5_kg(n_ent, n_rel, T, dev, seed=rank)
    model = S.TransE((n_ent, n_ent, n_rel), d, l1=True, init="device_nunif")
    model.add_hyperparam("margin", 2.0)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in model.params.items()}
    kg = DeviceKG(trip, dev)
    del trip
    nb = max(1, T // B5)
    runner = EpochRunner(model, upd, kg, nbatches=nb, seed=99 + rank)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t_build
    runner.run(args.warmup)
    runner.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if runner.pipelined:   # (fits at |E| = 50M with 8-bit entity sums: ~236 GB)
        t0 = time.perf_counter()
        runner.run(args.steps)
        runner.synchronize()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        prof = None
    else:
        # the two-launch epoch's kernel sequence launched eagerly with HIP events
        # between the kernels: per-kernel device time and applied rows of
        # exactly the timed epochs (kernels of ~0.3-1 ms: launch cost ~1%)
        elapsed, prof = eager_epochs(runner, kg, nb, d, args.steps)
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, world, dev)
    counter_cost = None
    if prof is not None and not args.c5_no_counter_split:
        # the counters' price at the same epochs: the next epoch's even batches
        # count their rows, the odd ones do not
        _, alt = eager_epochs(runner, kg, nb, d, 1, counters="alt")
        counter_cost = {
            "apply_us_counters": round(alt["apply_us_counters"], 3),
            "apply_us_no_counters": round(alt["apply_us_no_counters"], 3),
            "note": "epoch W+K+1, even batches with the per-row update counters "
                    "(skge/param.py:149-150, AdaGrad's updateCounts -- work the reference "
                    "does, so the timed epochs keep them; they also give U for k_apply's "
                    "8(d) bytes), odd batches without"}
    value = replica_value(T * args.steps, world, elapsed)
    prof_epochs = args.steps
    if prof is None:
        # the pipelined runner: the batch launch's time from the timed region's
        # epoch time minus the other kernels (as config 2), counters from one
        # more eager epoch
        prof = pipe_profile(runner, kg, nb, d, gpu_ms_per_epoch=1000.0 * elapsed / args.steps)
        prof_epochs = 1
    k = prof["dominant"]
    if rank == 0:
        traffic, traffic_src = pmc_traffic_epochs(PMC_KERNEL.get(k["name"], k["name"]),
                                                  "pmc_c5_epochs.json", args.warmup, args.steps)
        if traffic is None:
            traffic, traffic_src = pmc_traffic(PMC_KERNEL.get(k["name"], k["name"]), "pmc_c5.json")
        line = {
            "metric": "triples/sec (score+grad+update), synthetic TransE |E|=50M |R|=10k d=512, "
                      "B=131072 per GPU (BASELINE configs[4])" +
                      ("" if world == 1 else " -- %d independent replicas (weak; not one model)"
                       % world),
            "value": round(value, 1), "unit": "triples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic uniform KG (|E|=%d |R|=%d T=%d, torch generator seed rank); "
                    "device-drawn nunif params" % (n_ent, n_rel, T),
            "config": {"workload": "TransE-L1 d=%d PairwiseStochasticTrainer+AdaGrad, margin 2.0, "
                                   "lr 0.1, device RandomModeSampler(1,[0,1]); step = 1 epoch of "
                                   "%d batches" % (d, nb),
                       "global_batch": T // nb * world,
                       "parallelism": "replicas%d" % world if world > 1 else "1gpu"},
            "roofline": {"bound": "hbm", "kernel": k["name"],
                         "achieved": round(k["achieved_gbs"], 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(k["achieved_gbs"] / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "traffic_source": traffic_src,
                         "bytes_per_launch": round(k["bytes_per_launch"]),
                         "avg_launch_us": round(k["avg_us"], 3),
                         "avg_launch_source": prof.get("source"),
                         "bytes_formula": prof.get("formula")},
            "cpu_baseline": None if (args.no_cpu or world > 1) else
                            cpu_baseline_config5(args.cpu_seconds),   # N = 1 only
            "detail": {"runner": "pipelined" if runner.pipelined else "two-launch",
                       "timed_epochs": ("epochs %d..%d (after %d warm-up epochs), replays of "
                                        "the epoch graph; the per-kernel detail from one more "
                                        "eager epoch" if runner.pipelined else
                                        "epochs %d..%d (after %d warm-up epochs as replays "
                                        "of the epoch graph), launched eagerly with HIP "
                                        "events between the kernels")
                                       % (args.warmup + 1, args.warmup + args.steps,
                                          args.warmup),
                       "counter_cost": counter_cost,
                       "accumulator": {"entity": acc_label(runner.accE),
                                       "relation": acc_label(runner.accR)},
                       "build_s": round(t_build, 1),
                       "kernels": {n: {"avg_us": round(v["avg_us"], 3), "launches": v["launches"],
                                       "GB_s": round(v["achieved_gbs"], 1)}
                                   for n, v in prof["kernels"].items()},
                       # the kernels' device time per step (<= ms_per_step: the
                       # rest is launch gaps)
                       "kernels_ms_per_step": round(sum(v["avg_us"] * v["launches"]
                                                        for v in prof["kernels"].values()
                                                        if v["launches"] > 1)
                                                    / 1000.0 / prof_epochs, 3),
                       "gpu_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def eager_epochs(runner, kg, nb, d, epochs, opt_k=12, counters=True):
    """`epochs` epochs of the two-launch runner's graph (skge_epoch.hip
    skge_runner_create: per batch k_transe_*_sample_grad then k_apply, then
    the epoch-key advance) launched eagerly on the runner's stream, HIP events
    between the kernels and no host synchronisation until the end; AdaGrad
    update counters on (skge_table_t.upd_count, param.py:149-150), whose sum is
    the rows the applies updated.  Returns (wall seconds, profile): per kernel
    the mean device time over these launches and the SURVEY 8(d) bytes --
    sample_grad 4d(3B + P) + 20B per batch, k_apply k d U with U the counted
    rows -- so frac and ms_per_step come from the same epochs.  counters=False
    "alt" counts on even batches only and returns the mean k_apply time of
    the counting and the non-counting batches of the same epochs (the
    counters' price; neighbouring batches apply about as many rows)."""
    import torch
    from skge_amd import _lib as L
    lib = L.lib()
    st = runner.stream
    sp = L.stream_ptr(st)
    dev = runner.model.device
    te = L.SkgeTable.from_buffer_copy(runner.te)
    tr = L.SkgeTable.from_buffer_copy(runner.tr)
    ucE = torch.zeros(te.rows, dtype=torch.int32, device=dev)
    ucR = torch.zeros(tr.rows, dtype=torch.int32, device=dev)
    te.upd_count, tr.upd_count = L.ptr(ucE), L.ptr(ucR)
    tabs = (L.SkgeTable * 2)(te, tr)
    te0 = L.SkgeTable.from_buffer_copy(te)
    tr0 = L.SkgeTable.from_buffer_copy(tr)
    te0.upd_count = tr0.upd_count = None
    tabs0 = (L.SkgeTable * 2)(te0, tr0)
    # counters: True -> every apply counts its rows; "alt" -> even batches
    # count, odd ones do not (the counters' price at the same epochs)
    on = (lambda i: True) if counters is True else (lambda i: i % 2 == 0)
    nviol = torch.zeros(1, dtype=torch.int32, device=dev)
    T = kg.T
    bs = T // nb
    batches = [(s0, min(bs, T - s0)) for s0 in range(0, T, bs)]
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
          for _ in range(epochs * len(batches))]
    l1 = 1 if runner.model.l1 else 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(st):
        i = 0
        for _ in range(epochs):
            for start, cnt in batches:
                e = ev[i]
                i += 1
                e[0].record(st)
                L.check(lib.skge_transe_sample_grad(sp, l1, te, tr, d, L.ptr(kg.trip), T,
                                                    L.ptr(kg.slots), kg.capacity, start, cnt,
                                                    runner.seed, L.ptr(runner.epoch_key),
                                                    float(runner.model.margin), runner.ntries,
                                                    L.ptr(nviol), None, None), "sample_grad")
                e[1].record(st)
                L.check(lib.skge_accum_apply(sp, tabs if on(i - 1) else tabs0, 2,
                                             L.int_array(4 * cnt, cnt)), "apply")
                e[2].record(st)
            L.check(lib.skge_epoch_advance(sp, L.ptr(runner.epoch_key)), "advance")
    st.synchronize()
    elapsed = time.perf_counter() - t0
    runner.nviol_total.add_(nviol)
    n = len(ev)
    t_s = sum(e[0].elapsed_time(e[1]) for e in ev) * 1e3 / n
    t_a = sum(e[1].elapsed_time(e[2]) for e in ev) * 1e3 / n
    n_on = sum(1 for i in range(n) if on(i))
    U = (int(ucE.sum().item()) + int(ucR.sum().item())) / n_on
    b_s = sum(algorithmic_bytes(d, c, 2 * c, 0, 0) for _, c in batches) / len(batches)
    b_a = float(opt_k) * d * U
    if counters == "alt":
        t_on = sum(e[1].elapsed_time(e[2]) for i, e in enumerate(ev) if on(i)) * 1e3 / n_on
        t_off = sum(e[1].elapsed_time(e[2]) for i, e in enumerate(ev) if not on(i)) * 1e3 / (n - n_on)
        return elapsed, {"apply_us_counters": t_on, "apply_us_no_counters": t_off, "U": U}
    kern = {"transe_sample_grad": {"name": "transe_sample_grad", "avg_us": t_s, "launches": n,
                                   "bytes_per_launch": b_s,
                                   "achieved_gbs": b_s / (t_s * 1e-6) / 1e9},
            "accum_apply": {"name": "accum_apply", "avg_us": t_a, "launches": n,
                            "bytes_per_launch": b_a, "achieved_gbs": b_a / (t_a * 1e-6) / 1e9}}
    B = T / len(batches)
    return elapsed, {"kernels": kern, "dominant": max(kern.values(), key=lambda v: v["avg_us"]),
                     "epoch_bytes": (b_s + b_a) * len(batches),
                     "source": "HIP events between the kernels of the timed epochs (eager "
                               "launches of the epoch graph's sequence)",
                     "formula": {"launches_per_epoch": len(batches), "B": B, "P": 2 * B,
                                 "U_per_apply": U, "d": d, "k": opt_k,
                                 "expr": "sample_grad 4d(3B+P) + 20B; k_apply k d U"}}


def run_config5_sharded(args):
    """BASELINE.json configs[4] as named there: the |E|=50M x d=512 entity
    table (and its AdaGrad state) row-sharded over the ranks, R replicated,
    T=100M triples split over the ranks, B=131072 positives per rank per
    batch (global batch = G x 131072), TransE-L1 + AdaGrad, margin 2.0.
    The dataset and tables are fixed as G grows: scaling "strong"."""
    import torch
    import torch.distributed as dist
    world, rank, local, dev = setup_ranks()
    from skge_amd.shard import ShardedRunner, owned_rows
    n_ent, T = int(N5 * args.c5_scale), int(T5 * args.c5_scale)
    d, n_rel = D5, M5
    t_build = time.perf_counter()
    T_r = T // world + (1 if rank < T % world else 0)
    trip = make_config5_kg(n_ent, n_rel, T_r, dev, seed=rank)
    bnd = float(np.sqrt(6) / np.sqrt(n_ent + d))      # init_nunif of the FULL table
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    E = torch.empty((owned_rows(n_ent, world, rank), d), dtype=torch.float32, device=dev)
    E.uniform_(-bnd, bnd, generator=g)
    for r0 in range(0, E.shape[0], 1 << 20):            # TransE's post=normalize at init
        blk = E[r0:r0 + (1 << 20)]
        blk.div_(blk.norm(dim=1, keepdim=True))
    g.manual_seed(7)                                     # the same R on every rank
    R = torch.empty((n_rel, d), dtype=torch.float32, device=dev)
    R.uniform_(-float(np.sqrt(6) / np.sqrt(n_rel + d)), float(np.sqrt(6) / np.sqrt(n_rel + d)),
               generator=g)
    nb = max(1, T_r // B5)
    runner = ShardedRunner(n_ent, E, R, trip, nb, lr=0.1, margin=2.0, seed=99 + rank)
    del E, R
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t_build
    runner.run(args.warmup)
    runner.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.run(args.steps)
    runner.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, world, dev)
    value = T * args.steps / elapsed
    prof = shard_profile(runner, d)
    nviol = int(runner.nviol_total.item())
    if rank == 0:
        k = prof["dominant"]
        line = {
            "metric": "triples/sec (score+grad+update), synthetic TransE |E|=50M |R|=10k d=512, "
                      "table row-sharded over the GPUs (BASELINE configs[4])",
            "value": round(value, 1), "unit": "triples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic uniform KG (|E|=%d |R|=%d T=%d split over ranks, torch generator "
                    "seed rank); device-drawn nunif params" % (n_ent, n_rel, T),
            "config": {"workload": "TransE-L1 d=%d PairwiseStochasticTrainer+AdaGrad, margin 2.0, "
                                   "lr 0.1, device RandomModeSampler(1,[0,1]); E and AdaGrad state "
                                   "row-sharded (row %% G), R replicated; step = 1 epoch of %d "
                                   "batches of %d positives per rank" % (d, len(runner.batches), B5),
                       "global_batch": B5 * world, "parallelism": "rowshard%d" % world},
            "roofline": {"bound": "hbm", "kernel": k["name"],
                         "achieved": round(k["achieved_gbs"], 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(k["achieved_gbs"] / HBM_PEAK_GBS, 4),
                         "traffic": None, "bytes_per_launch": round(k["bytes_per_launch"]),
                         "avg_launch_us": round(k["avg_us"], 3)},
            "cpu_baseline": None if (args.no_cpu or world > 1) else
                            cpu_baseline_config5(args.cpu_seconds),   # N = 1 only
            "detail": {"runner": "row-sharded (skge_amd.shard)",
                       "bucket_capacity": runner.C,
                       "captured_graph": runner.graph is not None,
                       "build_s": round(t_build, 1),
                       "violations_per_pair": round(nviol / (2.0 * T_r * (args.warmup + args.steps)), 4),
                       "phases_ms_per_batch": {n: round(v, 4) for n, v in prof["phases_ms"].items()},
                       "kernels": {n: {"avg_us": round(v["avg_us"], 3),
                                       "GB_s": round(v["achieved_gbs"], 1)}
                                   for n, v in prof["kernels"].items()},
                       "gpu_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def shard_profile(runner, d, nbatch=6):
    """The phases of `nbatch` sharded steps (skge_amd.shard.sharded_step,
    replayed here eagerly with HIP events on the runner stream between
    phases; the collectives' time shows in the phases that wait for them) and
    the algorithmic bytes of each HIP kernel: route 52 B per positive (record +
    request ids + slots), gather 8d + 4 B per row served, score 20d + 20 B per
    positive (4 fetched rows + R row) + d + 16 B per contribution record + 2d
    per violating positive's R row, accum d + 20 B per record + 4d per
    non-empty record (packed sums read+written), apply 20d per applied row.
    Fixed-capacity layout: every all-to-all moves G x C slots."""
    import torch
    ops, ex, st = runner.ops, runner.ex, runner.stream
    names = ["route", "a2a_ids", "gather", "a2a_rows", "score", "a2a_contrib", "accum",
             "allreduce_R", "apply"]
    ms = {n: 0.0 for n in names}
    kb = {n: 0.0 for n in ("route", "gather", "score", "accum", "apply")}
    batches = [b for b in runner.batches if b[1] > 0][:nbatch]
    with torch.cuda.stream(st):
        runner.sample_epoch()
        for start, count in batches:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
            ev[0].record(st)
            send_ids, req_pos = ops.route(start, count)
            ev[1].record(st)
            recv_ids = ex.all_to_all(send_ids, ops.buf("recv_ids"))
            ev[2].record(st)
            rows = ops.gather(recv_ids)
            ev[3].record(st)
            fetched = ex.all_to_all(rows, ops.buf("fetched"))
            ev[4].record(st)
            contrib = ops.score(start, count, fetched, req_pos)
            ev[5].record(st)
            rc = ex.all_to_all(contrib, ops.buf("recv_contrib"))
            ev[6].record(st)
            ops.accum(recv_ids, rc)
            ev[7].record(st)
            for t in ops.rel_sums():
                ex.all_reduce_(t)
            ev[8].record(st)
            st.synchronize()
            valid = recv_ids >= 0
            nrecv = int(valid.sum().item())
            nsend = int((send_ids >= 0).sum().item())
            nz = int(((rc[:, :4].contiguous().view(torch.int32)[:, 0] > 0) & valid).sum().item())
            touched = int((runner.accE.cnt != 0).sum().item()) + int((runner.accR.cnt != 0).sum().item())
            ea = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ea[0].record(st)
            ops.apply()
            ea[1].record(st)
            st.synchronize()
            for i, n in enumerate(names):
                ms[n] += ea[0].elapsed_time(ea[1]) if n == "apply" else ev[i].elapsed_time(ev[i + 1])
            kb["route"] += 52.0 * count
            kb["gather"] += (8.0 * d + 4) * nrecv
            kb["score"] += (20.0 * d + 20) * count + (d + 16.0) * nsend + 2.0 * d * count
            kb["accum"] += (d + 20.0) * nrecv + 4.0 * d * nz
            kb["apply"] += 20.0 * d * touched
    n = max(len(batches), 1)
    kern = {}
    for k in kb:
        us = 1000.0 * ms[k] / n
        kern[k] = {"name": k, "avg_us": us, "bytes_per_launch": kb[k] / n,
                   "achieved_gbs": (kb[k] / n) / (us * 1e-6) / 1e9 if us > 0 else 0.0}
    return {"phases_ms": {k: v / n for k, v in ms.items()}, "kernels": kern,
            "dominant": max(kern.values(), key=lambda v: v["avg_us"])}


FP32_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: FP32 vector = FP32 matrix (MFMA) peak


def hole_positive_path(d):
    """The device pair loop runs HolE on k_hole_pos (one positive and both of
    its pairs per wave: 3 scores + 4 gradient correlations, computed for every
    positive) unless SKGE_HOLE_PAIRS=1 or d is outside its range."""
    return d % 4 == 0 and 4 <= d <= 256 and os.environ.get("SKGE_HOLE_PAIRS", "0") in ("", "0")


def model_flops(kind, d, P, V):
    """Algorithmic FLOPs of one batch of P pairs with V violators:
    HolE: 2 scoring correlations per pair + 6 gradient correlations per
    violating pair, 2d^2 each (direct form); on the per-positive path 2
    correlations per positive (A = ccorr(R, E[o]), B = ccorr(R, E[o']) score
    all three triples) + 2 per violating pair (3 for a positive whose second
    pair alone violates: counted as 2, a lower bound); RESCAL: W E_o for the 4 triples of
    a positive's 2 pairs, E_s W for the violators' entity gradients (computed
    for all 4 by the GEMM) and the 4 dW outer products: 24 d^2 per positive."""
    if kind == "hole":
        if hole_positive_path(d):   # k_hole_pos / k_hole_pipe
            return 2.0 * d * d * (2 * (P / 2.0) + 2 * V)
        return 2.0 * d * d * (2 * P + 6 * V)
    return 24.0 * d * d * (P / 2.0)


def run_config34(args):
    """BASELINE.json configs[2] / configs[3]: HolE (Sigmoid, margin 0.2) or
    RESCAL (Linear, margin 0.2) d=200, pairwise, AdaGrad lr 0.1, on the WN18
    shape at nb=100 -- whole epochs on the device pair loop (device sampler +
    explicit pairs + skge_pair_step per batch, one hipGraph per epoch)."""
    import torch
    import torch.distributed as dist
    world, rank, local, dev = setup_ranks()
    import skge_amd as S
    from skge_amd.device import DeviceKG, batch_sizes, make_runner
    kind = "hole" if args.config == 3 else "rescal"
    d, nb, margin = args.d, args.nb, 0.2
    trip = bench_kg(args, rank)
    np.random.seed(42 + rank)
    model = (S.HolE if kind == "hole" else S.RESCAL)((N_ENT, N_ENT, N_REL), d)
    model.add_hyperparam("margin", margin)
    upd = {pid: S.AdaGrad(p, 0.1) for pid, p in model.params.items()}
    kg = DeviceKG(trip, dev)
    runner = make_runner(model, upd, kg, nb, seed=1234 + rank, runner=args.runner)
    init = {pid: p.data.clone() for pid, p in model.params.items()}
    runner.run(args.warmup)
    runner.synchronize()
    for pid, p in model.params.items():
        p.data.copy_(init[pid])
        upd[pid].reset()
    runner.nviol_total.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.run(args.steps)
    runner.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(elapsed, world, dev)
    V = int(runner.nviol_total.item())
    value = replica_value(N_TRIPLES * args.steps, world, elapsed)
    P = 2 * N_TRIPLES * args.steps
    flops = model_flops(kind, d, P, V)
    tfs = flops / elapsed / 1e12 * world
    nl = runner.nlaunches
    rname = type(runner).__name__
    prof = None
    if kind == "hole" and getattr(runner, "pipelined", False):
        # the pipelined HolE runner's own counters over one more (eager) epoch;
        # the batch launches' time from the timed region's wall clock per epoch
        prof = pipe_profile(runner, kg, nb, d, gpu_ms_per_epoch=1000.0 * elapsed / args.steps,
                            hole=True)
    del runner
    large = None
    if args.large_nb > 0:
        # the same runner at a large batch (nb = 2: 70,721 positives per batch), where
        # the kernels are not latency-bound; starts from the initial parameters
        for pid, p in model.params.items():
            p.data.copy_(init[pid])
            upd[pid].reset()
        r2 = make_runner(model, upd, kg, args.large_nb, seed=1234 + rank, runner=args.runner)
        e2 = 3
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        r2.run(e2)
        r2.synchronize()
        torch.cuda.synchronize()
        t2 = time.perf_counter() - t2
        V2 = int(r2.nviol_total.item())
        f2 = model_flops(kind, d, 2 * N_TRIPLES * e2, V2)
        large = {"nbatches": args.large_nb, "batch": N_TRIPLES // args.large_nb,
                 "value": round(N_TRIPLES * e2 / t2, 1), "unit": "triples/s",
                 "ms_per_epoch": round(1000.0 * t2 / e2, 4),
                 "achieved_TFLOP_s": round(f2 / t2 / 1e12, 2),
                 "frac_of_peak": round(f2 / t2 / 1e12 / FP32_PEAK_TFS, 4),
                 "violations_per_pair": round(V2 / float(2 * N_TRIPLES * e2), 4),
                 "runner": type(r2).__name__}
        del r2
    if rank == 0:
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline(   # N = 1 only
            trip, d, nb, args.cpu_seconds, kind, margin)
        name = {"hole": "HolE", "rescal": "RESCAL"}[kind]
        tkern = "k_hole_pipe" if prof is not None else (
            "k_rescal_front" if kind == "rescal" else "k_hole")
        traffic, traffic_src = pmc_traffic(tkern, "pmc_c%d.json" % args.config)
        line = {
            "metric": "triples/sec (score+grad+update), WN18 %s d=%d pairwise, 1 MI355X "
                      "(BASELINE configs[%d])" % (name, d, args.config - 1) +
                      ("" if world == 1 else " -- %d independent replicas (weak; not one model: "
                       "no data-parallel runner for this model)" % world),
            "value": round(value, 1), "unit": "triples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": kg_label(args, "RandomState(rank)") + "; random-init params (nunif, seed 42)",
            "config": {"workload": "%s d=%d PairwiseStochasticTrainer+AdaGrad, %s, margin %g, "
                                   "lr 0.1, nb=%d (B=%d), device RandomModeSampler(1,[0,1]); "
                                   "step = 1 epoch on the device pair loop"
                                   % (name, d, "Sigmoid" if kind == "hole" else "Linear",
                                      margin, nb, N_TRIPLES // nb),
                       "global_batch": N_TRIPLES // nb,
                       "parallelism": "replicas%d" % world if world > 1 else "1gpu"},
            "roofline": ({"bound": "hbm", "kernel": "k_hole_pipe",
                          "achieved": round(prof["dominant"]["achieved_gbs"], 1),
                          "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(prof["dominant"]["achieved_gbs"] / HBM_PEAK_GBS, 4),
                          "traffic": None if traffic is None else round(traffic),
                          "traffic_source": traffic_src,
                          "bytes_per_launch": round(prof["dominant"]["bytes_per_launch"]),
                          "avg_launch_us": round(prof["dominant"]["avg_us"], 3),
                          "note": "row gathers, fp32 atomic rows (2.5 V lower bound) and "
                                  "applies, as config 2; the correlations run through the "
                                  "wave FFT (skge_hole_fft.h)"}
                         if prof is not None else
                         {"bound": "valu" if kind == "hole" else "mfma", "kernel": "whole step",
                          "achieved": round(tfs, 2), "peak": FP32_PEAK_TFS, "unit": "TFLOP/s",
                          "frac": round(tfs / FP32_PEAK_TFS, 4),
                          # HBM bytes per launch of the step's dominant kernel (rocprofv3 PMC)
                          "traffic": None if traffic is None else round(traffic),
                          "traffic_kernel": tkern, "traffic_source": traffic_src}),
            "cpu_baseline": cpu,
            "detail": {"violations_per_pair": round(V / float(P), 4),
                       "direct_form_TFLOP_s": round(tfs, 2),   # model_flops at the timed rate
                       "graph_nodes_per_step": nl,
                       "runner": rname,
                       "batches": len(batch_sizes(N_TRIPLES, nb)),
                       "large_batch": large},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def kernel_profile(model, upd, kg, nb, d, st, runner, opt_k=12):
    """Launch one epoch eagerly with HIP events around every kernel (on the
    stream the kernels run on) and count the algorithmic bytes of each launch
    from the touched-row counts."""
    import torch
    from skge_amd import _lib as L
    lib = L.lib()
    dev = model.device
    te, tr = runner.te, runner.tr
    tabs = (L.SkgeTable * 2)(te, tr)
    nviol = torch.zeros(1, dtype=torch.int32, device=dev)
    T = kg.T
    bs = T // nb
    sp = L.stream_ptr(st)
    times = {"transe_sample_grad": [], "accum_apply": []}
    bytes_ = {"transe_sample_grad": 0.0, "accum_apply": 0.0}     # SURVEY 8(d) share
    impl = {"transe_sample_grad": 0.0, "accum_apply": 0.0}       # implementation bytes
    total = 0.0
    accE, accR = runner.accE, runner.accR
    with torch.cuda.stream(st):
        for start in range(0, T, bs):
            cnt = min(bs, T - start)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            nviol.zero_()
            e[0].record(st)
            L.check(lib.skge_transe_sample_grad(sp, 1, te, tr, d, L.ptr(kg.trip), T, L.ptr(kg.slots),
                                                kg.capacity, start, cnt, 777, L.ptr(runner.epoch_key),
                                                2.0, 100, L.ptr(nviol), None, None))
            e[1].record(st)
            st.synchronize()
            UE = int((accE.cnt != 0).sum().item())
            UR = int((accR.cnt != 0).sum().item())
            V = int(nviol.item())
            e[2].record(st)
            L.check(lib.skge_accum_apply(sp, tabs, 2, L.int_array(4 * cnt, cnt)))
            e[3].record(st)
            st.synchronize()
            times["transe_sample_grad"].append(e[0].elapsed_time(e[1]) * 1e3)
            times["accum_apply"].append(e[2].elapsed_time(e[3]) * 1e3)
            P = 2 * cnt
            impl["transe_sample_grad"] += _score_bytes(d, cnt, V, runner.packed)
            impl["accum_apply"] += _apply_bytes(d, UE + UR, runner.packed)
            # 8(d): the gathers + indices are the scoring kernel's, k d U the apply's
            bytes_["transe_sample_grad"] += algorithmic_bytes(d, cnt, P, 0, 0)
            bytes_["accum_apply"] += float(opt_k) * d * (UE + UR)
            total += algorithmic_bytes(d, cnt, P, UE, UR, opt_k)
    kern = {}
    for n in times:
        t = np.array(times[n])
        avg = float(t.mean())
        bpl = bytes_[n] / len(t)
        ipl = impl[n] / len(t)
        kern[n] = {"name": n, "avg_us": avg, "launches": len(t), "bytes_per_launch": bpl,
                   "achieved_gbs": bpl / (avg * 1e-6) / 1e9, "impl_bytes_per_launch": ipl,
                   "impl_gbs": ipl / (avg * 1e-6) / 1e9}
    dom = max(kern.values(), key=lambda v: v["avg_us"])
    return {"kernels": kern, "dominant": dom, "epoch_bytes": total}


if __name__ == "__main__":
    main()
