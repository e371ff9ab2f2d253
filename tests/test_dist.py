"""world_size-2 gloo test of the sharded likelihood's host logic (CPU).

Each rank takes its contiguous shard (hddm_amd.dist.shard_range, the C ABI's
wfpt_shard_range), computes its {sum log p, #zero trials} partial with the
oracle (standing in for the per-GPU kernel, which needs a device), and the two
partials are all-reduced over gloo exactly as libwfpt_amd all-reduces them
over RCCL. The combined value must equal the unsharded reference likelihood.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, x, args, kn, out_q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import oracle
    from hddm_amd import dist as hdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = hdist.shard_range(x.size, world, rank)
    lp = oracle.pdf_array(x[lo:hi], *args, kn[0], 1, *kn[1:])
    zeros = int(np.isneginf(lp).sum())
    s = math.fsum(lp[np.isfinite(lp)]) if zeros == 0 else 0.0
    t = torch.tensor([s, float(zeros)], dtype=torch.float64)
    dist.all_reduce(t)  # the {sum, zeros} part of RCCL's 3-double sum in wfpt_wiener_like_allreduce
    total = -math.inf if t[1].item() > 0 else t[0].item()
    out_q.put((rank, total, hi - lo))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("inject_zero", [False, True])
def test_two_rank_allreduce_matches_unsharded(oracle_lib, inject_zero):
    rng = np.random.default_rng(1)
    x = rng.choice([-1.0, 1.0], 3001) * (0.35 + rng.gamma(2.0, 0.4, 3001))
    if inject_zero:
        x[2900] = 0.1  # below t - st/2: zero density on rank 1 only
    args = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.0, 0.1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, x, args, kn, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = oracle_lib.wiener_like(x, *args, *kn)
    assert sum(r[2] for r in res) == x.size
    for _, total, _ in res:
        if inject_zero:
            assert total == -math.inf and ref == -math.inf
        else:
            assert abs(total - ref) < 1e-9 * abs(ref)


@pytest.mark.gpu
def test_rccl_single_rank_allreduce_path(gpu, oracle_lib):
    """The RCCL path of wfpt_wiener_like_allreduce on one GPU (world 1): the
    3-double all-reduce must leave the local result unchanged, including the
    zero-trial (-inf) semantics."""
    from hddm_amd import _lib, dist as hdist
    ctx = _lib.context()
    hdist.init_comm(ctx, 0, 1)
    rng = np.random.default_rng(3)
    x = rng.choice([-1.0, 1.0], 50_000) * (0.35 + rng.gamma(2.0, 0.4, 50_000))
    args = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    ds = gpu.Dataset(x)
    a = ds.wiener_like_allreduce(*args, *kn)
    b = ds.wiener_like(*args, *kn)
    assert a == b
    ref = oracle_lib.pdf_array(x, *args, kn[0], 1, *kn[1:])
    assert abs(a - math.fsum(ref)) < 1e-11 * math.fsum(np.abs(ref))
    x[17] = 0.1
    ds0 = gpu.Dataset(x)
    assert ds0.wiener_like_allreduce(*args, 1e-4, 2, 2, 1, 1e-3, 0.0, 0.1) == -math.inf
