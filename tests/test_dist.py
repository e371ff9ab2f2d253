"""world_size-2 gloo tests of the sharded likelihood's combine (CPU).

Each rank takes its contiguous shard (hddm_amd.dist.shard_range, the C ABI's
wfpt_shard_range), computes its {sum log p, #zero trials, encoded errors}
triple with the oracle (standing in for the per-GPU kernels, which need a
device), the triples are summed over gloo exactly as libwfpt_amd sums them
over RCCL, and the library's own decode (wfpt_decode_result) turns the sum into
the value or the error every rank reports.
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


def _worker(rank, world, port, x, args, kn, inject, out_q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import oracle
    from hddm_amd import _lib
    from hddm_amd import dist as hdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = hdist.shard_range(x.size, world, rank)
    lp = oracle.pdf_array(x[lo:hi], *args, kn[0], 1, *kn[1:])
    zeros = int(np.isneginf(lp).sum())
    s = math.fsum(lp[np.isfinite(lp)])
    # this rank's {sum, zeros, encoded errors} triple, as finalize_kernel writes
    # it; the sum over ranks is what wfpt_wiener_like_allreduce's ncclAllReduce does
    err = inject.get(rank, 0.0)
    t = torch.tensor([s, float(zeros), err], dtype=torch.float64)
    dist.all_reduce(t)
    try:
        res = ("ok", _lib.decode_result(t.tolist()))  # the library's decode
    except NotImplementedError as e:
        res = ("error", str(e))
    out_q.put((rank, res, hi - lo))
    dist.barrier()
    dist.destroy_process_group()


def _run(x, args, kn, inject):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, x, args, kn, inject, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(r[2] for r in res) == x.size
    return [r[1] for r in res]


@pytest.mark.parametrize("inject_zero", [False, True])
def test_two_rank_allreduce_matches_unsharded(oracle_lib, inject_zero):
    """World-2 gloo: shard, per-rank triple, sum over ranks, the library's
    decode. Equals the unsharded reference; a zero-density trial on one rank
    gives -inf on every rank (wfpt.pyx:71-72)."""
    rng = np.random.default_rng(1)
    x = rng.choice([-1.0, 1.0], 3001) * (0.35 + rng.gamma(2.0, 0.4, 3001))
    if inject_zero:
        x[2900] = 0.1  # below t - st/2: zero density on rank 1 only
    args = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.0, 0.1)
    res = _run(x, args, kn, {})
    ref = oracle_lib.wiener_like(x, *args, *kn)
    for kind, total in res:
        assert kind == "ok"
        if inject_zero:
            assert total == -math.inf and ref == -math.inf
        else:
            assert abs(total - ref) < 1e-9 * abs(ref)


@pytest.mark.parametrize("inject,want", [
    ({0: 1.0}, ["WFPT_MAX_DEPTH"]),                          # depth error on rank 0 only
    ({0: 1.0, 1: 1.0}, ["WFPT_MAX_DEPTH"]),                  # on both: still depth, not budget
    ({1: 1048576.0}, ["WFPT_EVAL_BUDGET"]),                  # budget error on rank 1
    ({0: 1.0, 1: 1048576.0}, ["WFPT_MAX_DEPTH", "WFPT_EVAL_BUDGET"]),
])
def test_two_rank_error_propagation(inject, want):
    """A depth / budget failure on any rank fails every rank, and the two kinds
    stay distinguishable after the sum over ranks (summed bit flags
    made two depth errors read as a budget error)."""
    rng = np.random.default_rng(2)
    x = rng.choice([-1.0, 1.0], 500) * (0.35 + rng.gamma(2.0, 0.4, 500))
    res = _run(x, (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0), (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1), inject)
    for kind, msg in res:
        assert kind == "error"
        for w in want:
            assert w in msg
        for w in {"WFPT_MAX_DEPTH", "WFPT_EVAL_BUDGET"} - set(want):
            assert w not in msg


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


@pytest.mark.gpu
def test_rccl_allreduce_call_sequences(gpu):
    """Repeated all-reduce calls take the predicted sequences (lean level-0
    pass + unconditional redo pass once the dataset's last call refined
    nothing in-wave): bitwise the local wiener_like result, also when a call
    with refining parameters follows non-refining ones (redo inside the same
    launch sequence, no host round trip before the exchange)."""
    from hddm_amd import _lib, dist as hdist
    ctx = _lib.context()
    hdist.init_comm(ctx, 0, 1)
    np.random.seed(4)
    calm = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    heavy = (1.7431, 2.0137, 0.6119, 0.5386, 0.2108, 0.3567, 0.1981)
    x = gpu.gen_rts_from_cdf(*heavy, samples=100_000, dt=1e-3)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    ds = gpu.Dataset(x)
    ref_calm = gpu.Dataset(x).wiener_like(*calm, *kn)
    ref_heavy = gpu.Dataset(x).wiener_like(*heavy, *kn)
    seq = [calm, calm, calm, heavy, heavy, calm, calm, heavy]
    for p in seq:
        got = ds.wiener_like_allreduce(*p, *kn)
        assert got == (ref_calm if p is calm else ref_heavy), p
