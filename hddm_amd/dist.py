"""Multi-GPU plumbing: one process per GPU, RCCL over xGMI for the exchange.

The likelihood shards trivially (trials are independent): each
rank keeps a contiguous trial range resident and the only exchange is one
3-double ncclAllReduce of {sum log p, #zero-density trials, status} per call,
done inside libwfpt_amd (wfpt_wiener_like_allreduce). torch.distributed (gloo, on
the host) is used only to broadcast RCCL's 128-byte unique id and for
barriers / max-over-ranks timing in bench.py.
"""
import ctypes

import numpy as np

from . import _lib


def shard_range(n, world, rank):
    """Contiguous [lo, hi) of n trials for `rank` (wfpt_shard_range in the C ABI)."""
    return _lib.shard_range(n, world, rank)


def combine(partials):
    """Reference semantics of a sharded wiener_like (wfpt.pyx:66-76): any
    zero-density trial anywhere => -inf; otherwise the sum (NaN propagates).
    partials: iterable of (sum_logp_without_zero_trials, n_zero_trials)."""
    s, z = 0.0, 0
    for ps, pz in partials:
        s += ps
        z += int(pz)
    return -np.inf if z > 0 else s


def init_comm(ctx, rank, world, pg=None):
    """Create the RCCL communicator of `ctx` for (rank, world). The unique id is
    made on rank 0 and broadcast over the torch.distributed (gloo) group."""
    import torch.distributed as dist
    if world == 1:
        uid = ctypes.create_string_buffer(128)
        _lib.check(_lib.wfpt_comm_unique_id(uid))
        _lib.check(_lib.wfpt_comm_init(ctx.handle, 1, 0, uid))
        return
    obj = [None]
    if rank == 0:
        uid = ctypes.create_string_buffer(128)
        _lib.check(_lib.wfpt_comm_unique_id(uid))
        obj[0] = bytes(uid.raw)
    dist.broadcast_object_list(obj, src=0, group=pg)
    buf = ctypes.create_string_buffer(obj[0], 128)
    _lib.check(_lib.wfpt_comm_init(ctx.handle, int(world), int(rank), buf))
