"""Multi-GPU plumbing: trials sharded over GPUs, RCCL over xGMI for the exchange.

The likelihood shards trivially (trials are independent): each
GPU keeps a contiguous trial range resident and the only exchange is one
3-double ncclAllReduce of {sum log p, #zero-density trials, encoded errors}
per call, done inside libwfpt_amd. No PyTorch anywhere in this module:

* one process per GPU (`init_comm`): the RCCL unique id goes from rank 0 to
  the other ranks over the library's own TCP rendezvous
  (wfpt_comm_init_tcp: rank 0 listens on host:port);
* one process driving several GPUs, e.g. a single PyMC sampler (`Group`):
  ncclCommInitAll over the devices and grouped all-reduces
  (wfpt_comm_init_all / wfpt_wiener_like_allreduce_group).
"""
import ctypes
import os

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


def rendezvous_address():
    """(host, port) of the unique-id rendezvous: $WFPT_COMM_ADDR /
    $WFPT_COMM_PORT, else $MASTER_ADDR and $MASTER_PORT + 1 (the launcher's
    own store keeps MASTER_PORT), else 127.0.0.1:29511."""
    host = os.environ.get("WFPT_COMM_ADDR") or os.environ.get("MASTER_ADDR") or "127.0.0.1"
    port = os.environ.get("WFPT_COMM_PORT")
    if port is None:
        mp = os.environ.get("MASTER_PORT")
        port = int(mp) + 1 if mp else 29511
    return host, int(port)


def exchange_id(rank, world, uid=None, host=None, port=None, timeout_s=120.0):
    """The TCP rendezvous alone (wfpt_comm_exchange_id; no GPU involved):
    rank 0 passes its 128-byte id, every rank returns it."""
    h, p = rendezvous_address()
    host = host or h
    port = port or p
    buf = ctypes.create_string_buffer(bytes(uid) if uid is not None else b"", 128)
    _lib.check(_lib.wfpt_comm_exchange_id(int(world), int(rank), host.encode(), int(port),
                                          int(timeout_s * 1000), buf))
    return bytes(buf.raw)


def init_comm(ctx, rank, world, host=None, port=None, timeout_s=120.0):
    """RCCL communicator of `ctx` for (rank, world), one process per GPU. The
    unique id is made on rank 0 and reaches the other ranks over the
    library's TCP rendezvous (rendezvous_address())."""
    if world == 1:
        uid = ctypes.create_string_buffer(128)
        _lib.check(_lib.wfpt_comm_unique_id(uid))
        _lib.check(_lib.wfpt_comm_init(ctx.handle, 1, 0, uid))
        return
    h, p = rendezvous_address()
    _lib.check(_lib.wfpt_comm_init_tcp(ctx.handle, int(world), int(rank), (host or h).encode(),
                                       int(port or p), int(timeout_s * 1000)))


class Group:
    """One process driving several GPUs: one context and one resident shard
    per device, one communicator per device from ncclCommInitAll, and the
    global likelihood from one grouped all-reduce per call."""

    def __init__(self, devices):
        self.contexts = [_lib.context(d) for d in devices]
        n = len(self.contexts)
        self._handles = (_lib._VP * n)(*[c.handle for c in self.contexts])
        _lib.check(_lib.wfpt_comm_init_all(self._handles, n))

    def shards(self, x):
        """Resident shards of the signed RTs x, contiguous ranges in device
        order (hddm_amd.wfpt.Dataset per device)."""
        from .wfpt import Dataset
        x = np.ascontiguousarray(x, dtype=np.float64)
        n = len(self.contexts)
        out = []
        for r, c in enumerate(self.contexts):
            lo, hi = shard_range(x.size, n, r)
            out.append(Dataset(x[lo:hi], device=c.device))
        return out

    def wiener_like(self, shards, v, sv, a, z, sz, t, st, err, n_st=10, n_sz=10,
                    use_adaptive=1, simps_err=1e-8, p_outlier=0, w_outlier=0.1):
        """wiener_like over the union of the shards (wfpt.pyx:54-76 semantics)."""
        n = len(self.contexts)
        if len(shards) != n:
            raise ValueError("one shard per device")
        ds = (_lib._VP * n)(*[s.handle for s in shards])
        P = _lib.make_params(v, sv, a, z, sz, t, st, p_outlier)
        K = _lib.make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier)
        out = _lib._D()
        _lib.check(_lib.wfpt_wiener_like_allreduce_group(self._handles, ds, n, ctypes.byref(P),
                                                         ctypes.byref(K), ctypes.byref(out)))
        return out.value
