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


def _master_store():
    """A TCPStore master held by the test process on a port the OS assigned
    and that stays bound (a probed-then-released port can be taken by another
    socket before a rank binds it: EADDRINUSE); the ranks join it as clients.
    Returns (store, port); keep the store alive until the ranks have joined."""
    import torch.distributed as dist
    store = dist.TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False)
    return store, store.port


def _init_pg(rank, world, port):
    """A rank joins the test process's store (_master_store) and forms the
    gloo group through it."""
    import datetime
    import torch.distributed as dist
    store = dist.TCPStore("127.0.0.1", port, is_master=False,
                          timeout=datetime.timedelta(seconds=60))
    dist.init_process_group("gloo", store=store, rank=rank, world_size=world)


def _worker(rank, world, port, x, args, kn, inject, out_q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import oracle
    from hddm_amd import _lib
    from hddm_amd import dist as hdist
    _init_pg(rank, world, port)
    lo, hi = hdist.shard_range(x.size, world, rank)
    lp = oracle.pdf_array(x[lo:hi], *args, kn[0], 1, *kn[1:])
    zeros = int(np.isneginf(lp).sum())
    s = math.fsum(lp[np.isfinite(lp)])
    # this rank's {sum, zeros, encoded errors} triple, as finalize_kernel writes
    # it; the sum over ranks is what wfpt_wiener_like_allreduce's ncclAllReduce does
    err = inject.get(rank, 0.0)
    if err == "fail":
        # this rank's local pass failed: it still enters the exchange, with
        # the library's poisoned triple (wfpt_wiener_like_allreduce does the
        # same before its ncclAllReduce)
        triple = _lib.poisoned_result()
    else:
        triple = [s, float(zeros), err]
    t = torch.tensor(triple, dtype=torch.float64)
    dist.all_reduce(t)
    try:
        res = ("ok", _lib.decode_result(t.tolist()))  # the library's decode
    except NotImplementedError as e:
        res = ("error", str(e))
    except _lib.CommError as e:
        res = ("comm", str(e))
    out_q.put((rank, res, hi - lo))
    dist.barrier()
    dist.destroy_process_group()


def _device_worker(rank, world, port, x, args, kn, seq, out_q):
    """A rank whose triple is the library's own: its contiguous shard resident
    on the GPU and wfpt_wiener_like_local (the triple wiener_like_allreduce
    puts into its ncclAllReduce), summed over gloo, decoded by the library."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from hddm_amd import _lib, wfpt
    from hddm_amd import dist as hdist
    _init_pg(rank, world, port)
    lo, hi = hdist.shard_range(x.size, world, rank)
    ds = wfpt.Dataset(x[lo:hi])
    res = []
    for p in seq:  # lean / engine / mispredicted sequences on each rank's own history
        triple = ds.local_triple(*p, *kn)
        t = torch.tensor(triple, dtype=torch.float64)
        dist.all_reduce(t)
        res.append(_lib.decode_result(t.tolist()))
    out_q.put((rank, res, hi - lo))
    ds.close()
    dist.barrier()
    dist.destroy_process_group()


def _run(x, args, kn, inject, worker=None, extra=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store, port = _master_store()
    if worker is None:
        worker, extra = _worker, inject
    procs = [ctx.Process(target=worker, args=(r, 2, port, x, args, kn, extra, q))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
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


@pytest.mark.parametrize("inject", [{1: "fail"}, {0: "fail", 1: "fail"}, {0: "fail", 1: 1.0}])
def test_two_rank_local_failure_before_exchange(inject):
    """A rank whose local pass fails still enters the exchange with the
    poisoned triple: every rank decodes an error (none waits in the
    collective, none returns a number), the failed-rank count survives the
    sum, and a depth error elsewhere is still reported next to it."""
    rng = np.random.default_rng(7)
    x = rng.choice([-1.0, 1.0], 400) * (0.35 + rng.gamma(2.0, 0.4, 400))
    res = _run(x, (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0), (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1), inject)
    nfail = sum(1 for v in inject.values() if v == "fail")
    depth = any(v == 1.0 for v in inject.values())
    for kind, msg in res:
        assert kind == ("error" if depth else "comm"), (kind, msg)
        assert f"{nfail} rank(s) failed before the likelihood exchange" in msg
        assert ("WFPT_MAX_DEPTH" in msg) == depth


_RDV_CHILD = r"""
import sys, json
sys.path.insert(0, sys.argv[1])
from hddm_amd import dist as hdist
rank, world, port, uid = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), bytes.fromhex(sys.argv[5])
got = hdist.exchange_id(rank, world, uid=uid if rank == 0 else None, host="127.0.0.1",
                        port=port, timeout_s=60)
print(json.dumps({"id": got.hex(), "torch": "torch" in sys.modules}))
"""


@pytest.mark.parametrize("world", [2, 3])
def test_tcp_rendezvous_hands_rank0_id_to_every_rank(world):
    """The library's torch-free unique-id exchange (wfpt_comm_exchange_id,
    used by wfpt_comm_init_tcp): every rank receives rank 0's 128 bytes, in
    plain processes that never import torch."""
    import json
    import subprocess
    import sys
    port = _free_port()
    uid = bytes(np.random.default_rng(world).integers(0, 256, 128, dtype=np.uint8))
    procs = [subprocess.Popen([sys.executable, "-c", _RDV_CHILD, ROOT, str(r), str(world),
                               str(port), uid.hex()], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True)
             for r in reversed(range(world))]  # peers first: they retry until rank 0 listens
    outs = [p.communicate(timeout=120) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
        r = json.loads(o.strip().splitlines()[-1])
        assert bytes.fromhex(r["id"]) == uid
        assert r["torch"] is False


def test_tcp_rendezvous_survives_silent_and_foreign_clients():
    """rank 0 serves its peer although a client that connects and
    never speaks, and one that sends a valid-looking hello with another job
    token, reach it first: the silent one is dropped after its per-connection
    budget (well before the deadline), the foreign one is ignored, and the
    real peer (same WFPT_COMM_TOKEN) gets rank 0's id."""
    import json
    import socket
    import struct
    import subprocess
    import sys
    import time
    port = _free_port()
    uid = bytes(range(128))
    env = dict(os.environ, WFPT_COMM_TOKEN="job-a")
    p0 = subprocess.Popen([sys.executable, "-c", _RDV_CHILD, ROOT, "0", "2", str(port), uid.hex()],
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    t0 = time.time()
    silent = None
    while silent is None and time.time() - t0 < 60:
        try:
            silent = socket.create_connection(("127.0.0.1", port), timeout=1)
        except OSError:
            time.sleep(0.05)
    assert silent is not None
    foreign = socket.create_connection(("127.0.0.1", port), timeout=5)
    foreign.sendall(struct.pack("<4I", 0x77667074, 2, 1, 12345))
    p1 = subprocess.Popen([sys.executable, "-c", _RDV_CHILD, ROOT, "1", "2", str(port), uid.hex()],
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
    outs = [p.communicate(timeout=120) for p in (p0, p1)]
    for p, (o, e) in zip((p0, p1), outs):
        assert p.returncode == 0, e
        assert bytes.fromhex(json.loads(o.strip().splitlines()[-1])["id"]) == uid
    assert time.time() - t0 < 40  # not held until the 60 s deadline
    foreign.settimeout(1)
    try:
        got = foreign.recv(128)
    except OSError:
        got = b""
    assert got == b""  # the foreign hello never received the id
    silent.close()
    foreign.close()


def test_tcp_rendezvous_times_out_without_rank0():
    """A peer whose rank 0 never shows up fails with an error naming the
    rendezvous (no hang past its deadline)."""
    from hddm_amd import _lib, dist as hdist
    with pytest.raises(_lib.CommError, match="rendezvous"):
        hdist.exchange_id(1, 2, host="127.0.0.1", port=_free_port(), timeout_s=0.5)


def test_product_modules_do_not_import_torch():
    """North_star: the product path has no PyTorch (the multi-GPU plumbing
    included); bench.py and the tests may use it as harness."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import hddm_amd, hddm_amd.wfpt, hddm_amd.dist, hddm_amd.likelihoods, "
            "hddm_amd.hierarchical, hddm_amd.integration, hddm_amd.cdfdif_wrapper\n"
            "print('torch' in sys.modules)" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"


@pytest.mark.gpu
def test_rccl_local_failure_enters_exchange_and_recovers(gpu, monkeypatch):
    """On the GPU through RCCL (world 1): a local failure (injected after the
    local pass) still runs the collective with the poisoned triple and
    returns the rank's own error; the communicator and the dataset stay usable
    and the next call gives the local result bit for bit."""
    from hddm_amd import _lib, dist as hdist
    ctx = _lib.context()
    hdist.init_comm(ctx, 0, 1)
    rng = np.random.default_rng(8)
    x = rng.choice([-1.0, 1.0], 20_000) * (0.35 + rng.gamma(2.0, 0.4, 20_000))
    args = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    ds = gpu.Dataset(x)
    ref = ds.wiener_like(*args, *kn)
    monkeypatch.setenv("WFPT_FAULT", "allreduce_local")
    with pytest.raises(RuntimeError, match="injected local failure"):
        ds.wiener_like_allreduce(*args, *kn)
    monkeypatch.delenv("WFPT_FAULT")
    assert ds.wiener_like_allreduce(*args, *kn) == ref


@pytest.mark.gpu
def test_single_process_group_allreduce(gpu, oracle_lib):
    """The single-process multi-GPU API (ncclCommInitAll + grouped
    all-reduce) over the devices this box has: equals the
    unsharded reference total."""
    from hddm_amd import _lib, dist as hdist
    nd = min(_lib.device_count(), 8)
    grp = hdist.Group(list(range(nd)))
    rng = np.random.default_rng(9)
    x = rng.choice([-1.0, 1.0], 30_001) * (0.35 + rng.gamma(2.0, 0.4, 30_001))
    args = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    shards = grp.shards(x)
    assert sum(len(s) for s in shards) == x.size
    ref = oracle_lib.pdf_array(x, *args, kn[0], 1, *kn[1:])
    for _ in range(3):  # lean prediction from the second call on
        got = grp.wiener_like(shards, *args, *kn)
        assert abs(got - math.fsum(ref)) < 1e-11 * math.fsum(np.abs(ref))
    x2 = x.copy()
    x2[-1] = 0.1  # zero density on the last shard
    assert grp.wiener_like(grp.shards(x2), *args, 1e-4, 2, 2, 1, 1e-3, 0.0, 0.1) == -math.inf


@pytest.mark.gpu
def test_two_rank_gloo_with_device_triples(gpu, oracle_lib):
    """World-2 gloo on the single-GPU lease, each rank a process with its own
    context on the device: the per-rank triple is the library's (its shard's
    level-0 / engine / redo passes and finalize, wfpt_wiener_like_local), not
    the oracle's. The decoded sum equals the unsharded reference on every rank
    for a call sequence that takes the lean prediction, a misprediction onto
    refining parameters and back, and a zero-density trial (-inf)."""
    np.random.seed(12)
    calm = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)
    heavy = (1.7431, 2.0137, 0.6119, 0.5386, 0.2108, 0.3567, 0.1981)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
    x = gpu.gen_rts_from_cdf(*heavy, samples=60_001, dt=1e-3)
    seq = [calm, calm, heavy, heavy, calm]
    res = _run(x, None, kn, None, worker=_device_worker, extra=seq)
    for r, p in enumerate(seq):
        terms = oracle_lib.pdf_array(x, *p, kn[0], 1, *kn[1:])
        ref = math.fsum(terms)
        for got in res:
            assert abs(got[r] - ref) <= 1e-11 * math.fsum(np.abs(terms)), (r, got[r], ref)
    x0 = x.copy()
    x0[-5] = 0.05  # below t - st/2 on rank 1: -inf everywhere
    kn0 = kn[:5] + (0.0, 0.1)  # p_outlier 0: a zero Wiener density is a zero mixture density
    res0 = _run(x0, None, kn0, None, worker=_device_worker, extra=[calm])
    assert all(g[0] == -math.inf for g in res0)


def _node_worker(rank, world, port, x, node, params, kn, out_q):
    """A rank of the hierarchical-mode exchange: its contiguous trial shard as
    a node dataset with the global node ids, the library's per-node partial
    sums (wfpt_wiener_like_nodes_local), summed over gloo."""
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from hddm_amd import _lib, wfpt
    from hddm_amd import dist as hdist
    _init_pg(rank, world, port)
    lo, hi = hdist.shard_range(x.size, world, rank)
    ds = wfpt.Dataset(x[lo:hi], node_id=node[lo:hi], n_nodes=params.shape[0])
    v = torch.tensor(ds.wiener_like_nodes_local(params, *kn), dtype=torch.float64)
    dist.all_reduce(v)
    v = v.numpy()
    if v[-1] != 0:
        _lib.decode_result([0.0, 0.0, float(v[-1])])
    out_q.put((rank, v[:-1], hi - lo))
    ds.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_gloo_node_sums(gpu, oracle_lib):
    """Hierarchical mode across ranks (count = n_nodes): two
    processes on the device, each with a contiguous shard of a 61-node dataset
    (node 30 split between the ranks), their per-node partial sums summed over
    gloo equal the unsharded per-node sums and the reference's per-node fsum;
    a zero-density trial in a split node makes that node -inf on every rank."""
    rng = np.random.default_rng(14)
    m, per = 61, 150  # 9150 trials: the shard boundary 4575 splits node 30
    node = np.repeat(np.arange(m, dtype=np.int32), per)
    x = rng.choice([-1.0, 1.0], node.size) * (0.34 + rng.gamma(2.0, 0.4, node.size))
    params = np.tile([0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.05], (m, 1))
    params[:, 0] += 0.02 * np.arange(m)
    kn = (1e-4, 2, 2, 1, 1e-3, 0.1)
    want = gpu.Dataset(x, node_id=node, n_nodes=m).wiener_like_nodes(params, *kn)
    for xx, zero in ((x, False), (np.where(np.arange(x.size) == 4520, 0.05, x), True)):
        pz = params.copy()
        if zero:
            pz[:, 7] = 0.0  # no outlier mass: the zero density is -inf
            want = gpu.Dataset(xx, node_id=node, n_nodes=m).wiener_like_nodes(pz, *kn)
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        store, port = _master_store()
        procs = [ctx.Process(target=_node_worker, args=(r, 2, port, xx, node, pz, kn, q))
                 for r in range(2)]
        for p in procs:
            p.start()
        res = [q.get(timeout=100) for _ in procs]
        for p in procs:
            p.join(timeout=30)
            assert p.exitcode == 0
        for _, got, _ in res:
            fin = np.isfinite(want)
            assert np.array_equal(np.isneginf(got), np.isneginf(want))
            assert np.all(np.abs(got[fin] - want[fin]) <= 1e-11 * np.abs(want[fin]))
        if zero:
            assert np.isneginf(want[4520 // per])
        else:
            for j in (0, 30, 60):
                terms = oracle_lib.pdf_array(xx[node == j], *pz[j, :7], kn[0], 1, kn[1], kn[2],
                                             kn[3], kn[4], pz[j, 7], kn[5], n_threads=4)
                assert abs(want[j] - math.fsum(terms)) <= 1e-11 * math.fsum(np.abs(terms))


@pytest.mark.gpu
def test_rccl_single_rank_node_allreduce(gpu):
    """wfpt_wiener_like_nodes_allreduce over world-1 RCCL equals
    wiener_like_nodes bit for bit (one all-reduce of n_nodes + 1 doubles)."""
    from hddm_amd import _lib, dist as hdist
    ctx = _lib.context()
    hdist.init_comm(ctx, 0, 1)
    rng = np.random.default_rng(15)
    m = 40
    node = rng.integers(0, m, 8000).astype(np.int32)
    x = rng.choice([-1.0, 1.0], node.size) * (0.34 + rng.gamma(2.0, 0.4, node.size))
    params = np.tile([0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.05], (m, 1))
    ds = gpu.Dataset(x, node_id=node, n_nodes=m)
    a = ds.wiener_like_nodes(params)
    b = ds.wiener_like_nodes_allreduce(params)
    assert np.array_equal(a, b)


@pytest.mark.gpu
def test_rccl_node_allreduce_failure_paths(gpu, monkeypatch):
    """the node all-reduce's failure paths on world-1 RCCL. A
    local failure injected after the per-node pass was enqueued
    (WFPT_FAULT=nodes_allreduce_local) and a dataset whose node count differs
    from the call's n_nodes both enter the exchange poisoned (node_poison_kernel,
    node_status_kernel with poison) with the call's count, decode the
    failure and return the rank's own error; the communicator stays usable
    and the next call equals wiener_like_nodes bit for bit."""
    import ctypes
    from hddm_amd import _lib, dist as hdist
    ctx = _lib.context()
    hdist.init_comm(ctx, 0, 1)
    rng = np.random.default_rng(16)
    m = 24
    node = rng.integers(0, m, 5000).astype(np.int32)
    x = rng.choice([-1.0, 1.0], node.size) * (0.34 + rng.gamma(2.0, 0.4, node.size))
    params = np.tile([0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.05], (m, 1))
    params[:, 0] += 0.01 * np.arange(m)
    ds = gpu.Dataset(x, node_id=node, n_nodes=m)
    want = ds.wiener_like_nodes(params)
    monkeypatch.setenv("WFPT_FAULT", "nodes_allreduce_local")
    with pytest.raises(RuntimeError, match="injected local failure"):
        ds.wiener_like_nodes_allreduce(params)
    monkeypatch.delenv("WFPT_FAULT")
    assert np.array_equal(ds.wiener_like_nodes_allreduce(params), want)
    # a count that disagrees with the dataset: WFPT_ERR_ARG after the exchange
    big = np.vstack([params, params[:1]])
    table = (_lib.Params * (m + 1)).from_buffer_copy(np.ascontiguousarray(big).tobytes())
    K = _lib.make_knobs(1e-4, 2, 2, 1, 1e-3, 0.1)
    out = np.empty(m + 1)
    rc = _lib.wfpt_wiener_like_nodes_allreduce(ctx.handle, ds.handle, table, m + 1,
                                               ctypes.byref(K), _lib.dptr(out))
    assert rc == 2 and b"nodes" in _lib.wfpt_last_error()
    rc = _lib.wfpt_wiener_like_nodes_allreduce(ctx.handle, None, table, m + 1, ctypes.byref(K),
                                               _lib.dptr(out))
    assert rc == 2
    assert np.array_equal(ds.wiener_like_nodes_allreduce(params), want)
    # the same through the Python wrapper, which takes the count
    # from the table (every rank's) and leaves the dataset checks to the
    # library inside the collective: a mismatched table enters the exchange
    # poisoned and fails after it (ValueError = WFPT_ERR_ARG), then the
    # communicator works again
    with pytest.raises(ValueError, match="nodes"):
        ds.wiener_like_nodes_allreduce(big)
    flat = gpu.Dataset(x)  # no node ids: also poisoned, inside the exchange
    with pytest.raises(ValueError, match="node ids"):
        flat.wiener_like_nodes_allreduce(params)
    with pytest.raises(ValueError):  # not a table: refused before any collective
        ds.wiener_like_nodes_allreduce(params[:, :7])
    assert np.array_equal(ds.wiener_like_nodes_allreduce(params), want)


def test_bench_launcher_does_not_touch_gpu():
    """bench.py --gpus N without a torch.distributed environment starts
    torch.distributed.run with N ranks on 127.0.0.1 before loading the library
    or anything that initialises a GPU (a process that has touched the GPU
    must not hand over to another program on this pool)."""
    import subprocess
    import sys
    code = (
        "import atexit, os, sys\n"
        "os.environ.pop('WORLD_SIZE', None)\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "seen = []\n"
        "bench.subprocess.call = lambda cmd: seen.append(cmd) or 0\n"
        "sys.argv = ['bench.py', '--gpus', '8', '--steps', '2']\n"
        "try:\n"
        "    bench.main()\n"
        "except SystemExit as e:\n"
        "    assert e.code == 0, e.code\n"
        "loaded = sorted(m for m in sys.modules if m.startswith('hddm_amd') or m.startswith('torch'))\n"
        "print('CMD', seen[0])\n"
        "print('LOADED', loaded)\n" % ROOT)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    cmd = next(l for l in r.stdout.splitlines() if l.startswith("CMD"))
    loaded = next(l for l in r.stdout.splitlines() if l.startswith("LOADED"))
    assert "torch.distributed.run" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    assert loaded == "LOADED []", loaded


def test_c5_shards_are_the_same_trials_at_every_world_size(monkeypatch):
    """bench.py's C5 data: block b (C5_BLOCK trials) is sampled with seed
    20261015 + b, and rank r of N takes its contiguous shard of the blocks'
    concatenation, so every world size scores the same trials (value(N) /
    c5_n1.value is a speed-up on one workload). Checked with small blocks and
    a stand-in sampler (CPU)."""
    import bench
    from hddm_amd import dist as hdist

    def fake_rts(n, seed):
        return np.random.default_rng(seed).standard_normal(n)

    monkeypatch.setattr(bench, "make_rts", fake_rts)
    monkeypatch.setattr(bench, "C5_BLOCK", 1000)
    total = 8 * 1000
    whole = bench.c5_rts(0, total)
    assert whole.size == total
    assert np.array_equal(whole[3000:4000], fake_rts(1000, 20261015 + 3))
    for world in (2, 3, 4, 8):
        parts = [bench.c5_rts(*hdist.shard_range(total, world, r)) for r in range(world)]
        assert np.array_equal(np.concatenate(parts), whole), world
