"""ctypes binding to libwfpt_amd.so (include/wfpt_amd.h).

There is no CPU fallback: if the HIP library is missing this module raises
ImportError, and every device/driver failure raises RuntimeError with the
library's message (never a numeric stand-in).
"""
import ctypes
import os
import threading

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("WFPT_AMD_LIB", os.path.join(_PKG, "lib", "libwfpt_amd.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"hddm_amd: HIP library not found at {LIB_PATH}; build it with "
        "`python -m hddm_amd.build` (hipcc --offload-arch=gfx950)")

# Kernel arguments in device memory: every wave of the likelihood kernels
# reads its ~150-byte argument block with scalar loads at start; from the
# default host-side kernarg pool those are PCIe round trips (measured on
# MI355X: 2.5% of the full-DDM kernel time). Read by the HIP runtime when it
# initialises, i.e. at the first call into the library; an explicit setting
# wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

_lib = ctypes.CDLL(LIB_PATH)

WFPT_OK = 0
WFPT_MAX_DEPTH = 24

_D = ctypes.c_double
_I = ctypes.c_int
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_PD = ctypes.POINTER(ctypes.c_double)
_VP = ctypes.c_void_p


class Params(ctypes.Structure):
    _fields_ = [(n, _D) for n in ("v", "sv", "a", "z", "sz", "t", "st", "p_outlier")]


class Knobs(ctypes.Structure):
    _fields_ = [("err", _D), ("n_st", _I32), ("n_sz", _I32), ("use_adaptive", _I32),
                ("simps_err", _D), ("w_outlier", _D)]


_PP = ctypes.POINTER(Params)
_PK = ctypes.POINTER(Knobs)


def _sig(name, res, args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = args
    return f


wfpt_last_error = _sig("wfpt_last_error", ctypes.c_char_p, [])
wfpt_device_count = _sig("wfpt_device_count", _I, [ctypes.POINTER(_I)])
wfpt_open = _sig("wfpt_open", _I, [_I, ctypes.POINTER(_VP)])
wfpt_close = _sig("wfpt_close", None, [_VP])
wfpt_dataset_create = _sig("wfpt_dataset_create", _I,
                           [_VP, _PD, _I64, ctypes.POINTER(_I32), _I32, ctypes.POINTER(_VP)])
wfpt_dataset_create_ex = _sig("wfpt_dataset_create_ex", _I,
                              [_VP, _PD, _I64, ctypes.POINTER(_I32), _I32, _I,
                               ctypes.POINTER(_VP)])
WFPT_DS_INPUT_ORDER = 1
wfpt_dataset_destroy = _sig("wfpt_dataset_destroy", None, [_VP])
wfpt_dataset_size = _sig("wfpt_dataset_size", _I64, [_VP])
wfpt_shard_range = _sig("wfpt_shard_range", None,
                        [_I64, _I, _I, ctypes.POINTER(_I64), ctypes.POINTER(_I64)])
wfpt_wiener_like = _sig("wfpt_wiener_like", _I, [_VP, _VP, _PP, _PK, _PD])
wfpt_wiener_like_host = _sig("wfpt_wiener_like_host", _I, [_VP, _PD, _I64, _PP, _PK, _PD])
wfpt_wiener_like_nodes = _sig("wfpt_wiener_like_nodes", _I, [_VP, _VP, _PP, _PK, _PD])


def _raw(name, nargs):
    """The same entry point through a prototype of plain addresses (ints): the
    per-call paths (one likelihood per MCMC step) skip the per-argument ctypes
    object conversions (~1 us per call through byref / data_as)."""
    proto = ctypes.CFUNCTYPE(_I, *([ctypes.c_void_p] * nargs))
    return proto(ctypes.cast(getattr(_lib, name), ctypes.c_void_p).value)


raw_wiener_like = _raw("wfpt_wiener_like", 5)
raw_wiener_like_nodes = _raw("wfpt_wiener_like_nodes", 5)
wfpt_wiener_like_nodes_multi = _sig("wfpt_wiener_like_nodes_multi", _I,
                                    [_VP, _VP, _PP, _I32, _PK, _PD])
wfpt_wiener_like_nodes_multi_ex = _sig("wfpt_wiener_like_nodes_multi_ex", _I,
                                       [_VP, _VP, _PP, _I32, _PK, _PD, _PD])
_raw_multi_proto = ctypes.CFUNCTYPE(_I, _VP, _VP, _VP, _I32, _VP, _VP)
raw_wiener_like_nodes_multi = _raw_multi_proto(
    ctypes.cast(_lib.wfpt_wiener_like_nodes_multi, ctypes.c_void_p).value)
wfpt_pdf_array = _sig("wfpt_pdf_array", _I, [_VP, _PD, _I64, _PP, _PK, _I, _PD])
wfpt_full_pdf = _sig("wfpt_full_pdf", _I, [_VP, _D, _PP, _PK, _PD])
wfpt_wiener_like_multi = _sig("wfpt_wiener_like_multi", _I,
                              [_VP, _PD, _I64, ctypes.POINTER(_PD), _PD, _PK, _D, _PD])
wfpt_wiener_like_multi_resident = _sig("wfpt_wiener_like_multi_resident", _I,
                                       [_VP, _VP, ctypes.POINTER(_PD), _PD, _PK, _D, _PD])
wfpt_wiener_like_nodes_ex = _sig("wfpt_wiener_like_nodes_ex", _I, [_VP, _VP, _PP, _PK, _PD, _PD])
wfpt_wiener_like_multi_ex = _sig("wfpt_wiener_like_multi_ex", _I,
                                 [_VP, _PD, _I64, ctypes.POINTER(_PD), _PD, _PK, _D, _PD, _PD])
wfpt_wiener_like_multi_resident_ex = _sig("wfpt_wiener_like_multi_resident_ex", _I,
                                          [_VP, _VP, ctypes.POINTER(_PD), _PD, _PK, _D, _PD, _PD])
wfpt_dmat_cdf_array = _sig("wfpt_dmat_cdf_array", _I, [_VP, _PD, _I64, _PP, _D, _PD])
wfpt_comm_unique_id = _sig("wfpt_comm_unique_id", _I, [ctypes.c_char_p])
wfpt_comm_init = _sig("wfpt_comm_init", _I, [_VP, _I, _I, ctypes.c_char_p])
wfpt_wiener_like_allreduce = _sig("wfpt_wiener_like_allreduce", _I, [_VP, _VP, _PP, _PK, _PD])
wfpt_comm_exchange_id = _sig("wfpt_comm_exchange_id", _I,
                             [_I, _I, ctypes.c_char_p, _I, _I, ctypes.c_char_p])
wfpt_comm_init_tcp = _sig("wfpt_comm_init_tcp", _I, [_VP, _I, _I, ctypes.c_char_p, _I, _I])
wfpt_comm_init_all = _sig("wfpt_comm_init_all", _I, [ctypes.POINTER(_VP), _I])
wfpt_wiener_like_allreduce_group = _sig("wfpt_wiener_like_allreduce_group", _I,
                                        [ctypes.POINTER(_VP), ctypes.POINTER(_VP), _I, _PP, _PK,
                                         _PD])
wfpt_result_poison = _sig("wfpt_result_poison", _I, [_PD])
wfpt_profile_enable = _sig("wfpt_profile_enable", _I, [_VP, _I])
wfpt_profile_read = _sig("wfpt_profile_read", _I,
                         [_VP, _PD, ctypes.POINTER(_I64), ctypes.POINTER(_I64), _I])
try:  # diagnostics only: A/B runs may load an older library build without it
    wfpt_profile_lists = _sig("wfpt_profile_lists", _I, [_VP, ctypes.POINTER(_I64), _I])
    wfpt_debug_waves = _sig("wfpt_debug_waves", _I, [_VP, ctypes.POINTER(ctypes.c_uint64), _I64])
except AttributeError:
    wfpt_profile_lists = wfpt_debug_waves = None
wfpt_synchronize = _sig("wfpt_synchronize", _I, [_VP])
wfpt_wiener_like_trials = _sig("wfpt_wiener_like_trials", _I, [_VP, _VP, _PP, _PK, _PD, _PD])
wfpt_dataset_order = _sig("wfpt_dataset_order", _I, [_VP, ctypes.POINTER(_I64)])
wfpt_debug_partials = _sig("wfpt_debug_partials", _I,
                           [_VP, _PD, ctypes.POINTER(ctypes.c_int32), _I64])
wfpt_last_path = _sig("wfpt_last_path", _I, [_VP, ctypes.POINTER(_I)])
wfpt_wiener_like_local = _sig("wfpt_wiener_like_local", _I, [_VP, _VP, _PP, _PK, _PD])
wfpt_wiener_like_nodes_local = _sig("wfpt_wiener_like_nodes_local", _I, [_VP, _VP, _PP, _PK, _PD])
wfpt_wiener_like_nodes_allreduce = _sig("wfpt_wiener_like_nodes_allreduce", _I,
                                        [_VP, _VP, _PP, _I32, _PK, _PD])
# WFPT_PATH_* (include/wfpt_amd.h): kernels the last likelihood call launched
PATH_LEAN, PATH_ENGINE, PATH_SMALL, PATH_REDO = 1, 2, 4, 8
PATH_FOLD, PATH_DIRECT, PATH_FIXED, PATH_SPLIT = 16, 32, 64, 128
PATH_SMALL_SPLIT, PATH_NODE_SPLIT, PATH_NODE_RARE = 256, 512, 1024
wfpt_decode_result = _sig("wfpt_decode_result", _I, [_PD, _PD])

EXPORTED = [
    "wfpt_device_count", "wfpt_open", "wfpt_close", "wfpt_last_error", "wfpt_dataset_create",
    "wfpt_dataset_destroy", "wfpt_dataset_size", "wfpt_shard_range", "wfpt_wiener_like",
    "wfpt_wiener_like_host", "wfpt_wiener_like_nodes", "wfpt_pdf_array", "wfpt_full_pdf",
    "wfpt_wiener_like_multi", "wfpt_dmat_cdf_array", "wfpt_comm_unique_id", "wfpt_comm_init",
    "wfpt_wiener_like_allreduce", "wfpt_profile_enable", "wfpt_profile_read", "wfpt_synchronize",
    "wfpt_decode_result", "wfpt_profile_lists", "wfpt_debug_waves", "wfpt_dataset_create_ex",
    "wfpt_wiener_like_multi_resident", "wfpt_comm_exchange_id", "wfpt_comm_init_tcp",
    "wfpt_comm_init_all", "wfpt_wiener_like_allreduce_group", "wfpt_result_poison",
    "wfpt_wiener_like_nodes_ex", "wfpt_wiener_like_multi_ex", "wfpt_wiener_like_multi_resident_ex",
    "wfpt_wiener_like_trials", "wfpt_dataset_order", "wfpt_debug_partials", "wfpt_last_path",
    "wfpt_wiener_like_local", "wfpt_wiener_like_nodes_local", "wfpt_wiener_like_nodes_allreduce",
    "wfpt_wiener_like_nodes_multi", "wfpt_wiener_like_nodes_multi_ex",
]

# error encoding of a result triple (include/wfpt_amd.h: wfpt_decode_result)
DEPTH_ERROR = 1.0
BUDGET_ERROR = 1048576.0
PEER_FAILED = 1099511627776.0  # 2^40: a rank that failed before the exchange


def poisoned_result():
    """The triple a rank that failed before the exchange contributes
    (wfpt_result_poison)."""
    r = (ctypes.c_double * 3)()
    check(wfpt_result_poison(r))
    return [r[0], r[1], r[2]]


def decode_result(triple):
    """The library's decode of a (rank-summed) {sum, zeros, errors} triple."""
    r = (ctypes.c_double * 3)(*[float(v) for v in triple])
    out = _D()
    check(wfpt_decode_result(r, ctypes.byref(out)))
    return out.value


class CommError(RuntimeError):
    """A multi-GPU exchange failed (WFPT_ERR_COMM), e.g. another rank's local
    pass failed before the all-reduce."""


def check(rc):
    if rc != WFPT_OK:
        msg = wfpt_last_error().decode(errors="replace")
        if rc == 4:
            raise NotImplementedError(f"wfpt_amd: {msg}")
        if rc == 2:
            raise ValueError(f"wfpt_amd: {msg}")
        if rc == 3:
            raise CommError(f"wfpt_amd error {rc}: {msg}")
        raise RuntimeError(f"wfpt_amd error {rc}: {msg}")


def dptr(a):
    return a.ctypes.data_as(_PD)


class Context:
    """One HIP device + stream + workspaces (wfpt_ctx)."""

    def __init__(self, device=0):
        h = _VP()
        check(wfpt_open(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = int(device)

    def close(self):
        if self.handle:
            wfpt_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    PROF_EVENTS = 1
    PROF_EVALS = 2

    def profile(self, flags=1):
        """flags: PROF_EVENTS (per-launch HIP-event time) | PROF_EVALS (count pdf_sv evals)."""
        check(wfpt_profile_enable(self.handle, int(flags)))

    def profile_read(self, reset=False):
        ms, nl, ne = _D(), _I64(), _I64()
        check(wfpt_profile_read(self.handle, ctypes.byref(ms), ctypes.byref(nl),
                                ctypes.byref(ne), 1 if reset else 0))
        return ms.value, nl.value, ne.value

    def profile_lists(self, reset=False):
        """Deferred-pass list sizes (include/wfpt_amd.h: wfpt_profile_lists)."""
        a = (_I64 * 16)()
        if wfpt_profile_lists is None:
            return {}
        check(wfpt_profile_lists(self.handle, a, 1 if reset else 0))
        v = list(a)
        return {"segments": v[0], "node_deferred": v[3],
                "tasks1": v[1], "tasks2": v[2], "records": v[4], "exact": v[5],
                "walk": v[6], "zwalks": v[7], "zwalks0": v[8], "zwalks1": v[9],
                "zwalks2": v[10], "phase_kcycles": v[11:16]}

    def debug_waves(self, n):
        """Per-wave engine records of diagnostic builds (wfpt_debug_waves): (n, 8) uint64."""
        out = np.zeros((n, 8), dtype=np.uint64)
        check(wfpt_debug_waves(self.handle, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n))
        return out

    def synchronize(self):
        check(wfpt_synchronize(self.handle))

    def last_path(self):
        """WFPT_PATH_* bits of the kernels the last likelihood call launched."""
        v = _I()
        check(wfpt_last_path(self.handle, ctypes.byref(v)))
        return v.value

    def partials(self, n):
        """The first n chunk partials {sum, zero word} of the last summing call."""
        part = np.empty(n, dtype=np.float64)
        zero = np.empty(n, dtype=np.int32)
        check(wfpt_debug_partials(self.handle, dptr(part),
                                  zero.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n))
        return part, zero


_ctx_lock = threading.Lock()
_contexts = {}


def default_device():
    env = os.environ.get("WFPT_DEVICE")
    if env is not None:
        return int(env)
    return 0


def context(device=None):
    """Process-wide context for `device` (default: $WFPT_DEVICE or 0)."""
    dev = default_device() if device is None else int(device)
    with _ctx_lock:
        c = _contexts.get(dev)
        if c is None:
            c = Context(dev)
            _contexts[dev] = c
        return c


def device_count():
    n = _I()
    check(wfpt_device_count(ctypes.byref(n)))
    return n.value


def shard_range(n, nranks, rank):
    lo, hi = _I64(), _I64()
    wfpt_shard_range(int(n), int(nranks), int(rank), ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def make_params(v, sv, a, z, sz, t, st, p_outlier=0.0):
    return Params(float(v), float(sv), float(a), float(z), float(sz), float(t), float(st),
                  float(p_outlier))


def make_knobs(err, n_st, n_sz, use_adaptive, simps_err, w_outlier):
    return Knobs(float(err), int(n_st), int(n_sz), 1 if use_adaptive else 0, float(simps_err),
                 float(w_outlier))
