"""C-ABI boundary and host-side logic (CPU; no compute calls need a GPU)."""
import ctypes
import inspect
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "wfpt_amd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wfpt_[a-z_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    from hddm_amd import _lib
    declared = header_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(_lib._lib, name), f"{name} declared in include/wfpt_amd.h but not exported"
    assert sorted(_lib.EXPORTED) == declared
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (wfpt_\w+)", out))
    assert set(declared) <= exported


def test_struct_layouts_match_header():
    from hddm_amd import _lib
    assert ctypes.sizeof(_lib.Params) == 8 * 8
    assert _lib.Knobs.n_st.offset == 8 and _lib.Knobs.simps_err.offset == 24
    assert ctypes.sizeof(_lib.Knobs) == 40


def test_library_is_gfx950_code_object():
    from hddm_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_reference_signatures():
    """Same parameter names, order and defaults as src/wfpt.pyx / pdf.pxi."""
    from hddm_amd import wfpt
    sig = lambda f: [(p.name, p.default) for p in inspect.signature(f).parameters.values()]
    E = inspect.Parameter.empty
    assert sig(wfpt.wiener_like) == [
        ("x", E), ("v", E), ("sv", E), ("a", E), ("z", E), ("sz", E), ("t", E), ("st", E),
        ("err", E), ("n_st", 10), ("n_sz", 10), ("use_adaptive", 1), ("simps_err", 1e-8),
        ("p_outlier", 0), ("w_outlier", 0.1)]
    assert sig(wfpt.pdf_array) == [
        ("x", E), ("v", E), ("sv", E), ("a", E), ("z", E), ("sz", E), ("t", E), ("st", E),
        ("err", 1e-4), ("logp", 0), ("n_st", 2), ("n_sz", 2), ("use_adaptive", 1),
        ("simps_err", 1e-3), ("p_outlier", 0), ("w_outlier", 0)]
    assert sig(wfpt.full_pdf) == [
        ("x", E), ("v", E), ("sv", E), ("a", E), ("z", E), ("sz", E), ("t", E), ("st", E),
        ("err", E), ("n_st", 2), ("n_sz", 2), ("use_adaptive", 1), ("simps_err", 1e-3)]
    assert sig(wfpt.wiener_like_multi)[9] == ("multi", None)
    assert sig(wfpt.gen_rts_from_cdf)[7:] == [("samples", 1000), ("cdf_lb", -6), ("cdf_ub", 6),
                                             ("dt", 1e-2)]


def test_buffer_argument_checks_without_gpu():
    from hddm_amd import wfpt
    with pytest.raises(TypeError):
        wfpt.pdf_array([1.0, 2.0], 0.5, 0, 2, 0.5, 0, 0.3, 0)
    with pytest.raises(ValueError):
        wfpt.pdf_array(np.ones(3, dtype=np.float32), 0.5, 0, 2, 0.5, 0, 0.3, 0)
    with pytest.raises(ValueError):
        wfpt.wiener_like(np.ones((2, 2)), 0.5, 0, 2, 0.5, 0, 0.3, 0, 1e-4)


def test_no_cpu_fallback_without_device():
    """On a host without a GPU the product path raises; it never computes on the CPU."""
    from hddm_amd import _lib, wfpt
    try:
        n = _lib.device_count()
    except RuntimeError:
        n = 0
    if n > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        wfpt.wiener_like(np.array([0.8]), 0.5, 0, 2, 0.5, 0, 0.3, 0, 1e-4)


def test_missing_library_fails_loudly(tmp_path):
    code = ("import os, sys; sys.path.insert(0, %r); "
            "os.environ['WFPT_AMD_LIB']=%r\n"
            "try:\n import hddm_amd.wfpt\nexcept ImportError as e:\n print('IMPORTERROR', e)\n"
            % (ROOT, str(tmp_path / "nope.so")))
    out = subprocess.run(["python", "-c", code], capture_output=True, text=True).stdout
    assert "IMPORTERROR" in out


@pytest.mark.parametrize("n,world", [(0, 1), (1, 1), (10, 3), (1_000_001, 8), (7, 8)])
def test_shard_ranges_partition(n, world):
    from hddm_amd import dist
    spans = [dist.shard_range(n, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (lo, hi), (lo2, _) in zip(spans, spans[1:]):
        assert hi == lo2 and hi >= lo
    sizes = [hi - lo for lo, hi in spans]
    assert max(sizes) - min(sizes) <= 1


def test_combine_semantics():
    from hddm_amd import dist
    assert dist.combine([(-3.0, 0), (-4.5, 0)]) == -7.5
    assert dist.combine([(-3.0, 0), (-4.5, 2)]) == -np.inf
    assert dist.combine([(float("nan"), 0), (-1.0, 1)]) == -np.inf  # zero beats NaN (wfpt.pyx:71)
    assert np.isnan(dist.combine([(float("nan"), 0), (-1.0, 0)]))


def test_new_entry_points_reject_null_arguments_without_gpu():
    """The r04 entry points (per-trial check, stored order, chunk partials,
    launched path, rank-local parts, per-node all-reduce) validate their
    arguments before touching a device: WFPT_ERR_ARG with a message."""
    from hddm_amd import _lib
    two = 2
    assert _lib.wfpt_wiener_like_trials(None, None, None, None, None, None) == two
    assert _lib.wfpt_dataset_order(None, None) == two
    assert _lib.wfpt_debug_partials(None, None, None, 0) == two
    assert _lib.wfpt_last_path(None, None) == two
    assert _lib.wfpt_wiener_like_local(None, None, None, None, None) == two
    assert _lib.wfpt_wiener_like_nodes_local(None, None, None, None, None) == two
    assert _lib.wfpt_wiener_like_nodes_allreduce(None, None, None, 0, None, None) == two
    assert b"null" in _lib.wfpt_last_error()


def test_raw_prototypes_bind_the_declared_entry_points():
    """The binding's per-step fast path (raw-address prototypes) calls the
    same C entry points as the declared ctypes functions, and a closed
    dataset still gets the C ABI's argument error (no crash on a NULL)."""
    from hddm_amd import _lib
    for raw, decl in ((_lib.raw_wiener_like, _lib.wfpt_wiener_like),
                      (_lib.raw_wiener_like_nodes, _lib.wfpt_wiener_like_nodes)):
        assert (ctypes.cast(raw, ctypes.c_void_p).value ==
                ctypes.cast(decl, ctypes.c_void_p).value)
    # NULL context / dataset through the raw prototype: WFPT_ERR_ARG, no device
    k = _lib.make_knobs(1e-4, 2, 2, 1, 1e-3, 0.1)
    p = _lib.make_params(0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.05)
    out = ctypes.c_double()
    rc = _lib.raw_wiener_like(None, None, ctypes.addressof(p), ctypes.addressof(k),
                              ctypes.addressof(out))
    assert rc == 2
