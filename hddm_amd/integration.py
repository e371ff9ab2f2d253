"""Drop-in installation into an HDDM process.

HDDM reaches the likelihood through the compiled `wfpt` module (imported as
`import wfpt` by hddm/__init__.py:16, hddm/models/hddm_rl.py:8 and
hddm/models/rl.py:8; called as `hddm.wfpt.<name>` at call time, e.g.
hddm/likelihoods.py:54-60,86) and the CDF through `cdfdif_wrapper`
(hddm/__init__.py:11,19; hddm/likelihoods.py:91). `install()` rebinds only the
hot-path attributes of those module objects, so every holder of the module sees
the MI355X functions while the names this engine does not provide
(`wiener_like_rl*`, `wiener_like_contaminant`, `gen_cdf_using_pdf`, `split_cdf`,
wfpt.pyx:79-421) keep the reference's implementations.
"""
import importlib
import sys

HOT_PATH = ("pdf_array", "wiener_like", "full_pdf", "wiener_like_multi", "gen_rts_from_cdf")
CDF_PATH = ("dmat_cdf_array",)


class Installation:
    """What install() changed; `uninstall()` puts it back."""

    def __init__(self):
        self._attrs = []      # (module, name, previous value or _MISSING)
        self._modules = []    # (sys.modules key, previous entry or _MISSING)

    def uninstall(self):
        for mod, name, old in reversed(self._attrs):
            if old is _MISSING:
                delattr(mod, name)
            else:
                setattr(mod, name, old)
        for key, old in reversed(self._modules):
            if old is _MISSING:
                sys.modules.pop(key, None)
            else:
                sys.modules[key] = old
        self._attrs, self._modules = [], []


_MISSING = object()


def _find(name, given):
    if given is not None:
        return given
    mod = sys.modules.get(name)
    if mod is not None:
        return mod
    try:
        return importlib.import_module(name)
    except ImportError:
        return None


def _patch(inst, key, target, ours, names):
    if target is None or target is ours:
        # no reference module in this process: ours under its name
        inst._modules.append((key, sys.modules.get(key, _MISSING)))
        sys.modules[key] = ours
        return ours
    for n in names:
        inst._attrs.append((target, n, getattr(target, n, _MISSING)))
        setattr(target, n, getattr(ours, n))
    return target


def install(wfpt_module=None, cdfdif_module=None, likelihoods_module=None):
    """Route HDDM's likelihood and CDF calls to libwfpt_amd.so.

    `wfpt_module` / `cdfdif_module` default to the already-imported (or
    importable) reference extensions `wfpt` and `cdfdif_wrapper`; when one is
    absent, the MI355X module is registered under its name instead. Call before
    or after `import hddm`: attributes are looked up per call. Returns an
    Installation whose `uninstall()` restores the previous state.

    If `hddm.likelihoods` is already imported (or given), its
    `generate_wfpt_stochastic_class` (called by HDDM models at construction,
    hddm/models/base.py:727,738) and `Wfpt` are rebound too, to this package's
    factory: the same PyMC class (kabuki's stochastic_from_dist with pdf, cdf,
    cdf_vec, random and the quantile methods), whose logp keeps each node's
    RTs resident on the GPU instead of uploading them per call. HDDM is never
    imported here."""
    from . import cdfdif_wrapper as amd_cdf
    from . import likelihoods as amd_lk
    from . import wfpt as amd_wfpt
    inst = Installation()
    _patch(inst, "wfpt", _find("wfpt", wfpt_module), amd_wfpt, HOT_PATH)
    _patch(inst, "cdfdif_wrapper", _find("cdfdif_wrapper", cdfdif_module), amd_cdf, CDF_PATH)
    lk = likelihoods_module if likelihoods_module is not None else sys.modules.get("hddm.likelihoods")
    if lk is not None:
        inst._attrs.append((lk, "generate_wfpt_stochastic_class",
                            getattr(lk, "generate_wfpt_stochastic_class", _MISSING)))
        lk.generate_wfpt_stochastic_class = amd_lk.generate_wfpt_stochastic_class
        if hasattr(lk, "Wfpt"):
            inst._attrs.append((lk, "Wfpt", lk.Wfpt))
            lk.Wfpt = amd_lk.generate_wfpt_stochastic_class()
    return inst
