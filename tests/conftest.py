import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def ref():
    """The reference's own kernels (oracle/_ref), or skip when not built."""
    import oracle
    R = oracle.load_ref()
    if R is None:
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    return R


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    out = {k: dict(np.load(os.path.join(d, k + ".npz"), allow_pickle=False))
           for k in ("full_pdf_grid", "wiener_like", "pdf_array", "datasets")}
    with open(os.path.join(d, "matlab_values.json")) as fh:
        out["matlab"] = json.load(fh)
    return out


@pytest.fixture(scope="session")
def gpu():
    """hddm_amd bound to a real device; fails loudly (never falls back)."""
    from hddm_amd import _lib, wfpt
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible to a @gpu test")
    return wfpt
