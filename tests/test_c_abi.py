"""The C ABI from a plain C program (tests/c/abi_smoke.c): compiles and links
against include/wfpt_amd.h and libwfpt_amd.so with gcc (CPU), and on the GPU
returns the reference's numbers and status conventions."""
import math
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "hddm_amd", "lib")


def _build(tmp_path):
    exe = str(tmp_path / "abi_smoke")
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_smoke.c"), "-o", exe, "-L", LIBDIR,
                    "-lwfpt_amd", f"-Wl,-rpath,{LIBDIR}", "-lm"], check=True)
    return exe


def test_c_client_compiles_and_links(tmp_path):
    assert os.path.exists(_build(tmp_path))


@pytest.mark.gpu
def test_c_client_matches_reference(tmp_path, oracle_lib):
    exe = _build(tmp_path)
    env = dict(os.environ, HIP_FORCE_DEV_KERNARG="1")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr
    l1, l2 = out.stdout.strip().splitlines()
    lp_res, lp_host, lp_arr = map(float, l1.split())
    rc_null, rc_cdf, rc_po, po_is_neginf = map(int, l2.split())
    n = 1000
    i = np.arange(n)
    rt = np.where(i % 3 == 0, -1.0, 1.0) * (0.35 + 0.002 * i)
    ref = oracle_lib.pdf_array(rt, 0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 1e-4, 1, 2, 2, 1, 1e-3,
                               0.05, 0.1)
    tot = math.fsum(ref)
    for v in (lp_res, lp_host, lp_arr):
        assert abs(v - tot) < 1e-10 * abs(tot), (v, tot)
    assert (rc_null, rc_cdf, rc_po, po_is_neginf) == (2, 2, 0, 1)
