"""The exact path's correctly rounded libm (hddm_amd/csrc/wfpt_crlibm.hpp), on the host.

The header is compiled with gcc (tests/c/crlibm_check.cpp) and checked:
  * against exact arithmetic (Python decimal / fractions at 60+ digits, rounded
    once): every sampled result must be the correctly rounded double;
  * against this host's glibc (what the reference's CPU build calls): the
    disagreement rate must be glibc's own misrounding rate (< 0.2%), far below
    OCML's 1-24% (tools/libm_probe.hip).
The same source is compiled for gfx950 into the exact path; IEEE operations and
fma() give the same bits on both.
"""
import decimal
import os
import subprocess
from fractions import Fraction

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "crlibm_check.cpp")

D = decimal.Decimal
CTX = decimal.Context(prec=70)
decimal.getcontext().prec = 70  # unary minus etc. use the thread context
PI = D("3.14159265358979323846264338327950288419716939937510582097494459230781640628620899863")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("crlibm") / "crlibm_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-o", exe, SRC, "-lm"], check=True)
    return exe


def run(exe, fn, x, tmp):
    inp, out = os.path.join(tmp, "in.bin"), os.path.join(tmp, "out.bin")
    np.ascontiguousarray(x, dtype=np.float64).tofile(inp)
    subprocess.run([exe, inp, str(fn), out], check=True)
    r = np.fromfile(out).reshape(-1, 2)
    return r[:, 0], r[:, 1]


def exact(fn, x):
    d = D(float(x))
    if fn == 0:
        return float(CTX.exp(d))
    if fn == 1:
        return float(CTX.ln(d))
    if fn == 2:
        two_pi = CTX.multiply(D(2), PI)
        r = CTX.remainder_near(d, two_pi)
        term, s, n = r, D(0), 1
        r2 = CTX.multiply(r, r)
        while abs(term) > D(10) ** -80:
            s = CTX.add(s, term)
            term = CTX.divide(CTX.multiply(-term, r2), D((n + 1) * (n + 2)))
            n += 2
        return float(s)
    return float(Fraction(float(x)) ** 3)


CASES = [
    (0, "exp", lambda r, n: np.concatenate([r.uniform(-745.2, 709.7, n), r.uniform(-1, 1, n // 4),
                                            r.uniform(-745.2, -708.0, n // 4)])),
    (1, "log", lambda r, n: np.concatenate([10.0 ** r.uniform(-320, 300, n), 1 + r.uniform(-0.05, 0.05, n // 4),
                                            r.uniform(1e-3, 10, n // 4)])),
    (2, "sin", lambda r, n: np.concatenate([r.uniform(0, 60, n), np.pi * np.arange(1, 40) * 1.0,
                                            r.uniform(0, 1e-3, n // 8)])),
    (3, "cube", lambda r, n: np.concatenate([10.0 ** r.uniform(-120, 100, n), r.uniform(0, 3, n)])),
]


@pytest.mark.parametrize("fn,name,gen", CASES, ids=[c[1] for c in CASES])
def test_correctly_rounded_vs_exact(checker, tmp_path, fn, name, gen):
    rng = np.random.default_rng(100 + fn)
    x = gen(rng, 1500)
    cr, _ = run(checker, fn, x, str(tmp_path))
    bad = [(xi, c, exact(fn, xi)) for xi, c in zip(x, cr) if c != exact(fn, xi)]
    assert not bad, f"{name}: {len(bad)} misrounded, e.g. {bad[:3]}"


@pytest.mark.parametrize("fn,name,gen", CASES, ids=[c[1] for c in CASES])
def test_agrees_with_glibc(checker, tmp_path, fn, name, gen):
    rng = np.random.default_rng(200 + fn)
    x = gen(rng, 200_000)
    cr, glibc = run(checker, fn, x, str(tmp_path))
    both_nan = np.isnan(cr) & np.isnan(glibc)
    differ = np.mean((cr != glibc) & ~both_nan)
    assert differ < 2e-3, f"{name}: differs from glibc in {differ:.2e} of calls"
    # never by more than one ulp
    a = cr[~both_nan].view(np.int64)
    b = glibc[~both_nan].view(np.int64)
    assert np.max(np.abs(a - b)) <= 1
