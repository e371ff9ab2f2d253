"""ORACLE — TEST INFRASTRUCTURE ONLY.

Recipe that compiles the reference's own WFPT kernels (src/pdf.pxi +
src/integrate.pxi, read where they lie under /root/reference) into
oracle/_ref/ref_shim<EXT_SUFFIX>. Outputs go only into oracle/_ref/ (git-ignored).

Mirrors the reference build of setup.py:4-7 (Cython -> C++, g++ -O2); the one
addition, -fopenmp, only parallelises the shim's pdf_array_prange (the
all-threads CPU calibration), not the reference's own loops. Cython's `include "integrate.pxi"` is resolved through the
include path, so nothing from the reference is copied into this repository.

Usage:  python oracle/build_ref.py [--reference /root/reference]
"""
import argparse
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_ref")


def build(reference="/root/reference", quiet=False):
    src = os.path.join(reference, "src")
    if not os.path.isfile(os.path.join(src, "integrate.pxi")):
        raise FileNotFoundError(f"reference sources not found under {src}")
    import numpy as np
    os.makedirs(OUT, exist_ok=True)
    cpp = os.path.join(OUT, "ref_shim.cpp")
    so = os.path.join(OUT, "ref_shim" + sysconfig.get_config_var("EXT_SUFFIX"))
    pyx = os.path.join(HERE, "ref_shim.pyx")
    if (os.path.exists(so) and os.path.getmtime(so) > os.path.getmtime(pyx)
            and os.path.getmtime(so) > os.path.getmtime(os.path.join(src, "integrate.pxi"))
            and os.path.getmtime(so) > os.path.getmtime(os.path.join(src, "pdf.pxi"))):
        return so
    run = (lambda c: subprocess.run(c, check=True, stdout=subprocess.DEVNULL)) if quiet else \
        (lambda c: subprocess.run(c, check=True))
    run([sys.executable, "-m", "cython", "--cplus", "-2", "-I", src, "-o", cpp, pyx])
    # -fopenmp only parallelises pdf_array_prange (the all-threads calibration
    # row); every kernel and the serial loops compile as with setup.py:4-7
    run(["g++", "-O2", "-fwrapv", "-fPIC", "-DNDEBUG", "-shared", "-fopenmp",
         "-DNPY_NO_DEPRECATED_API=NPY_1_7_API_VERSION",
         "-I", sysconfig.get_paths()["include"], "-I", np.get_include(),
         cpp, "-o", so])
    return so


def build_cdfdif(reference="/root/reference", quiet=False):
    """The reference's own `cdfdif_wrapper` extension (src/cdfdif_wrapper.pyx +
    src/cdfdif.c, setup.py:9-13) compiled where the sources lie, into
    oracle/_ref/cdfdif_wrapper<EXT_SUFFIX>. It imports nothing from hddm."""
    src = os.path.join(reference, "src")
    pyx = os.path.join(src, "cdfdif_wrapper.pyx")
    csrc = os.path.join(src, "cdfdif.c")
    if not os.path.isfile(pyx):
        raise FileNotFoundError(f"reference sources not found under {src}")
    import numpy as np
    os.makedirs(OUT, exist_ok=True)
    c = os.path.join(OUT, "cdfdif_wrapper.c")
    so = os.path.join(OUT, "cdfdif_wrapper" + sysconfig.get_config_var("EXT_SUFFIX"))
    if (os.path.exists(so) and os.path.getmtime(so) > os.path.getmtime(pyx)
            and os.path.getmtime(so) > os.path.getmtime(csrc)):
        return so
    run = (lambda c_: subprocess.run(c_, check=True, stdout=subprocess.DEVNULL)) if quiet else \
        (lambda c_: subprocess.run(c_, check=True))
    run([sys.executable, "-m", "cython", "-2", "-I", src, "-o", c, pyx])
    run(["gcc", "-O2", "-fwrapv", "-fPIC", "-DNDEBUG", "-shared",
         "-DNPY_NO_DEPRECATED_API=NPY_1_7_API_VERSION",
         "-I", src, "-I", sysconfig.get_paths()["include"], "-I", np.get_include(),
         c, csrc, "-o", so, "-lm"])
    return so


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ref = ap.parse_args().reference
    print(build(ref))
    print(build_cdfdif(ref))
