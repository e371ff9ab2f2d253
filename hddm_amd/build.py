"""Build libwfpt_amd.so in-tree (hipcc, gfx950 only).

    python -m hddm_amd.build [--force]

The library lands in hddm_amd/lib/ (git-ignored, shipped to the GPU box with
the working tree). No CMake, no JIT cache: the .so that the tests and bench
load is exactly the one built here.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libwfpt_amd.so")
SOURCES = ["wfpt_kernels.hip", "cdfdif_kernels.hip", "wfpt_capi.cpp", "wfpt_rendezvous.cpp"]
DEPS = SOURCES + ["wfpt_device.hpp", "wfpt_internal.h", "wfpt_crlibm.hpp", "wfpt_exact.hpp"]
ARCH = os.environ.get("WFPT_OFFLOAD_ARCH", "gfx950")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
          f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result"]


def source_digest(defines=()):
    """sha1 over the compiler flags and every source the library is built from:
    identifies a build independently of the binary's bytes (profiles measured
    on one build are matched to the library by it)."""
    import hashlib
    h = hashlib.sha1(" ".join(CFLAGS + list(defines)).encode())
    for f in DEPS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(ROOT, "include", "wfpt_amd.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()


def built_digest(lib=LIB):
    """The source digest recorded next to a built library (None if absent)."""
    try:
        with open(lib + ".src") as fh:
            return fh.read().strip()
    except OSError:
        return None


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, defines=(), out=None):
    """Compile libwfpt_amd.so. `defines` (e.g. ["WFPT_FAST_WAVES=3"]; entries
    starting with '-' are extra compiler flags) and `out` build experiment
    variants next to the default library."""
    os.makedirs(LIBDIR, exist_ok=True)
    lib = out or LIB
    deps = [os.path.join(CSRC, f) for f in DEPS] + [os.path.join(ROOT, "include", "wfpt_amd.h")]
    if not force and not _stale(lib, deps):
        if built_digest(lib) is None:  # built before digests were recorded
            with open(lib + ".src", "w") as fh:
                fh.write(source_digest(defines) + "\n")
        return lib
    objs, procs = [], []
    tag = os.path.splitext(os.path.basename(lib))[0]
    for src in SOURCES:  # the translation units compile concurrently
        obj = os.path.join(LIBDIR, tag + "_" + os.path.splitext(src)[0] + ".o")
        flags = [f for d in defines if d.startswith("-") for f in d.split()]
        cmd = [HIPCC, *CFLAGS, *flags, *[f"-D{d}" for d in defines if not d.startswith("-")],
               "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    tmp = lib + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs,
           "-L/opt/rocm/lib", "-lrccl", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    with open(lib + ".src", "w") as fh:
        fh.write(source_digest(defines) + "\n")
    for o in objs:
        os.remove(o)
    return lib


# Diagnostic builds that tests load in a child process (WFPT_AMD_LIB); never
# the product. pubdiag: segment_publish_kernel's non-last blocks store their
# sums after the completion word (tests/test_parity_trials.py:
# test_stale_check_detects_late_publication).
VARIANTS = {"pubdiag": ["WFPT_PUB_DIAG=1"]}


def variant_path(name):
    return os.path.join(LIBDIR, f"libwfpt_amd_{name}.so")


def build_variants(force=False, verbose=False):
    return [build(force=force, verbose=verbose, defines=d, out=variant_path(k))
            for k, d in VARIANTS.items()]


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--variants" in sys.argv:
        print(build_variants(force="--force" in sys.argv, verbose=True))
