"""Host C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5
"Race detection / sanitizers"; CPU only — GPU sanitizers are not available).

tests/c/sanitize_driver.cpp is linked from the real sources — the oracle
(oracle/wfpt_oracle.c), the exact path (wfpt_exact.hpp, wfpt_crlibm.hpp), the C
ABI's host code (wfpt_capi.cpp, wfpt_rendezvous.cpp; the kernel objects only
for their host launch stubs) — with the sanitizers on the host side
(`-Xarch_host -fsanitize=...` for HIP sources, one clang toolchain for all of
it), and run here without a GPU. Any sanitizer report fails the test
(halt_on_error; UBSan non-recoverable).
"""
import os
import socket
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/lib/llvm/bin/clang"
HIPCC = "/opt/rocm/bin/hipcc"
SAN = "-fsanitize=address,undefined"
NOREC = "-fno-sanitize-recover=undefined"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if not (os.path.exists(CLANG) and os.path.exists(HIPCC)):
        pytest.skip("ROCm clang / hipcc not present")
    d = tmp_path_factory.mktemp("san")
    csrc = os.path.join(ROOT, "hddm_amd", "csrc")
    objs = []
    o = str(d / "oracle.o")
    subprocess.run([CLANG, "-O1", "-g", "-ffp-contract=off", "-fno-fast-math", SAN, NOREC,
                    "-c", os.path.join(ROOT, "oracle", "wfpt_oracle.c"), "-o", o], check=True)
    objs.append(o)
    hip_flags = ["-std=c++17", "-ffp-contract=off", "-fno-fast-math", "--offload-arch=gfx950",
                 "-Xarch_host", "-O1", "-Xarch_host", "-g", "-Xarch_host", SAN, "-Xarch_host",
                 NOREC]
    for src in ("wfpt_capi.cpp", "wfpt_rendezvous.cpp", "wfpt_kernels.hip",
                "cdfdif_kernels.hip"):
        o = str(d / (os.path.splitext(src)[0] + ".o"))
        # no GPU runs here: the device code only has to exist (-O0 keeps the
        # build short); the host side is what is sanitized
        subprocess.run([HIPCC, *hip_flags, "-Xarch_device", "-O0", "-c",
                        os.path.join(csrc, src), "-o", o], check=True)
        objs.append(o)
    o = str(d / "driver.o")
    subprocess.run([HIPCC, *hip_flags, "-x", "c++", "-c",
                    os.path.join(ROOT, "tests", "c", "sanitize_driver.cpp"), "-o", o], check=True)
    objs.append(o)
    exe = str(d / "sanitize_driver")
    subprocess.run([HIPCC, "--offload-arch=gfx950", SAN, "-o", exe, *objs, "-L/opt/rocm/lib",
                    "-lrccl", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib", "-lm",
                    "-lpthread"], check=True)
    return exe


def test_host_code_is_sanitizer_clean(driver):
    env = dict(os.environ,
               ASAN_OPTIONS="halt_on_error=1:detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    out = subprocess.run([driver, str(_free_port())], capture_output=True, text=True, env=env,
                         timeout=600)
    report = out.stdout + out.stderr
    assert "ERROR: AddressSanitizer" not in report, report[-4000:]
    assert "runtime error" not in report, report[-4000:]
    assert out.returncode == 0, report[-4000:]
    assert "all checks passed" in out.stdout
