"""CPU-baseline calibration, run in the BUILD container only.

Times the oracle's C restatement (oracle/wfpt_oracle.c, what bench.py's
cpu_baseline runs on the GPU box: kind "port") next to the reference's own
kernels (oracle/_ref, compiled from /root/reference/src by oracle/build_ref.py)
on the same cores, the same inputs and the same loop shape (serial
wiener_like), and records the ratio port/reference. Best of several
interleaved rounds (the container is shared and noisy).

    python tools/calibrate_cpu.py > profiles/r03/cpu_calibration.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KN = (1e-4, 2, 2, 1, 1e-3, 0.05, 0.1)
SIMPLE = (0.5, 0.0, 2.0, 0.5, 0.0, 0.3, 0.0)
FULL = (0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1)


def rate(fn, n, budget=1.5):
    fn()
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget:
            return n * reps / el


def main():
    import oracle
    oracle.build()
    R = oracle.load_ref()
    if R is None:
        sys.exit("oracle/_ref not built: calibration needs the reference tree")
    rng = np.random.default_rng(20261015)
    out = {"host": os.uname().nodename, "cpu": None, "rows": []}
    try:
        with open("/proc/cpuinfo") as fh:
            out["cpu"] = next(l.split(":", 1)[1].strip() for l in fh if l.startswith("model name"))
    except Exception:
        pass
    for name, args, n in (("simple", SIMPLE, 200_000), ("full", FULL, 20_000)):
        x = np.sign(rng.uniform(-0.27, 0.73, n)) * (0.3 + rng.gamma(2.0, 0.45, n))
        port, ref = [], []
        for _ in range(5):  # interleaved best-of-5
            port.append(rate(lambda: oracle.wiener_like(x, *args, *KN), n))
            ref.append(rate(lambda: R.wiener_like(x, *args, *KN), n))
        assert oracle.wiener_like(x, *args, *KN) == R.wiener_like(x, *args, *KN)
        out["rows"].append({"dataset": name, "trials": n, "threads": 1,
                            "loop": "serial wiener_like (wfpt.pyx:66-76)",
                            "port_trials_per_s": max(port), "reference_trials_per_s": max(ref),
                            "port_over_reference": max(port) / max(ref)})
    # all host threads: the port's OpenMP pdf_array (what bench.py's
    # cpu_baseline "value" runs) next to the reference's full_pdf under the
    # prange of wfpt.pyx:40 compiled with -fopenmp (ref_shim.pdf_array_prange)
    nt = len(os.sched_getaffinity(0))
    out["threads_all"] = nt
    for name, args, n in (("simple", SIMPLE, 2_000_000), ("full", FULL, 200_000)):
        x = np.sign(rng.uniform(-0.27, 0.73, n)) * (0.3 + rng.gamma(2.0, 0.45, n))
        kn = (KN[0], KN[1], KN[2], KN[3], KN[4])
        port, ref = [], []
        for _ in range(5):
            port.append(rate(lambda: oracle.pdf_array(x, *args, kn[0], 0, kn[1], kn[2], kn[3],
                                                      kn[4], 0, 0, n_threads=nt), n))
            ref.append(rate(lambda: R.pdf_array_prange(x, *args, kn[0], kn[1], kn[2], kn[3],
                                                       kn[4], nt), n))
        a_ = oracle.pdf_array(x, *args, kn[0], 0, kn[1], kn[2], kn[3], kn[4], 0, 0, n_threads=nt)
        b_ = R.pdf_array_prange(x, *args, kn[0], kn[1], kn[2], kn[3], kn[4], nt)
        assert np.array_equal(a_, b_)
        out["rows"].append({"dataset": name, "trials": n, "threads": nt,
                            "loop": "pdf_array densities, OpenMP over trials (wfpt.pyx:40 "
                                    "prange; -fopenmp is not the reference's own build)",
                            "port_trials_per_s": max(port), "reference_trials_per_s": max(ref),
                            "port_over_reference": max(port) / max(ref)})
    # the DMAT CDF (cdfdif_wrapper.dmat_cdf_array): oracle/cdfdif_oracle.c vs
    # the reference's own extension, 1 thread
    C = oracle.load_ref_cdfdif()
    if C is not None:
        for name, args in (("cdf full", FULL), ("cdf simple", SIMPLE)):
            n = 4000
            x = np.sign(rng.uniform(-0.27, 0.73, n)) * (0.3 + rng.gamma(2.0, 0.45, n))
            x = np.clip(x, -4.9, 4.9)
            port, ref = [], []
            for _ in range(5):
                port.append(rate(lambda: oracle.dmat_cdf_array(x, *args, 0.05, 0.1), n))
                ref.append(rate(lambda: C.dmat_cdf_array(x, *args, 0.05, 0.1), n))
            assert np.array_equal(oracle.dmat_cdf_array(x, *args, 0.05, 0.1),
                                  C.dmat_cdf_array(x, *args, 0.05, 0.1))
            out["rows"].append({"dataset": name, "trials": n, "threads": 1,
                                "loop": "dmat_cdf_array (cdfdif_wrapper.pyx:44-51)",
                                "port_trials_per_s": max(port),
                                "reference_trials_per_s": max(ref),
                                "port_over_reference": max(port) / max(ref)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
