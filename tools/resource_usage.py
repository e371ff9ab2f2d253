"""Register / scratch / LDS / occupancy of the gfx950 kernels, from the
compiler's own resource-usage remarks (the numbers the code object carries).

    python tools/resource_usage.py [name-filter ...] [-D NAME=VAL ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hddm_amd", "csrc", "wfpt_kernels.hip")
FIELDS = ("VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
          "LDS Size [bytes/block]")


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def usage(defines=()):
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
               "-fPIC", "--offload-arch=gfx950", *[f"-D{d}" for d in defines], "-c", SRC, "-o",
               os.path.join(td, "k.o"), "-Rpass-analysis=kernel-resource-usage"]
        txt = subprocess.run(cmd, capture_output=True, text=True, cwd=td).stderr
    rows, cur = [], None
    for line in txt.splitlines():
        m = re.search(r"remark: (Function Name|[A-Za-z ]+(?:\[[^\]]*\])?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None and key in FIELDS:
            cur[key] = val
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        r["name"] = n
    return rows


def main():
    args = sys.argv[1:]
    defines, filt = [], []
    while args:
        a = args.pop(0)
        if a == "-D":
            defines.append(args.pop(0))
        else:
            filt.append(a)
    for r in usage(defines):
        if filt and not any(f in r["name"] for f in filt):
            continue
        print(f"{r['name'][:70]:70s} " + " ".join(f"{k.split()[0]}={r.get(k, '-')}" for k in FIELDS))


if __name__ == "__main__":
    main()
