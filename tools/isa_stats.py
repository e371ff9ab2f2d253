"""Static ISA statistics of one kernel (device assembly via hipcc -S).

    python tools/isa_stats.py [kernel-substring] [-D...]
Prints VGPR/SGPR counts, occupancy and the instruction histogram.
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else "fast_kernelILi3ELb0ELi0E"
    defs = [a for a in sys.argv[2:] if a.startswith("-D")]
    out = "/tmp/wfpt_isa.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-fast-math", "--offload-arch=gfx950", "--cuda-device-only", "-S", *defs,
                    "-o", out, os.path.join(ROOT, "hddm_amd/csrc/wfpt_kernels.hip")], check=True,
                   stderr=subprocess.DEVNULL)
    s = open(out).read()
    for m in re.finditer(r"^(_Z\w*" + re.escape(pat) + r"\w*):", s, re.M):
        name = m.group(1)
        end = s.index(".Lfunc_end", m.end())
        body = s[m.end():end].splitlines()
        ins = [l.strip().split()[0] for l in body
               if l.startswith("\t") and not l.strip().startswith((".", ";"))]
        info = s[end:end + 4000]
        g = lambda k: (re.search(k + r":\s*(\d+)", info) or [None, "?"])[1]
        print(f"{name}: {len(ins)} instrs, VGPR {g('NumVgprs')}, SGPR {g('TotalNumSgprs')}, "
              f"scratch {g('ScratchSize')}, occupancy {g('Occupancy')}")
        for k, v in collections.Counter(ins).most_common(int(os.environ.get("TOP", "25"))):
            print(f"   {k:28s}{v}")


if __name__ == "__main__":
    main()
