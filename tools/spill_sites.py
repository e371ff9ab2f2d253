"""Scratch spill / reload sites of one kernel, attributed to source lines.

    python tools/spill_sites.py [kernel-substring] [-D...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else "lean_kernelILi3ELb0ELi0E"
    defs = [a for a in sys.argv[2:] if a.startswith("-D")]
    out = "/tmp/wfpt_spill.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-fast-math", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-gline-tables-only", *defs, "-o", out,
                    os.path.join(ROOT, "hddm_amd/csrc/wfpt_kernels.hip")], check=True,
                   stderr=subprocess.DEVNULL)
    s = open(out).read()
    files = {m.group(1): m.group(3).split("/")[-1]
             for m in re.finditer(r'\.file\s+(\d+)\s+("[^"]*"\s+)?"([^"]+)"', s)}
    m = re.search(r"^(_Z\w*" + re.escape(pat) + r"\w*):", s, re.M)
    end = s.index(".Lfunc_end", m.end())
    cur = None
    for i, l in enumerate(s[m.end():end].splitlines()):
        mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if mm:
            cur = f"{files.get(mm.group(1), mm.group(1))}:{mm.group(2)}"
        elif "scratch_" in l:
            print(i, cur, l.strip()[:90])


if __name__ == "__main__":
    main()
