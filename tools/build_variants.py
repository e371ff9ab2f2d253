"""Build named library variants for A/B runs (hddm_amd/lib/variants/libwfpt_<name>.so).

    python tools/build_variants.py name=DEF1,DEF2 name2=DEF ...   (DEF: NAME=VAL)
"""
import concurrent.futures as cf
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from hddm_amd import build as hb
    d = os.path.join(hb.LIBDIR, "variants")
    os.makedirs(d, exist_ok=True)
    specs = {}
    for a in sys.argv[1:]:
        name, _, defs = a.partition("=")
        specs[name] = [x for x in defs.split(",") if x]
    with cf.ThreadPoolExecutor(3) as ex:
        fs = {ex.submit(hb.build, True, False, v, os.path.join(d, f"libwfpt_{k}.so")): k
              for k, v in specs.items()}
        for f in cf.as_completed(fs):
            print(fs[f], f.result(), flush=True)


if __name__ == "__main__":
    main()
