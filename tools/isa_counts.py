"""Static instruction counts per kernel from a gfx950 assembly listing
(`make -C odelib_amd/csrc asm UNIT=inst_chain20`): total, v_accvgpr moves, fp64 VALU,
DPP movs, scratch accesses.  CPU only.

    python tools/isa_counts.py odelib_amd/csrc/inst_chain20-gfx950.s --match 'k_integrate_split|Li1ELb1ELb1'
"""
from __future__ import annotations

import argparse
import json
import re


def kernels(path: str, match: str):
    txt = open(path).read()
    for m in re.finditer(r"^(_ZN2oe\w+):", txt, re.M):
        name = m.group(1)
        if not re.search(match, name):
            continue
        end = txt.find(".Lfunc_end", m.end())
        ins = [l.split()[0] for l in txt[m.end():end].splitlines()
               if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
        yield name, {
            "instructions": len(ins),
            "v_accvgpr": sum(i.startswith("v_accvgpr") for i in ins),
            "valu_f64": sum(i.startswith("v_") and i.endswith("_f64") for i in ins),
            "dpp_mov": sum(i.startswith("v_mov_b32_dpp") for i in ins),
            "scratch": sum(i.startswith("scratch_") for i in ins),
            "salu": sum(i.startswith("s_") for i in ins),
        }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--match", default=".")
    a = ap.parse_args()
    for name, c in kernels(a.asm, a.match):
        print(json.dumps({"kernel": name, **c}))


if __name__ == "__main__":
    main()
