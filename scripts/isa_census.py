#!/usr/bin/env python3
"""Static ISA census of a kernel's step loop (gfx950 assembly).

  python scripts/isa_census.py [--kernel 'dual_fill_ck_kernel<1>'] [--out profiles/r06/isa_census_dual_fill_ck.json]

The step loop is the innermost loop (a backward branch with no other loop
inside it) with the most DPP moves -- every step hands values across lanes by
DPP -- then the most v_pk_maximum3_f16 (a local fill's full 16-row argmax tree),
then the fewest VALU instructions (no lane masks): for the dual fills the
unmasked two-step body of full stripes (ta_dual.hip run_steps), one of the
copies the compiler makes of it per stripe count and pass kind.  Reported per
loop iteration and per step: VALU by opcode, SALU by opcode, s_nop (count and
wait states), LDS / global / scratch instructions, and VALU lane-operations per
cell (VALU x 64 / cells the iteration computes: 2 steps x 16 rows x 2 pairs
per lane x 64 lanes).  Uses the same translation-unit builds (and cache) as
scripts/valu_roof.py."""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import valu_roof  # noqa: E402

ROOT = valu_roof.ROOT


def function_lines(text, sym):
    funcs = re.split(r"\n(?=_Z\w+:)", text)
    body = [f for f in funcs if f.split(":")[0].find(sym) >= 0 and "s_endpgm" in f][0].split(".Lfunc_end")[0]
    return body.splitlines()


def loops(lines):
    """(first, last) line index pairs of the backward branches' loops."""
    labels = {m.group(1): k for k, ln in enumerate(lines) if (m := re.match(r"^(\.LBB\w+):", ln))}
    out = []
    for k, ln in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < k:
                out.append((labels[t], k))
    return out


def opcodes(lines, a, b):
    c = collections.Counter()
    for x in lines[a:b + 1]:
        tok = x.strip().split()
        if tok and not tok[0].startswith((";", ".")) and re.match(r"^[a-z]", tok[0]):
            c[tok[0]] += 1
            if tok[0] == "s_nop":
                c["(s_nop wait states)"] += int(tok[1], 0) + 1
    return c


def step_loop(lines):
    """The innermost loop with the most DPP moves, then the most three-input maxima, then the
    fewest VALU."""
    ls = loops(lines)
    inner = [(a, b) for a, b in ls if not any(a <= c and d <= b and (c, d) != (a, b) for c, d in ls)]
    best = None
    for a, b in inner:
        c = opcodes(lines, a, b)
        dpp = sum(n for o, n in c.items() if "_dpp" in o)
        valu = sum(n for o, n in c.items() if o.startswith("v_"))
        key = (dpp, c["v_pk_maximum3_f16"], -valu)
        if best is None or key > best[0]:
            best = (key, (a, b), c)
    return best[1], best[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="dual_fill_ck_kernel<1>")
    ap.add_argument("--steps", type=int, default=2, help="steps per loop iteration (the dual fills: 2)")
    ap.add_argument("--cells-per-step", type=int, default=16 * 2 * 64, help="cells per step and wave")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06", "isa_census_dual_fill_ck.json"))
    a = ap.parse_args()
    src, defines, sym = valu_roof.KERNELS[a.kernel]
    lines = function_lines(valu_roof.asm_of(src, defines), sym)
    (lo, hi), c = step_loop(lines)
    cls = lambda p: {o: n for o, n in sorted(c.items(), key=lambda kv: -kv[1]) if o.startswith(p)}  # noqa: E731
    valu, salu = cls("v_"), {o: n for o, n in cls("s_").items() if o != "s_nop"}
    nv = sum(valu.values())
    res = {
        "kernel": a.kernel, "source": f"bioinfo1_amd/csrc/{src} {' '.join(defines)}",
        "method": __doc__.split("\n\n")[1].strip(),
        "loop_lines": [lo, hi], "steps_per_iteration": a.steps,
        "valu_per_step": round(nv / a.steps, 2),
        "salu_per_step": round(sum(salu.values()) / a.steps, 2),
        "s_nop_per_step": round(c.get("s_nop", 0) / a.steps, 2),
        "s_nop_wait_states_per_step": round(c.get("(s_nop wait states)", 0) / a.steps, 2),
        "lds_per_step": round(sum(n for o, n in c.items() if o.startswith("ds_")) / a.steps, 2),
        "global_per_step": round(sum(n for o, n in c.items() if o.startswith(("global_", "buffer_"))) / a.steps, 2),
        "scratch_per_step": round(sum(n for o, n in c.items() if o.startswith("scratch_")) / a.steps, 2),
        "valu_lane_ops_per_cell": round(nv / a.steps * 64 / a.cells_per_step, 3),
        "valu": valu, "salu": salu,
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("valu", "salu", "method")}))
    print("VALU:", list(valu.items())[:20])
    print("SALU:", list(salu.items())[:15])


if __name__ == "__main__":
    main()
