#!/usr/bin/env python3
"""The VALU issue roof of a fill kernel, from measured per-opcode rates.

  python scripts/valu_roof.py [--rates profiles/r03_valu_rates.txt] [--out profiles/valu_roof.json]

1. Per-opcode issue cost: scripts/exp/ubench/valu_rates (run on the MI355X)
   prints cycles per wave64 instruction per SIMD for the opcodes the kernels
   use (8 independent chains x 8 waves per SIMD: throughput, not latency).
   The measured values sit ~5-30 % above the issue class (loop overhead);
   each opcode is assigned its class, 2 or 4 cycles (the nearest of 2, 4, 8, 16).
2. Instruction mix: a static census of the kernel's step loop (the innermost
   loop with the most DPP hand-offs, scripts/isa_census.py) in the gfx950
   assembly of its translation unit.
3. Mixed roof: cycles per wave-instruction = census-weighted mean of the
   classes; peak = 256 CU x 4 SIMD x 64 lanes x 2.4 GHz / that mean, in VALU
   lane-operations per second -- the number bench.py's valu.frac divides by.
Opcodes the ubench does not cover count as 2 cycles (packed ones as 4): that
can only raise the roof, i.e. lower the reported fraction."""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "bioinfo1_amd", "csrc")
SIMDS, CLOCK = 256 * 4, 2.4e9

# kernel (as rocprofv3 names it; bench.py dominant_kernel) -> (source, defines, symbol substring)
KERNELS = {
    "dual_fill_kernel<1, true, true>": ("ta_dual.hip", ["-DTA_DUAL_MODE=1", "-DTA_DUAL_CIGAR=1", "-DTA_DUAL_BLK"],
                                        "dual_fill_kernelILi1ELb1ELb1E"),
    "dual_fill_ck_kernel<1>": ("ta_dual.hip", ["-DTA_DUAL_MODE=1", "-DTA_DUAL_CIGAR=1", "-DTA_DUAL_BLK", "-DTA_DUAL_CK=1"],
                               "dual_fill_ck_kernelILi1E"),
    "dual_fill_ck_kernel<0>": ("ta_dual.hip", ["-DTA_DUAL_MODE=0", "-DTA_DUAL_CIGAR=1", "-DTA_DUAL_BLK", "-DTA_DUAL_CK=1"],
                               "dual_fill_ck_kernelILi0E"),
    "dual_fill_ck_kernel<2>": ("ta_dual.hip", ["-DTA_DUAL_MODE=2", "-DTA_DUAL_CIGAR=1", "-DTA_DUAL_BLK", "-DTA_DUAL_CK=1"],
                               "dual_fill_ck_kernelILi2E"),
    "dual_fill_kernel<1, true, false>": ("ta_dual.hip", ["-DTA_DUAL_MODE=1", "-DTA_DUAL_CIGAR=1"],
                                         "dual_fill_kernelILi1ELb1ELb0E"),
    "dual_fill_kernel<2, true, false>": ("ta_dual.hip", ["-DTA_DUAL_MODE=2", "-DTA_DUAL_CIGAR=1"],
                                         "dual_fill_kernelILi2ELb1ELb0E"),
    "flex_fill_kernel<2, true>": ("ta_flex.hip", ["-DTA_FLEX_MODE=2", "-DTA_FLEX_CIGAR=1"], "flex_fill_kernelILi2ELb1E"),
    "flex_fill_kernel<1, true>": ("ta_flex.hip", ["-DTA_FLEX_MODE=1", "-DTA_FLEX_CIGAR=1"], "flex_fill_kernelILi1ELb1E"),
    "flex_fill_ck_kernel<2>": ("ta_flex.hip", ["-DTA_FLEX_MODE=2", "-DTA_FLEX_CIGAR=1", "-DTA_FLEX_CK=1"], "flex_fill_ck_kernelILi2E"),
    "flex_fill_ck_kernel<1>": ("ta_flex.hip", ["-DTA_FLEX_MODE=1", "-DTA_FLEX_CIGAR=1", "-DTA_FLEX_CK=1"], "flex_fill_ck_kernelILi1E"),
    "affine_dual_fill_kernel<2, true>": ("ta_affine.hip", [], "affine_dual_fill_kernelILi2ELb1E"),
}


def parse_rates(path):
    rates = {}
    for ln in open(path):
        m = re.match(r"^(\S.*?)\s+[\d.]+ ms .*=> ([\d.]+) cycles", ln)
        if not m:
            continue
        name, cyc = m.group(1).strip(), float(m.group(2))
        if "(x2)" in name:  # two instructions per link: name the first opcode only when the second is known
            continue
        name = name.split(" ")[0].split("(")[0]
        rates.setdefault(name, cyc)
    return rates


# Opcodes measured only in a pair, or whose single-op kernel is not a throughput test:
#  v_mov_b32      -- "v_mov_b32+v_add_u32 (x2)" averages 2.33 with v_add_u32 at 2.89: ~1.8, class 2
#  v_readlane_b32 -- its pair kernel chains every lane read through one SGPR (serialised);
#                    a VOP3 cross-lane read, counted as class 4
#  v_cndmask_b32  -- the VOP2 form's kernel reads a VCC nothing writes (22.9, an artifact);
#                    the VOP3 form with an SGPR mask runs 4.30, and the e32 form is counted alike
DERIVED = {"v_mov_b32": 2.0, "v_readlane_b32": 4.0, "v_cndmask_b32": None}


def issue_class(c):
    return min((2, 4, 8, 16), key=lambda k: abs(k - c))


def base_op(op):
    op = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    return op


def asm_of(src, defines):
    """gfx950 assembly of a translation unit (cached per source + defines)."""
    key = src.rsplit(".", 1)[0] + "".join(d.replace("-D", "_").replace("=", "") for d in defines)
    out = os.path.join("/tmp/valu_roof", key)
    os.makedirs(out, exist_ok=True)
    stem = src.rsplit(".", 1)[0]
    s_file = f"{out}/{stem}-hip-amdgcn-amd-amdhsa-gfx950.s"
    if not os.path.exists(s_file) or os.path.getmtime(s_file) < os.path.getmtime(os.path.join(CS, src)):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", *defines,
                               "--cuda-device-only", "-S", os.path.join(CS, src), "-o", s_file], cwd=out,
                              stderr=subprocess.DEVNULL)
    return open(s_file).read()


def census(src, defines, sym):
    """VALU opcodes of the kernel's step loop (scripts/isa_census.py step_loop: the innermost
    loop with the most DPP moves, then the most three-input maxima, then the fewest VALU)."""
    import isa_census

    lines = isa_census.function_lines(asm_of(src, defines), sym)
    _, c = isa_census.step_loop(lines)
    return collections.Counter({o: n for o, n in c.items() if o.startswith("v_")})


def roof(mix, rates):
    tot = cyc = 0.0
    per = {}
    for op, n in mix.items():
        b = base_op(op)
        if op.endswith("_dpp"):
            b = "v_mov_b32_dpp" if op.startswith("v_mov") else b
        meas = rates.get(op)  # an encoding measured on its own (v_cndmask_b32_e64)
        if meas is None and b in DERIVED:
            meas = DERIVED[b] if DERIVED[b] is not None else rates.get(b + "_e64")
        if meas is None:
            meas = rates.get(b)
        if meas is None and op.endswith("_dpp"):
            meas = rates.get("v_mov_b32_dpp")
        k = issue_class(meas) if meas is not None else (4 if b.startswith("v_pk_") else 2)
        per[op] = {"count": n, "measured_cycles": meas, "class_cycles": k}
        tot += n
        cyc += n * k
    mean = cyc / tot
    return mean, per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default=os.path.join(ROOT, "profiles", "r03_valu_rates.txt"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "valu_roof.json"))
    a = ap.parse_args()
    rates = parse_rates(a.rates)
    res = {"rates_source": os.path.relpath(a.rates, ROOT), "method": __doc__.split("\n\n")[1].strip(),
           "kernels": {}}
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(len(KERNELS)) as ex:  # compile the translation units in parallel
        mixes = dict(zip(KERNELS, ex.map(lambda kv: census(*kv[1]), KERNELS.items())))
    for tag in KERNELS:
        mix = mixes[tag]
        mean, per = roof(mix, rates)
        peak = SIMDS * 64 * CLOCK / mean / 1e12
        four = sum(v["count"] for v in per.values() if v["class_cycles"] >= 4) / sum(v["count"] for v in per.values())
        res["kernels"][tag] = {"mean_cycles_per_wave_instr": round(mean, 3), "peak_lane_tops": round(peak, 2),
                               "share_4cycle_ops": round(four, 3), "hot_loop_valu_instrs": sum(mix.values()),
                               "mix": dict(sorted(per.items(), key=lambda kv: -kv[1]["count"]))}
        print(f"{tag}: mean {mean:.3f} cycles/wave-instr, 4-cycle share {four:.2f}, peak {peak:.1f} T lane-ops/s")
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
