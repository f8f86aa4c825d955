#!/usr/bin/env python3
"""Static instruction census of the loops in a compiled kernel.

  TA_CENSUS_FLAGS="-DTA_TU_MISC" python scripts/isa_census.py <kernel-substring> [asm.s]

Builds bioinfo1_amd/csrc/ta_kernels.hip with -save-temps (unless an .s is
given), finds the kernel whose symbol contains the substring, and for each
innermost loop (header label .. last backward branch to it) prints the count
of VALU / SALU / VMEM / LDS / DPP instructions.  Used to track VALU ops per
DP cell (a step updates 16 rows = 16 cells per lane)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def asm_text(path=None):
    if path:
        return open(path).read()
    out = "/tmp/ta_census"
    os.makedirs(out, exist_ok=True)
    extra = os.environ.get("TA_CENSUS_FLAGS", "-DTA_FILL_MODE=1 -DTA_FILL_CIGAR=1").split()
    src = os.environ.get("TA_CENSUS_SRC", "ta_kernels")  # or ta_dual (with -DTA_DUAL_MODE=.. -DTA_DUAL_CIGAR=..)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", *extra, "-c",
                           os.path.join(ROOT, f"bioinfo1_amd/csrc/{src}.hip"), "-o", f"{out}/k.o", "-save-temps"],
                          cwd=out, stderr=subprocess.DEVNULL)
    return open(f"{out}/{src}-hip-amdgcn-amd-amdhsa-gfx950.s").read()


def classify(op):
    if op.startswith("v_") and "_dpp" in op:
        return "DPP"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "LANE"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("s_waitcnt", "s_nop", "s_cbranch", "s_branch", "s_endpgm")):
        return "CTRL"
    if op.startswith(("s_load", "s_buffer")):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    return "OTHER"


def main():
    sub = sys.argv[1]
    text = asm_text(sys.argv[2] if len(sys.argv) > 2 else None)
    funcs = re.split(r"\n(?=_Z\w+:)", text)
    f = [x for x in funcs if x.split(":")[0].find(sub) >= 0 and "s_endpgm" in x]
    if not f:
        sys.exit(f"no kernel matching {sub}")
    body = f[0].split(".Lfunc_end")[0]  # whole kernel (it may hold several s_endpgm)
    lines = body.splitlines()
    labels = {}
    for k, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = k
    loops = []
    for k, ln in enumerate(lines):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < k:
                loops.append((labels[tgt], k))
    print(f"{f[0].split(':')[0][:90]}")
    # DP step loops: one step = 2 DPP moves (the wave_shr:1 hand-offs); static
    # counts include the rarely taken chunk-load branches
    seen = set()
    for a, b in sorted(set(loops)):
        c = collections.Counter()
        for ln in lines[a:b + 1]:
            t = ln.strip().split()
            if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
                c[classify(t[0])] += 1
        steps = c["DPP"] // 2
        if steps == 0 or (c["DPP"], c["VALU"]) in seen:
            continue
        seen.add((c["DPP"], c["VALU"]))
        tot = sum(c.values())
        nop = sum(1 for ln in lines[a:b + 1] if ln.strip().startswith("s_nop"))
        mov = sum(1 for ln in lines[a:b + 1] if ln.strip().startswith("v_mov_b32_e32"))
        print(f"  step loop lines {a}-{b}: {steps} step(s), per step: VALU={c['VALU'] / steps:.1f} "
              f"SALU={c['SALU'] / steps:.1f} VMEM={c['VMEM'] / steps:.1f} total={tot / steps:.1f} "
              f"(s_nop={nop / steps:.1f} v_mov={mov / steps:.1f})")


if __name__ == "__main__":
    main()
