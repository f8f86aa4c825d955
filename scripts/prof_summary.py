#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run into profiles/<round>_*.

  python scripts/prof_summary.py gpurun_out/<tag> <round-tag> <workload-tag>

Writes profiles/<round-tag>_kernel_stats.csv (the rocprofv3 --stats summary),
profiles/<round-tag>_pmc.json (per-kernel average counters per dispatch) and
merges the dominant fill kernel's HBM traffic per step and its VALU
instructions per DP cell into profiles/traffic_by_kernel.json and
profiles/valu_by_kernel.json, keyed "<kernel>|<workload-tag>" with the kernel
named as rocprofv3 prints it (bench.py dominant_kernel reads the same key, so a
line never quotes another kernel's counters).  profiles/traffic.json and
valu.json are the r01-r04 tables keyed by workload alone (history).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come
from separate passes; FETCH_SIZE is reported in KB and reads 1/2 of the bytes
of wide coalesced streaming reads on gfx950, so it is doubled; WRITE_SIZE (KB)
is taken as is."""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pat):
    r = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return r[0] if r else None


def pmc_avgs(d):
    f = find(d, "*counter_collection.csv")
    if not f:
        return {}
    acc = defaultdict(lambda: defaultdict(list))
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "?")
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def bench_line(d):
    for name in ("prof_trace.log", "prof_sq.log"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            for ln in open(p):
                if ln.startswith("{"):
                    return json.loads(ln)
    return None


def short_name(k):
    """'void ta::(anonymous namespace)::dual_fill_kernel<1, true, true>(ta::FillArgs)'
    -> 'dual_fill_kernel<1, true, true>' (bench.py dominant_kernel's form)"""
    k = k.split("(ta::")[0] if "(ta::" in k else k
    return k.replace("void ", "").replace("ta::(anonymous namespace)::", "").strip()


def merge(path, key, entry):
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[key] = entry
    with open(path, "w") as fh:
        json.dump(dict(sorted(d.items())), fh, indent=1)


def main():
    src, rtag, wtag = sys.argv[1], sys.argv[2], sys.argv[3]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    st = find(os.path.join(src, "prof_trace"), "*kernel_stats.csv")
    if st:
        shutil.copy(st, os.path.join(prof, f"{rtag}_kernel_stats.csv"))
    pmc = {}
    for part in ("prof_fetch", "prof_write", "prof_sq", "prof_busy", "prof_wait"):
        for k, cs in pmc_avgs(os.path.join(src, part)).items():
            pmc.setdefault(k, {}).update(cs)
    with open(os.path.join(prof, f"{rtag}_pmc.json"), "w") as fh:
        json.dump(pmc, fh, indent=1)
    fill = {k: v for k, v in pmc.items() if "fill_kernel" in k or "fill_ck_kernel" in k}
    if fill:
        # the dominant fill launch (dual and int32 fills both match; the int32
        # one may be the near-empty fallback launch for '-' queries)
        k, cs = max(fill.items(), key=lambda kv: kv[1].get("SQ_INSTS_VALU", 0))
        bl = bench_line(src)
        # per-dispatch averages x dispatches per step = the step's fill (every
        # step repeats the same chunk dispatches)
        per_step = bl.get("chunks", 1) if bl else 1
        tr = None
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            tr = int((2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024 * per_step)
        key = f"{short_name(k)}|{wtag}"
        # the source the counters were measured on (bench.py quotes them only while it matches)
        sys.path.insert(0, ROOT)
        import bench

        meta = {"profile": rtag, "kernel": k, "dispatches_per_step": per_step,
                "src_hash": bench.kernel_src_hash(short_name(k))}
        if bl and (bl.get("roofline") or {}).get("kernel") not in (None, short_name(k)):
            print("WARNING: bench line names", bl["roofline"]["kernel"], "but the dominant PMC kernel is", k)
        merge(os.path.join(prof, "traffic_by_kernel.json"), key, dict(value=tr, **meta))
        if "SQ_INSTS_VALU" in cs:
            # SQ_INSTS_VALU counts wave-instructions; cells per step from the bench line
            cells = bl["config"]["cells_per_gpu"]
            # per lane-cell: wave-instr x 64 lanes / cells
            merge(os.path.join(prof, "valu_by_kernel.json"), key,
                  dict(value=round(cs["SQ_INSTS_VALU"] * 64 * per_step / cells, 3), **meta))
        print(k, json.dumps(cs, indent=1))
    print("summary written to", prof)


if __name__ == "__main__":
    main()
