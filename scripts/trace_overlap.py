#!/usr/bin/env python3
"""How much of each kernel's time ran beside another kernel, from a rocprofv3
--kernel-trace CSV (the pipelined config 2: batch k's band walk and run
formatter beside batch k+1's fill).

  python scripts/trace_overlap.py <dir-with-kernel_trace.csv> [--out file.txt]

Prints, per kernel name: dispatches, mean duration, and the fraction of its
busy time during which a dual fill dispatch was also running; and the mean gap
between consecutive fill dispatches (the pipelined step's fill-to-fill time)."""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("ta::(anonymous namespace)::", "")
    return name.split("(ta::")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    ks = []
    with open(f) as fh:
        for row in csv.DictReader(fh):
            ks.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), short(row["Kernel_Name"])))
    ks.sort()
    fills = [(s, e) for s, e, n in ks if n.startswith("dual_fill_kernel")]
    out = []
    by = defaultdict(list)
    for s, e, n in ks:
        by[n].append((s, e))
    for n, iv in sorted(by.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        tot = sum(e - s for s, e in iv)
        ov = 0
        if not n.startswith("dual_fill_kernel"):
            for s, e in iv:
                for fs, fe in fills:
                    ov += max(0, min(e, fe) - max(s, fs))
        out.append(f"{n:45s} dispatches {len(iv):4d}  mean {tot / len(iv) / 1e3:9.1f} us  "
                   f"beside a fill {100.0 * ov / tot if tot else 0:5.1f} %")
    if len(fills) > 1:
        gaps = [b[0] - a[0] for a, b in zip(fills, fills[1:])]
        out.append(f"fill start to next fill start: median {statistics.median(gaps) / 1e3:.1f} us over {len(gaps)}")
    txt = "\n".join(out)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
