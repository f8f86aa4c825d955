"""Summaries of scripts/exp/prof_quick.sh: per kernel, mean duration and the
SQ counters per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]


def short(name):
    name = name.replace("void ", "").replace("ta::(anonymous namespace)::", "")
    return name.split("(ta::")[0][:60]


dur = defaultdict(list)
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:60s} n={len(v):4d} mean {sum(v) / len(v) / 1e3:9.1f} us")
ctr = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "sq*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in ctr.items():
    print(k, {n: round(sum(v) / len(v)) for n, v in c.items()})
