#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc passes (scripts/pmc_walk.sh output):
  scripts/pmc_sum.py <gpurun_out/tag> <profiles/out.json> "<what>"
Kernel names as rocprofv3 prints them, namespace and parameters dropped."""
import csv
import glob
import json
import sys
from collections import defaultdict

src, dst, what = sys.argv[1], sys.argv[2], sys.argv[3]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(src + "/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, cs in acc.items():
    name = k.replace("ta::(anonymous namespace)::", "").replace("void ", "").split("(ta::")[0]
    out[name] = {c: sum(v) / len(v) for c, v in sorted(cs.items())}
json.dump({"what": what, "kernels": out}, open(dst, "w"), indent=1)
for k, v in out.items():
    print(k, {c: "%.4g" % x for c, x in v.items() if c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES")})
