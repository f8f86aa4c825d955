#!/usr/bin/env python3
"""Shrink a scripts/profile.sh output directory on the GPU box before it is
copied back (gpurun returns at most 64 MiB): in every counter_collection.csv
keep only the rows of this repository's kernels (ta:: / tm:: symbols), keep
every *_stats.csv and the logs, and delete the other trace files (the
per-dispatch traces of the synthetic-input generator dominate their size).

  python scripts/prof_compact.py gpurun_out/<tag>"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
        base = os.path.basename(f)
        if base.endswith("counter_collection.csv"):
            with open(f) as fh:
                rows = list(csv.DictReader(fh))
            keep = [r for r in rows if "ta::" in r.get("Kernel_Name", "") or "tm::" in r.get("Kernel_Name", "")]
            if rows:
                with open(f, "w", newline="") as fh:
                    w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
                    w.writeheader()
                    w.writerows(keep)
        elif not base.endswith("_stats.csv"):
            os.remove(f)
    for f in glob.glob(os.path.join(d, "**", "*"), recursive=True):
        if os.path.isfile(f) and not f.endswith((".csv", ".log", ".json")):
            os.remove(f)


if __name__ == "__main__":
    main()
