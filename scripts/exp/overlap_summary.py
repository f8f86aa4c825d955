"""Overlap of the pipelined steps from a rocprofv3 kernel trace (bench.py without --serial):
per walk dispatch, the share of its time during which a fill ran.  Usage: overlap_summary.py <trace.csv> <out.json>"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows]
fills = [(s, e) for s, e, n, q in k if "dual_fill_ck_kernel" in n]
walks = [(s, e) for s, e, n, q in k if "traceback_ck_kernel" in n]
ov = []
for s, e in walks:
    t = sum(max(0, min(e, fe) - max(s, fs)) for fs, fe in fills)
    ov.append(t / max(e - s, 1))
span = max(e for s, e, n, q in k if "ta::" in n) - min(s for s, e, n, q in k if "ta::" in n)
out = {"trace": sys.argv[1], "fills": len(fills), "walks": len(walks),
       "fill_queues": sorted({q for s, e, n, q in k if "dual_fill_ck_kernel" in n}),
       "walk_queues": sorted({q for s, e, n, q in k if "traceback_ck_kernel" in n}),
       "walk_share_overlapping_a_fill": [round(x, 3) for x in ov],
       "walks_mostly_overlapped": sum(x > 0.5 for x in ov),
       "mean_fill_us": round(sum(e - s for s, e in fills) / max(len(fills), 1) / 1e3, 1),
       "mean_walk_us": round(sum(e - s for s, e in walks) / max(len(walks), 1) / 1e3, 1)}
pw = [(s, e) for (s, e), x in zip(walks, ov) if x > 0.5]
pf = [(fs, fe) for fs, fe in fills if any(min(fe, e) > max(fs, s) for s, e in walks)]
out["pipelined_walk_us"] = round(sum(e - s for s, e in pw) / max(len(pw), 1) / 1e3, 1)
out["pipelined_fill_us"] = round(sum(e - s for s, e in pf) / max(len(pf), 1) / 1e3, 1)
if pf:  # fill starts of the overlapped stretch: the per-batch period
    st = sorted(s for s, e in pf)
    out["pipelined_fill_period_us"] = round((st[-1] - st[0]) / max(len(st) - 1, 1) / 1e3, 1)
sw = [(s, e) for (s, e), x in zip(walks, ov) if x == 0.0]
sf = [(fs, fe) for fs, fe in fills if (fs, fe) not in pf]
out["serial_walk_us"] = round(sum(e - s for s, e in sw) / max(len(sw), 1) / 1e3, 1)
out["serial_fill_us"] = round(sum(e - s for s, e in sf) / max(len(sf), 1) / 1e3, 1)
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out)[:600])
