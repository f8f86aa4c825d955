#!/usr/bin/env bash
# One PMC pass (VALU/SALU instruction counts) of a bench command on the GPU box:
#   scripts/pmc_quick.sh <tag> [bench args...]  -> gpurun_out/<tag>/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-q}"; shift || true
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS --output-format csv -d "$OUT/pmc" -o run \
  -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-parity --no-host --no-score-only "$@" > "$OUT/pmc.log" 2>&1
rc=$?; echo "pmc rc=$rc"
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
out = sys.argv[1]
f = glob.glob(out + "/pmc/**/*counter_collection.csv", recursive=True)
acc = defaultdict(lambda: defaultdict(list))
for row in csv.DictReader(open(f[0])):
    acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
bl = [json.loads(l) for l in open(out + "/pmc.log") if l.startswith("{")][-1]
cells = bl["config"]["cells_per_gpu"]; ch = bl.get("chunks", 1)
pairs = bl["config"]["pairs_per_gpu"]
for k, cs in acc.items():
    if "traceback" in k:
        v = sum(cs["SQ_INSTS_VALU"]) / len(cs["SQ_INSTS_VALU"])
        s = sum(cs["SQ_INSTS_SALU"]) / len(cs["SQ_INSTS_SALU"])
        l = sum(cs["SQ_INSTS_LDS"]) / len(cs["SQ_INSTS_LDS"])
        print(k[:70], "per pair: VALU %.0f SALU %.0f LDS %.0f" % (v * ch / pairs, s * ch / pairs, l * ch / pairs))
    if "fill" in k:
        v = sum(cs["SQ_INSTS_VALU"]) / len(cs["SQ_INSTS_VALU"])
        s = sum(cs["SQ_INSTS_SALU"]) / len(cs["SQ_INSTS_SALU"])
        print(k[:70], "VALU/cell %.3f SALU/cell %.3f" % (v * 64 * ch / cells, s * 64 * ch / cells))
PY
