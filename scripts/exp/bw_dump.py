"""Experiment (with the TA_BW_DUMP library build): the band walk's raw events
(one byte each in place of the CIGAR) of config 2's uniform batch, merged into
runs here and compared with the lane walk's CIGAR (TA_PLAN_NO_BLK); for the
first few differing pairs, the item sequences around the first difference."""
import re
import sys

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import TA_PLAN_NO_BLK, Aligner, DevicePlan  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000


def items_of_events(ev):
    out = []
    for v in ev:
        kd, mop = v >> 2, v & 3
        out += [2] * kd
        if mop != 3:
            out.append(mop)
    return out


def items_of_cigar(s):
    out = []
    for cnt, op in re.findall(r"(\d+)([MID])", s):
        out += ["MID".index(op)] * int(cnt)
    return out[::-1]  # walk order


al = Aligner(0)
b = synth.uniform_batch(N, 1000, 1000, 0x5EED)
res = {}
for flags in (0, TA_PLAN_NO_BLK):
    plan = DevicePlan(al, b, 1, 1, -1, -1, True, flags=flags)
    plan.run()
    res[flags] = plan.results()
    plan.close()
bad = 0
for k in range(N):
    ev = list(res[0].cigar(k))
    got = items_of_events(ev)
    want = items_of_cigar(res[TA_PLAN_NO_BLK].cigar(k).decode())
    if got != want:
        bad += 1
        if bad <= 3:
            i = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), min(len(got), len(want)))
            # the event holding item i
            acc, e = 0, 0
            while e < len(ev) and acc + (ev[e] >> 2) + (0 if ev[e] & 3 == 3 else 1) <= i:
                acc += (ev[e] >> 2) + (0 if ev[e] & 3 == 3 else 1)
                e += 1
            print(f"pair {k}: items {len(got)} vs {len(want)}, first diff at item {i} (event {e} of {len(ev)})")
            print("  got :", "".join("MID"[x] for x in got[max(0, i - 30):i + 30]))
            print("  want:", "".join("MID"[x] for x in want[max(0, i - 30):i + 30]))
            print("  events:", [(v >> 2, v & 3) for v in ev[max(0, e - 6):e + 6]])
print(f"event lists differing from the lane walk: {bad} of {N}")
