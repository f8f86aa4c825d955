"""Experiment: the band walk (flags 0) against the lane walk (TA_PLAN_NO_BLK)
on config 2's uniform batch -- the number of pairs whose CIGAR differs and the
first few differing CIGARs, the first differing character marked."""
import sys

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import TA_PLAN_NO_BLK, Aligner, DevicePlan  # noqa: E402

al = Aligner(0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
b = synth.uniform_batch(N, 1000, 1000, 0x5EED)
res = {}
for flags in (0, TA_PLAN_NO_BLK):
    plan = DevicePlan(al, b, 1, 1, -1, -1, True, flags=flags)
    plan.run()
    res[flags] = plan.results()
    plan.close()
a, r = res[0], res[TA_PLAN_NO_BLK]
bad = [k for k in range(N) if a.cigar(k) != r.cigar(k)]
print(f"differing {len(bad)} of {N}")
for k in bad[:4]:
    x, y = a.cigar(k).decode(), r.cigar(k).decode()
    i = next((i for i in range(min(len(x), len(y))) if x[i] != y[i]), min(len(x), len(y)))
    print(f"pair {k} len {len(x)} vs {len(y)} first diff at {i}")
    print("  band:", x[max(0, i - 60):i], "|", x[i:i + 60])
    print("  lane:", y[max(0, i - 60):i], "|", y[i:i + 60])
