"""HostPipeline with and without the traceback/fill overlap, alternating, config 2."""
import sys, json
sys.path.insert(0, ".")
import bench
from bioinfo1_amd.align import Aligner

args = bench.parse(["--no-cpu"])
D = bench.Dist(args)
batch, aux, _ = bench.make_batch(args, D)
al = Aligner(0)
sc = (1, -1, -1)
for rnd in range(3):
    for ov in (False, True):
        r = bench.host_to_host_pipelined(al, batch, 1, sc, True, args, 0, reps=30, overlap=ov)
        print(rnd, "overlap" if ov else "serial ", r["value"], r["ms_per_batch"], r["parity"]["bit_exact"], flush=True)
