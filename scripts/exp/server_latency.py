"""Experiment: single-call latency of the resident single-pair server
(ta_server_*) and its device-side phase times, per shape."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Server  # noqa: E402

srv = Server(0, 1)
for n, m in ((5, 9), (64, 64), (200, 200), (1000, 1000)):
    b = synth.related_batch(1, n, m, seed=5)
    q, t = b.query(0), b.target(0)
    for _ in range(50):
        srv.align(q, t, 1, -1, -1)
    reps = 2000 if n < 500 else 200
    lat, ph = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        srv.align(q, t, 1, -1, -1)
        lat.append((time.perf_counter() - t0) * 1e6)
        ph.append(srv.last_times(0))
    ph = np.array(ph)
    print(f"{n}x{m}: host p50 {np.percentile(lat, 50):.1f} us p99 {np.percentile(lat, 99):.1f}; device p50 "
          f"request+copy {np.median(ph[:, 0]):.2f} fill+walk {np.median(ph[:, 1]):.2f} "
          f"results {np.median(ph[:, 2]):.2f} fence {np.median(ph[:, 3]):.2f} us", flush=True)
srv.close()
