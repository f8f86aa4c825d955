#!/usr/bin/env python3
"""Benchmark of the team::Align hot path on MI355X (BASELINE.json).

Default workload = BASELINE config 2: one "step" is one pass of the path over
one batch -- the DP fill kernels and the traceback/CIGAR kernel for 10,000
synthetic 1 kb x 1 kb read-vs-window pairs per GPU, Smith-Waterman (local),
match/mismatch/gap = 1/-1/-1, CIGAR on -- with the inputs resident in HBM
before the timed region.

Multi-GPU: one process per GPU.  `--gpus N` without a
torch.distributed environment starts the N ranks itself (torch.distributed.run
as a child process, before this process touches the GPU) and exits with its
status; every rank checks WORLD_SIZE == --gpus.  Config 2 is weak-scaled (each
rank aligns its own 10,000-pair range of the seeded stream); config 4
(`--workload cfg4`) strong-scales one fixed read set (the config-3 stand-in)
range-split by cells (bioinfo1_amd/shard.py).  In every step each rank's
results -- the fixed per-pair records (score, target_begin, cigar_len) and the
CIGAR bytes, compacted on the device -- are all-gathered over RCCL inside the
timed region: the records of step k right after its kernels, its CIGAR bytes
(whose sizes the records carry) once step k+1 is enqueued, so neither stalls
the GPU; all gathers are drained before the clock stops.  value = total cells
of all ranks / max over ranks of the step time.

Also reported (rank 0):
  roofline      -- the dominant fill kernel: algorithmic bytes per launch /
                   its HIP-event duration on its launch stream, against the
                   8 TB/s HBM peak; traffic = rocprofv3 PMC HBM bytes per launch
                   of this same command (profiles/traffic.json, collected by
                   scripts/profile.sh; rocprof counters cannot be read in-process).
  valu          -- the same kernel against the VALU int32 issue roof (the roof
                   that binds this integer DP; ops/cell from profiles/valu.json).
  pipeline      -- the timed steps run through align.DevicePipeline (batch k's
                   traceback beside batch k+1's fill, one workspace per slot)
                   when two workspaces fit in HBM; the same steps one batch
                   after the other are reported beside it (serial_*).
  host_to_host  -- the same batch through ta_align_batch from pinned host memory
                   to host results (PCIe both ways), SURVEY §8d's GCUPS definition.
  cpu_baseline  -- the reference team::Align (oracle/_ref, compiled from the
                   reference sources), OpenMP over pairs on the box's host cores,
                   plus a 1-thread figure, on bounded samples of the same batch.
  parity        -- results against the committed golden digest made by the
                   reference (tests/golden/), the CPU oracle, or (config 4) the
                   1-GPU result of the same read set.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process (HIP's default, 4, is what the box exports): the
# pipelines (align.DevicePipeline / HostPipeline) keep fills, tracebacks,
# uploads and downloads on streams of their own, and streams beyond the queue
# count share queues -- two streams on one queue run one after the other.  Set
# before anything initialises HIP.
_HWQ = int(os.environ.get("TA_BENCH_HW_QUEUES", "16"))  # (experiments: another count)
_HWQ_ORIG = os.environ.get("GPU_MAX_HW_QUEUES")  # (the drop-in runs keep the process default, 4 on
# the box, as a plain library user does; 16 measured the same, r06h)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _HWQ or "TA_BENCH_HW_QUEUES" in os.environ:
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(_HWQ, 32))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, Chip-level parameters)
# VALU issue roof of the dominant fill kernel: profiles/valu_roof.json (scripts/valu_roof.py) weights the
# measured issue cost of every opcode of the kernel's hot loop (scripts/exp/ubench/valu_rates on the
# MI355X: packed 16-bit ops, v_perm/v_bfi/v_max*/DPP 4 cycles per wave64 instruction, v_add/v_xor/
# v_mov/v_cmp 2) by the kernel's instruction mix.  Fallback when a kernel has no entry: every
# instruction 4 cycles, 256 CU x 4 SIMD x 16 lanes x 2.4 GHz = 39.3 T lane-ops/s.
VALU_PEAK_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12
METRIC = "GCUPS (DP cell updates/s) at 1/2/4/8 GPUs; bit-exact score+CIGAR"
MODES = {"global": 0, "local": 1, "semiGlobal": 2}
DTYPE = "int32 semantics; packed int16 arithmetic where range-proven (fits_int16), else int32"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="cfg2", choices=["cfg2", "cfg3", "cfg4", "cfg5", "cfg3map", "dropin"],
                    help="cfg2: 1kx1k pairs (headline); cfg3: E. coli stand-in, ONT-like reads vs true-origin "
                         "windows, semiGlobal, per GPU; cfg4: ONE such read set range-split by cells over the GPUs "
                         "(strong scaling); cfg5: 10kx10k related semiGlobal pairs (--pairs 100000 = the stated "
                         "size, generated in HBM); cfg3map: config 3 end to end (minimizers, FindLIS, alignment); "
                         "dropin: single-call team::Align latency/throughput vs the reference Align")
    ap.add_argument("--pairs", type=int, default=0, help="pairs per GPU (cfg4: in total; 0 = the workload's default)")
    ap.add_argument("--qlen", type=int, default=1000)
    ap.add_argument("--tlen", type=int, default=1000)
    ap.add_argument("--mode", default=None, choices=["global", "local", "semiGlobal"])
    ap.add_argument("--scoring", default="1,-1,-1")
    ap.add_argument("--related", action="store_true", help="config-2 related variant (5%% sub/ins/del)")
    ap.add_argument("--no-cigar", action="store_true", help="score-only (cigar == nullptr) mode")
    ap.add_argument("--cpu-pairs", type=int, default=10000, help="CPU-baseline sample size (pairs), all threads")
    ap.add_argument("--cpu-pairs-1t", type=int, default=400, help="CPU-baseline sample size (pairs), 1 thread")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host-to-host (PCIe-inclusive) measurement")
    ap.add_argument("--no-score-only", action="store_true", help="skip the config-2 score-only measurement")
    ap.add_argument("--workspace-gb", type=float, default=0.0,
                    help="device budget (GB) for the traceback codes; 0 = the library default (half the free "
                         "HBM, <= 64 GiB) -- cfg3/4/5 default to 240; batches above it run in chunks")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--check-all", action="store_true",
                    help="cfg5: check every pair's CIGAR path and score on the host (oracle cigar_check)")
    ap.add_argument("--gap-open", type=int, default=None,
                    help="affine-gap extension (no reference counterpart): a gap of length L costs "
                         "gap_open + L*gap, gap = the third --scoring value (config 5's 'affine gaps')")
    ap.add_argument("--serial", action="store_true",
                    help="one batch after the other (no DevicePipeline overlap of a traceback with the next fill)")
    ap.add_argument("--flags", type=int, default=0, help="ta_plan_create TA_PLAN_* kernel-selection flags")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL, default) or gloo (rehearsal only)")
    a = ap.parse_args(argv)
    if a.workload == "cfg2":
        a.pairs = a.pairs or 10000
        a.mode = a.mode or "local"
    elif a.workload in ("cfg3", "cfg4", "cfg3map"):
        a.pairs = a.pairs or 10000
        a.mode = a.mode or "semiGlobal"
        a.cpu_pairs = min(a.cpu_pairs, 200)
        a.cpu_pairs_1t = min(a.cpu_pairs_1t, 20)
        a.workspace_gb = a.workspace_gb or 240.0
    elif a.workload == "cfg5":
        # a slice of config 5's 100k pairs that fills the GPU in one chunk: 8,192 pairs (4,096
        # two-pair waves, 197 GB of 2-bit codes); affine 4,096 (4-bit codes, 197 GB)
        a.pairs = a.pairs or (8192 if a.gap_open is None else 4096)
        a.mode = a.mode or "semiGlobal"
        a.qlen = a.tlen = 10000
        a.related = True
        a.cpu_pairs = min(a.cpu_pairs, 64 if a.gap_open is None else 32)
        a.cpu_pairs_1t = min(a.cpu_pairs_1t, 4)
        a.workspace_gb = a.workspace_gb or 240.0
    return a


# --------------------------------------------------------------------------- ranks

def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """--gpus N outside torch.distributed: start the N ranks as a child process
    (nothing here has touched the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


class Dist:
    """This process's rank, device and collective helpers (RCCL or gloo)."""

    def __init__(self, args):
        import torch

        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = args.dist_backend
        self.dist = None
        # TA_BENCH_ONE_GPU=1: every rank on device 0 (multi-rank rehearsal on a 1-GPU box, gloo)
        self.dev_index = 0 if os.environ.get("TA_BENCH_ONE_GPU") == "1" else self.local_rank
        torch.cuda.set_device(self.dev_index)
        self.dev = torch.device("cuda", self.dev_index)
        # TA_BENCH_FORCE_DIST=1 (tests only): a world of one under torch.distributed.run still
        # initialises the process group and gathers every step, which exercises the RCCL
        # branch of ResultGather on a one-GPU box (two RCCL ranks cannot share one device)
        if self.world > 1 or os.environ.get("TA_BENCH_FORCE_DIST") == "1":
            import torch.distributed as dist

            dist.init_process_group(self.backend, device_id=self.dev if self.backend == "nccl" else None)
            self.dist = dist
        # collectives run on device tensors with RCCL, on host tensors with gloo
        self.cdev = self.dev if self.backend == "nccl" else torch.device("cpu")

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def all_gather_flat(self, out, t, async_op):
        """out = concatenation over ranks of t (equal sizes)."""
        if self.backend == "nccl":
            return self.dist.all_gather_into_tensor(out, t, async_op=async_op)
        parts = list(out.chunk(self.world))
        return self.dist.all_gather(parts, t, async_op=async_op)

    def close(self):
        if self.dist:
            self.dist.barrier()
            self.dist.destroy_process_group()


class ResultGather:
    """Every step's results of every rank gathered to rank 0, the only consumer
    (SURVEY §8e); the other ranks receive nothing.

    Records of step k (score, target_begin, cigar_len per pair, plus the pair
    and CIGAR-byte counts): one ``gather`` to rank 0 right after the step's
    kernels.  CIGAR bytes of step k (compacted on the device,
    ta_compact_cigars): point-to-point, exactly each rank's byte count (RCCL
    has no gatherv; rank 0 learns the counts from step k's records), posted
    once step k+1 is enqueued, so neither stalls the GPU.  With RCCL every
    transfer runs on a side stream that waits only for the event recorded
    after step k's compaction: the compute stream never waits for a gather,
    and a send never waits for step k+1's kernels.  All transfers are drained
    before the clock stops."""

    def __init__(self, D: Dist, P_max: int, cigar: bool):
        import torch

        self.torch, self.D, self.P, self.cigar = torch, D, P_max, cigar
        self.root = D.rank == 0
        self.nccl = D.backend == "nccl"
        self.side = torch.cuda.Stream(D.dev) if self.nccl else None
        self.pending = []
        self.recv_bytes = 0  # bytes this rank received over all steps (0 on ranks > 0)

    def _ctx(self):
        import contextlib

        return self.torch.cuda.stream(self.side) if self.nccl else contextlib.nullcontext()

    def post(self, plan):
        torch, D, P = self.torch, self.D, self.P
        rec = torch.zeros(3 * P + 2, dtype=torch.int32, device=D.dev)
        n = plan.P
        rec[:n] = plan.score
        rec[P:P + n] = plan.target_begin
        dst = None
        if self.cigar:
            rec[2 * P:2 * P + n] = plan.cigar_len
            dst, off = plan.compact_cigars()
            rec[3 * P + 1] = off[-1].to(torch.int32)
        rec[3 * P] = n
        st = {"dst": dst, "works": []}
        if self.nccl:
            ready = torch.cuda.Event()
            ready.record()  # step k's records and compacted bytes, on the compute stream
            st["ready"] = ready
            with self._ctx():
                self.side.wait_event(ready)
                # this rank's own pair / byte counts, to the host without waiting for step k+1
                cnt = torch.empty(2, dtype=torch.int32, pin_memory=True)
                cnt.copy_(rec[3 * P:], non_blocking=True)
                cev = torch.cuda.Event()
                cev.record()
                st.update(cnt=cnt, cev=cev)
                outs = [torch.empty_like(rec) for _ in range(D.world)] if self.root else None
                st["works"].append(D.dist.gather(rec, outs, dst=0, async_op=True))
                if self.root:
                    st["works"][-1].wait()  # the side stream waits, not the compute stream
                    tot = torch.empty((D.world, 2), dtype=torch.int32, pin_memory=True)
                    tot.copy_(torch.stack([o[3 * P:] for o in outs]), non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                    st.update(outs=outs, tot=tot, ev=ev)
            st["rec"] = rec
        else:
            rec_h = rec.cpu()
            st.update(cnt=rec_h[3 * P:].clone(), cev=None)
            outs = [torch.empty_like(rec_h) for _ in range(D.world)] if self.root else None
            D.dist.gather(rec_h, outs, dst=0)
            if self.root:
                st.update(outs=outs, tot=torch.stack([o[3 * P:] for o in outs]), ev=None)
        if self.root:
            self.recv_bytes += (D.world - 1) * rec.numel() * 4
        if self.cigar and self.pending and "bytes" not in self.pending[-1]:
            self._post_bytes(self.pending[-1])
        self.pending.append(st)

    def _post_bytes(self, st):
        torch, D = self.torch, self.D
        dev = D.dev if self.nccl else torch.device("cpu")
        dst = st["dst"]
        if self.root:
            if st["ev"] is not None:
                st["ev"].synchronize()  # step k's records are in: the GPU is already busy with step k+1
            nbytes = [int(x) for x in st["tot"][:, 1].tolist()]
        else:
            nbytes = None
        with self._ctx():
            if self.root:
                mine = dst[:nbytes[0]] if nbytes[0] else dst[:0]
                bufs = [mine if self.nccl else mine.cpu()]
                ops = []
                for r in range(1, D.world):
                    words = (nbytes[r] + 3) // 4
                    b = torch.empty(words, dtype=torch.int32, device=dev)
                    bufs.append(b)
                    if words:
                        ops.append(D.dist.P2POp(D.dist.irecv, b, r))
                    self.recv_bytes += 4 * words
                st["bufs"] = bufs
                st["nbytes"] = nbytes
            else:
                # this rank's byte count (its records' last word); whole int32 words go (rank 0 drops the slack)
                if st["cev"] is not None:
                    st["cev"].synchronize()  # step k's count only: the GPU is already busy with step k+1
                words = (int(st["cnt"][1]) + 3) // 4
                ops = []
                if words:
                    w = dst[:4 * words].view(torch.int32) if self.nccl else dst[:4 * words].cpu().view(torch.int32)
                    st["send"] = w
                    ops.append(D.dist.P2POp(D.dist.isend, w, 0))
            if ops and self.nccl:
                st["works"] += D.dist.batch_isend_irecv(ops)
            for op in ops if not self.nccl else ():
                # gloo (the CPU / one-GPU rehearsal): blocking transfers -- a large asynchronous
                # send left in flight under the next step's gather stalls gloo's pair
                (D.dist.recv if op.op is D.dist.irecv else D.dist.send)(op.tensor, op.peer)
        st["bytes"] = True

    def drain(self):
        for st in self.pending:
            if self.cigar and "bytes" not in st:
                self._post_bytes(st)
        with self._ctx():  # RCCL: the side stream waits for the transfers, then the compute stream for it
            for st in self.pending:
                for w in st["works"]:
                    w.wait()
        if self.nccl:
            self.torch.cuda.current_stream(self.D.dev).wait_stream(self.side)

    def last(self):
        """Rank 0: rank-ordered (scores, target_begins, cigar_lens, cigar bytes) of the last step."""
        assert self.root, "results are gathered to rank 0 only"
        st = self.pending[-1]
        P, W = self.P, self.D.world
        rec = self.torch.stack(st["outs"]).cpu().numpy()
        n = rec[:, 3 * P]
        sc = np.concatenate([rec[r, :n[r]] for r in range(W)])
        tb = np.concatenate([rec[r, P:P + n[r]] for r in range(W)]).view(np.uint32)
        cl = np.concatenate([rec[r, 2 * P:2 * P + n[r]] for r in range(W)]).view(np.uint32)
        cig = None
        if self.cigar:
            parts = []
            for r, b in enumerate(st["bufs"]):
                parts.append(b.cpu().numpy().view(np.uint8)[:st["nbytes"][r]].tobytes())
            cig = b"".join(parts)
        return sc, tb, cl, cig

    def clear_old(self, keep=2):
        # finished steps (their byte transfers posted) can go; waits keep the allocator safe
        while len(self.pending) > keep and "bytes" in self.pending[0]:
            st = self.pending.pop(0)
            with self._ctx():
                for w in st["works"]:
                    w.wait()


# --------------------------------------------------------------------------- inputs

def make_batch(args, D, cells_split=None):
    """This rank's batch (host PairBatch) and, for cfg5, its inputs in HBM."""
    from bioinfo1_amd import shard, synth

    P, rank, world = args.pairs, D.rank, D.world
    if args.workload == "cfg3":
        return synth.cfg3_batch(P, first_read=rank * P)[0], None, (rank * P, (rank + 1) * P)
    if args.workload == "cfg4":
        full = synth.cfg3_batch(P)[0]
        cells = full.qlen.astype(np.int64) * full.tlen.astype(np.int64)
        lo, hi = shard.range_split(cells, world)[rank]
        return full.slice(lo, hi), full, (lo, hi)
    if args.workload == "cfg5":
        import torch

        q, t = synth.related_batch_torch(P, args.qlen, args.tlen, 0x5EED, first_pair=rank * P, device=D.dev)
        ql = np.full(P, args.qlen, np.uint32)
        tl = np.full(P, args.tlen, np.uint32)
        qoff = np.arange(P, dtype=np.uint64) * np.uint64(args.qlen)
        toff = np.arange(P, dtype=np.uint64) * np.uint64(args.tlen)
        shapes = synth.PairBatch(np.zeros(0, np.uint8), qoff, ql, np.zeros(0, np.uint8), toff, tl)
        dev_in = (q, torch.from_numpy(qoff.view(np.int64)).to(D.dev), t,
                  torch.from_numpy(toff.view(np.int64)).to(D.dev))
        return shapes, dev_in, (rank * P, (rank + 1) * P)
    gen = synth.related_batch if args.related else synth.uniform_batch
    return gen(P, args.qlen, args.tlen, 0x5EED, first_pair=rank * P), None, (rank * P, (rank + 1) * P)


def host_batch_of(batch, dev_in, k=None):
    """A host PairBatch of (the first k pairs of) a batch whose bytes live in
    HBM (cfg5: fixed shape, pairs back to back)."""
    from bioinfo1_amd import synth

    k = batch.n_pairs if k is None else min(k, batch.n_pairs)
    if dev_in is None:
        return batch if k == batch.n_pairs else batch.slice(0, k)
    q, _, t, _ = dev_in
    n, m = int(batch.qlen[0]), int(batch.tlen[0])
    return synth.PairBatch(q[:k * n].cpu().numpy(), batch.qoff[:k].copy(), batch.qlen[:k].copy(),
                           t[:k * m].cpu().numpy(), batch.toff[:k].copy(), batch.tlen[:k].copy())


def input_variants(plan, batch, count=3):
    """Batches of the plan's shapes for back-to-back steps: the
    same pairs rotated by ``shift`` positions (pair p of a variant is pair
    (p + shift) % P of the batch), made on the device from the plan's own
    inputs.  Only for batches of one (n, m) shape, where a rotation keeps every
    pair's planned lengths; else just the batch.  Returns [(inputs, shift)]."""
    import torch

    P = plan.P
    if P < count or not (np.all(batch.qlen == batch.qlen[0]) and np.all(batch.tlen == batch.tlen[0])):
        return [((plan.qbytes, plan.qoff, plan.tbytes, plan.toff), 0)]
    n, m = int(batch.qlen[0]), int(batch.tlen[0])
    out = [((plan.qbytes, plan.qoff, plan.tbytes, plan.toff), 0)]
    for v in range(1, count):
        sh = v * P // count
        out.append(((torch.roll(plan.qbytes[:P * n], -sh * n), plan.qoff,
                     torch.roll(plan.tbytes[:P * m], -sh * m), plan.toff), sh))
    return out


def rotated(res, shift):
    """A BatchResult of a rotated variant read back in the batch's own pair
    order: (scores, target_begins, cigar_lens, cigar_of)."""
    P = res.scores.shape[0]
    idx = (np.arange(P) - shift) % P
    return (res.scores[idx], res.target_begins[idx], res.cigar_lens[idx] if res.cigar_lens is not None else None,
            lambda b: res.cigar(int(idx[b])))


# --------------------------------------------------------------------------- checks and baselines

def fill_alg_bytes(batch, cigar: bool, affine: bool = False) -> int:
    """Algorithmic HBM bytes of one fill launch: the sequence
    bytes read, the 2-bit (affine: 4-bit) traceback code per DP cell written
    (cigar on) and 16 B of per-pair results (score, target_begin, goal cell)."""
    n = batch.qlen.astype(np.int64)
    m = batch.tlen.astype(np.int64)
    b = n + m + 16
    if cigar:
        b = b + ((n * m + 1) // 2 if affine else (n * m + 3) // 4)
    return int(b.sum())


def cpu_threads() -> int:
    """The host cores this process may use: OMP_NUM_THREADS when the box sets
    it (the GPU box allots 16 CPUs per GPU), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() else len(os.sched_getaffinity(0))


def cpu_baseline(batch, mode, sc, cigar, pairs, pairs_1t, gap_open=None):
    from oracle.pyoracle import Oracle, Reference

    affine = gap_open is not None
    impl = Reference() if Reference.available() and not affine else Oracle()

    def run(k, threads):
        sample = batch.slice(0, min(k, batch.n_pairs))
        t0 = time.perf_counter()
        if affine:  # the reference has no affine Align: the CPU definition (oracle/affine_oracle.c) is the baseline
            res = impl.align_affine_batch(sample, mode, sc[0], sc[1], gap_open, sc[2], cigar, n_threads=threads)
        else:
            res = impl.align_batch(sample, mode, *sc, cigar, n_threads=threads)
        dt = time.perf_counter() - t0
        assert not res.status.any()
        return sample, dt

    thr = cpu_threads()
    sample, dt = run(pairs, thr)
    s1, dt1 = run(pairs_1t, 1)
    aff = len(os.sched_getaffinity(0))
    value = sample.cells / dt / 1e9
    return {"value": round(value, 4), "unit": "GCUPS", "cores": thr, "kind": impl.kind,
            "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            # (VERDICT r04 item 7 asked for a run on every CPU of the affinity mask; the GPU box grants
            # 16 CPUs per GPU -- OMP_NUM_THREADS=16 -- and its rules keep worker pools within that share,
            # so the all-mask figure is the measured per-thread rate scaled linearly: an upper bound)
            "value_all_affinity": None,
            "value_all_affinity_bound": round(value / thr * aff, 2) if thr else None,
            "all_affinity_note": (f"not measured: the box grants {thr} of its {aff} affinity CPUs to this job; "
                                  f"value_all_affinity_bound = value / {thr} threads x {aff} CPUs (perfect scaling, "
                                  "an upper bound on the reference's CPU rate on the whole node)"),
            "sample": f"first {sample.n_pairs} pairs of the same batch ({sample.cells:.3g} cells), OpenMP over pairs "
                      f"(schedule dynamic) on {thr} threads, {dt:.2f} s wall",
            "value_1thread": round(s1.cells / dt1 / 1e9, 4),
            "sample_1thread": f"first {s1.n_pairs} pairs ({s1.cells:.3g} cells), 1 thread, {dt1:.2f} s",
            "impl": "oracle/_ref/libref_align.so (reference team_alignment.cpp, g++ -O3)" if impl.kind == "reference"
            else ("oracle/liboracle.so (affine_oracle.c: the extension's CPU definition)" if affine
                  else "oracle/liboracle.so (C restatement)")}


def digest_name(args, n_pairs):
    if args.workload == "cfg2" and (args.mode, args.scoring, args.qlen, args.tlen) == ("local", "1,-1,-1", 1000, 1000) \
            and n_pairs == 10000:
        return ("cfg2_related_local" if args.related else "cfg2_local"), 10000
    if args.workload in ("cfg3", "cfg4") and (args.mode, args.scoring) == ("semiGlobal", "1,-1,-1") and n_pairs >= 64:
        return "cfg3_semi_sample", 64
    if args.workload in ("cfg3", "cfg4") and (args.mode, args.scoring) == ("local", "1,-1,-1") and n_pairs >= 64:
        return "cfg3_local_sample", 64
    if args.workload == "cfg5" and (args.mode, args.scoring) == ("semiGlobal", "1,-1,-1") and n_pairs >= 32:
        return "cfg5_semi_sample", 32
    return None, 0


def parity_vs_digest(scores, tbs, clens, cigar_of, name, k):
    """The first k pairs against the committed golden digest (made by the
    reference) of the same seeded batch."""
    with open(os.path.join(ROOT, "tests", "golden", f"digest_{name}.json")) as f:
        meta = json.load(f)
    d = np.load(os.path.join(ROOT, "tests", "golden", f"digest_{name}.npz"))
    ok = bool(np.array_equal(scores[:k], d["scores"]) and np.array_equal(tbs[:k], d["target_begins"])
              and np.array_equal(clens[:k], d["cigar_lens"]))
    h = hashlib.sha256()
    for p in range(k):
        c = cigar_of(p)
        h.update(len(c).to_bytes(4, "little"))
        h.update(c)
    ok = ok and h.hexdigest() == meta["cigar_sha256"]
    return {"golden": f"tests/golden/digest_{name}", "pairs_checked": k, "bit_exact": ok}


def strided_name(args):
    """The stratified reference digest (pairs spread over the whole stated-size
    stream, tests/golden/make_golden.py) that covers this workload, or None."""
    if args.gap_open is not None or args.scoring != "1,-1,-1":
        return None
    if args.workload == "cfg5" and args.mode == "semiGlobal" and (args.qlen, args.tlen) == (10000, 10000):
        return "cfg5_semi_strided"
    if args.workload in ("cfg3", "cfg4"):
        return {"semiGlobal": "cfg3_semi_strided", "local": "cfg3_local_strided"}.get(args.mode)
    return None


def parity_strided(scores, tbs, clens, cigar_of, name, lo, hi, chunk_of=None, n_chunks=None):
    """The pairs of the stratified digest `name` that fall in this run's stream
    range [lo, hi) (pair p of the run is stream position lo + p), each against
    the reference's score, target_begin, CIGAR length and CIGAR CRC32; with all
    of them present also the SHA-256 over the whole sample.  chunk_of (per
    pair) shows which chunks of the plan the checked pairs ran in."""
    import zlib

    with open(os.path.join(ROOT, "tests", "golden", f"digest_{name}.json")) as f:
        meta = json.load(f)
    d = np.load(os.path.join(ROOT, "tests", "golden", f"digest_{name}.npz"))
    idx = d["indices"]
    sel = np.nonzero((idx >= lo) & (idx < hi))[0]
    loc = (idx[sel] - lo).astype(np.int64)
    cig = [cigar_of(int(p)) for p in loc]
    ok = bool(np.array_equal(scores[loc], d["scores"][sel]) and np.array_equal(tbs[loc], d["target_begins"][sel])
              and np.array_equal(clens[loc], d["cigar_lens"][sel])
              and all(zlib.crc32(c) == int(d["cigar_crc32"][k]) for c, k in zip(cig, sel)))
    if len(sel) == len(idx):
        h = hashlib.sha256()
        for c in cig:
            h.update(len(c).to_bytes(4, "little"))
            h.update(c)
        ok = ok and h.hexdigest() == meta["cigar_sha256"]
    out = {"golden": f"tests/golden/digest_{name}", "pairs_checked": int(len(sel)), "sample_size": int(len(idx)),
           "stream_positions": f"{int(idx[sel].min()) if len(sel) else '-'}..{int(idx[sel].max()) if len(sel) else '-'}",
           "bit_exact": ok}
    if chunk_of is not None and len(sel):
        out["chunks_covered"] = int(len(np.unique(chunk_of[loc])))
        out["chunks"] = int(n_chunks)
    return out


def parity_vs_oracle(res, batch, mode, sc, gap_open, k):
    """Affine extension (no reference digest exists for gap_open != 0): the
    first k pairs against the CPU definition (oracle/affine_oracle.c)."""
    from oracle.pyoracle import Oracle

    sub = batch.slice(0, min(k, batch.n_pairs))
    want = Oracle().align_affine_batch(sub, mode, sc[0], sc[1], gap_open, sc[2], res.cigar_lens is not None)
    ok = bool(np.array_equal(res.scores[: sub.n_pairs], want.scores)
              and np.array_equal(res.target_begins[: sub.n_pairs], want.target_begins))
    if res.cigar_lens is not None:
        ok = ok and all(res.cigar(p) == want.cigar(p) for p in range(sub.n_pairs))
    return {"oracle": "oracle/affine_oracle.c (definition; parity vs the reference unpinned for gap_open != 0)",
            "pairs_checked": sub.n_pairs, "bit_exact": ok}


def check_all(res, batch, mode, sc, gap_open):
    """Every pair: the CIGAR is a valid path of the mode whose score is the
    reported score (oracle cigar_check; size-independent), on host cores."""
    from oracle.pyoracle import affine_cigar_check_batch, cigar_check_batch

    t0 = time.perf_counter()
    if gap_open is None:
        st = cigar_check_batch(batch, mode, *sc, res.scores, res.target_begins, res.arena, res.cigar_offsets,
                               res.cigar_lens)
    else:
        st = affine_cigar_check_batch(batch, mode, sc[0], sc[1], gap_open, sc[2], res.scores, res.target_begins,
                                      res.arena, res.cigar_offsets, res.cigar_lens)
    return {"pairs_checked": int(batch.n_pairs), "bad": int(np.count_nonzero(st)), "check_s": round(time.perf_counter() - t0, 2),
            "checker": "oracle cigar_check (path validity + rescoring of every CIGAR)"}


def dominant_kernel(plan, mode, cigar, affine):
    """The fill kernel that carries most of the plan's cells, named as rocprofv3
    prints it (template arguments included, namespace and parameters dropped):
    the key of its counter entries in profiles/{traffic,valu}_by_kernel.json and
    of its issue roof in profiles/valu_roof.json."""
    c = str(cigar).lower()
    if affine:
        return f"affine_dual_fill_kernel<{mode}, {c}>" if plan.dual_pairs else f"affine_fill_kernel<{mode}, {c}>"
    if plan.flex_pairs and plan.flex_pairs * 2 >= plan.P:
        if cigar and getattr(plan, "ck", False):
            return f"flex_fill_ck_kernel<{mode}>"  # (checkpoints instead of codes)
        return f"flex_fill_kernel<{mode}, {c}>"
    if plan.dual_pairs * 2 >= plan.P:
        if cigar and getattr(plan, "ck", False):
            return f"dual_fill_ck_kernel<{mode}>"  # (checkpoints instead of codes)
        return f"dual_fill_kernel<{mode}, {c}, {'true' if (cigar and plan.blk) else 'false'}>"
    return f"fill_kernel<{mode}, {c}, false>"


# The translation unit each kernel is compiled from (build.sh), by rocprof-name prefix.
KERNEL_TU = (("dual_fill_ck_kernel", "ta_dual.hip"), ("dual_fill_kernel", "ta_dual.hip"),
             ("flex_fill_ck_kernel", "ta_flex.hip"), ("flex_fill_kernel", "ta_flex.hip"), ("affine_", "ta_affine.hip"),
             ("traceback_ck_kernel", "ta_walk_ck.hip"), ("fill_kernel", "ta_kernels.hip"),
             ("traceback", "ta_kernels.hip"), ("format_runs_kernel", "ta_kernels.hip"))
CSRC = os.path.join(ROOT, "bioinfo1_amd", "csrc")


def kernel_src_hash(kernel, csrc=CSRC, build=os.path.join(ROOT, "build.sh")):
    """sha256 (16 hex) over what a kernel's counters depend on: its translation
    unit and every csrc header it includes (transitively), the planner and the
    launch code (chunking, grids), and build.sh (flags, -D variants).  A counter
    entry (profiles/{traffic,valu}_by_kernel.json) carries the hash of the source
    it was measured on; bench.py quotes it only while the hash still matches."""
    import re

    tu = next((f for pre, f in KERNEL_TU if kernel.startswith(pre)), None)
    if tu is None:
        return None
    seen, todo = [], [tu, "ta_planner.cpp", "ta_api.hip"]
    while todo:
        f = todo.pop(0)
        path = os.path.join(csrc, f)
        if f in seen or not os.path.exists(path):
            continue
        seen.append(f)
        todo += re.findall(r'^#include "([^"/]+)"', open(path).read(), re.M)
    h = hashlib.sha256()
    for f in sorted(seen) + [None]:
        h.update(open(os.path.join(csrc, f) if f else build, "rb").read())
    return h.hexdigest()[:16]


def profile_entry(name, kernel, tag):
    """profiles/<name>: {"<kernel>|<workload tag>": {"value", "profile", "src_hash", ...}}
    -- counters of THIS kernel (rocprof name, dominant_kernel) on THIS workload,
    written by scripts/prof_summary.py.  Returns (entry, None), or (None, why)
    when there is no entry or it was measured on other source ("stale")."""
    e = load_profile(name, f"{kernel}|{tag}")
    if not isinstance(e, dict):
        return None, f"not profiled for {kernel} on this workload"
    want = kernel_src_hash(kernel)
    if e.get("src_hash") != want:
        return None, (f"stale: profiles/{e.get('profile')}_pmc.json was measured on source {e.get('src_hash')}, "
                      f"the loaded kernel is built from {want} (scripts/profile.sh + prof_summary.py to refresh)")
    return e, None


MODES_INV = {0: "kGlobal", 1: "kLocal", 2: "kSemi"}


def load_profile(name, tag):
    p = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f).get(tag)


# --------------------------------------------------------------------------- workloads

def main_align(args, D):
    import torch

    from bioinfo1_amd.align import Aligner, DevicePlan, HostBatchRunner

    mode = MODES[args.mode]
    sc = tuple(int(x) for x in args.scoring.split(","))
    cigar = not args.no_cigar
    affine = args.gap_open is not None
    batch, aux, (lo, hi) = make_batch(args, D)
    dev_in = aux if args.workload == "cfg5" else None
    full = aux if args.workload == "cfg4" else None
    al = Aligner(D.dev_index)
    budget = int(args.workspace_gb * 2**30)
    plan = DevicePlan(al, batch, mode, *sc, cigar, workspace_budget=budget, gap_open=args.gap_open,
                      flags=args.flags, inputs=dev_in)
    stream = torch.cuda.current_stream(D.dev)
    P_max = plan.P
    if args.workload == "cfg4" and D.world > 1:
        from bioinfo1_amd import shard

        cells = full.qlen.astype(np.int64) * full.tlen.astype(np.int64)
        P_max = max(h - l for l, h in shard.range_split(cells, D.world))
    gather = ResultGather(D, P_max, cigar) if D.dist else None
    # two-slot pipeline (align.DevicePipeline): batch k's traceback beside batch k+1's fill, when
    # a second workspace fits in HBM (config 5's 197 GB of codes does not)
    pipe = None
    if cigar and not args.serial:
        free_b, _ = torch.cuda.mem_get_info(D.dev)
        if free_b > 2 * plan.workspace_bytes + 8 * 2**30:
            from bioinfo1_amd.align import DevicePipeline

            pipe = DevicePipeline(D.dev_index, batch, mode, *sc, cigar, workspace_budget=budget,
                                  gap_open=args.gap_open, flags=args.flags, inputs=dev_in, first=plan)

    # back-to-back steps align different batches of the same shapes in turn (three rotations
    # of the batch; only for one-shape batches), so a slot never realigns the batch it
    # held last -- what the pipeline checks below rely on
    variants = input_variants(plan, batch) if (pipe and args.workload == "cfg2") else None
    torch.cuda.synchronize(D.dev)  # (the variants are resident before the pipeline's fill stream reads them)
    held = {}  # slot plan id -> variant it aligned last
    state = {"k": 0, "last": plan}

    def step():
        v = state["k"] % len(variants) if variants else 0
        state["k"] += 1
        if pipe:
            p = pipe.step(inputs=variants[v][0]) if variants else pipe.step()
        else:
            p = plan
            plan.run()
        held[id(p)] = v
        state["last"] = p
        if gather:
            gather.post(p)
            gather.clear_old()

    # parity of this rank's own results (rank 0: the digest covers the first pairs of the stream),
    # from one step BEFORE the warmup: the checks take ~1 s of host time, and a GPU left idle that
    # long starts the next steps at a lower clock -- the warmup steps run right before the clock
    step()
    if gather:
        gather.drain()
    torch.cuda.synchronize(D.dev)
    parity = None
    if D.rank == 0 and not args.no_parity:
        res = plan.results()
        name, k = digest_name(args, plan.P)
        if name and cigar and not affine and lo == 0:
            shift = variants[held.get(id(plan), 0)][1] if variants else 0
            parity = parity_vs_digest(*rotated(res, shift), name, k)
            sname = strided_name(args)
            if sname:
                parity["digest_stratified"] = parity_strided(res.scores, res.target_begins, res.cigar_lens,
                                                             res.cigar, sname, lo, hi, plan.pair_chunks(),
                                                             plan.chunks)
                parity["bit_exact"] = parity["bit_exact"] and parity["digest_stratified"]["bit_exact"]
        elif affine and cigar:
            parity = parity_vs_oracle(res, host_batch_of(batch, dev_in, 16), mode, sc, args.gap_open, 16)
    D.barrier()
    for _ in range(args.warmup):
        step()
    if gather:
        gather.drain()
    torch.cuda.synchronize(D.dev)
    D.barrier()
    torch.cuda.synchronize(D.dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if gather:
        gather.drain()
    torch.cuda.synchronize(D.dev)
    D.barrier()
    torch.cuda.synchronize(D.dev)
    elapsed = D.max(time.perf_counter() - t0)
    (pipe or plan).check()  # raises if a kernel reported an internal failure during the timed steps
    ms = elapsed / max(args.steps, 1) * 1e3
    cells_job = (full.cells if args.workload == "cfg4" else batch.cells * D.world)
    gcups = cells_job / (ms / 1e3) / 1e9

    gathered = None
    if gather and D.rank == 0:
        gathered = gather.last()

    pipeline = None
    if pipe and D.rank == 0:
        # every slot's last batch (a different input variant per slot) against the reference
        # digest, read back through its rotation -- before the serial steps below reuse slot 0
        slots = []
        name, k = digest_name(args, plan.P)
        for q in pipe.plans:
            v = held.get(id(q), 0)
            shift = variants[v][1] if variants else 0
            ent = {"variant": v, "rotation": shift}
            if name and cigar and not affine and lo == 0 and not args.no_parity:
                ent["bit_exact"] = parity_vs_digest(*rotated(q.results(), shift), name, k)["bit_exact"]
            slots.append(ent)
        # the same steps one batch after the other (no overlap), alternating the same inputs
        # (after warmup steps of their own: the slot checks above left the GPU idle)
        for j in range(max(args.warmup, 2)):
            plan.run()
        torch.cuda.synchronize(D.dev)
        t1 = time.perf_counter()
        for j in range(args.steps):
            if variants:
                plan.set_inputs(variants[j % len(variants)][0])
            plan.run()
        torch.cuda.synchronize(D.dev)
        s_ms = (time.perf_counter() - t1) / max(args.steps, 1) * 1e3
        if variants:
            plan.set_inputs(variants[0][0])
        pipeline = {"depth": len(pipe.plans), "serial_ms_per_step": round(s_ms, 4),
                    "serial_value": round(batch.cells / (s_ms / 1e3) / 1e9, 2),
                    "input_variants": len(variants) if variants else 1,
                    "inputs": ("step k aligns variant k % 3: the batch's pairs rotated by 0, P/3, 2P/3 positions "
                               "(distinct bytes at every pair position), all resident in HBM before the clock starts"
                               if variants else "one batch, realigned every step"),
                    "slots": slots,
                    "slots_bit_exact": all(e.get("bit_exact", True) for e in slots),
                    "path": "align.DevicePipeline: one Aligner context (workspace) per slot; fills on a fill stream, "
                            "tracebacks on a walk stream, batch k's traceback beside batch k+1's fill"}
    out = None
    if D.rank == 0:
        # dominant kernel (fill) timed on its own launch stream with HIP events
        kt, tt = [], []
        for _ in range(max(min(args.steps, 10), 3)):
            f_ms = t_ms = 0.0
            for c in range(plan.chunks):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record(stream)
                plan.run_fill(c)
                e1.record(stream)
                if cigar:
                    plan.run_traceback(c)
                e2.record(stream)
                e2.synchronize()
                f_ms += e0.elapsed_time(e1)
                t_ms += e1.elapsed_time(e2)
            kt.append(f_ms)
            tt.append(t_ms)
        fill_ms = float(np.mean(kt))
        alg = fill_alg_bytes(batch, cigar, affine)
        achieved = alg / (fill_ms / 1e3) / 1e9
        tag = (f"{args.mode}_{'cigar' if cigar else 'score'}_{args.pairs}x{args.qlen}x{args.tlen}"
               if args.workload not in ("cfg3", "cfg4")
               else f"cfg3_{'' if args.mode == 'semiGlobal' else args.mode + '_'}{'cigar' if cigar else 'score'}_{plan.P}")
        if affine:
            tag = "affine_" + tag
        kern = dominant_kernel(plan, mode, cigar, affine)
        tr, tr_why = profile_entry("traffic_by_kernel.json", kern, tag)
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": tr["value"] if tr else None,
                "traffic_source": (f"rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE (separate passes) of {kern} on this "
                                   f"workload, bytes per step's fill: profiles/{tr['profile']}_pmc.json "
                                   f"(profiles/traffic_by_kernel.json, source {tr['src_hash']}; scripts/profile.sh)")
                if tr else tr_why,
                "src_hash": kernel_src_hash(kern),
                "kernel": kern, "kernel_ms": round(fill_ms, 4),
                "launches_per_step": plan.chunks,
                "kernel_ms_per_dispatch": round(fill_ms / max(plan.chunks, 1), 4),
                "alg_bytes_per_launch": alg,
                "per_launch_note": "one launch = the step's fill dispatches (one per chunk); traffic and "
                                   "ops/cell are rocprof per-dispatch averages x launches_per_step",
                "note": "integer DP: VALU-bound, not HBM- or MFMA-bound (see valu)"}
        ve, ve_why = profile_entry("valu_by_kernel.json", kern, tag)
        ops = ve["value"] if ve else None
        kroof = (load_profile("valu_roof.json", "kernels") or {}).get(kern)
        peak = kroof["peak_lane_tops"] if kroof else VALU_PEAK_TOPS
        valu = {"kernel_gcups": round(batch.cells / (fill_ms / 1e3) / 1e9, 2),
                "peak_lane_tops": round(peak, 2),
                "peak_basis": ("profiles/valu_roof.json: measured per-opcode issue cost (profiles/r03_valu_rates.txt) "
                               f"weighted by the kernel's instruction mix, {kroof['mean_cycles_per_wave_instr']} "
                               "cycles per wave64 instruction") if kroof else "every instruction 4 cycles (fallback)",
                "valu_ops_per_cell": ops,
                "valu_ops_source": (f"rocprofv3 SQ_INSTS_VALU x 64 / cells of {kern} on this workload: "
                                    f"profiles/{ve['profile']}_pmc.json, source {ve['src_hash']}") if ve else ve_why,
                "achieved_lane_tops": round(batch.cells * ops / (fill_ms / 1e3) / 1e12, 2) if ops else None,
                "frac": round(batch.cells * ops / (fill_ms / 1e3) / 1e12 / peak, 4) if ops else None}
        extra = {}
        if gathered is not None:
            extra["gather"] = check_gathered(args, gathered, state["last"], full, al, mode, sc, cigar)
        if D.world == 1 and not args.no_host and args.workload == "cfg2" and not affine:
            extra["host_to_host"] = host_to_host_pipelined(al, batch, mode, sc, cigar, args, budget)
            extra["host_to_host_single_call"] = host_to_host(HostBatchRunner(al, batch, mode, *sc, cigar), batch, args)
        if D.world == 1 and args.workload == "cfg2" and cigar and not affine and not args.no_score_only:
            extra["score_only"] = score_only(al, batch, mode, sc, args, budget, stream)
        if args.check_all and cigar:
            extra["check_all"] = check_all(plan.results(), host_batch_of(batch, dev_in), mode, sc, args.gap_open)
        cpu = None
        if D.world == 1 and not args.no_cpu:
            cpu = cpu_baseline(host_batch_of(batch, dev_in, args.cpu_pairs), mode, sc, cigar,
                               args.cpu_pairs, args.cpu_pairs_1t, args.gap_open)
        strong = args.workload == "cfg4"
        out = {
            "metric": METRIC, "value": round(gcups, 2), "unit": "GCUPS", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": DTYPE, "data": "synthetic",
            "config": {"workload": workload_name(args, cigar, plan.P, full), "pairs_per_gpu": plan.P,
                       "qlen": args.qlen if args.workload not in ("cfg3", "cfg4") else "1-20 kb reads",
                       "tlen": args.tlen if args.workload not in ("cfg3", "cfg4") else "true-origin window",
                       "mode": args.mode, "cigar": cigar, "cells_per_gpu": batch.cells, "cells_total": cells_job,
                       "parallelism": (f"one read set range-split by cells over {D.world} GPU(s)" if strong else
                                       f"pairs range-split over {D.world} GPU(s)")
                       + (", per-pair records and CIGAR bytes gathered to rank 0 every step (RCCL)" if D.world > 1 else "")},
            "fill_ms": round(fill_ms, 4), "traceback_ms": round(float(np.mean(tt)), 4) if cigar else None,
            "batch_latency_ms": round(fill_ms + (float(np.mean(tt)) if cigar else 0.0), 4),
            "chunks": plan.chunks, "workspace_gb": round(plan.workspace_bytes / 2**30, 2),
            "plan": {"dual_pairs": plan.dual_pairs, "flex_pairs": plan.flex_pairs, "fused_traceback": plan.fused},
            "pipeline": pipeline,
            "roofline": roof, "valu": valu, "cpu_baseline": cpu, "parity": parity, **extra,
            "device": torch.cuda.get_device_name(D.dev),
        }
    if pipe:
        pipe.close()
    plan.close()
    al.close()
    D.close()
    if out is not None:
        print(json.dumps(out), flush=True)
        if out.get("parity") and not out["parity"].get("bit_exact", True):
            sys.exit(1)
        if out.get("pipeline") and not out["pipeline"]["slots_bit_exact"]:
            sys.exit(1)
        g = out.get("gather")
        if g and not g.get("bit_exact", True):
            sys.exit(1)
        for k in ("score_only", "host_to_host"):
            par = (out.get(k) or {}).get("parity")
            if par and not par.get("bit_exact", True):
                sys.exit(1)


def check_gathered(args, gathered, plan, full, al, mode, sc, cigar):
    """Rank 0 after the timed steps: the gathered results of all ranks.  cfg4:
    byte-identical to the same read set aligned on this one GPU,
    and its first 64 pairs to the reference digest.  cfg2: this rank's slice
    of the gather equals its own results."""
    sc_g, tb_g, cl_g, cig_g = gathered
    if args.workload == "cfg4":
        from bioinfo1_amd.align import DevicePlan

        one = DevicePlan(al, full, mode, *sc, cigar, workspace_budget=int(args.workspace_gb * 2**30))
        one.run()
        r = one.results()
        one.close()
        ok = bool(np.array_equal(sc_g, r.scores) and np.array_equal(tb_g, r.target_begins))
        if cigar:
            ok = ok and np.array_equal(cl_g, r.cigar_lens) and cig_g == b"".join(r.cigars())
        res = {"vs": "1-GPU result of the whole read set", "pairs": int(full.n_pairs), "bit_exact": ok,
               "cigar_bytes": len(cig_g) if cig_g is not None else 0}
        name, k = digest_name(args, full.n_pairs)
        if name and cigar:
            offs = np.concatenate([[0], np.cumsum(cl_g.astype(np.int64))])
            d = parity_vs_digest(sc_g, tb_g, cl_g, lambda p: cig_g[offs[p]:offs[p + 1]], name, k)
            res["digest"] = d
            res["bit_exact"] = res["bit_exact"] and d["bit_exact"]
            sname = strided_name(args)
            if sname:
                ds = parity_strided(sc_g, tb_g, cl_g, lambda p: cig_g[offs[p]:offs[p + 1]], sname, 0, full.n_pairs)
                res["digest_stratified"] = ds
                res["bit_exact"] = res["bit_exact"] and ds["bit_exact"]
        return res
    r = plan.results()
    n = plan.P
    ok = bool(np.array_equal(sc_g[:n], r.scores) and np.array_equal(tb_g[:n], r.target_begins))
    if cigar:
        ok = ok and np.array_equal(cl_g[:n], r.cigar_lens) and cig_g[:int(r.cigar_lens.sum())] == b"".join(r.cigars())
    return {"vs": "rank 0's own results (its slice of the gather)", "pairs_gathered": int(sc_g.shape[0]),
            "bit_exact": ok, "cigar_bytes": len(cig_g) if cig_g is not None else 0}


def score_only(al, batch, mode, sc, args, budget, stream):
    """config 2 is measured in both CIGAR and score-only mode.
    The same HBM-resident batch, fill only (no codes written, no traceback);
    scores and target_begins against the reference digest."""
    import torch

    from bioinfo1_amd.align import DevicePlan

    p = DevicePlan(al, batch, mode, *sc, False, workspace_budget=budget)
    for _ in range(2):
        p.run()
    torch.cuda.synchronize(stream.device)
    reps = max(args.steps, 10)
    t0 = time.perf_counter()
    for _ in range(reps):
        p.run()
    torch.cuda.synchronize(stream.device)
    dt = (time.perf_counter() - t0) / reps
    p.check()
    r = p.results()
    p.close()
    par = None
    name, k = digest_name(args, batch.n_pairs)
    if name:
        d = np.load(os.path.join(ROOT, "tests", "golden", f"digest_{name}.npz"))
        par = {"golden": f"tests/golden/digest_{name}", "pairs_checked": k,
               "bit_exact": bool(np.array_equal(r.scores[:k], d["scores"])
                                 and np.array_equal(r.target_begins[:k], d["target_begins"]))}
    return {"value": round(batch.cells / dt / 1e9, 2), "unit": "GCUPS", "ms_per_step": round(dt * 1e3, 4),
            "steps": reps, "parity": par}


def host_to_host(runner, batch, args, reps=10):
    """SURVEY §8d's GCUPS: inputs resident on the host (pinned) to results
    (score, target_begin, CIGARs) on the host, one ta_align_batch per batch."""
    runner.run()
    runner.run()
    t0 = time.perf_counter()
    for _ in range(reps):
        runner.run()
    dt = (time.perf_counter() - t0) / reps
    r = runner.results()
    name, k = digest_name(args, batch.n_pairs)
    par = parity_vs_digest(r.scores, r.target_begins, r.cigar_lens, r.cigar, name, k) if (name and r.cigar_lens is not None) else None
    return {"value": round(batch.cells / dt / 1e9, 2), "unit": "GCUPS", "ms_per_batch": round(dt * 1e3, 4),
            "batches": reps, "path": "ta_align_batch: pinned host SoA in -> H2D -> kernels -> D2H -> host results "
                                     "(CIGARs compacted on the device)", "parity": par}


def host_to_host_pipelined(al, batch, mode, sc, cigar, args, budget, reps=10, overlap=True):
    """SURVEY §8d's GCUPS with the PCIe transfers overlapped (align.HostPipeline):
    every step uploads the batch from pinned host memory, runs the kernels and
    downloads every record and the compacted CIGAR bytes into pinned host memory;
    step k's upload and step k-1's download run beside the kernels."""
    from bioinfo1_amd.align import HostPipeline

    hp = HostPipeline(al, batch, mode, *sc, cigar, workspace_budget=budget, overlap=overlap)
    for _ in range(2):
        hp.step()
    hp.drain()
    t0 = time.perf_counter()
    for _ in range(reps):
        hp.step()
    hp.drain()
    dt = (time.perf_counter() - t0) / reps
    r = hp.results()
    hp.close()
    name, k = digest_name(args, batch.n_pairs)
    par = parity_vs_digest(r.scores, r.target_begins, r.cigar_lens, r.cigar, name, k) if (name and r.cigar_lens is not None) else None
    up = batch.qbytes.nbytes + batch.tbytes.nbytes
    down = 12 * batch.n_pairs + (int(r.cigar_lens.sum()) if r.cigar_lens is not None else 0)
    return {"value": round(batch.cells / dt / 1e9, 2), "unit": "GCUPS", "ms_per_batch": round(dt * 1e3, 4),
            "batches": reps, "pcie_bytes_per_batch": {"host_to_device": up, "device_to_host": down},
            "path": "align.HostPipeline: pinned host bytes -> H2D (upload stream) -> kernels + device CIGAR "
                    "compaction (compute stream) -> records + exact CIGAR bytes D2H (download stream), two "
                    "plans alternating", "parity": par}


def workload_name(args, cigar, n_pairs, full):
    tail = f"{args.mode}, scoring {args.scoring}, CIGAR {'on' if cigar else 'off'}"
    if args.workload == "cfg3":
        return (f"config 3 stand-in: {args.pairs} ONT-like reads per GPU (log-normal 1-20 kb, median 9 kb, 10% error, "
                f"50% reverse) of a 4.64 Mb synthetic genome vs their true-origin windows, {tail}")
    if args.workload == "cfg4":
        return (f"config 4: one set of {full.n_pairs} ONT-like reads (config-3 stand-in) vs true-origin windows, "
                f"range-split by cells over the GPUs, {tail}")
    pre = {"cfg2": "config 2: " if (args.qlen, args.tlen, args.pairs) == (1000, 1000, 10000) else "",
           "cfg5": (("config 5" if args.pairs >= 100000 else "config 5 slice") + " (linear gap): "
                    if args.gap_open is None else
                    ("config 5" if args.pairs >= 100000 else "config 5 slice")
                    + f", affine gaps (open {args.gap_open}, extend {args.scoring.split(',')[2]}): ")}[args.workload]
    return pre + (f"{n_pairs} {'related' if args.related else 'uniform'} {args.qlen}x{args.tlen} pairs per GPU, "
                  f"{tail}")


def _dropin_env(extra):
    e = dict(os.environ, **extra)
    e.pop("GPU_MAX_HW_QUEUES", None)
    if _HWQ_ORIG is not None:
        e["GPU_MAX_HW_QUEUES"] = _HWQ_ORIG
    return e


def main_dropin(args):
    """Single-call team::Align (the reference mapper's calling pattern) through
    our drop-in library vs the reference's own Align, same harness, same pairs."""
    res = {}
    # amd: the drop-in as shipped (pairs up to 4096 x 16384 on the resident single-pair server), run as
    # a plain library user runs it -- the process default of hardware queues, 4 on the box;
    # amd_batch_path: the same library with TEAM_ALIGN_SERVER=0 (concurrent calls combined into batches);
    # amd_queues16: one thread under GPU_MAX_HW_QUEUES=16 (what bench.py sets for its pipelines).
    # Before the timed runs, 2 s of 1 kb calls from 16 threads: a fresh box's idle GPU runs a
    # latency-bound 5x9 round trip at 19 us, one that has been busy at 13 (r06h: the same run's
    # later variants, and the queue count made no difference)
    amd = os.path.join(ROOT, "build", "dropin_amd")
    if os.path.exists(amd):
        subprocess.run([amd, "16", "2.0", "1000x1000", str(MODES[args.mode or "local"])], capture_output=True,
                       timeout=300, check=True, env=_dropin_env({}))
    for name, exe, env, threads in (("amd", amd, {}, (1, 8, 16)),
                                    ("amd_batch_path", amd, {"TEAM_ALIGN_SERVER": "0"}, (1, 8, 16)),
                                    ("amd_queues16", amd, {"GPU_MAX_HW_QUEUES": "16"}, (1,)),
                                    ("reference", os.path.join(ROOT, "oracle", "_ref", "dropin_ref"), {}, (1, 8, 16))):
        if not os.path.exists(exe):
            continue
        rows = []
        for thr in threads:  # 16: the host cores a GPU box grants this job
            e = _dropin_env({k: v for k, v in env.items() if k != "GPU_MAX_HW_QUEUES"})
            e.update({k: v for k, v in env.items() if k == "GPU_MAX_HW_QUEUES"})
            p = subprocess.run([exe, str(thr), "1.0", "5x9,200x200,1000x1000", str(MODES[args.mode or "local"])],
                               capture_output=True, text=True, timeout=300, check=True, env=e)
            rows += [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
        res[name] = rows
    same = None
    if "amd" in res and "reference" in res:
        key = lambda r: (r["shape"], r["threads"])  # noqa: E731
        ref = {key(r): r["score_checksum"] for r in res["reference"]}
        same = all(ref.get(key(r)) == r["score_checksum"] for v in ("amd", "amd_batch_path", "amd_queues16")
                   for r in res.get(v, []))
    print(json.dumps({"metric": "team::Align single-call throughput (drop-in, one pair per call)", "unit": "calls/s",
                      "mode": args.mode or "local", "score_checksums_equal": same, "results": res}), flush=True)


def main_mapper(args, D):
    """config 3 end to end: the team_mapper pipeline on the GPU (minimizers ->
    seed hits -> FindLIS -> one alignment batch) for this rank's reads against
    the whole 4.64 Mb genome (index replicated per GPU, reads range-split)."""
    import torch

    from bioinfo1_amd import mapper as M
    from bioinfo1_amd import shard, synth

    mode = MODES[args.mode]
    sc = tuple(int(x) for x in args.scoring.split(","))
    g = synth.genome(synth.ECOLI_LEN)
    rs = synth.ont_reads(args.pairs, g, first_read=D.rank * args.pairs)
    reads = (rs.bytes if rs.bytes.size else np.zeros(1, np.uint8), rs.off.copy(), rs.len.copy())  # SoA, packed once
    mp = M.Mapper(D.dev_index)
    t0 = time.perf_counter()
    idx = M.Index(mp, "ecoli_syn", g.tobytes(), 15, 5, 0.001)
    index_s = time.perf_counter() - t0
    opt = M.Options.make(type=mode, match=sc[0], mismatch=sc[1], gap=sc[2], want_cigar=not args.no_cigar,
                         fastq_rules=True)

    def step():
        r = idx.map_batch(reads, opt)
        if D.world > 1:  # gather every rank's records and CIGAR bytes in read order (RCCL over xGMI)
            n_cig = int(r.cigar_len.sum()) if opt.want_cigar else 0
            cig = torch.from_numpy(r.arena[:n_cig]).to(D.cdev) if opt.want_cigar else None
            t = lambda a: torch.from_numpy(a.view(np.int32)).to(D.cdev)  # noqa: E731
            shard.gather_results(D.dist, t(r.scores), t(r.t_begin), t(r.cigar_len), cig, device=D.cdev)
        return r

    for _ in range(args.warmup):
        step()
    D.barrier()
    torch.cuda.synchronize(D.dev)
    t0 = time.perf_counter()
    stages = {}
    for _ in range(args.steps):
        r = step()
        st, cells = mp.stage_times()
        plan_stats = mp.align_plan_stats()
        for k, v in st.items():
            stages[k] = stages.get(k, 0.0) + v / args.steps
    torch.cuda.synchronize(D.dev)
    D.barrier()
    elapsed = D.max(time.perf_counter() - t0)
    ms = elapsed / max(args.steps, 1) * 1e3
    out = None
    if D.rank == 0:
        extra = {}
        if D.world == 1 and not args.no_cpu:
            extra = mapper_cpu_baseline_and_parity(g, rs, 24, args.mode, os.path.join(ROOT, "gpurun_out", "cfg3map"))
        out = {
            "metric": METRIC, "value": round(cells * D.world / (ms / 1e3) / 1e9, 2), "unit": "GCUPS",
            "n_gpus": D.world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": DTYPE, "data": "synthetic",
            "config": {"workload": f"config 3 end to end: {args.pairs} ONT-like reads per GPU (log-normal 1-20 kb, "
                                   f"10% error, 50% reverse, FASTQ rules) mapped to a 4.64 Mb synthetic genome: GPU "
                                   f"minimizers, seed matching, FindLIS, {args.mode} alignment of the chained windows "
                                   f"with CIGAR {'off' if args.no_cigar else 'on'}; host reads in, host results out",
                       "reads_per_gpu": args.pairs, "mode": args.mode, "aligned_cells_per_gpu": cells,
                       "parallelism": f"reads range-split over {D.world} GPU(s), index replicated, RCCL all-gather "
                                      f"of per-read records and CIGAR bytes"},
            "reads_mapped": int(r.mapped.sum()), "reads_per_s": round(args.pairs * D.world / (ms / 1e3), 1),
            "index_build_s": round(index_s, 3), "stage_ms": {k: round(v, 3) for k, v in stages.items()},
            "align_plan": plan_stats,
            "roofline": None, "device": torch.cuda.get_device_name(D.dev), **extra,
        }
    idx.close()
    mp.close()
    D.close()
    if out is not None:
        print(json.dumps(out), flush=True)


def write_fastx(path, recs, fastq):
    with open(path, "wb") as f:
        for name, seq in recs:
            if fastq:
                f.write(b"@" + name + b"\n" + seq + b"\n+\n" + b"I" * len(seq) + b"\n")
            else:
                f.write(b">" + name + b"\n" + seq + b"\n")


def mapper_cpu_baseline_and_parity(genome, reads, sample, mode_name, tmpdir):
    """oracle/_ref/ref_mapper (the reference's Minimize + Align, restated glue,
    sequential) on the first `sample` reads, timed; and team_mapper_amd on the
    same files, whose PAF lines must be byte-identical."""
    from bioinfo1_amd import mapper as M
    from oracle.pymapper import REF_MAPPER_BIN

    os.makedirs(tmpdir, exist_ok=True)
    gp, rp = os.path.join(tmpdir, "genome.fasta"), os.path.join(tmpdir, "reads.fastq")
    write_fastx(gp, [(b"ecoli_syn", genome.tobytes())], False)
    write_fastx(rp, [(b"read%d" % r, reads.read(r)) for r in range(sample)], True)
    args = ["-a", mode_name, "-c", gp, rp]
    res = {}
    if os.path.exists(REF_MAPPER_BIN):
        env = dict(os.environ, REF_MAPPER_TIMING="1")
        t0 = time.perf_counter()
        ref = subprocess.run([REF_MAPPER_BIN] + args, capture_output=True, env=env, check=True)
        wall = time.perf_counter() - t0
        tm = dict(kv.split("=") for kv in ref.stderr.decode().split("ref_mapper_timing ")[1].split())
        cells = int(tm["aligned_cells"])
        res["cpu_baseline"] = {"value": round(cells / float(tm["map_s"]) / 1e9, 4), "unit": "GCUPS", "cores": 1,
                               "kind": "reference",
                               "sample": f"first {sample} reads ({cells:.3g} aligned cells): reference Minimize + Align "
                                         f"with the restated team_mapper glue, sequential; index build "
                                         f"{float(tm['index_s']):.2f} s excluded, {wall:.1f} s wall",
                               "impl": "oracle/_ref/ref_mapper"}
        gpu = M.run_cli(args, timeout=300)
        res["parity"] = {"golden": f"oracle/_ref/ref_mapper PAF on the first {sample} reads",
                         "lines": ref.stdout.count(b"\n"), "bit_exact": gpu.returncode == 0 and gpu.stdout == ref.stdout}
    return res


def main():
    args = parse()
    if args.workload == "dropin":
        return main_dropin(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(3)
    D = Dist(args)
    if args.workload == "cfg3map":
        return main_mapper(args, D)
    return main_align(args, D)


if __name__ == "__main__":
    main()
