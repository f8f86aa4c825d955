#!/usr/bin/env python3
"""Benchmark of the team::Align hot path on MI355X (BASELINE.json config 2).

One "step" = one pass of the path over one batch: the DP fill kernel and the
traceback/CIGAR kernel for 10,000 synthetic 1 kb x 1 kb read-vs-window pairs,
Smith-Waterman (local), match/mismatch/gap = 1/-1/-1, CIGAR on -- inputs
resident in HBM before the timed region, results (score, target_begin,
CIGAR) left in HBM.  With N GPUs (torch.distributed.run, one process per
GPU, RCCL) every rank aligns its own 10,000 pairs (weak scaling: pairs are
independent, the batch is range-split by pair index) and the fixed-size
per-pair records of every step are all-gathered over RCCL inside the timed
region (asynchronously: step k's gather overlaps step k+1; drained before
the clock stops).  --pipeline runs the K steps as one pipelined sequence of K batches
(ta_plan_execute_batches: batch k's traceback beside batch k+1's fill, each
batch with its own outputs).  batch_latency_ms = one batch alone (fill +
traceback kernels, HIP events).

Prints ONE JSON line (rank 0).  value = whole-job GCUPS = (sum of n*m over
all ranks' pairs) / (max over ranks of the step time).

Also reported, on rank 0:
  roofline      -- the fill kernel's algorithmic bytes per launch / its
                   average duration (HIP events on the launch stream) against
                   the 8 TB/s HBM peak; traffic = PMC-measured HBM bytes per
                   launch from profiles/ when present.
  valu          -- the same kernel against the VALU int32 roofline (the roof
                   that actually binds this integer DP).
  cpu_baseline  -- the reference team::Align (oracle/_ref, compiled from the
                   reference sources) or, where it was not built, our C
                   restatement (oracle/), on the node's host cores, OpenMP
                   over pairs, on a bounded sample of the same batch.
  parity        -- this run's first step compared with the committed golden
                   digest of the same seeded batch (tests/golden/).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bioinfo1_amd import synth  # noqa: E402
from bioinfo1_amd.align import Aligner, DevicePlan  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, Chip-level parameters)
# int32 VALU: a wave64 integer instruction occupies its SIMD for 4 cycles (measured:
# SQ_ACTIVE_INST_VALU == SQ_INSTS_VALU quad-cycles at ~100% busy), i.e. 16 lanes/clk/SIMD:
# 256 CU x 4 SIMD x 16 lanes x 2.4 GHz = 39.3 T lane-ops/s
VALU_PEAK_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="cfg2", choices=["cfg2", "cfg3", "cfg5", "cfg3map"],
                    help="cfg2: 1kx1k pairs (headline); cfg3: E. coli stand-in, ONT-like reads vs true-origin "
                         "windows, semiGlobal; cfg5: 10kx10k related semiGlobal (a sample of the 100k pairs); "
                         "cfg3map: config 3 end to end -- minimizer seeding, FindLIS chaining and semiGlobal "
                         "alignment of the same reads against the 4.64 Mb genome (team_mapper pipeline)")
    ap.add_argument("--pairs", type=int, default=0, help="pairs per GPU (0 = the workload's default)")
    ap.add_argument("--qlen", type=int, default=1000)
    ap.add_argument("--tlen", type=int, default=1000)
    ap.add_argument("--mode", default=None, choices=["global", "local", "semiGlobal"])
    ap.add_argument("--scoring", default="1,-1,-1")
    ap.add_argument("--related", action="store_true", help="config-2 related variant (5%% sub/ins/del)")
    ap.add_argument("--no-cigar", action="store_true", help="score-only (cigar == nullptr) mode")
    ap.add_argument("--cpu-pairs", type=int, default=10000, help="CPU-baseline sample size (pairs)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, host cores)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workspace-gb", type=float, default=0.0,
                    help="device budget (GB) for the 2-bit traceback codes; 0 = the library default (85%% of free HBM); batches above it run in chunks")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--gap-open", type=int, default=None,
                    help="affine-gap extension (no reference counterpart): a gap of length L costs "
                         "gap_open + L*gap, gap = the third --scoring value (config 5's 'affine gaps')")
    ap.add_argument("--pipeline", action="store_true",
                    help="run the K steps as one ta_plan_execute_batches call (batch k's traceback on a "
                         "second stream beside batch k+1's fill) instead of ta_plan_execute per step; "
                         "measured slower on config 2 (DESIGN.md 3.8)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL, default) or gloo (rehearsal only)")
    a = ap.parse_args()
    if a.workload == "cfg2":
        a.pairs = a.pairs or 10000
        a.mode = a.mode or "local"
    elif a.workload in ("cfg3", "cfg3map"):
        a.pairs = a.pairs or 10000
        a.mode = a.mode or "semiGlobal"
        a.cpu_pairs = min(a.cpu_pairs, 200)
    else:
        # a slice of config 5's 100k pairs that fills the GPU in one chunk: 8,192 pairs (4,096
        # two-pair waves, 197 GB of 2-bit codes); affine 4,096 (4-bit codes, 197 GB)
        a.pairs = a.pairs or (8192 if a.gap_open is None else 4096)
        a.mode = a.mode or "semiGlobal"
        a.qlen = a.tlen = 10000
        a.related = True
        a.cpu_pairs = min(a.cpu_pairs, 64 if a.gap_open is None else 32)
    return a


MODES = {"global": 0, "local": 1, "semiGlobal": 2}


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


def cpu_baseline(batch, mode, sc, cigar, pairs, threads, gap_open=None):
    from oracle.pyoracle import Oracle, Reference

    affine = gap_open is not None
    impl = Reference() if Reference.available() and not affine else Oracle()
    sample = batch.slice(0, min(pairs, batch.n_pairs))
    t0 = time.perf_counter()
    if affine:  # the reference has no affine Align: the CPU definition (oracle/affine_oracle.c) is the baseline
        res = impl.align_affine_batch(sample, mode, sc[0], sc[1], gap_open, sc[2], cigar, n_threads=threads)
    else:
        res = impl.align_batch(sample, mode, *sc, cigar, n_threads=threads)
    dt = time.perf_counter() - t0
    assert not res.status.any()
    return {"value": round(sample.cells / dt / 1e9, 4), "unit": "GCUPS", "cores": threads, "kind": impl.kind,
            "sample": f"first {sample.n_pairs} pairs of the same batch ({sample.cells:.3g} cells), "
                      f"OpenMP over pairs, {dt:.2f} s wall",
            "impl": "oracle/_ref/libref_align.so (reference team_alignment.cpp, g++ -O3)" if impl.kind == "reference"
            else ("oracle/liboracle.so (affine_oracle.c: the extension's CPU definition)" if affine
                  else "oracle/liboracle.so (C restatement)")}


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


def parity_vs_digest(res, batch, args):
    """Compare against the committed golden digest (made by the reference) of
    this seeded batch, or of its first pairs (per-pair streams make the
    digest batches prefixes of the bench batches)."""
    name, k = None, batch.n_pairs
    if args.workload == "cfg2" and (args.mode, args.scoring, args.qlen, args.tlen) == ("local", "1,-1,-1", 1000, 1000) \
            and batch.n_pairs == 10000:
        name = "cfg2_related_local" if args.related else "cfg2_local"
    elif args.workload == "cfg3" and (args.mode, args.scoring) == ("semiGlobal", "1,-1,-1") and batch.n_pairs >= 64:
        name, k = "cfg3_semi_sample", 64
    elif args.workload == "cfg5" and (args.mode, args.scoring) == ("semiGlobal", "1,-1,-1") and batch.n_pairs >= 32:
        name, k = "cfg5_semi_sample", 32
    if name is None or res.cigar_lens is None or (args.gap_open or 0) != 0:
        return None
    import hashlib

    with open(os.path.join(ROOT, "tests", "golden", f"digest_{name}.json")) as f:
        meta = json.load(f)
    d = np.load(os.path.join(ROOT, "tests", "golden", f"digest_{name}.npz"))
    ok = bool(np.array_equal(res.scores[:k], d["scores"]) and np.array_equal(res.target_begins[:k], d["target_begins"])
              and np.array_equal(res.cigar_lens[:k], d["cigar_lens"]))
    h = hashlib.sha256()
    for p in range(k):
        c = res.cigar(p)
        h.update(len(c).to_bytes(4, "little"))
        h.update(c)
    ok = ok and h.hexdigest() == meta["cigar_sha256"]
    return {"golden": f"tests/golden/digest_{name}", "pairs_checked": k, "bit_exact": ok}


def workload_name(args, cigar):
    tail = f"{args.mode}, scoring {args.scoring}, CIGAR {'on' if cigar else 'off'}"
    if args.workload == "cfg3":
        return (f"config 3 stand-in: {args.pairs} ONT-like reads per GPU (log-normal 1-20 kb, median 9 kb, 10% error, "
                f"50% reverse) of a 4.64 Mb synthetic genome vs their true-origin windows, {tail}")
    pre = {"cfg2": "config 2: " if (args.qlen, args.tlen, args.pairs) == (1000, 1000, 10000) else "",
           "cfg5": ("config 5 sample (linear gap): " if args.gap_open is None else
                    f"config 5 sample, affine gaps (open {args.gap_open}, extend {args.scoring.split(',')[2]}): ")}[args.workload]
    return pre + (f"{args.pairs} {'related' if args.related else 'uniform'} {args.qlen}x{args.tlen} pairs per GPU, "
                  f"{tail}")


def load_traffic(tag):
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        t = json.load(f)
    return t.get(tag)


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
    import subprocess

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


def main_mapper(args):
    """config 3 end to end: the team_mapper pipeline on the GPU (minimizers ->
    seed hits -> FindLIS -> one alignment batch) for this rank's reads against
    the whole 4.64 Mb genome (index replicated per GPU, reads range-split)."""
    from bioinfo1_amd import mapper as M

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(args.dist_backend)
    dev_index = 0 if os.environ.get("TA_BENCH_ONE_GPU") == "1" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    mode = MODES[args.mode]
    sc = tuple(int(x) for x in args.scoring.split(","))
    g = synth.genome(synth.ECOLI_LEN)
    rs = synth.ont_reads(args.pairs, g, first_read=rank * args.pairs)
    reads = (rs.bytes if rs.bytes.size else np.zeros(1, np.uint8), rs.off.copy(), rs.len.copy())  # SoA, packed once
    mp = M.Mapper(dev_index)
    t0 = time.perf_counter()
    idx = M.Index(mp, "ecoli_syn", g.tobytes(), 15, 5, 0.001)
    index_s = time.perf_counter() - t0
    opt = M.Options.make(type=mode, match=sc[0], mismatch=sc[1], gap=sc[2], want_cigar=not args.no_cigar,
                         fastq_rules=True)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    def step():
        r = idx.map_batch(reads, opt)
        if world > 1:  # config 4: gather every rank's records and CIGAR bytes in read order (RCCL over xGMI)
            from bioinfo1_amd import shard

            n_cig = int(r.cigar_len.sum()) if opt.want_cigar else 0
            cig = torch.from_numpy(r.arena[:n_cig]).to(coll_dev) if opt.want_cigar else None
            t = lambda a: torch.from_numpy(a.view(np.int32)).to(coll_dev)  # noqa: E731
            shard.gather_results(dist, t(r.scores), t(r.t_begin), t(r.cigar_len), cig, device=coll_dev)
        return r

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    stages = {}
    for _ in range(args.steps):
        r = step()
        st, cells = mp.stage_times()
        for k, v in st.items():
            stages[k] = stages.get(k, 0.0) + v / args.steps
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    ms = elapsed / max(args.steps, 1) * 1e3
    out = None
    if rank == 0:
        extra = {}
        if world == 1 and not args.no_cpu:
            extra = mapper_cpu_baseline_and_parity(g, rs, 24, args.mode, os.path.join(ROOT, "gpurun_out", "cfg3map"))
        out = {
            "metric": "GCUPS (DP cell updates/s) at 1/2/4/8 GPUs; bit-exact score+CIGAR",
            "value": round(cells * world / (ms / 1e3) / 1e9, 2), "unit": "GCUPS", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": f"config 3 end to end: {args.pairs} ONT-like reads per GPU (log-normal 1-20 kb, "
                                   f"10% error, 50% reverse, FASTQ rules) mapped to a 4.64 Mb synthetic genome: GPU "
                                   f"minimizers, seed matching, FindLIS, {args.mode} alignment of the chained windows "
                                   f"with CIGAR {'off' if args.no_cigar else 'on'}; host reads in, host results out",
                       "reads_per_gpu": args.pairs, "mode": args.mode, "aligned_cells_per_gpu": cells,
                       "parallelism": f"reads range-split over {world} GPU(s), index replicated, RCCL all-gather "
                                      f"of per-read records and CIGAR bytes (config 4 when world = 8)"},
            "reads_mapped": int(r.mapped.sum()), "reads_per_s": round(args.pairs * world / (ms / 1e3), 1),
            "index_build_s": round(index_s, 3), "stage_ms": {k: round(v, 3) for k, v in stages.items()},
            "roofline": None, "device": torch.cuda.get_device_name(dev), **extra,
        }
    idx.close()
    mp.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.workload == "cfg3map":
        return main_mapper(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(args.dist_backend)
    # TA_BENCH_ONE_GPU=1: every rank on device 0 (multi-rank rehearsal on a 1-GPU box, gloo)
    dev_index = 0 if os.environ.get("TA_BENCH_ONE_GPU") == "1" else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    mode = MODES[args.mode]
    sc = tuple(int(x) for x in args.scoring.split(","))
    cigar = not args.no_cigar

    # this rank's slice of the whole job: pairs [rank*P, (rank+1)*P) of the seeded stream
    P = args.pairs
    if args.workload == "cfg3":
        batch = synth.cfg3_batch(P, first_read=rank * P)[0]
    else:
        gen = synth.related_batch if args.related else synth.uniform_batch
        batch = gen(P, args.qlen, args.tlen, 0x5EED, first_pair=rank * P)

    al = Aligner(dev_index)
    plan = DevicePlan(al, batch, mode, *sc, cigar, workspace_budget=int(args.workspace_gb * 2**30),
                      gap_open=args.gap_open)
    stream = torch.cuda.current_stream(dev)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # gloo: host tensors
    # Steps = batches.  --pipeline: ta_plan_execute_batches runs batch k's
    # traceback beside batch k+1's fill; every batch has its own output
    # buffers, so all K results stay intact and are gathered at the end.
    pipelined = cigar and args.gap_open is None and args.pipeline
    n_sets = max(args.steps, args.warmup, 2)
    outs = [plan] + [plan.output_set() for _ in range(n_sets - 1)] if pipelined else None

    def gather(sets):
        if world > 1:  # range-split results -> every rank (RCCL all-gather over xGMI)
            rec = torch.empty((len(sets), 3, P), dtype=torch.int32, device=dev)
            for k, o in enumerate(sets):
                rec[k, 0].copy_(o.score)
                rec[k, 1].copy_(o.target_begin)
                rec[k, 2].copy_(o.cigar_len if cigar else o.score)
            rec = rec.to(coll_dev)
            out = torch.empty((world * len(sets), 3, P), dtype=torch.int32, device=coll_dev)
            # asynchronous: step k's gather overlaps step k+1's kernels; drained before the clock stops
            pending.append((rec, out, dist.all_gather_into_tensor(out, rec, async_op=True)))

    pending = []

    def drain():
        for _, _, h in pending:
            h.wait()
        pending.clear()

    def run_steps(k):
        if k <= 0:
            return
        if pipelined:
            plan.run_batches(outs[:k])
            gather(outs[:k])
        else:
            for _ in range(k):
                plan.run()
                gather([plan])

    run_steps(args.warmup)
    drain()
    parity = None
    if rank == 0 and not args.no_parity:
        if args.warmup < (2 if pipelined else 1):
            # compute only (rank 0 alone: no collective here)
            plan.run_batches(outs[:2]) if pipelined else plan.run()
        parity = parity_vs_digest(plan.results(), batch, args)
        if parity is not None and pipelined:  # batch 1 ran beside batch 0 (capped traceback grid on its own)
            p1 = parity_vs_digest(outs[1].results(), batch, args)
            parity["pairs_checked"] += p1["pairs_checked"]
            parity["bit_exact"] = parity["bit_exact"] and p1["bit_exact"]
            parity["batches_checked"] = 2
        if parity is None and args.gap_open is not None:
            parity = parity_vs_oracle(plan.results(), batch, mode, sc, args.gap_open, 16)

    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(args.steps)
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    ms = elapsed / max(args.steps, 1) * 1e3
    cells_job = batch.cells * world
    gcups = cells_job / (ms / 1e3) / 1e9

    out = None
    if rank == 0:
        # dominant kernel (fill) timed on its own launch stream with HIP events
        kt, tt = [], []
        for _ in range(max(args.steps, 3)):
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
        alg = fill_alg_bytes(batch, cigar, args.gap_open is not None)
        achieved = alg / (fill_ms / 1e3) / 1e9 if alg else None
        tag = (f"{args.mode}_{'cigar' if cigar else 'score'}_{args.pairs}x{args.qlen}x{args.tlen}" if args.workload != "cfg3"
               else f"cfg3_{'cigar' if cigar else 'score'}_{args.pairs}")
        if args.gap_open is not None:
            tag = "affine_" + tag
        traffic = load_traffic(tag)
        roof = {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic, "kernel": ("affine_dual_fill_kernel" if plan.dual_pairs else "affine_fill_kernel")
                if args.gap_open is not None else "fill_kernel",
                "kernel_ms": round(fill_ms, 4),
                "alg_bytes_per_launch": alg,
                "note": "integer DP: VALU-bound, not HBM- or MFMA-bound (see valu)"}
        ops_per_cell = None
        pv = os.path.join(ROOT, "profiles", "valu.json")
        if os.path.exists(pv):
            with open(pv) as f:
                ops_per_cell = json.load(f).get(tag)
        valu = {"kernel_gcups": round(batch.cells / (fill_ms / 1e3) / 1e9, 2), "peak_int32_tops": round(VALU_PEAK_TOPS, 1),
                "valu_ops_per_cell": ops_per_cell,
                "frac": round(batch.cells * ops_per_cell / (fill_ms / 1e3) / 1e12 / VALU_PEAK_TOPS, 4)
                if ops_per_cell else None}
        cpu = None
        if world == 1 and not args.no_cpu:
            thr = args.cpu_threads or min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(batch, mode, sc, cigar, args.cpu_pairs, thr, args.gap_open)
        out = {
            "metric": "GCUPS (DP cell updates/s) at 1/2/4/8 GPUs; bit-exact score+CIGAR",
            "value": round(gcups, 2), "unit": "GCUPS", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32", "data": "synthetic",
            "config": {"workload": workload_name(args, cigar),
                       "pairs_per_gpu": args.pairs, "qlen": args.qlen if args.workload != "cfg3" else "1-20 kb reads",
                       "tlen": args.tlen if args.workload != "cfg3" else "true-origin window", "mode": args.mode,
                       "cigar": cigar, "cells_per_gpu": batch.cells,
                       "parallelism": f"pairs range-split over {world} GPU(s), RCCL all-gather of per-pair records"},
            "fill_ms": round(fill_ms, 4), "traceback_ms": round(float(np.mean(tt)), 4) if cigar else None,
            "pipelined": pipelined,
            "batch_latency_ms": round(fill_ms + (float(np.mean(tt)) if cigar else 0.0), 4),
            "chunks": plan.chunks, "workspace_gb": round(plan.workspace_bytes / 2**30, 2),
            "roofline": roof, "valu": valu, "cpu_baseline": cpu, "parity": parity,
            "device": torch.cuda.get_device_name(dev),
        }
    plan.close()
    al.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if out is not None:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
