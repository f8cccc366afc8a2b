#!/usr/bin/env python
"""Benchmark of the MI355X classify hot path (BASELINE.json metric, configs[1]).

Workload (config 2): 1M x 150 bp paired reads vs a RefSeq-viral-sized (~10 GB) reference DB, DB
resident in HBM, reads resident in HBM when the timed region starts. Synthetic data (no network):
species genomes + two 2%-diverged strains each, gene blocks shared by a species' strains, the DB
built on the GPU in the reference's on-disk format (mtb_build_db), reads sampled from the genomes
with 0.5% substitutions plus 10% random reads.

One step = one pass of the whole path over the batch: K0 read metadata, K1 extract, K2 k-mer
radix sort, K4 match (count + emit), K5/K6 per-read sort + assignment, taxcnt compaction; with
N > 1 ranks, plus an RCCL all-gather of the per-read result records (weak scaling: every rank
classifies its own batch against its own DB replica).

Prints one JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from metabuli_work_amd import synth  # noqa: E402
from metabuli_work_amd._abi import RESULT_DTYPE, default_params  # noqa: E402
from metabuli_work_amd.classifier import Classifier, LocalParameters  # noqa: E402
from metabuli_work_amd.dbbuild import build_db  # noqa: E402
from metabuli_work_amd.gpu_synth import make_genomes_gpu, make_long_reads_gpu, make_reads_gpu  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01", "stage_traffic.json")
# the six timed kernels of mtb_last_kernel_ms, by join path (mtb_last_stats[10])
KERNELS_SORT = ["extract", "filter", "kmer_sort", "match_join", "match_transpose", "match_sort", "assign"]
KERNELS_PROBE = ["extract", "filter", "kmer_sort", "probe_join", "match_transpose", "match_sort", "assign"]


def kernel_names(work):
    return KERNELS_PROBE if work.get("join_path", 1) == 0 else KERNELS_SORT


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=1_000_000, help="read pairs per rank per step")
    ap.add_argument("--species", type=int, default=25000)
    ap.add_argument("--mean-genome", type=int, default=75000)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="read pairs timed on the CPU oracle (0 = off)")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--long-reads", type=int, default=50_000,
                    help="ONT-style reads (N50 ~10 kb) per rank for the long-read line (0 = off)")
    ap.add_argument("--db-parts", type=int, default=0,
                    help="config-5 mode: the DB range-partitioned into this many parts (= the number of ranks; "
                         "on one GPU every part is timed in turn)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    t0 = time.time()
    par = default_params(kmer_format=2, seq_mode=2)
    taxo, gen, seq, off_t, lens = make_genomes_gpu(args.species, args.mean_genome, 2, args.seed, dev)
    rseed = args.seed * 1000 + 1 + (0 if args.db_parts > 1 else 17 * rank)  # config 5: one batch on all ranks
    s1, o1, s2, o2 = make_reads_gpu(seq, off_t, args.pairs, rseed, dev)
    torch.cuda.synchronize()
    log(rank, f"[bench] genomes {seq.numel() / 1e9:.2f} Gbp in {len(lens) * 2} genomes, blocks "
              f"{len(gen.blk_genome)}; reads {args.pairs} pairs ({time.time() - t0:.1f}s)")
    if args.long_reads > 0:
        ls1, lo1, long_n50 = make_long_reads_gpu(seq, off_t, args.long_reads, args.seed * 1000 + 17 * rank + 7, dev)
    hdb = build_db(gen, taxo, par, device=local, device_seq=(seq, off_t))
    del seq
    torch.cuda.empty_cache()
    db_bytes = hdb.nbytes
    log(rank, f"[bench] DB built: {hdb.n_kmers / 1e9:.3f}G k-mers, {db_bytes / 1e9:.2f} GB "
              f"(diffIdx+info) ({time.time() - t0:.1f}s)")
    lp = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1)
    if args.db_parts > 1:
        return run_partitioned(args, lp, hdb, (s1, o1, s2, o2), world, rank, local, dev)
    clf = Classifier(lp, db_host=hdb.c_struct(), device=local)
    log(rank, f"[bench] DB resident in HBM ({time.time() - t0:.1f}s)")

    n = args.pairs
    gathered = None
    res_dev = torch.empty(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    if world > 1:
        gathered = torch.empty(world * res_dev.numel(), dtype=torch.uint8, device=dev)

    def step():
        clf.classify_batch(s1, o1, s2, o2, device_input=True, fetch=False)
        if world > 1:
            clf.copy_results(res_dev.data_ptr(), on_device=True)
            dist.all_gather_into_tensor(gathered, res_dev)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kern = np.zeros(7)
    stage = np.zeros(5)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
        kern += clf.kernel_ms()
        stage += clf.stage_ms()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern /= max(1, args.steps)
    stage /= max(1, args.steps)
    Q, M = clf.last_counts()
    work = clf.stats()
    KERNELS = kernel_names(work)
    ms_per_step = elapsed / max(1, args.steps) * 1e3
    value = world * n * args.steps / elapsed

    # ---- roofline of the dominant kernel: algorithmic bytes per launch / event-timed duration ----
    read_bytes = 2 * n * 150 + 2 * 8 * (n + 1)
    R = int(2 * 252 * n)  # reserved slots: getQueryKmerNumber(150) = (147/3 - 8 + 1) * 6 = 252 per mate
    D = hdb.n_kmers
    alg = {
        "filter": 8 * R + 4 * R + 20 * Q,                  # keys in, one 4-B membership word per window,
                                                            # the present (key, slot, DB lower bound) out
        # probe join: per query its (key, slot, lower bound), 8 DB values + taxIDs from there,
        # its staged matches (+ rank) out
        "probe_join": 20 * Q + 96 * Q + 28 * M,
        "extract": read_bytes + 8 * R,                      # reads in, one 8-B key per window out
        "kmer_sort": 2 * 3 * 12 * Q,                        # three passes over the (key, slot) pairs
        "match_join": 12 * Q + 12 * D + 28 * M,             # queries, the DB (values + taxIDs) streamed through
                                                            # the block windows once, staged matches written
        "match_transpose": 2 * 24 * M + 4 * M + 8 * n,      # staged matches (+ rank) read, written to segments
        "match_sort": 2 * 24 * M + 8 * (n + 1),             # each read's matches read and written once
        "assign": 24 * M + 32 * n + 4 * n + 8 * n,          # sorted matches read, results + lengths written
    }
    dom = int(np.argmax(kern))
    dname = KERNELS[dom]
    achieved = alg[dname] / (kern[dom] * 1e-3) / 1e9
    # HBM traffic of the same stage per step from rocprofv3 FETCH_SIZE/WRITE_SIZE passes over this
    # workload (tools/pmc_passes.sh + tools/stage_profile.py, committed under profiles/)
    traffic, traffic_src = None, None
    try:
        with open(TRAFFIC_FILE) as f:
            tf = json.load(f)
        if tf.get("pairs") == n and tf.get("species") == args.species and dname in tf["stages"]:
            traffic = tf["stages"][dname]["hbm_bytes"]
            traffic_src = os.path.relpath(TRAFFIC_FILE, ROOT)
    except (OSError, ValueError, KeyError):
        pass
    roofline = {"bound": "hbm", "kernel": dname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": traffic_src, "alg_bytes_per_launch": int(alg[dname]),
                "avg_launch_ms": round(float(kern[dom]), 3)}

    # ---- CPU baseline: the oracle (restated reference algorithm, OpenMP) on a bounded sample ----
    cpu = None
    parity = None
    odb = None
    cores = 1
    if rank == 0 and args.cpu_sample > 0:
        from tests import oracle_ctypes as oc  # checker / baseline only

        S = min(args.cpu_sample, n)
        h1 = s1[:S * 150].cpu().numpy()
        h2 = s2[:S * 150].cpu().numpy()
        ho = o1[:S + 1].cpu().numpy().astype(np.uint64)
        reads = synth.Reads(h1, ho, h2, ho.copy(), np.zeros(S, np.int32))
        cores = len(os.sched_getaffinity(0))
        cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
        oc.lib().orc_set_threads(cores)
        opar = lp.to_c()
        opar.threads = cores
        odb = oc.OracleDb.from_host(hdb.c_struct())  # kept open for the long-read baseline below
        stage_s = np.zeros(4)
        tc0 = time.perf_counter()
        ores, otc = oc.classify(odb, opar, reads, stage_s=stage_s)
        cpu_t = time.perf_counter() - tc0
        cpu = {"value": round(S / cpu_t, 1), "unit": "reads/s", "cores": cores, "kind": "port",
               "sample": f"first {S} read pairs of the rank-0 batch, same DB; oracle/ (OpenMP C++ restatement "
                         f"of the reference path), {cpu_t:.1f}s wall",
               "stage_s": [round(x, 3) for x in stage_s]}
        gb = clf.classify_batch(h1, ho, h2, ho.copy())
        parity = bool(np.array_equal(gb.results["classification"], ores["classification"])
                      and np.array_equal(gb.results["score"].view(np.uint32), ores["score"].view(np.uint32))
                      and np.array_equal(gb.taxcnt, otc))

    # ---- long reads (seq mode 3, same DB): reads/s of the same pipeline on ~10 kb reads ----
    long_line = None
    if args.long_reads > 0:
        clf.close()
        lpl = LocalParameters(seqMode=3, kmerFormat=2, skipRedundancy=1)
        clfl = Classifier(lpl, db_host=hdb.c_struct(), device=local)
        for _ in range(max(1, args.warmup)):
            clfl.classify_batch(ls1, lo1, device_input=True, fetch=False)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        lsteps = max(1, min(args.steps, 3))
        kl = np.zeros(7)
        tl0 = time.perf_counter()
        for _ in range(lsteps):
            clfl.classify_batch(ls1, lo1, device_input=True, fetch=False)
            kl += clfl.kernel_ms()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        tl = time.perf_counter() - tl0
        if world > 1:
            t = torch.tensor([tl], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tl = float(t.item())
        lq, lm = clfl.last_counts()
        lwork = clfl.stats()
        long_cpu = None
        if rank == 0 and args.cpu_sample > 0:
            # the oracle on the first reads of the long batch (~10 s of 16-core work), and the GPU's
            # results for the same reads compared with it
            LS = max(1, min(args.long_reads, args.cpu_sample // 50))
            lo_h = lo1[:LS + 1].cpu().numpy().astype(np.uint64)
            ls_h = ls1[:int(lo_h[-1])].cpu().numpy()
            lreads = synth.Reads(ls_h, lo_h, None, None, np.zeros(LS, np.int32))
            lopar = lpl.to_c()
            lopar.threads = cores
            tc0 = time.perf_counter()
            lres, ltc = oc.classify(odb, lopar, lreads)
            lcpu_t = time.perf_counter() - tc0
            gl = clfl.classify_batch(ls_h, lo_h)
            long_cpu = {"value": round(LS / lcpu_t, 1), "unit": "reads/s", "cores": cores, "kind": "port",
                        "sample": f"first {LS} long reads of the rank-0 batch, same DB, {lcpu_t:.1f}s wall",
                        "parity_sample": bool(np.array_equal(gl.results["classification"], lres["classification"])
                                              and np.array_equal(gl.results["score"].view(np.uint32),
                                                                 lres["score"].view(np.uint32))
                                              and np.array_equal(gl.taxcnt, ltc))}
        long_line = {"value": round(world * args.long_reads * lsteps / tl, 1), "unit": "reads/s",
                     "ms_per_step": round(tl / lsteps * 1e3, 3), "steps": lsteps,
                     "reads_per_gpu": args.long_reads, "bases_per_gpu": int(lo1[-1].item()), "n50": long_n50,
                     "query_kmers": lq, "matches": lm,
                     "kernel_ms": {k: round(float(v) / lsteps, 3) for k, v in zip(kernel_names(lwork), kl)},
                     "cpu_baseline": long_cpu, "work": lwork,
                     "workload": "config-4-shaped ONT reads (lognormal N50 ~10 kb, 5% subs, 1% indels) vs the "
                                 "same DB, seq mode 3"}
        clfl.close()
    if odb is not None:
        odb.close()

    if rank == 0:
        out = {
            "metric": "reads/sec classified (150bp & 10kb) vs GTDB-scale DB at 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "reads/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "config 2: 1M x 150bp paired reads vs RefSeq-viral-sized DB (~10 GB), "
                                   "format 2, DB + reads resident in HBM",
                       "read_pairs_per_gpu": n, "read_len": 150, "db_kmers": D,
                       "db_bytes": db_bytes, "query_kmers": Q, "matches": M,
                       "parallelism": f"reads sharded, DB replicated x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernel_ms": {k: round(float(v), 3) for k, v in zip(KERNELS, kern)},
            "stage_ms": {k: round(float(v), 3) for k, v in zip(["extract", "sort", "match", "assign", "total"], stage)},
            "parity_sample": parity,
            "work": work,
            "long_reads": long_line,
        }
        print(json.dumps(out), flush=True)
    clf.close()
    if world > 1:
        dist.destroy_process_group()


def run_partitioned(args, lp, hdb, batch, world, rank, local, dev):
    """Config-5 shape: the DB cut into P AA-aligned k-mer ranges, one per rank. Every
    rank matches the WHOLE batch against its range (MTB_MATCH_ONLY), the matches go all-to-all to
    the owners of their reads (RCCL), each owner sorts + scores its 1/P of the reads
    (mtb_assign_chunks), and the result records are gathered. With world == P this runs for real;
    on one GPU (world == 1) each part is timed in turn: a rank's step = its match-only pass over
    the batch + the assignment of its owned reads (their matches from all parts); the all-to-all
    is not timed there and its bytes are reported instead."""
    from metabuli_work_amd.dist import classify_partitioned, gather_records, owner_bounds

    P = args.db_parts
    s1, o1, s2, o2 = batch
    n = args.pairs
    if world > 1 and world != P:
        raise SystemExit("--db-parts must equal the number of ranks (or run on one GPU)")
    out = {"metric": "reads/sec classified (150bp & 10kb) vs GTDB-scale DB at 1/2/4/8 MI355X", "unit": "reads/s",
           "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "u64", "data": "synthetic"}
    if world > 1:
        # same batch on every rank (rank-independent seed), each holding DB part `rank`
        clf = Classifier(lp, db_host=hdb.c_struct(), device=local, db_part=(rank, P))
        sizes = [b - a for a, b in owner_bounds(n, world)]
        res = torch.empty((sizes[rank], RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)

        def step():
            _, br = classify_partitioned(clf, s1, o1, s2, o2, device_input=True, on_device=True)
            clf.copy_results(res.data_ptr(), on_device=True)
            gather_records(res, sizes)

        for _ in range(args.warmup):
            step()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        clf.close()
        out.update(value=round(n * args.steps / el, 1), ms_per_step=round(el / args.steps * 1e3, 3),
                   config={"workload": f"config-5 shape: {n} read pairs x 150 bp per step vs the bench DB "
                                       f"range-partitioned over {P} GPUs (match all-to-all + result gather)",
                           "db_kmers": hdb.n_kmers, "parallelism": f"DB range-partitioned x{P}"})
        if rank == 0:
            print(json.dumps(out), flush=True)
        dist.destroy_process_group()
        return
    # one GPU: the owners' assignment inputs = the full DB's matches of their reads
    full = Classifier(lp, db_host=hdb.c_struct(), device=local)
    full.classify_batch(s1, o1, s2, o2, device_input=True, match_only=True)
    _, Mf = full.last_counts()
    mt = torch.empty((Mf, 24), dtype=torch.uint8, device=dev)
    ct = torch.empty(n, dtype=torch.int32, device=dev)
    qt = torch.empty(n, dtype=torch.int32, device=dev)
    full.copy_matches(mt, ct, qt)
    full.close()
    cs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(ct.to(torch.int64), 0, out=cs[1:])
    bounds = owner_bounds(n, P)
    parts = []
    for p in range(P):
        clf = Classifier(lp, db_host=hdb.c_struct(), device=local, db_part=(p, P))
        lo, hi = bounds[p]
        a, b = int(cs[lo].item()), int(cs[hi].item())
        om, oc_, oq = mt[a:b].contiguous(), ct[lo:hi].contiguous(), qt[lo:hi].contiguous()
        for _ in range(args.warmup):
            clf.classify_batch(s1, o1, s2, o2, device_input=True, match_only=True)
            clf.assign_chunks(om, b - a, oc_, 1, oq, hi - lo, fetch=False)
        torch.cuda.synchronize()
        tm = ta = 0.0
        kern = np.zeros(7)
        for _ in range(args.steps):
            t0 = time.perf_counter()
            clf.classify_batch(s1, o1, s2, o2, device_input=True, match_only=True)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            kern += clf.kernel_ms()
            clf.assign_chunks(om, b - a, oc_, 1, oq, hi - lo, fetch=False)
            torch.cuda.synchronize()
            tm += t1 - t0
            ta += time.perf_counter() - t1
        _, Mp = clf.last_counts()
        clf.classify_batch(s1, o1, s2, o2, device_input=True, match_only=True)
        _, Mp = clf.last_counts()
        parts.append({"part": p, "db_kmers": clf.db_kmers, "match_only_ms": round(tm / args.steps * 1e3, 3),
                      "assign_ms": round(ta / args.steps * 1e3, 3), "matches": Mp,
                      "a2a_send_bytes": int(Mp * 24 * (P - 1) // P),
                      "kernel_ms": {k: round(float(v) / args.steps, 3)
                                    for k, v in zip(KERNELS_SORT[:5], kern[:5])}})
        clf.close()
        log(rank, f"[bench] part {p}/{P}: {parts[-1]}")
    step_ms = max(q["match_only_ms"] + q["assign_ms"] for q in parts)
    out.update(value=round(n / (step_ms * 1e-3), 1), ms_per_step=round(step_ms, 3),
               config={"workload": f"config-5 shape on ONE GPU: {n} read pairs x 150 bp vs the bench DB range-"
                                   f"partitioned into {P} parts, each part's rank step timed in turn (the "
                                   "all-to-all over xGMI is not timed: a2a_send_bytes)",
                       "db_kmers": hdb.n_kmers, "parallelism": f"DB range-partitioned x{P} (simulated)"},
               parts=parts)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
