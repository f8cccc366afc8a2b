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
import gc
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
from metabuli_work_amd.dist import gather_results  # noqa: E402
from metabuli_work_amd.gpu_synth import make_genomes_gpu, make_long_reads_gpu, make_reads_gpu  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# per-stage HBM bytes of one batch from this round's rocprofv3 FETCH_SIZE / WRITE_SIZE passes
# (tools/measure_r04.sh + tools/stage_profile.py), one file per workload
# this round's PMC passes first; a workload not re-measured this round falls back to the previous one
TRAFFIC_DIRS = [os.path.join(ROOT, "profiles", d) for d in ("r06", "r05", "r04")]
# the six timed kernels of mtb_last_kernel_ms, by join path (mtb_last_stats[10])
KERNELS_SORT = ["extract", "filter", "kmer_sort", "match_join", "match_transpose", "match_sort", "assign"]
KERNELS_PROBE = ["extract", "filter", "kmer_sort", "probe_join", "match_transpose", "match_sort", "assign"]


def kernel_names(work):
    return KERNELS_PROBE if work.get("join_path", 1) == 0 else KERNELS_SORT


class ResultGather:
    """C1 of a multi-GPU step: each batch's result records and pooled taxID:count
    lists are copied device-to-device into step buffers (the records' offsets rebased onto the step
    pool), then gathered to every rank in one go (dist.gather_results: RCCL all-gathers)."""

    def __init__(self, dev, n_reads):
        self.dev = dev
        self.pool = torch.empty((4 * n_reads + 1024, 8), dtype=torch.uint8, device=dev)
        self.used = 0

    def reset(self):
        self.used = 0

    def add(self, clf, rec):
        clf.copy_results(rec.data_ptr(), on_device=True)
        nt = clf.n_taxcnt()
        if self.used + nt > self.pool.shape[0]:  # grow (rare: > 4 entries per read on average)
            bigger = torch.empty((2 * (self.used + nt), 8), dtype=torch.uint8, device=self.dev)
            bigger[:self.used] = self.pool[:self.used]
            self.pool = bigger
        clf.copy_taxcnt(self.pool[self.used:].data_ptr(), on_device=True)
        if self.used:
            rec.view(torch.int32).view(-1, 8)[:, 4] += self.used
        self.used += nt

    def gather(self, rec):
        return gather_results(rec, self.pool[:self.used])


VARIANT_BATCH = {"syncmer": 3_333_334, "conserved": 3_333_334, "related": 2_000_000, "em": 2_000_000}


def variant_batch(args, variant):
    """Read pairs per mtb_classify_batch of a config-3 DB variant (or the --em line): --variant-batch,
    else the variant's own QuerySplit (VARIANT_BATCH: the largest that fits HBM beside its DB)."""
    return args.variant_batch or VARIANT_BATCH.get(variant, 2_000_000)


def cpu_model() -> str:
    """The host CPU's model name and the machine's logical CPUs (state nproc and the CPU
    model beside the cores the baseline used)."""
    name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    name = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return f"{name} (nproc {os.cpu_count()})"


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def alg_bytes(bases, n, Qall, Q, M, D, live=None, probe=False, mates=2, dbread=0):
    """Algorithmic bytes per launch of each timed kernel for a batch of n reads of `bases` bases in
    all (Qall = windows the scanners emitted, the reference's "Query k-mer number"; Q = kept query
    k-mers, whose AA 8-mer the DB holds; M matches; live = matches K6 reads after K5's pruning; D
    DB k-mers)."""
    read_bytes = bases + mates * 8 * (n + 1)
    live = M if live is None else live
    return {
        # fused K1 + K1F (k_extract_filter): the reads in, one membership word per emitted window
        # (the window keys never reach HBM), the present (key, slot) pairs out (+ the 8-B DB lower
        # bound for the probe join)
        "filter": read_bytes + 4 * Qall + (20 if probe else 12) * Q,
        # probe join: per query its (key, slot, lower bound), 8 DB values + taxIDs from there,
        # its staged matches (+ rank) out
        "probe_join": 20 * Q + 96 * Q + 28 * M,
        "extract": read_bytes,                               # K0 read metadata (the keys stay in the fused K1F)
        "kmer_sort": 2 * 3 * 12 * Q,                        # three passes over the (key, slot) pairs
        # queries, the DB (12-B value + taxID records) read once through the block windows, or, when
        # the DB is much larger than the query stream (D > 12 Q), each query's run: its two
        # run-index entries (4 B) and the run's first two records (24 B); the 16-B segment matches
        # written into the reads' segments (direct join)
        # the DB-sweep join (MTB_JOIN=sweep) reads the records of every tile that holds queries once,
        # coalesced (dbread of them: all D at these batch sizes)
        "match_join": 12 * Q + (12 * dbread if dbread else 28 * Q if D > 12 * Q else 12 * D) + 16 * M,
        "match_transpose": 2 * 24 * M + 4 * M + 8 * n,      # staged matches (+ rank) read, written to segments
        "match_sort": 16 * M + 24 * live + 8 * (n + 1),     # each read's segment matches read, live ones written
        "assign": 24 * live + 32 * n + 4 * n + 8 * n,       # live sorted matches read, results + lengths
    }


def load_traffic(workload, kmers, batch):
    """Per-stage HBM bytes of one batch of this workload (profiles/r05/ or r04/stage_traffic_<workload>.json,
    separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes over the same workload: tools/measure_r05.sh),
    when the profiled DB and batch shape match this run's (the synthetic DB's size varies by a few
    k-mers per build)."""
    for d in TRAFFIC_DIRS:
        path = os.path.join(d, f"stage_traffic_{workload}.json")
        try:
            with open(path) as f:
                tf = json.load(f)
        except (OSError, ValueError):
            continue
        if tf.get("batch") != batch or abs(tf.get("kmers", 0) - kmers) > 1e-3 * max(kmers, 1):
            continue
        return tf, os.path.relpath(path, ROOT)
    return None, None


def roofline_of(kern, names, alg, traffic):
    """Roofline of the dominant kernel: algorithmic bytes per launch / its event-timed duration
    (kern: per-launch ms of the timed kernels)."""
    dom = int(np.argmax(kern))
    dname = names[dom]
    achieved = alg[dname] / (kern[dom] * 1e-3) / 1e9
    tf, src = traffic
    hbm = tf["stages"][dname]["hbm_bytes"] if tf and dname in tf.get("stages", {}) else None
    out = {"bound": "hbm", "kernel": dname, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": hbm,
           "traffic_source": src if hbm is not None else None, "alg_bytes_per_launch": int(alg[dname]),
           "avg_launch_ms": round(float(kern[dom]), 3)}
    if hbm is not None:  # the HBM bytes it moves (random reads move 128-B lines) over its time
        out["traffic_gb_per_s"] = round(hbm / (kern[dom] * 1e-3) / 1e9, 1)
    return out


# the random-line ceiling (tools/rand_gather.hip, tools/calib_random_fetch.sh): independent 4-B loads at
# pseudo-random 64-B-aligned offsets of a buffer the size of the structure a kernel probes; every such
# load is one 128-B memory-side read request (TCC_EA0_RDREQ_128B = loads), so the ceiling is the HBM's
# bandwidth at 128-B lines (6.1-6.3 TB/s; a coalesced stream on the same box: 5.82 TB/s)
RANDOM_CALIBRATION = os.path.join(ROOT, "profiles", "r05", "random_fetch_calibration.json")
RANDOM_LINE_BYTES = 128
# the random kernels and the buffer their random reads land in (GB): K1F the 14.4-GB link lines (round 6;
# the nearest calibrated buffer prices it), the unstaged K4 the 144-GB DB records (and the run index)
RANDOM_KERNELS = {"filter": 14.4, "match_join": 144.0}


def random_ceilings():
    """{buffer_gb: ceiling TB/s at 128-B lines} of the calibration's plain random loads."""
    try:
        with open(RANDOM_CALIBRATION) as f:
            runs = json.load(f)["runs"]
    except (OSError, ValueError, KeyError):
        return {}
    return {r["buffer_gb"]: r["tb_per_s_at_128B"] for r in runs if r.get("kind") == "load4"}


def random_roofline(kern, names, traffic, Q=0, sweep=False):
    """The random-access kernels against the chip's measured random-line ceiling, in bytes: the
    kernel's HBM bytes per launch from the PMC passes (FETCH_SIZE doubled: a random read moves a
    128-B line; WRITE_SIZE: a scattered 16-B store or atomic is one 32-B write request) over its
    event-timed duration, against the random 128-B-line bandwidth over a buffer of the size it
    probes. Reads, writes and atomics are each counted at the bytes they move, so frac <= 1 unless
    the kernel beats the calibration itself. No PMC pass for the workload: no entry."""
    ceil = random_ceilings()
    tf, src = traffic
    if not ceil or not tf:
        return None
    out = {}
    for k, gb in RANDOM_KERNELS.items():
        if k not in names or k not in tf.get("stages", {}) or (k == "match_join" and sweep):
            continue
        st = tf["stages"][k]
        ms = float(kern[names.index(k)])
        if ms <= 0 or not st.get("hbm_bytes"):
            continue
        c_gb = min(ceil, key=lambda g: abs(g - gb))
        got = st["hbm_bytes"] / (ms * 1e-3) / 1e12
        e = {"traffic_tb_per_s": round(got, 3), "ceiling_tb_per_s_at_128B": ceil[c_gb], "ceiling_buffer_gb": c_gb,
             "frac": round(got / ceil[c_gb], 3), "hbm_bytes_per_launch": int(st["hbm_bytes"]),
             "avg_launch_ms": round(ms, 3), "traffic_source": src,
             "ceiling_source": os.path.relpath(RANDOM_CALIBRATION, ROOT)}
        if Q > 0 and st.get("fetch_bytes"):
            e["lines_fetched_per_query"] = round(st["fetch_bytes"] / RANDOM_LINE_BYTES / Q, 3)
        out[k] = e
    return out or None


class Tally:
    """Per-launch averages of a timed loop's batches: kernel and stage ms and work counts."""

    def __init__(self):
        self.kern = np.zeros(7)
        self.stage = np.zeros(5)
        self.w = {k: 0.0 for k in ("qall", "q", "m", "live", "matched", "gallop", "bases", "reads", "slots", "dbread")}
        self.launches = 0

    def add(self, clf, bases, reads):
        self.kern += clf.kernel_ms()
        self.stage += clf.stage_ms()
        qall, m = clf.last_counts()
        st = clf.stats()
        for k, v in (("qall", qall), ("q", st["query_kmers"]), ("m", m), ("live", st["live_matches"]),
                     ("matched", st["matched_queries"]), ("gallop", st["gallop_queries"]), ("bases", bases),
                     ("reads", reads), ("slots", st["slots"]), ("dbread", st["db_records_read"])):
            self.w[k] += v
        self.launches += 1

    def avg(self, k):
        return self.w[k] / max(1, self.launches)

    def kern_avg(self):
        return self.kern / max(1, self.launches)

    def stage_avg(self):
        return self.stage / max(1, self.launches)

    def rooflines(self, names, D, traffic, mates):
        kern = self.kern_avg()
        alg = alg_bytes(self.avg("bases"), self.avg("reads"), self.avg("qall"), self.avg("q"), self.avg("m"), D,
                        live=self.avg("live"), probe=names is KERNELS_PROBE, mates=mates, dbread=self.avg("dbread"))
        return (roofline_of(kern, names, alg, traffic),
                random_roofline(kern, names, traffic, Q=self.avg("q"), sweep=self.avg("dbread") > 0))


# ---------------------------------------------------------------------------------------------
def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(gpus: int, argv, port: int):
    """The command that runs this bench as `gpus` ranks on one node, one process per GPU (the
    driver's own form: torch.distributed.run, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def resolve_world(gpus, env):
    """How this process runs, from --gpus and the launcher's environment: ("launch", N) when it must
    start N ranks itself (--gpus N > 1 and no WORLD_SIZE: the parent never touches the GPU), else
    ("run", world). A WORLD_SIZE that disagrees with an explicit --gpus is an error: the line's n_gpus
    would not be the GPU count asked for."""
    ws = env.get("WORLD_SIZE")
    if gpus is not None and gpus < 1:
        raise ValueError(f"--gpus must be >= 1 (got {gpus})")
    if ws is None:
        return ("launch", gpus) if gpus is not None and gpus > 1 else ("run", 1)
    ws = int(ws)
    if gpus is not None and gpus != ws:
        raise ValueError(f"--gpus {gpus} but WORLD_SIZE={ws}: launch with --nproc-per-node {gpus}, or drop --gpus")
    return "run", ws


def launch_ranks(gpus: int, argv) -> int:
    """Start `gpus` ranks as a child torch.distributed.run (before any GPU call in this process) and
    return its exit code."""
    import subprocess
    if os.environ.get("MTB_BENCH_ONE_DEVICE") != "1":
        have = torch.cuda.device_count()  # counts devices without initialising the GPU (this image)
        if have < gpus:
            raise SystemExit(f"[bench] --gpus {gpus} but {have} GPU(s) visible")
    cmd = launcher_cmd(gpus, argv, free_port())
    print(f"[bench] launching {gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks, one process each). N > 1 without WORLD_SIZE: the bench starts the N ranks "
                         "itself through torch.distributed.run; under a launcher it must equal WORLD_SIZE "
                         "(default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=1_000_000, help="config 2: read pairs per rank per step")
    ap.add_argument("--species", type=int, default=25000)
    ap.add_argument("--mean-genome", type=int, default=75000)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="read pairs timed on the CPU oracle (0 = off)")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--long-reads", type=int, default=125_000,
                    help="config 4: ONT-style reads (N50 ~10 kb) per rank for the long-read line (1M / 8; 0 = off)")
    ap.add_argument("--long-batch", type=int, default=62_500,
                    help="long reads per mtb_classify_batch (62.5k: 2 batches per 125k-read shard; 25k: 494.6k vs 527.8k "
                         "reads/s same box, profiles/r03/long_batch_sweep.json)")
    ap.add_argument("--db-parts", type=int, default=0,
                    help="config-5 mode: the DB range-partitioned into this many parts (= the number of ranks; "
                         "on one GPU every part is timed in turn)")
    ap.add_argument("--skip-config2", action="store_true", help="config 3 only (experiments)")
    ap.add_argument("--gtdb-kmers", type=float, default=12e9,
                    help="config 3: k-mers of the GTDB-scale DB (0 = skip config 3; config 2 is then the headline)")
    ap.add_argument("--gtdb-pairs", type=int, default=10_000_000, help="config 3: read pairs per rank per step")
    ap.add_argument("--gtdb-batch", type=int, default=3_333_334,
                    help="config 3 (and config 5): read pairs per mtb_classify_batch (the QuerySplit: three per "
                         "10M-pair step, 88 GB of workspace beside the 171 GB of DB arrays since K6's scratch lives "
                         "in dead buffers; 2M: 22.99M, 3M: 23.16M, 3.33M: 24.06M, 4M: 23.72M reads/s, "
                         "profiles/r04/batch_sweep.json)")
    ap.add_argument("--gtdb-contexts", type=int, default=1,
                    help="experiments: config-3 batches spread over this many contexts on the GPU (mtb_clone), "
                         "each driven by a thread of its own (two batches in flight)")
    ap.add_argument("--variant-batch", type=int, default=0,
                    help="config-3 DB variants and --em: read pairs per mtb_classify_batch (0: per variant, "
                         "VARIANT_BATCH — the largest that fits HBM beside the DB: related 2M (100.7 GB of "
                         "workspace; 16.01M at 1M, 16.63M at 2M reads/s), syncmer and conserved 3.33M "
                         "(40.86 -> 42.02M and 22.20 -> 22.75M against 2M, same box); --em 2M)")
    ap.add_argument("--gtdb-species", type=int, default=129_671)
    ap.add_argument("--gtdb-true-species", type=int, default=1000)
    ap.add_argument("--gtdb-genome", type=int, default=3_000_000)
    ap.add_argument("--gtdb-cpu-sample", type=int, default=1_000_000, help="config 3: read pairs timed on the oracle")
    ap.add_argument("--variants", default="syncmer,related,conserved",
                    help="extra config-3 lines, comma-separated (GTDB_VARIANTS; empty = none)")
    ap.add_argument("--variant-cpu-sample", type=int, default=200_000,
                    help="read pairs of each variant line timed on the oracle (parity sample)")
    ap.add_argument("--e2e-pairs", type=int, default=10_000_000,
                    help="config 3 file -> TSV line: read pairs written as BGZF / plain FASTQ (0 = off)")
    ap.add_argument("--e2e-contexts", type=int, default=2,
                    help="contexts on the GPU for the file -> TSV lines (mtb_clone: two batches in flight)")
    ap.add_argument("--e2e-repeat", type=int, default=3,
                    help="file -> TSV runs per format (A/B: the line reports the median, and every run)")
    ap.add_argument("--e2e-gzip-pairs", type=int, default=10_000_000,
                    help="config 3 file -> TSV line: read pairs written as single-member gzip FASTQ (0 = off)")
    ap.add_argument("--em-pairs", type=int, default=10_000_000,
                    help="config 3 --em line: read pairs classified with em and reassigned (0 = off)")
    ap.add_argument("--variant-only", default="", help="experiments: run this config-3 variant line alone")
    ap.add_argument("--c5-kmers", type=float, default=35e9,
                    help="config 5: k-mers of the range-partitioned DB (> one GPU's HBM; 0 = off)")
    ap.add_argument("--c5-pairs", type=int, default=10_000_000, help="config 5: read pairs per step")
    ap.add_argument("--c5-parts", type=int, default=8,
                    help="config 5 on one GPU: DB parts, each timed in turn (with N >= 4 GPUs: one part per rank)")
    ap.add_argument("--c5-sample", type=int, default=24_000, help="config 5: read pairs of the oracle parity sample")
    ap.add_argument("--c5-only", action="store_true", help="experiments: run the config-5 line alone")
    ap.add_argument("--ab", default="", help="experiments: 'name=K=V,K=V;name2=...' same-box A/B of the headline")
    ap.add_argument("--ab-repeat", type=int, default=2, help="--ab: rounds over the specs")
    ap.add_argument("--ab-skewed", action="store_true", help="--ab on the skewed-abundance reads (--skew-sigma)")
    ap.add_argument("--skewed-pairs", type=int, default=10_000_000,
                    help="config 3: read pairs of the skewed-abundance line (log-normal genome abundance; 0 = off)")
    ap.add_argument("--skew-sigma", type=float, default=2.0,
                    help="skewed line: sigma of the log-normal per-genome abundance")
    ap.add_argument("--cold-gtdb", type=int, default=1,
                    help="config 3: open the GTDB-scale DB from host diffIdx/info/split (mtb_open_host) and time it")
    ap.add_argument("--cold-settle-s", type=float, default=8.0,
                    help="GTDB cold open: idle seconds after freeing the resident DB (the driver's wipe of freed HBM)")
    ap.add_argument("--cold-pairs", type=int, default=10_000_000,
                    help="cold one-shot line: read pairs of the file classified by a freshly opened context (0 = off)")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--detail", default=DEFAULT_DETAIL,
                    help="side file for the full result tree (per-kernel splits, work counters, config-5 parts, "
                         "e2e host stages); the stdout line keeps the headline and one-line summaries")
    args = ap.parse_args()

    how, world = resolve_world(args.gpus, os.environ)
    if how == "launch":
        sys.exit(launch_ranks(world, sys.argv[1:]))
    if args.launch_probe:  # tests: each rank reports what the launcher gave it, before any GPU call
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": world,
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}), flush=True)
        return
    if world > 1 and args.detail == DEFAULT_DETAIL:
        args.detail = DEFAULT_DETAIL.replace(".json", f"_n{world}.json")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 paths on a one-GPU box (never the measurement): MTB_BENCH_BACKEND=gloo and
    # MTB_BENCH_ONE_DEVICE=1 put every rank on cuda:0
    if os.environ.get("MTB_BENCH_ONE_DEVICE") == "1":
        local = 0
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)  # before the process group: RCCL's communicator binds this rank's GPU
    if world > 1:
        backend = os.environ.get("MTB_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, init_method="env://", device_id=dev if backend == "nccl" else None)
        if args.db_parts <= 1:
            # the scaling runs time the headline lines (config 3 short and long reads) only: the CPU
            # baseline, the config-2 line, the DB variants, the file -> TSV and --em lines are
            # single-GPU measurements (their per-rank DB rebuilds and host files would only
            # lengthen the run)
            args.cpu_sample = 0
            args.skip_config2 = True
            args.variants = ""
            args.e2e_pairs = args.e2e_gzip_pairs = args.em_pairs = args.cold_pairs = args.skewed_pairs = 0
    if args.c5_only:
        c5 = run_config5(args, world, rank, local, dev)
        if rank == 0:
            print(json.dumps(c5))
        return
    if args.ab:  # experiments: the headline DB built once, environments A/B'd on it; one JSON line
        v = run_gtdb(args, world, rank, local, dev)
        if rank == 0:
            print(json.dumps(v))
        return
    if args.variant_only:
        v = run_gtdb(args, world, rank, local, dev, variant=args.variant_only)
        if rank == 0:
            print(json.dumps(v))
        return
    c2 = run_config2(args, world, rank, local, dev) if not args.skip_config2 or args.db_parts > 1 else None
    if args.db_parts > 1:
        return
    torch.cuda.empty_cache()
    c3 = run_gtdb(args, world, rank, local, dev) if args.gtdb_kmers > 0 else None
    if c3 is not None:
        c3["variants"] = {}
        for v in [x for x in args.variants.split(",") if x]:
            torch.cuda.empty_cache()
            c3["variants"][v] = run_gtdb(args, world, rank, local, dev, variant=v)
    c5 = None
    if args.c5_kmers > 0 and (world == 1 or world >= 4):  # two GPUs cannot hold a > 288 GB DB's halves
        torch.cuda.empty_cache()
        c5 = run_config5(args, world, rank, local, dev)
    if rank == 0:
        head = c3 if c3 is not None else c2
        if head is None:
            return
        out = {
            "metric": "reads/sec classified (150bp & 10kb) vs GTDB-scale DB at 1/2/4/8 MI355X",
            "value": head["value"], "unit": "reads/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        }
        for k, v in head.items():
            if k not in ("value", "ms_per_step"):
                out[k] = v
        if c2 is not None and c2.get("cold_run"):
            out["cold_run"] = c2["cold_run"]
        if c3 is not None and c2 is not None:
            out["config2"] = {k: v for k, v in c2.items() if k not in ("long_reads", "cold_run")}
        if c3 is not None and c3.get("long_reads") is not None:
            out["long_reads"] = c3["long_reads"]
            if c2 is not None and c2.get("long_reads") is not None:
                out["config2"]["long_reads"] = c2["long_reads"]
        else:
            out["long_reads"] = c2.get("long_reads") if c2 is not None else None
        out["config5"] = c5
        print(json.dumps(compact_line(out, args.detail)), flush=True)
    if world > 1:
        dist.destroy_process_group()


DEFAULT_DETAIL = os.path.join(ROOT, "profiles", "r06", "bench_detail.json")
LINE_CAP = 8000  # the driver keeps only the tail of stdout (~15.5 KB): the one JSON line stays well under it


def count_label(x) -> str:
    """A count as the labels print it: 10000000 -> "10M", 3333334 -> "3.33M", 200000 -> "200k",
    12.0e9 -> "12.0G" (k-mers keep one decimal in G)."""
    x = float(x)
    if x >= 1e9:
        return f"{x / 1e9:.1f}G"
    if x >= 1e6:
        v = x / 1e6
        return f"{v:.0f}M" if abs(v - round(v)) < 5e-3 else f"{v:.3g}M"
    if x >= 1e3:
        v = x / 1e3
        return f"{v:.0f}k" if abs(v - round(v)) < 5e-3 else f"{v:.3g}k"
    return f"{int(x)}"


def hbm_note(nbytes) -> str:
    """Whether a DB's resident bytes fit one MI355X (288 GB of HBM)."""
    return "more than one GPU's 288 GB HBM" if nbytes > 288e9 else "fits one GPU's 288 GB HBM"


def config3_label(pairs, read_len, db_kmers, species, batch, what="config 3") -> str:
    """config.workload of a config-3 line, from the run's own parameters."""
    return (f"{what}: {count_label(pairs)} x {read_len}bp paired reads per GPU vs a GTDB-scale DB "
            f"({count_label(db_kmers)} k-mers, {species:,}-species skeleton taxonomy), format 2, DB + reads "
            f"resident in HBM, {batch}-pair batches")


def config5_label(pairs, read_len, db_kmers, parts) -> str:
    return (f"config 5: {count_label(pairs)} x {read_len}bp read pairs per step vs a {count_label(db_kmers)}-k-mer "
            f"GTDB-shaped DB ({db_kmers * 12 / 1e9:.0f} GB of records: {hbm_note(db_kmers * 12)}), range-partitioned "
            f"into {parts} AA-aligned parts")


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _roof(r):
    return _pick(r, ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "traffic_source",
                     "alg_bytes_per_launch", "avg_launch_ms", "traffic_gb_per_s"))


def _cpu(c):
    if not isinstance(c, dict):
        return c
    s = _pick(c, ("value", "unit", "cores", "cpu_model", "kind", "sample"))
    if isinstance(s.get("sample"), str) and len(s["sample"]) > 240:
        s["sample"] = s["sample"][:237] + "..."
    return s


def _line(v):
    """One-line summary of a secondary bench line (config 2, a DB variant, config 4)."""
    if not isinstance(v, dict):
        return v
    s = _pick(v, ("value", "unit", "ms_per_step", "parity_sample"))
    if "roofline" in v:
        s["roofline"] = _pick(v["roofline"], ("kernel", "frac", "achieved"))
    if "cpu_baseline" in v and isinstance(v["cpu_baseline"], dict):
        s["cpu_baseline"] = _pick(v["cpu_baseline"], ("value", "cores", "kind"))
    return s


def compact_line(out, detail_path):
    """The stdout JSON line: the headline with its roofline, CPU baseline and parity sample, the
    long-read line in full, one-line summaries of the rest. Everything else (kernel and stage splits,
    work counters, config-5 parts, e2e host stages) goes to the detail file the line names."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(out, f, indent=1)
        except OSError as e:
            log(0, f"[bench] detail file not written: {e}")
            detail_path = None
    line = _pick(out, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                       "scaling", "vs_baseline", "dtype", "data", "config", "parity_sample"))
    line["roofline"] = _roof(out.get("roofline"))
    line["cpu_baseline"] = _cpu(out.get("cpu_baseline"))
    if isinstance(out.get("random_roofline"), dict):
        line["random_roofline"] = {k: _pick(v, ("frac", "traffic_tb_per_s", "ceiling_tb_per_s_at_128B",
                                                "lines_fetched_per_query"))
                                   for k, v in out["random_roofline"].items()}
    if isinstance(out.get("pipeline_roofline"), dict):
        line["pipeline_roofline"] = _pick(out["pipeline_roofline"], ("achieved", "frac", "alg_bytes"))
    if "kernel_ms" in out:
        line["kernel_ms"] = out["kernel_ms"]
    lr = out.get("long_reads")
    if isinstance(lr, dict):
        line["long_reads"] = _pick(lr, ("value", "unit", "ms_per_step", "parity_sample", "workload"))
        line["long_reads"]["roofline"] = _roof(lr.get("roofline"))
        line["long_reads"]["cpu_baseline"] = _cpu(lr.get("cpu_baseline"))
        if "parity_sample" not in lr and isinstance(lr.get("cpu_baseline"), dict):
            line["long_reads"]["parity_sample"] = lr["cpu_baseline"].get("parity_sample")
    if isinstance(out.get("config2"), dict):
        line["config2"] = _line(out["config2"])
    if out.get("variants"):
        line["variants"] = {k: _line(v) for k, v in out["variants"].items()}
    e2e = out.get("end_to_end")
    if isinstance(e2e, dict):
        line["end_to_end"] = {k: (_pick(v, ("reads_per_s", "tsv_matches_oracle", "first_run_reads_per_s"))
                                  if isinstance(v, dict) else v) for k, v in e2e.items() if k != "note"}
    if isinstance(out.get("cold_run"), dict):
        line["cold_run"] = _pick(out["cold_run"], ("open_s", "first_run_reads_per_s", "steady_reads_per_s",
                                                   "tsv_matches_oracle"))
    if isinstance(out.get("em"), dict):
        line["em"] = _pick(out["em"], ("classify_with_mappings_reads_per_s", "em_s", "reassigned"))
    c5 = out.get("config5")
    if isinstance(c5, dict):
        line["config5"] = _pick(c5, ("value", "unit", "ms_per_step", "parity_sample", "scaling"))
        cfg = c5.get("config", {})
        if "read_pairs" in cfg and "db_kmers" in cfg and "parts" in cfg:
            line["config5"]["workload"] = (f"{count_label(cfg['read_pairs'])} pairs vs a {count_label(cfg['db_kmers'])}"
                                           f"-k-mer DB in {cfg['parts']} AA-aligned parts (detail: config5)")
    line["detail"] = os.path.relpath(detail_path, ROOT) if detail_path else None
    # never overflow the driver's capture: drop the summaries, least important first
    for k in ("end_to_end", "em", "random_roofline", "pipeline_roofline", "kernel_ms", "variants", "config5",
              "config2", "cold_run"):
        if len(json.dumps(line)) <= LINE_CAP:
            break
        line.pop(k, None)
    if isinstance(line.get("config"), dict) and len(json.dumps(line)) > LINE_CAP:
        line["config"] = _pick(line["config"], ("workload", "read_pairs_per_gpu", "batch_pairs", "db_kmers",
                                                "parallelism"))
    return line


def run_config2(args, world, rank, local, dev):
    """Config 2 (1M x 150 bp pairs vs the RefSeq-viral-sized DB) + the long-read line; returns the
    line's fields (rank 0)."""
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
    res_dev = torch.empty((n, RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    c1 = ResultGather(dev, n) if world > 1 else None

    def step():
        clf.classify_batch(s1, o1, s2, o2, device_input=True, fetch=False)
        if world > 1:  # C1: result records + taxID:count lists to every rank (rank 0 writes the TSV)
            c1.reset()
            c1.add(clf, res_dev)
            c1.gather(res_dev)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    tally = Tally()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
        tally.add(clf, 2 * 150 * n, n)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern, stage = tally.kern_avg(), tally.stage_avg()
    Qref, M = clf.last_counts()  # Qref: the reference's "Query k-mer number" (all non-blank windows)
    work = clf.stats()
    Q = work["query_kmers"]      # the query k-mers K4 consumes (AA 8-mer in the DB)
    work["run_index_fallback_rate"] = round(tally.avg("gallop") / max(1, tally.avg("q")), 6)
    KERNELS = kernel_names(work)
    ms_per_step = elapsed / max(1, args.steps) * 1e3
    value = world * n * args.steps / elapsed

    D = hdb.n_kmers
    roofline, rand_roof = tally.rooflines(KERNELS, D, load_traffic("config2", D, n), mates=2)

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
        cpu = {"value": round(S / cpu_t, 1), "unit": "reads/s", "cores": cores, "cpu_model": cpu_model(), "kind": "port",
               "sample": f"first {S} read pairs of the rank-0 batch, same DB; oracle/ (OpenMP C++ restatement "
                         f"of the reference path), {cpu_t:.1f}s wall",
               "stage_s": [round(x, 3) for x in stage_s]}
        gb = clf.classify_batch(h1, ho, h2, ho.copy())
        parity = bool(np.array_equal(gb.results["classification"], ores["classification"])
                      and np.array_equal(gb.results["score"].view(np.uint32), ores["score"].view(np.uint32))
                      and np.array_equal(gb.taxcnt, otc))

    # ---- long reads (seq mode 3, same DB): reads/s of the same pipeline on ~10 kb reads ----
    long_line = None
    clf.close()
    cold = None
    if rank == 0 and world == 1 and args.cold_pairs > 0:
        cold = run_cold(args, hdb, par, lp, s1, s2, n, (ores, otc) if parity is not None else None)
    if args.long_reads > 0:
        long_line = run_long_reads(args, lambda lpl: Classifier(lpl, db_host=hdb.c_struct(), device=local), ls1, lo1,
                                   long_n50, world, rank, dev, odb, cores, "the config-2 DB", hdb.n_kmers,
                                   "config2_long")
    if odb is not None:
        odb.close()

    out = {
        "value": round(value, 1), "ms_per_step": round(ms_per_step, 3),
        "config": {"workload": f"config 2: {count_label(n)} x 150bp paired reads vs a RefSeq-viral-sized DB "
                               f"({count_label(D)} k-mers, {db_bytes / 1e9:.1f} GB of diffIdx + info), format 2, "
                               "DB + reads resident in HBM",
                   "read_pairs_per_gpu": n, "read_len": 150, "db_kmers": D,
                   "db_bytes": db_bytes, "query_kmers": Q, "matches": M,
                   "parallelism": f"reads sharded, DB replicated x{world}"},
        "roofline": roofline,
        "random_roofline": rand_roof,
        "cpu_baseline": cpu,
        "kernel_ms": {k: round(float(v), 3) for k, v in zip(KERNELS, kern)},
        "stage_ms": {k: round(float(v), 3) for k, v in zip(["extract", "sort", "match", "assign", "total"], stage)},
        "parity_sample": parity,
        "work": work,
        "long_reads": long_line,
        "cold_run": cold,
    }
    return out


def run_cold(args, hdb, par, lp, s1, s2, n, check=None):
    """A one-shot classify as a user runs it: the config-2 DB written as the
    reference's files (diffIdx, info, split, taxID_list, taxonomy/*.dmp; /dev/shm, so the page cache
    and not a disk is read), mtb_open from that directory into a fresh context, then the context's
    first mtb_start_classify over a 10M-pair plain FASTQ (the config-2 batch's pairs, repeated) and a
    second, steady one. open_s has its phases (mtb_open_phases); first_run is what one CLI call pays
    after the open; steady is a warm context's rate."""
    import shutil
    import tempfile

    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    d = tempfile.mkdtemp(prefix="mtb_cold_", dir=base)
    L = 150
    try:
        tw = time.perf_counter()
        hdb.write(os.path.join(d, "db"), par)
        reps = max(1, args.cold_pairs // n)
        off = np.arange(n + 1, dtype=np.uint64) * L
        for mate, (sq, pre) in enumerate(((s1, "a"), (s2, "b"))):
            body = synth.fastq_bytes(sq[:n * L].cpu().numpy(), off, prefix=pre)
            with open(os.path.join(d, f"q{mate + 1}.fq"), "wb") as f:
                for _ in range(reps):
                    f.write(body)
            del body
        prep = time.perf_counter() - tw
        q1, q2 = os.path.join(d, "q1.fq"), os.path.join(d, "q2.fq")
        lpc = LocalParameters(seqMode=2, filenames=[q1, q2, os.path.join(d, "db")])
        t0 = time.perf_counter()
        clf = Classifier(lpc, db_dir=os.path.join(d, "db"))
        open_s = time.perf_counter() - t0
        phases = clf.open_phases()
        tsv = os.path.join(d, "out.tsv")
        runs = []
        try:
            for _ in range(3):
                t1 = time.perf_counter()
                got = clf.startClassify(tsv, report_tsv=os.path.join(d, "report.tsv"))
                runs.append((time.perf_counter() - t1, dict(clf.last_run)))
                if len(runs) == 1 and check is not None:
                    ok = tsv_matches_oracle(tsv, *check)
        finally:
            clf.close()
        steady = sorted(w for w, _ in runs[1:])[len(runs[1:]) // 2]
        out = {"open_s": round(open_s, 3), "open_phases_s": phases,
               "first_run_reads_per_s": round(got / runs[0][0], 1), "steady_reads_per_s": round(got / steady, 1),
               "one_shot_reads_per_s": round(got / (open_s + runs[0][0]), 1),
               "read_pairs": got, "db_kmers": hdb.n_kmers, "db_file_bytes": hdb.nbytes,
               "first_run": {k: round(v, 3) for k, v in runs[0][1].items() if k.endswith("_s")},
               "first_run_batches": int(runs[0][1]["batches"]), "file_prep_s": round(prep, 1),
               "tsv_matches_oracle": ok if check is not None else None,
               "what": "config-2 DB as files in /dev/shm, mtb_open into a fresh context, its first startClassify "
                       f"over {got} read pairs (plain FASTQ), then two more (steady: the faster)"}
        log(0, f"[bench] cold run: open {open_s:.2f}s {phases}, first {out['first_run_reads_per_s'] / 1e6:.2f}M, "
               f"steady {out['steady_reads_per_s'] / 1e6:.2f}M pairs/s")
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def run_ab(args, rdb, lp, s1, s2, o1, spans, L, local, rank):
    """--ab 'name=K=V,K=V;name2=...': a same-box A/B on the headline workload with the GTDB-scale DB
    built once — per spec a fresh context opened under its environment (knobs read at open, or per
    batch), one warm-up step and --steps timed steps, specs interleaved --ab-repeat times. Returns
    {name: [ {value, kernel_ms}, ... ]}."""
    specs = []
    for part in args.ab.split(";"):
        name, _, envs = part.partition("=")
        kv = dict(e.split("=", 1) for e in envs.split(",") if e)
        specs.append((name, kv))
    N = spans[-1][1]
    offs = {b - a: o1[:b - a + 1].contiguous() for a, b in spans}
    out = {name: [] for name, _ in specs}
    for rep in range(args.ab_repeat):
        for name, kv in specs:
            old = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            try:
                clf = Classifier(lp, db_resident=rdb, device=local)
                tally = Tally()

                def step(timed):
                    for a, b in spans:
                        ob = offs[b - a]
                        clf.classify_batch(s1[a * L:b * L], ob, s2[a * L:b * L], ob, device_input=True, fetch=False)
                        if timed:
                            tally.add(clf, 2 * L * (b - a), b - a)
                step(False)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    step(True)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                names = kernel_names(clf.stats())
                r = {"value": round(N * args.steps / el, 1),
                     "kernel_ms": {k: round(float(v), 3) for k, v in zip(names, tally.kern_avg())}}
                clf.close()
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            out[name].append(r)
            log(rank, f"[bench ab] {name} #{rep}: {r['value'] / 1e6:.3f}M reads/s {r['kernel_ms']}")
    return {"ab": out, "value": max(max(x["value"] for x in v) for v in out.values())}


def run_skewed(args, clf, reads, s1, s2, o1, B, L, world, rank, lp, odb):
    """Config 3 with a skewed-abundance sample: the same GTDB-scale DB and
    context, reads drawn with a log-normal per-genome abundance (sigma --skew-sigma) so a few species
    get tens of x coverage per batch, as real samples do. Timed as the headline (its QuerySplits); then
    one untimed batch of each sample with MTB_DUP_STATS=1 counts the query k-mers whose AA rank /
    whole value repeats another's in its K4 block — the work the reference's identical-query and
    same-AA reuse saves (KmerMatcher.cpp:277-353) — and a 200k-pair oracle parity sample."""
    k1, ko1, k2, ko2 = reads
    N = ko1.numel() - 1
    spans = [(a, min(N, a + B)) for a in range(0, N, B)]
    offs = {b - a: ko1[:b - a + 1].contiguous() for a, b in spans}
    tally = Tally()

    def step(timed):
        for a, b in spans:
            ob = offs[b - a]
            clf.classify_batch(k1[a * L:b * L], ob, k2[a * L:b * L], ob, device_input=True, fetch=False)
            if timed:
                tally.add(clf, 2 * L * (b - a), b - a)

    step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=k1.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    value = world * N * args.steps / el
    dup = {}
    os.environ["MTB_DUP_STATS"] = "1"
    try:
        for name, (q1, q2, qo) in (("skewed", (k1, k2, ko1)), ("uniform", (s1, s2, o1))):
            b = min(B, qo.numel() - 1)
            ob = qo[:b + 1].contiguous()
            clf.classify_batch(q1[:b * L], ob, q2[:b * L], ob, device_input=True, fetch=False)
            st = clf.stats()
            dup[name] = {"query_kmers": st["query_kmers"], "dup_aa_queries": st["dup_aa_queries"],
                         "dup_key_queries": st["dup_key_queries"],
                         "dup_aa_rate": round(st["dup_aa_queries"] / max(1, st["query_kmers"]), 5),
                         "dup_key_rate": round(st["dup_key_queries"] / max(1, st["query_kmers"]), 5)}
    finally:
        os.environ.pop("MTB_DUP_STATS", None)
    parity = None
    if odb is not None and args.variant_cpu_sample > 0:
        from tests import oracle_ctypes as oc  # checker only
        S = min(args.variant_cpu_sample, N)
        h1, h2 = k1[:S * L].cpu().numpy(), k2[:S * L].cpu().numpy()
        ho = ko1[:S + 1].cpu().numpy().astype(np.uint64)
        sample = synth.Reads(h1, ho, h2, ho.copy(), np.zeros(S, np.int32))
        ores, otc = oc.classify(odb, lp.to_c(), sample)
        gb = clf.classify_batch(h1, ho, h2, ho.copy())
        parity = bool(np.array_equal(gb.results["classification"], ores["classification"])
                      and np.array_equal(gb.results["score"].view(np.uint32), ores["score"].view(np.uint32))
                      and np.array_equal(gb.taxcnt, otc))
    kern = tally.kern_avg()
    names = kernel_names(clf.stats())
    out = {"value": round(value, 1), "unit": "reads/s", "ms_per_step": round(el / args.steps * 1e3, 3),
           "read_pairs_per_gpu": N, "batch_pairs": B, "abundance_sigma": args.skew_sigma,
           "kernel_ms": {k: round(float(v), 3) for k, v in zip(names, kern)},
           "query_kmers_per_batch": int(tally.avg("q")), "matches_per_batch": int(tally.avg("m")),
           "duplicates": dup, "parity_sample": parity,
           "what": "the headline DB and context, reads drawn with log-normal per-genome abundance "
                   f"(sigma {args.skew_sigma}): a few species at tens of x coverage per batch"}
    log(rank, f"[bench] config 3 skewed: {value / 1e6:.2f}M reads/s, duplicates {dup}, parity {parity}")
    return out


def run_cold_gtdb(args, host, odb, lp, local, reads, ores, otc):
    """The GTDB-scale DB opened as the reference opens its DB on every run (KmerMatcher.cpp:127-138,
    212-265; Classifier.cpp:6-32): from diffIdx / info / split — here the host copy the oracle holds
    (encode_into_oracle: the resident DB re-encoded, 12G k-mers, ~108 GB) — through mtb_open_host
    into a fresh context, after the resident DB was freed. open_phases_s has mtb_open_phases: the
    uploads (read_s), the chunked K3 decode into records (decode_s), the AA directory, the probe
    lines, the run index and the taxonomy. A parity check follows: the oracle sample's reads through
    the new context against the oracle's results."""
    diff, info, split = odb.arrays
    h = host.c_struct()
    h.diff_idx, h.n_diff_idx = diff.ctypes.data, len(diff)
    h.info, h.n_info = info.ctypes.data, len(info)
    h.split, h.n_split = split.ctypes.data, len(split) // 3
    t0 = time.perf_counter()
    clf = Classifier(lp, db_host=h, device=local)
    open_s = time.perf_counter() - t0
    try:
        phases = clf.open_phases()
        S = min(len(reads.off1) - 1, 200_000)
        gb = clf.classify_batch(reads.seq1, reads.off1[:S + 1], reads.seq2, reads.off2[:S + 1])
        ok = bool(np.array_equal(gb.results["classification"], ores["classification"][:S])
                  and np.array_equal(gb.results["score"].view(np.uint32), ores["score"].view(np.uint32)[:S]))
        n = clf.db_kmers
    finally:
        clf.close()
    out = {"open_s": round(open_s, 3), "open_phases_s": phases, "db_kmers": n,
           "db_bytes": int(diff.nbytes + info.nbytes), "diff_idx_words": len(diff),
           "parity_sample_pairs": S, "parity_sample": ok,
           "what": f"the config-3 DB ({n} k-mers) as diffIdx/info/split in host memory, mtb_open_host into a "
                   "fresh context (the resident copy freed first): what a CLI run pays before its first batch"}
    log(0, f"[bench] GTDB-scale cold open: {open_s:.2f}s {phases}, parity {ok}")
    return out


def run_long_reads(args, open_clf, ls1, lo1, n50, world, rank, dev, odb, cores, db_name, db_kmers, workload):
    """Config 4 (BASELINE.json configs[3]: 1M ONT-style reads sharded across 8 GPUs): the rank's
    shard of args.long_reads reads (125k = 1M / 8 by default) in seq mode 3, classified in batches
    of at most args.long_batch reads (the reference's RAM-bounded QuerySplits, Classifier.cpp:81-133)
    against the replicated DB, plus, with N > 1, the C1 all-gather of the shard's result records and
    taxID:count lists (ResultGather) — weak scaling at 125k reads per GPU. On rank 0 with an oracle
    DB, the oracle on the first reads of the shard (~10 s of 16-core work) with the GPU's results for
    the same reads compared to it."""
    lpl = LocalParameters(seqMode=3, kmerFormat=2, skipRedundancy=1)
    clfl = open_clf(lpl)
    nl_all = lo1.numel() - 1
    lb = max(1, args.long_batch)
    cuts = []  # cut before the timed region
    for a in range(0, nl_all, lb):
        b = min(nl_all, a + lb)
        base = int(lo1[a].item())
        cuts.append((a, b, ls1[base:int(lo1[b].item())], (lo1[a:b + 1] - base).contiguous(),
                     int(lo1[b].item()) - base))
    res_all = torch.empty((nl_all, RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    c1 = ResultGather(dev, nl_all) if world > 1 else None

    def long_step(tally=None):
        if c1 is not None:
            c1.reset()
        for a, b, cs, co, nb in cuts:
            clfl.classify_batch(cs, co, device_input=True, fetch=False)
            if tally is not None:
                tally.add(clfl, nb, b - a)
            if c1 is not None:
                c1.add(clfl, res_all[a:b])
        if c1 is not None:
            c1.gather(res_all)

    for _ in range(max(1, args.warmup)):
        long_step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    lsteps = max(1, min(args.steps, 3))
    tally = Tally()
    tl0 = time.perf_counter()
    for _ in range(lsteps):
        long_step(tally)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    tl = time.perf_counter() - tl0
    if world > 1:
        t = torch.tensor([tl], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tl = float(t.item())
    lwork = clfl.stats()
    names = kernel_names(lwork)
    roofline, rand_roof = tally.rooflines(names, db_kmers, load_traffic(workload, db_kmers, lb), mates=1)
    long_cpu = None
    if rank == 0 and args.cpu_sample > 0 and odb is not None:
        from tests import oracle_ctypes as oc  # checker / baseline only

        LS = max(1, min(nl_all, args.cpu_sample // 50))
        lo_h = lo1[:LS + 1].cpu().numpy().astype(np.uint64)
        ls_h = ls1[:int(lo_h[-1])].cpu().numpy()
        lreads = synth.Reads(ls_h, lo_h, None, None, np.zeros(LS, np.int32))
        lopar = lpl.to_c()
        lopar.threads = cores
        tc0 = time.perf_counter()
        lres, ltc = oc.classify(odb, lopar, lreads)
        lcpu_t = time.perf_counter() - tc0
        gl = clfl.classify_batch(ls_h, lo_h)
        long_cpu = {"value": round(LS / lcpu_t, 1), "unit": "reads/s", "cores": cores, "cpu_model": cpu_model(), "kind": "port",
                    "sample": f"first {LS} long reads of the rank-0 shard, same DB, {lcpu_t:.1f}s wall",
                    "parity_sample": bool(np.array_equal(gl.results["classification"], lres["classification"])
                                          and np.array_equal(gl.results["score"].view(np.uint32),
                                                             lres["score"].view(np.uint32))
                                          and np.array_equal(gl.taxcnt, ltc))}
    clfl.close()
    kl = tally.kern_avg()
    return {"value": round(world * nl_all * lsteps / tl, 1), "unit": "reads/s",
            "ms_per_step": round(tl / lsteps * 1e3, 3), "steps": lsteps,
            "reads_per_gpu": nl_all, "bases_per_gpu": int(lo1[-1].item()), "n50": n50,
            "batch_reads": lb, "batches_per_step": len(cuts),
            "query_kmers_per_batch": int(tally.avg("q")), "matches_per_batch": int(tally.avg("m")),
            "kernel_ms": {k: round(float(v), 3) for k, v in zip(names, kl)},  # per batch (launch)
            "roofline": roofline, "random_roofline": rand_roof,
            "cpu_baseline": long_cpu, "work": lwork,
            "parallelism": f"reads sharded ({nl_all} per GPU), DB replicated x{world}, result all-gather",
            "workload": f"config 4: ONT-style reads (lognormal N50 ~10 kb, 5% subs, 1% indels), {nl_all} per GPU "
                        f"(1M / 8 at 8 GPUs), vs {db_name}, seq mode 3"}


GTDB_VARIANTS = {  # extra config-3 lines: the DB format users run, GTDB-like sharing
    "syncmer": {"syncmer": 1, "smer_len": 5, "per_genus": 1, "species_div": 0.0,
                "what": "Syncmer 1 DB (closed syncmers, s = 5: GTDB R226's DB format), reads classified with syncmer"},
    "related": {"syncmer": 0, "smer_len": 5, "per_genus": 20, "species_div": 0.05,
                "what": "true-signal species in genera of 20 sister species, each 5% diverged from its genus "
                        "genome (~10% between sisters, GTDB's 5-15% within a genus): DB AA runs carry several "
                        "species"},
    "conserved": {"syncmer": 0, "smer_len": 5, "per_genus": 1, "species_div": 0.0, "conserved": 1_000_000,
                  "what": "heavy-tailed sharing: 1M AA 8-mers of the true-signal genomes are also held by 100 to "
                          "10,000 filler species each (log-uniform), as conserved genes' AA 8-mers are across "
                          "GTDB: DB runs of 10^2-10^4 k-mers, queries selecting among thousands of candidates"},
}


def run_gtdb(args, world, rank, local, dev, variant=None):
    """Config 3, the configuration BASELINE.json's metric names: 10M x 150 bp pairs per
    GPU vs a GTDB-scale DB (~12G k-mers over a 129,671-species skeleton taxonomy: 1000 species x 2
    strains x ~3 Mbp of true-signal genomes through the GPU builder, the rest random valid metamers),
    built in place in HBM (gtdb_synth.build_gtdb_scale) and used there (mtb_open_resident). One step
    = the rank's 10M pairs as 1M-pair QuerySplits (Classifier.cpp:81-133), plus, with N > 1, the
    all-gather of the per-read result records."""
    from metabuli_work_amd.gtdb_synth import build_gtdb_scale, encode_into_oracle, run_length_histogram

    t0 = time.time()
    N, B = args.gtdb_pairs, min(variant_batch(args, variant) if variant else args.gtdb_batch, args.gtdb_pairs)
    got = {}

    def grab(seq, off):  # reads sampled from the true-signal genomes before they are freed
        got["reads"] = make_reads_gpu(seq, off, N, args.seed * 1000 + 31 + 17 * rank, dev,
                                      abundance_sigma=args.skew_sigma if args.ab and args.ab_skewed else 0.0)
        if args.skewed_pairs > 0 and not variant:  # a skewed-abundance sample of the same genomes
            got["skewed"] = make_reads_gpu(seq, off, min(N, args.skewed_pairs), args.seed * 1000 + 41 + 17 * rank, dev,
                                           abundance_sigma=args.skew_sigma)
        if args.long_reads > 0 and not variant:
            got["long"] = make_long_reads_gpu(seq, off, args.long_reads, args.seed * 1000 + 37 + 17 * rank, dev)

    vr = GTDB_VARIANTS[variant] if variant else {"syncmer": 0, "smer_len": 5, "per_genus": 1, "species_div": 0.0}
    tag = f"config 3 [{variant}]" if variant else "config 3"
    rdb = build_gtdb_scale(dev, n_true_species=args.gtdb_true_species, genome_len=args.gtdb_genome,
                           total_species=args.gtdb_species, target_kmers=int(args.gtdb_kmers), seed=args.seed + 1,
                           before_free=grab, log=lambda m: log(rank, f"[bench] {m} ({time.time() - t0:.1f}s)"),
                           syncmer=vr["syncmer"], smer_len=vr["smer_len"], per_genus=vr["per_genus"],
                           species_div=vr["species_div"], conserved=vr.get("conserved", 0))
    s1, o1, s2, o2 = got.pop("reads")
    lp = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1, syncmer=vr["syncmer"], smerLen=vr["smer_len"])
    clf = Classifier(lp, db_resident=rdb, device=local)
    db_n, db_n_true = rdb.n, rdb.n_true  # (the resident DB may be freed before the line is built)
    log(rank, f"[bench] GTDB-scale context open ({time.time() - t0:.1f}s)")
    L = 150
    spans = [(a, min(N, a + B)) for a in range(0, N, B)]
    offs = {}
    for a, b in spans:
        if b - a not in offs:
            offs[b - a] = o1[:b - a + 1].contiguous()
    res_all = torch.empty((N, RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    c1 = ResultGather(dev, N) if world > 1 else None
    tally = Tally()

    if args.ab and not variant:  # experiments: same-box A/B of environments on this DB, then stop
        clf.close()
        return run_ab(args, rdb, lp, s1, s2, o1, spans, L, local, rank)
    peers = [clf.clone() for _ in range(args.gtdb_contexts - 1)] if not variant and world == 1 else []

    def step(timed):
        if world > 1:
            c1.reset()
        if peers:  # experiments: batch k on context k mod K, one host thread per context
            import threading
            ctxs = [clf] + peers

            def run(ci):
                for a, b in spans[ci::len(ctxs)]:
                    ob = offs[b - a]
                    ctxs[ci].classify_batch(s1[a * L:b * L], ob, s2[a * L:b * L], ob, device_input=True, fetch=False)
                    if timed and ci == 0:
                        tally.add(clf, 2 * L * (b - a), b - a)
            th = [threading.Thread(target=run, args=(ci,)) for ci in range(len(ctxs))]
            for t in th:
                t.start()
            for t in th:
                t.join()
            return
        for a, b in spans:
            ob = offs[b - a]
            clf.classify_batch(s1[a * L:b * L], ob, s2[a * L:b * L], ob, device_input=True, fetch=False)
            if timed:
                tally.add(clf, 2 * L * (b - a), b - a)
            if world > 1:
                c1.add(clf, res_all[a:b])
        if world > 1:
            c1.gather(res_all)

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern, stage = tally.kern_avg(), tally.stage_avg()
    Qb, Mb = tally.avg("q"), tally.avg("m")  # per 1M-pair batch
    work = clf.stats()
    work["workspace_bytes"] = clf.workspace_bytes  # the context's batch workspace after the timed batches
    work["join_env"] = os.environ.get("MTB_JOIN", "") + ("/nofilter" if os.environ.get("MTB_FILTER") == "0" else "")
    # run-index fallback rate: query k-mers whose DB run the join found by a gallop (all timed batches)
    work["run_index_fallback_rate"] = round(tally.avg("gallop") / max(1, Qb), 6)
    names = kernel_names(work)
    roofline, rand_roof = tally.rooflines(names, rdb.n, load_traffic(variant or "gtdb", rdb.n, B), mates=2)
    value = world * N * args.steps / elapsed
    log(rank, f"[bench] {tag}: {value / 1e6:.2f}M reads/s, {elapsed / args.steps * 1e3:.1f} ms/step, "
              f"kernels {dict(zip(names, np.round(kern, 2)))}")
    # whole pipeline against HBM: reads + query k-mers written and read (2 x 16 B) +
    # the DB bytes the join asks for (28 B per query: two run-index entries, two records) + matches
    # written and read (2 x 24 B) + 16 B per read, over the batch's device time (all stages)
    pipe_bytes = 2 * L * B + 32 * Qb + 28 * Qb + 48 * Mb + 16 * B
    pipe = {"achieved": round(pipe_bytes / (stage[4] * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(pipe_bytes / (stage[4] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_batch": int(pipe_bytes),
            "device_ms_per_batch": round(float(stage[4]), 3)}

    cpu = parity = odb = None
    cores = 1
    cpu_sample = args.variant_cpu_sample if variant else args.gtdb_cpu_sample
    if rank == 0 and args.cpu_sample > 0 and cpu_sample > 0:
        from tests import oracle_ctypes as oc  # checker / baseline only

        S = min(cpu_sample, N)
        h1 = s1[:S * L].cpu().numpy()
        h2 = s2[:S * L].cpu().numpy()
        ho = o1[:S + 1].cpu().numpy().astype(np.uint64)
        reads = synth.Reads(h1, ho, h2, ho.copy(), np.zeros(S, np.int32))
        cores = len(os.sched_getaffinity(0))
        cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
        oc.lib().orc_set_threads(cores)
        opar = lp.to_c()
        opar.threads = cores
        te = time.perf_counter()
        if variant:
            # parity only: the oracle on the sub-DB of the sample's AA runs (gtdb_synth.SubDb; a query
            # k-mer matches only DB k-mers of its own AA 8-mer), no CPU baseline (the headline line has it)
            from metabuli_work_amd.gtdb_synth import SubDb
            ext, _, _ = oc.extract(opar, reads)
            sub = SubDb.of_kmers(rdb.host, ext, dev)
            sub.collect(rdb)
            sdb, sub_n = sub.oracle_db(oc.OracleDb)
            ores, otc = oc.classify(sdb, opar, reads)
            sdb.close()
            log(rank, f"[bench] {tag} oracle on the sample's {sub_n}-k-mer sub-DB ({time.perf_counter() - te:.1f}s)")
        else:
            odb = encode_into_oracle(rdb, oc.OracleDb)
            log(rank, f"[bench] oracle DB encoded on the host ({time.perf_counter() - te:.1f}s)")
            stage_s = np.zeros(4)
            tc0 = time.perf_counter()
            ores, otc = oc.classify(odb, opar, reads, stage_s=stage_s)
            cpu_t = time.perf_counter() - tc0
            cpu = {"value": round(S / cpu_t, 1), "unit": "reads/s", "cores": cores, "cpu_model": cpu_model(), "kind": "port",
                   "sample": f"first {S} read pairs of the rank-0 batch, same GTDB-scale DB re-encoded as diffIdx/"
                             f"info/split; oracle/ (OpenMP C++ restatement of the reference path), {cpu_t:.1f}s wall",
                   "stage_s": [round(x, 3) for x in stage_s]}
        gb = clf.classify_batch(h1, ho, h2, ho.copy())
        parity = bool(np.array_equal(gb.results["classification"], ores["classification"])
                      and np.array_equal(gb.results["score"].view(np.uint32), ores["score"].view(np.uint32))
                      and np.array_equal(gb.taxcnt, otc))
        log(rank, f"[bench] {tag} CPU oracle: {cpu['value'] if cpu else '-'} reads/s, parity {parity}")
    skewed = None
    if "skewed" in got:
        skewed = run_skewed(args, clf, got.pop("skewed"), s1, s2, o1, B, L, world, rank, lp,
                            odb if rank == 0 else None)
    e2e = None
    for c in peers:
        c.close()
    if rank == 0 and not variant and (args.e2e_pairs > 0 or args.e2e_gzip_pairs > 0):
        # the file pipeline is another workload for this context: its 3.33M-pair workspace goes back
        # first (mtb_release_workspace, untimed), as a server switching workloads would, instead of
        # inside the pipeline's first run
        clf.release_workspace()
        e2e = run_e2e(args, clf, s1, s2, L, N, (ores, otc) if cpu is not None else None)
    clf.close()
    em_line = None
    if rank == 0 and not variant and args.em_pairs > 0:
        em_line = run_em(args, rdb, lp, s1, s2, o1, L, min(N, args.em_pairs), min(B, variant_batch(args, "em")), local)
    long_line = None
    if "long" in got and not variant:
        ls1, lo1, n50 = got.pop("long")
        long_line = run_long_reads(args, lambda lpl: Classifier(lpl, db_resident=rdb, device=local), ls1, lo1, n50,
                                   world, rank, dev, odb, cores, "the GTDB-scale DB", rdb.n, "long")
        log(rank, f"[bench] config 3 long reads: {long_line['value']} reads/s")
    cold_gtdb = None
    if odb is not None and args.cold_gtdb:
        # the resident DB goes first: the open builds its own records, probe lines and run index
        host = rdb.host
        clf = peers = None  # closed contexts still hold the resident records (Classifier._resident)
        del rdb
        gc.collect()
        torch.cuda.empty_cache()
        # let the driver finish wiping the ~170 GB just freed (untimed): freed HBM is cleared in the
        # background at ~33 GB/s and an allocation that needs it waits for that (tools/alloc_probe.hip:
        # 144 GB allocated 4.3 s after a free, 0.000 s fresh or after 6 s idle); a fresh process
        # opening its DB has nothing being wiped
        torch.cuda.synchronize()
        time.sleep(args.cold_settle_s)
        cold_gtdb = run_cold_gtdb(args, host, odb, lp, local, reads, ores, otc)
        rdb = None
    if odb is not None:
        odb.close()
    out = {
        "value": round(value, 1), "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "config": {"workload": config3_label(N, L, db_n, args.gtdb_species, B, tag),
                   "read_pairs_per_gpu": N, "batch_pairs": B, "read_len": L, "db_kmers": db_n,
                   "db_true_signal_kmers": db_n_true, "db_resident_bytes": db_n * 12,
                   "query_kmers_per_batch": int(Qb), "matches_per_batch": int(Mb),
                   "parallelism": f"reads sharded, DB replicated x{world}"},
        "roofline": roofline,
        "random_roofline": rand_roof,
        "cpu_baseline": cpu,
        "kernel_ms": {k: round(float(v), 3) for k, v in zip(names, kern)},
        "stage_ms": {k: round(float(v), 3) for k, v in zip(["extract", "sort", "match", "assign", "total"], stage)},
        "parity_sample": parity,
        "work": work,
        "long_reads": long_line,
        "end_to_end": e2e,
        "em": em_line,
        "pipeline_roofline": pipe,
        "cold_run_gtdb": cold_gtdb,
        "skewed": skewed,
    }
    if variant:
        out = {"variant": variant, "what": vr["what"], "value": out["value"], "unit": "reads/s",
               "ms_per_step": out["ms_per_step"], "config": out["config"], "roofline": roofline,
               "pipeline_roofline": pipe, "random_roofline": rand_roof, "cpu_baseline": cpu, "parity_sample": parity,
               "kernel_ms": out["kernel_ms"], "work": work}
        if rank == 0 and variant == "conserved":  # the heavy tail: DB AA runs by length
            out["db_run_lengths"] = run_length_histogram(rdb)
    del rdb
    torch.cuda.empty_cache()
    return out


def run_em(args, rdb, lp, s1, s2, o1, L, N, B, local):
    """--em at config 3: the reads classified with em = 1 in B-pair batches, their
    mappings collected (Reporter::writeMappings), then mtb_em timed: the EM iterations and the
    reassignment on the device over all N reads' mappings (Classifier::em + reclassify)."""
    import dataclasses
    lpe = dataclasses.replace(lp, em=1)
    clf = Classifier(lpe, db_resident=rdb, device=local)
    maps = []
    t_map = 0.0
    ob = o1[:B + 1].contiguous()
    b0 = min(N, B)  # warm-up batch: the new context's workspace grows to size outside the timing
    clf.classify_batch(s1[:b0 * L], o1[:b0 + 1].contiguous(), s2[:b0 * L], o1[:b0 + 1].contiguous(),
                       device_input=True, fetch=False)
    clf.em_mappings(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in range(0, N, B):
        b = min(N, a + B)
        obb = ob if b - a == B else o1[:b - a + 1].contiguous()
        clf.classify_batch(s1[a * L:b * L], obb, s2[a * L:b * L], obb, device_input=True, fetch=False)
        tm = time.perf_counter()
        maps.append(clf.em_mappings(a))
        t_map += time.perf_counter() - tm
    torch.cuda.synchronize()
    t_cls = time.perf_counter() - t0
    maps = np.concatenate(maps)
    clf.em(maps[:1], N)  # species k-mer counts (a pass over the DB, once per context) outside the timing
    t1 = time.perf_counter()
    reads, sp, st = clf.em(maps, N)
    t_em = time.perf_counter() - t1
    clf.close()
    out = {"reads": int(N), "mappings": int(len(maps)), "top_species": int(st["n_species"]),
           "iterations": int(st["iterations"]), "query_count": int(st["query_count"]),
           "em_s": round(t_em, 3), "classify_with_mappings_reads_per_s": round(N / t_cls, 1),
           "mapping_fetch_s": round(t_map, 3),
           "reassigned": int((reads["mapped"] == 1).sum()),
           "note": "mtb_em wall time (host setup + device iterations + reassignment) over all mappings; "
                   "classification with em = 1 timed per batch with the mapping copy"}
    log(0, f"[bench] em: {out}")
    return out


def tsv_matches_oracle(tsv, ores, otc):
    """The first len(ores) lines of a classification TSV against the oracle's results for the same
    reads, field by field (Reporter::writeReadClassification, Reporter.cpp:38-83: classified flag,
    taxID, query length, score as %g, taxID:count list)."""
    n = len(ores)
    with open(tsv) as f:
        f.readline()
        for i in range(n):
            fld = f.readline().rstrip("\n").split("\t")
            o = ores[i]
            cl = bool(o["is_classified"])
            if fld[0] != ("1" if cl else "0") or int(fld[2]) != (int(o["classification"]) if cl else 0):
                return False
            if int(fld[3]) != int(o["query_length"]) or fld[4] != "%g" % float(o["score"]):
                return False
            if cl:
                a = int(o["taxcnt_offset"])
                want = "".join(f"{int(t)}:{int(c)} " for t, c in otc[a:a + int(o["taxcnt_len"])])
                if fld[6] != want:
                    return False
    return True


def run_e2e(args, clf, s1, s2, L, N, check=None):
    """File -> TSV (SURVEY §8(d) "end-to-end reads/s including host parse and write"): the rank's
    first read pairs written as FASTQ mate files (BGZF, plain, single-member gzip), then
    Classifier.startClassify = the native pipeline (mtb_start_classify: readers/parsers, pinned
    batches uploaded on a copy stream, mtb_classify_batch, TSV writer + report) timed wall-clock.
    Files live in /dev/shm (page cache speed, no disk in the measurement). With check = (ores, otc),
    the oracle's results for the first read pairs, the TSV's first lines are compared with them."""
    import shutil
    import tempfile

    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    d = tempfile.mkdtemp(prefix="mtb_e2e_", dir=base)
    out = {}
    peers = [clf.clone() for _ in range(max(1, args.e2e_contexts) - 1)]  # the same DB, own workspaces
    warm = bool(peers)  # the first run grows the peers' workspaces: untimed (a server keeps its contexts warm)
    try:
        n_max = min(N, max(args.e2e_pairs, args.e2e_gzip_pairs))
        h1 = s1[:n_max * L].cpu().numpy()
        h2 = s2[:n_max * L].cpu().numpy()
        for mode, n in (("bgzf", args.e2e_pairs), ("plain", args.e2e_pairs), ("gzip", args.e2e_gzip_pairs)):
            n = min(n, n_max)
            if n <= 0:
                continue
            off = np.arange(n + 1, dtype=np.uint64) * L
            p1, p2 = os.path.join(d, f"q1.{mode}"), os.path.join(d, f"q2.{mode}")
            tw = time.perf_counter()
            synth.write_compressed(p1, synth.fastq_bytes(h1[:n * L], off, prefix="a"), mode)
            synth.write_compressed(p2, synth.fastq_bytes(h2[:n * L], off, prefix="b"), mode)
            prep = time.perf_counter() - tw
            size = os.path.getsize(p1) + os.path.getsize(p2)
            clf.par = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1, filenames=[p1, p2, d])
            tsv, rep = os.path.join(d, "out.tsv"), os.path.join(d, "report.tsv")
            runs = []
            for _ in range(max(1, args.e2e_repeat) + int(warm)):
                t0 = time.perf_counter()
                got = clf.startClassify(tsv, report_tsv=rep, peers=peers)
                runs.append((time.perf_counter() - t0, clf.last_run))
            cold = None
            if warm:  # the first run of the process: pinned slots and the peers' workspaces grown in it
                cold = round(got / runs[0][0], 1)
                runs, warm = runs[1:], False
            runs_rate = [round(got / w, 1) for w, _ in runs]
            wall, lr = sorted(runs, key=lambda x: x[0])[len(runs) // 2]  # the median run
            with open(tsv, "rb") as f:
                lines = sum(buf.count(b"\n") for buf in iter(lambda: f.read(1 << 24), b""))
            out[mode] = {"reads_per_s": round(got / wall, 1), "read_pairs": got, "wall_s": round(wall, 3),
                         "native_wall_s": round(lr["wall_s"], 3), "runs_reads_per_s": runs_rate,
                         "input_bytes": size, "batches": int(lr["batches"]), "gpu_s": round(lr["gpu_s"], 3),
                         "input_wait_s": round(lr["input_wait_s"], 3), "write_s": round(lr["write_s"], 3),
                         "host_stages_s": {k: round(lr[k], 3) for k in ("source_s", "scan_s", "parse_s", "fill_s",
                                                                        "first_batch_s")},
                         "tsv_lines_ok": lines == got + 1, "file_prep_s": round(prep, 1)}
            if cold is not None:
                out[mode]["first_run_reads_per_s"] = cold
                out[mode]["first_run_note"] = (
                    "the process's first startClassify after the headline (whose context gave its workspace back "
                    "before, untimed: mtb_release_workspace): both contexts grow their workspaces and the pinned "
                    "slots and parse buffers are allocated; later runs reuse all of it. A fresh context's one-shot "
                    "run: cold_run")
            if check is not None:  # the file's first reads are the oracle sample's
                out[mode]["tsv_oracle_lines"] = len(check[0])
                out[mode]["tsv_matches_oracle"] = tsv_matches_oracle(tsv, *check)
            log(0, f"[bench] end to end ({mode}): {got / wall / 1e6:.2f}M read pairs/s, {out[mode]}")
            for p in (p1, p2, tsv, rep):
                os.remove(p)
    finally:
        shutil.rmtree(d, ignore_errors=True)
        for c in peers:
            c.close()
    out["contexts"] = 1 + len(peers)
    out["note"] = ("file -> TSV wall clock of mtb_start_classify_multi on the GPU box's host (16 threads), mate "
                   f"files in /dev/shm, DB resident in HBM, {1 + len(peers)} context(s) on the GPU sharing it "
                   "(mtb_clone: two batches in flight); headline value is the device-resident rate")
    return out


XGMI_LINK_GBS = 153.0  # per xGMI link and direction (the prompt's MI355X figure: 7 links per GPU)


def run_config5(args, world, rank, local, dev):
    """Config 5 (BASELINE.json configs[4]): 10M x 150 bp pairs vs a DB larger than one GPU's HBM —
    35G k-mers of the GTDB-shaped synthetic DB (420 GB of 12-B records) — range-partitioned into P
    AA-aligned parts (the per-thread split seek of KmerMatcher.cpp:180-192,255-271
    generalised to GPUs). Each part is built in place in HBM (gtdb_synth.GtdbRecipe: whole chunks of
    the AA-rank space, plus the guard k-mer) and opened alone (mtb_open_resident, db_part). Per
    1M-pair batch every part matches the whole batch (MTB_MATCH_ONLY), the per-read match segments go
    all-to-all to the owners of the reads (1/P of the batch each), which sort and score them
    (mtb_assign_chunks); the owners' result records are gathered at the end of the step (C1).

    N >= 4 GPUs: one part per rank, for real (RCCL all-to-all and all-gather over xGMI), P = N.
    One GPU: P parts built and timed in turn, a rank's step = its part's match-only passes over the
    10 batches + its owned reads' assignment; the matches are kept (HBM, or host memory when they do
    not fit) between the two phases; the all-to-all is not measurable on one GPU: its bytes are
    reported and its time estimated at one xGMI link per peer (XGMI_LINK_GBS) and added.
    Parity: the oracle on the sub-DB of the sample reads' AA runs (gtdb_synth.SubDb: the runs are
    collected from each part while it is resident) against the owners' results for those reads."""
    from metabuli_work_amd.dist import classify_partitioned, owner_bounds
    from metabuli_work_amd.gtdb_synth import GtdbRecipe, SubDb

    t0 = time.time()
    P = world if world > 1 else args.c5_parts
    N, B, L = args.c5_pairs, min(args.gtdb_batch, args.c5_pairs), 150
    got = {}

    def grab(seq, off):  # the same batch on every rank (rank-independent seed), as the path needs
        got["reads"] = make_reads_gpu(seq, off, N, args.seed * 1000 + 53, dev)

    rc = GtdbRecipe(dev, n_true_species=args.gtdb_true_species, genome_len=args.gtdb_genome,
                    total_species=args.gtdb_species, target_kmers=int(args.c5_kmers), seed=args.seed + 2,
                    n_chunks=32 * P, before_free=grab, log=lambda m: log(rank, f"[bench] c5 {m} ({time.time() - t0:.1f}s)"))
    s1, o1, s2, o2 = got.pop("reads")
    parts = rc.part_chunks(P)
    sizes = rc.chunk_sizes()
    part_kmers = [sum(sizes[a:b]) for a, b in parts]
    D = sum(sizes)
    lp = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1)
    spans = [(a, min(N, a + B)) for a in range(0, N, B)]
    offs = {}
    for a, b in spans:
        if b - a not in offs:
            offs[b - a] = o1[:b - a + 1].contiguous()
    # parity sample: the first S/P reads of every owner's range of batch 0
    obs = [owner_bounds(b - a, P) for a, b in spans]  # each batch's owner ranges (the last batch may be shorter)
    own0 = obs[0]
    per_owner = max(1, min(args.c5_sample // P, min(hi - lo for lo, hi in own0)))
    samp = np.concatenate([np.arange(lo, lo + per_owner) for lo, _ in own0])
    sub = None
    if rank == 0 and args.c5_sample > 0:
        from tests import oracle_ctypes as oc  # checker only
        idx = torch.from_numpy(samp).to(dev)
        pos = (idx[:, None] * L + torch.arange(L, device=dev)[None, :]).reshape(-1)
        h1, h2 = s1[pos].cpu().numpy(), s2[pos].cpu().numpy()
        ho = (np.arange(len(samp) + 1, dtype=np.uint64) * L)
        sample = synth.Reads(h1, ho, h2, ho.copy(), np.zeros(len(samp), np.int32))
        ext, _, _ = oc.extract(lp.to_c(), sample)
        sub = SubDb.of_kmers(rc.host, ext, dev)
        del ext
    common = {"workload": config5_label(N, 150, D, P),
              "read_pairs": N, "batch_pairs": B, "db_kmers": D, "db_resident_bytes": D * 12, "parts": P,
              "part_kmers": part_kmers}

    if world > 1:  # ---- one part per rank, for real ----
        c0, c1 = parts[rank]
        part = rc.build(c0, c1, guard=True)
        rc.free_true()
        clf = Classifier(lp, db_resident=part, device=local, db_part=(rank, P))
        own = np.cumsum([0] + [o[rank][1] - o[rank][0] for o in obs])  # the last span may be shorter
        res = torch.empty((int(own[-1]), RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        c1g = ResultGather(dev, int(own[-1]))

        def step():
            c1g.reset()
            for k, (a, b) in enumerate(spans):
                o = offs[b - a]
                classify_partitioned(clf, s1[a * L:b * L], o, s2[a * L:b * L], o, device_input=True, on_device=True)
                c1g.add(clf, res[int(own[k]):int(own[k + 1])])
            c1g.gather(res)

        for _ in range(max(1, args.warmup)):
            step()
        dist.barrier()
        torch.cuda.synchronize()
        steps = max(1, min(args.steps, 3))
        ts = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([time.perf_counter() - ts], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        clf.close()
        del part
        torch.cuda.empty_cache()
        return {"value": round(N * steps / el, 1), "unit": "reads/s", "ms_per_step": round(el / steps * 1e3, 3),
                "steps": steps, "config": dict(common, parallelism=f"DB range-partitioned x{P} (one part per GPU), "
                                                                     "match all-to-all + result all-gather over RCCL"),
                "scaling": "strong"}

    # ---- one GPU: every part in turn ----
    match_ms = np.zeros((P, len(spans)))
    kern = np.zeros((P, 7))
    build_s, store, qlens, part_stats = [], [], [], []
    store_host = False
    keep_clf = None
    for p, (c0, c1) in enumerate(parts):
        tb = time.perf_counter()
        part = rc.build(c0, c1, guard=True)
        clf = Classifier(lp, db_resident=part, device=local, db_part=(p, P))
        torch.cuda.synchronize()
        build_s.append(round(time.perf_counter() - tb, 2))
        b0 = spans[0][1] - spans[0][0]
        clf.classify_batch(s1[:b0 * L], offs[b0], s2[:b0 * L], offs[b0], device_input=True,
                           match_only=True)  # warm-up: the workspace grows outside the timing
        row, mt_tot = [], 0
        for k, (a, b) in enumerate(spans):
            o = offs[b - a]
            torch.cuda.synchronize()
            tm = time.perf_counter()
            clf.classify_batch(s1[a * L:b * L], o, s2[a * L:b * L], o, device_input=True, match_only=True)
            _, m = clf.last_counts()
            mt = torch.empty((m, 24), dtype=torch.uint8, device=dev)  # classify_partitioned's copy
            ct = torch.empty(b - a, dtype=torch.int32, device=dev)
            qt = torch.empty(b - a, dtype=torch.int32, device=dev)
            clf.copy_matches(mt, ct, qt)
            torch.cuda.synchronize()
            match_ms[p, k] = (time.perf_counter() - tm) * 1e3
            kern[p] += clf.kernel_ms()
            mt_tot += m
            if p == 0 and k == 0:  # all parts' matches of all batches: in HBM if they fit
                free, _ = torch.cuda.mem_get_info(dev)
                store_host = m * 24 * P * len(spans) * 1.3 > free - 60e9
            if store_host:
                mt = mt.cpu()
            row.append((mt, ct))
            if p == 0:
                qlens.append(qt)
        store.append(row)
        part_stats.append({"part": p, "chunks": [c0, c1], "db_kmers": part.n, "matches": int(mt_tot),
                           "build_open_s": build_s[-1], "match_only_ms_per_batch": round(float(match_ms[p].mean()), 3),
                           "kernel_ms_per_batch": {k: round(float(v) / len(spans), 3)
                                                   for k, v in zip(KERNELS_SORT[:5], kern[p][:5])}})
        if sub is not None:
            sub.collect(part, *part.rank_range, db_end=(p == P - 1))
        log(rank, f"[bench] c5 part {p}/{P}: {part_stats[-1]} ({time.time() - t0:.1f}s)")
        if p < P - 1:
            clf.close()
            del part
            torch.cuda.empty_cache()
        else:
            keep_clf, keep_part = clf, part  # the owners' K5 + K6 run in this context
    rc.free_true()
    assign_ms = np.zeros((P, len(spans)))
    a2a_ms = np.zeros((P, len(spans)))
    a2a_bytes = np.zeros(P)
    csum = {}
    for p in range(P):
        for k in range(len(spans)):
            c = store[p][k][1].to(torch.int64)
            cs = torch.zeros(c.numel() + 1, dtype=torch.int64, device=dev)
            torch.cumsum(c, 0, out=cs[1:])
            csum[p, k] = cs[[lo for lo, _ in obs[k]] + [obs[k][-1][1]]].cpu().tolist()

    def recv(r, k):
        lo, hi = obs[k][r]
        ms = [store[p][k][0][csum[p, k][r]:csum[p, k][r + 1]] for p in range(P)]
        m = torch.cat([x.to(dev, non_blocking=True) for x in ms])
        cnt = torch.cat([store[p][k][1][lo:hi] for p in range(P)])
        return m, cnt, qlens[k][lo:hi].contiguous()

    for r in range(P):
        for k in range(len(spans)):
            # the all-to-all (not measurable on one GPU): rank r sends each peer q the matches of q's
            # reads against part r and receives q's part's matches of its own reads; one link per peer
            ob = obs[k]
            sends = [(csum[r, k][q + 1] - csum[r, k][q]) * 24 + 4 * (ob[q][1] - ob[q][0]) for q in range(P) if q != r]
            recvs = [(csum[q, k][r + 1] - csum[q, k][r]) * 24 + 4 * (ob[r][1] - ob[r][0]) for q in range(P) if q != r]
            a2a_bytes[r] += sum(sends)
            a2a_ms[r, k] = max(max(sends), max(recvs)) / (XGMI_LINK_GBS * 1e9) * 1e3
            m, cnt, ql = recv(r, k)
            torch.cuda.synchronize()
            ta = time.perf_counter()
            keep_clf.assign_chunks(m, m.shape[0], cnt, P, ql, ob[r][1] - ob[r][0], fetch=False)
            torch.cuda.synchronize()
            assign_ms[r, k] = (time.perf_counter() - ta) * 1e3
            del m, cnt, ql
    rank_ms = match_ms.sum(1) + a2a_ms.sum(1) + assign_ms.sum(1)  # rank r holds part r and owns reads r
    step_ms = float(rank_ms.max())
    parity = None
    if sub is not None:
        from tests import oracle_ctypes as oc  # checker only
        rs, ts = [], []
        for r in range(P):
            m, cnt, ql = recv(r, 0)
            br = keep_clf.assign_chunks(m, m.shape[0], cnt, P, ql, obs[0][r][1] - obs[0][r][0])
            res_r = br.results[:per_owner].copy()
            tc_r = [br.taxcnt[int(x["taxcnt_offset"]):int(x["taxcnt_offset"]) + int(x["taxcnt_len"])] for x in res_r]
            rs.append(res_r)
            ts.extend(tc_r)
        gres = np.concatenate(rs)
        sdb, sub_n = sub.oracle_db(oc.OracleDb)
        opar = lp.to_c()
        opar.threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "64")))
        ores, otc = oc.classify(sdb, opar, sample)
        sdb.close()
        otl = [otc[int(x["taxcnt_offset"]):int(x["taxcnt_offset"]) + int(x["taxcnt_len"])] for x in ores]
        parity = bool(np.array_equal(gres["classification"], ores["classification"])
                      and np.array_equal(gres["score"].view(np.uint32), ores["score"].view(np.uint32))
                      and all(np.array_equal(a, b) for a, b in zip(ts, otl)))
        log(rank, f"[bench] c5 parity ({len(samp)} pairs, sub-DB {sub_n} k-mers): {parity}")
    keep_clf.close()
    del keep_part, store
    torch.cuda.empty_cache()
    out = {"value": round(N / (step_ms * 1e-3), 1), "unit": "reads/s", "ms_per_step": round(step_ms, 3),
           "config": dict(common, parallelism=f"DB range-partitioned x{P}, simulated on one GPU: each part built "
                                              "and timed in turn"),
           "rank_step_ms": {"match_only": [round(float(x), 2) for x in match_ms.sum(1)],
                            "all_to_all_estimate": [round(float(x), 2) for x in a2a_ms.sum(1)],
                            "assign": [round(float(x), 2) for x in assign_ms.sum(1)]},
           "a2a_send_bytes_per_step": [int(x) for x in a2a_bytes],
           "a2a_note": f"not measurable on one GPU: time estimated as the largest per-peer volume over one "
                       f"{XGMI_LINK_GBS:.0f} GB/s xGMI link, added to each rank's step",
           "matches_kept_in": "host memory" if store_host else "HBM",
           "parts": part_stats,
           "parity_sample": parity,
           "parity_note": f"{len(samp)} read pairs ({per_owner} per owner of batch 0): the owners' results vs the "
                          "oracle on the sub-DB of the sample's AA runs collected from every part (gtdb_synth.SubDb)",
           "cpu_baseline": None, "scaling": "strong"}
    log(rank, f"[bench] config 5: {out['value'] / 1e6:.2f}M reads/s, step {step_ms:.1f} ms ({time.time() - t0:.1f}s)")
    return out


def run_partitioned(args, lp, hdb, batch, world, rank, local, dev):
    """Config-5 shape: the DB cut into P AA-aligned k-mer ranges, one per rank. Every
    rank matches the WHOLE batch against its range (MTB_MATCH_ONLY), the matches go all-to-all to
    the owners of their reads (RCCL), each owner sorts + scores its 1/P of the reads
    (mtb_assign_chunks), and the result records are gathered. With world == P this runs for real;
    on one GPU (world == 1) each part is timed in turn: a rank's step = its match-only pass over
    the batch + the assignment of its owned reads (their matches from all parts); the all-to-all
    is not timed there and its bytes are reported instead."""
    from metabuli_work_amd.dist import classify_partitioned, owner_bounds

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
        c1 = ResultGather(dev, sizes[rank])

        def step():
            classify_partitioned(clf, s1, o1, s2, o2, device_input=True, on_device=True)
            c1.reset()
            c1.add(clf, res)
            c1.gather(res)  # C1: records + taxID:count lists

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
