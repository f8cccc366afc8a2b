"""Range-partitioned DB across GPUs.

CPU: the partition bounds are AA-aligned split entries (IndexCreator.cpp:843-851) and balanced;
the match all-to-all (gloo, world 2) delivers every read's segments to its owner in the layout
mtb_assign_chunks takes. GPU: contexts holding DB parts 0..P-1 produce, together, exactly the
full DB's matches, and scoring the exchanged chunks gives the oracle's results bit for bit; the
same through two gloo ranks sharing cuda:0 (dist.classify_partitioned).
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from metabuli_work_amd._abi import MATCH_DTYPE, info_seq
from metabuli_work_amd._lib import MtbError, lib
from metabuli_work_amd.dist import MATCH_BYTES, exchange_matches, owner_bounds
from tests import oracle_ctypes as oc

MTB_ERR_DB = -4


def _db_values(db_dir):
    """All DB k-mer values, diffIdx decoded as getNextTargetKmer does (KmerMatcher.h:282-297)."""
    diff = np.fromfile(os.path.join(db_dir, "diffIdx"), np.uint16).astype(np.uint64)
    term = np.nonzero(diff & np.uint64(0x8000))[0]
    starts = np.concatenate([[0], term[:-1] + 1])
    kidx = np.repeat(np.arange(len(term)), term - starts + 1)
    shift = (term[kidx] - np.arange(len(diff))) * 15
    return np.cumsum(np.add.reduceat((diff & np.uint64(0x7FFF)) << shift.astype(np.uint64), starts), dtype=np.uint64)


def _bounds(split, D, parts):
    start = np.zeros(parts + 1, np.uint64)
    entry = np.zeros(parts, np.uint64)
    rc = lib().mtb_partition_bounds(split.ctypes.data, len(split) // 3, D, parts, start.ctypes.data,
                                    entry.ctypes.data)
    return rc, start, entry


@pytest.mark.parametrize("db_name", ["fmt2", "fmt1", "fmt2_syncmer"])
@pytest.mark.parametrize("parts", [2, 3, 8])
def test_partition_bounds_aa_aligned(make_db, db_name, parts):
    db_dir, _, _ = make_db(db_name)
    vals = _db_values(db_dir)
    split = np.fromfile(os.path.join(db_dir, "split"), np.uint64)
    rc, start, entry = _bounds(split, len(vals), parts)
    assert rc == 0
    assert start[0] == 0 and start[-1] == len(vals)
    assert np.all(np.diff(start.astype(np.int64)) > 0)
    aa = vals >> np.uint64(24)
    for p in range(1, parts):
        s = int(start[p])
        assert aa[s - 1] != aa[s], "a boundary splits an AA run"
        e = split[3 * int(entry[p]):3 * int(entry[p]) + 3]
        assert e[0] == vals[s] and e[2] == s + 1  # the split entry names the part's first k-mer
    sizes = np.diff(start.astype(np.int64))
    assert sizes.max() < 1.5 * len(vals) / parts + 1000


def test_partition_bounds_too_many_parts(make_db):
    db_dir, _, _ = make_db("fmt2")
    vals = _db_values(db_dir)
    split = np.fromfile(os.path.join(db_dir, "split"), np.uint64)[:3 * 4].copy()  # 3 usable entries
    rc, _, _ = _bounds(split, len(vals), 8)
    assert rc == MTB_ERR_DB
    assert b"too few" in lib().mtb_last_error()
    rc, start, _ = _bounds(split, len(vals), 1)
    assert rc == 0 and list(start) == [0, len(vals)]


# ---- the match all-to-all on CPU (gloo, world 2) ---------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _synthetic_segments(rank, n, seed):
    """Per-read match counts and records tagged (source rank, read, k) in the qinfo/target fields."""
    rng = np.random.default_rng(seed + rank)
    counts = rng.integers(0, 6, size=n).astype(np.int32)
    counts[rng.random(n) < 0.2] = 0
    m = np.zeros(int(counts.sum()), MATCH_DTYPE)
    read = np.repeat(np.arange(n), counts)
    k = np.arange(len(m)) - np.repeat(np.cumsum(counts) - counts, counts)
    m["qinfo"] = (read + 1).astype(np.uint64) << np.uint64(32)
    m["target_id"] = rank
    m["species_id"] = k
    return counts, m


def _a2a_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    counts, m = _synthetic_segments(rank, n, 7)
    t = torch.from_numpy(m.view(np.uint8).reshape(-1, MATCH_BYTES).copy())
    rm, rc = exchange_matches(t, torch.from_numpy(counts), owner_bounds(n, world))
    q.put((rank, rm.numpy().copy(), rc.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 257), (8, 257), (8, 5)])
def test_exchange_matches_gloo(world, n):
    """(8, 5): three owners hold no reads — their receive layout is empty, every rank still sends
    them a zero-length chunk."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (m, c)) for r, m, c in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    src = [_synthetic_segments(r, n, 7) for r in range(world)]
    for owner, (lo, hi) in enumerate(owner_bounds(n, world)):
        rm, rc = got[owner]
        rm = rm.view(MATCH_DTYPE).reshape(-1)
        rc = rc.reshape(world, hi - lo)
        expect = []
        for r in range(world):
            counts, m = src[r]
            assert np.array_equal(rc[r], counts[lo:hi])  # chunk r = rank r's counts of the owned reads
            sel = (info_seq(m["qinfo"]) > lo) & (info_seq(m["qinfo"]) <= hi)
            expect.append(m[sel])
        assert np.array_equal(rm, np.concatenate(expect))


# ---- GPU: parts 0..P-1 against the full DB and the oracle ------------------------------------
def _reads(gen, seed, n=1200):
    from metabuli_work_amd import synth
    return synth.make_reads(gen, n, paired=True, seed=seed, short_frac=0.03, rate_n=0.002)


@pytest.mark.gpu
@pytest.mark.parametrize("db_name", ["fmt2", "fmt2_syncmer", "fmt1"])
@pytest.mark.parametrize("parts", [2, 3])
def test_partitioned_db_parity(make_db, db_name, parts):
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from tests.test_gpu_parity import _match_sorted, compare_results

    db_dir, _, gen = make_db(db_name)
    par = LocalParameters(seqMode=2).load_db_parameters(db_dir)
    reads = _reads(gen, 41)
    n = len(reads.off1) - 1
    odb = oc.OracleDb(db_dir)
    opar = par.to_c()
    okmers, ql1, ql2 = oc.extract(opar, reads)
    omatches = oc.match(odb, opar, okmers)
    ores, otc = oc.assign(odb, opar, omatches, ql1, ql2)
    odb.close()
    chunks, counts, qlen = [], [], None
    clfs = [Classifier(par, db_dir=db_dir, db_part=(p, parts)) for p in range(parts)]
    try:
        assert sum(c.db_kmers for c in clfs) == len(_db_values(db_dir)) + parts - 1  # + one guard k-mer per cut
        for c in clfs:
            c.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, match_only=True)
            _, M = c.last_counts()
            m = np.zeros(M, MATCH_DTYPE)
            cnt = np.zeros(n, np.uint32)
            ql = np.zeros(n, np.uint32)
            c.copy_matches(m, cnt, ql)
            assert np.array_equal(np.repeat(np.arange(1, n + 1), cnt), info_seq(m["qinfo"]))  # grouped by read
            chunks.append(m)
            counts.append(cnt)
            qlen = ql
        allm = np.concatenate(chunks)
        assert len(allm) == len(omatches)
        assert np.array_equal(_match_sorted(allm), _match_sorted(omatches))
        assert np.array_equal(qlen, ql1 + ql2)
        br = clfs[-1].assign_chunks(allm, len(allm), np.concatenate(counts), parts, qlen, n)
        compare_results(br.results, br.taxcnt, ores, otc)
        with pytest.raises(MtbError, match="pruned"):  # K5 dropped dead matches: no full match array
            clfs[-1].matches()
        br = clfs[-1].assign_chunks(allm, len(allm), np.concatenate(counts), parts, qlen, n, keep_stages=True)
        compare_results(br.results, br.taxcnt, ores, otc)
        assert np.array_equal(clfs[-1].matches(), omatches)  # every match, compareMatches order
        # a match-only batch keeps no results of its own; an ordinary batch afterwards still works
        br2 = clfs[0].classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        assert br2.matches == len(chunks[0])
    finally:
        for c in clfs:
            c.close()


def _part_worker(rank, world, port, db_dir, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from metabuli_work_amd import synth
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from metabuli_work_amd.dist import classify_partitioned, gather_results

    taxo = synth.make_taxonomy(14, 2, seed=11)
    gen = synth.make_genomes(taxo, genome_len=24000, seed=12)
    reads = _reads(gen, seed)
    par = LocalParameters(seqMode=2).load_db_parameters(db_dir)
    with Classifier(par, db_dir=db_dir, device=0, db_part=(rank, world)) as clf:
        (lo, hi), br = classify_partitioned(clf, reads.seq1, reads.off1, reads.seq2, reads.off2, on_device=False)
        rec = torch.from_numpy(br.results.view(np.uint8).reshape(-1, 32).copy())
        tc = torch.from_numpy(br.taxcnt.view(np.uint8).reshape(-1, 8).copy())
        allres, alltc = gather_results(rec, tc)  # C1 with the taxID:count lists, offsets rebased
    q.put((rank, allres.numpy().copy(), alltc.numpy().copy()))
    dist.destroy_process_group()


def _replica_worker(rank, world, port, db_dir, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from metabuli_work_amd import synth
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from metabuli_work_amd.dist import classify_sharded

    taxo = synth.make_taxonomy(14, 2, seed=11)
    gen = synth.make_genomes(taxo, genome_len=24000, seed=12)
    reads = _reads(gen, seed)
    par = LocalParameters(seqMode=2).load_db_parameters(db_dir)
    with Classifier(par, db_dir=db_dir, device=0) as clf:  # a full DB replica per rank
        res, tc = classify_sharded(clf, reads.seq1, reads.off1, reads.seq2, reads.off2)
    q.put((rank, res.view(np.uint8).copy(), tc.view(np.uint8).copy()))
    dist.destroy_process_group()


def _long_reads(gen, seed):
    from metabuli_work_amd import synth
    return synth.make_long_reads(gen, 90, n50=3000, min_len=400, seed=seed)


def _long_replica_worker(rank, world, port, db_dir, seed, q):
    """Config 4's shape: seq-mode-3 reads, DB replicated, batches dealt round-robin over the ranks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from metabuli_work_amd import synth
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from metabuli_work_amd.dist import classify_batches_sharded, shard_reads

    taxo = synth.make_taxonomy(14, 2, seed=11)
    gen = synth.make_genomes(taxo, genome_len=24000, seed=12)
    reads = _long_reads(gen, seed)
    par = LocalParameters(seqMode=3).load_db_parameters(db_dir)
    cuts = [(a, min(reads.n, a + 13)) for a in range(0, reads.n, 13)]  # 7 batches: ranks take 4 and 3
    batches = [(lambda a=a, b=b: shard_reads(reads.seq1, reads.off1, a, b) + (None, None)) for a, b in cuts]
    with Classifier(par, db_dir=db_dir, device=0) as clf:
        res, tc = classify_batches_sharded(clf, batches)
    q.put((rank, res.view(np.uint8).copy(), tc.view(np.uint8).copy()))
    dist.destroy_process_group()


def _run_two_ranks(target, db_dir, seed):
    from metabuli_work_amd._abi import RESULT_DTYPE, TAXCNT_DTYPE

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, db_dir, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {r: (a, b) for r, a, b in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got[0][0].view(RESULT_DTYPE).reshape(-1), got[0][1].view(TAXCNT_DTYPE).reshape(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["partitioned", "replicated", "replicated_long"])
def test_classify_two_ranks(make_db, mode):
    """Two processes on cuda:0 over gloo. partitioned: each holds half of the DB, matches go
    all-to-all to the read owners (config 5); replicated: each holds the whole DB and classifies
    half of the reads (configs 2-3); replicated_long: seq-mode-3 long reads in batches dealt
    round-robin over the ranks (config 4, classify_batches_sharded). Either way rank 0's gathered results AND taxID:count lists
    are the oracle's, element by element — what one GPU writes to the TSV."""
    from tests.test_gpu_parity import compare_results
    from metabuli_work_amd.classifier import LocalParameters

    db_dir, taxo, gen = make_db("fmt2")  # DB_CONFIGS["fmt2"]: 14 species x 2 strains, 24 kb, seeds 11/12
    long = mode == "replicated_long"
    reads = _long_reads(gen, 43) if long else _reads(gen, 43)
    par_c = LocalParameters(seqMode=3 if long else 2).load_db_parameters(db_dir).to_c()
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par_c, reads)
    odb.close()
    target = {"partitioned": _part_worker, "replicated": _replica_worker, "replicated_long": _long_replica_worker}[mode]
    res, tc = _run_two_ranks(target, db_dir, 43)
    assert len(res) == len(ores)
    assert int(res["taxcnt_len"].sum()) == len(tc)
    compare_results(res, tc, ores, otc)


@pytest.mark.gpu
@pytest.mark.parametrize("db_name,parts,cap,batch,peer", [("fmt2", 2, False, 700, ""), ("fmt2", 3, False, 700, ""),
                                                          ("fmt1", 2, False, 700, ""), ("fmt2_syncmer", 3, False, 700, ""),
                                                          ("fmt2", 2, True, 700, ""), ("fmt2", 3, False, 37, ""),
                                                          ("fmt2", 3, False, 700, "host"), ("fmt2", 2, True, 700, "host")])
def test_start_classify_partitioned(make_db, tmp_path, monkeypatch, db_name, parts, cap, batch, peer):
    """mtb_start_classify_partitioned (SURVEY §8(e), config 5 natively): one context per DB part (all
    on cuda:0 here), every batch matched by each part, the segments handed to the owners of their
    reads and scored there; the TSV and report are byte-identical to the one-context run over the
    whole DB, and its classifications are the oracle's. cap: one part's workspace capped so its
    pieces halve (the whole group splits the batch). batch 37: ~60 small batches through the
    workers' per-batch barriers (worker 0 must not refill the shared pieces before every part has
    left the last batch's loop). peer "host": MTB_PEER_COPY=host, every device-to-device copy (the
    batch to the further parts, the segments to their owners) staged through pinned host memory, as on
    a node where hipDeviceCanAccessPeer is false for a pair."""
    if peer:
        monkeypatch.setenv("MTB_PEER_COPY", peer)
    from metabuli_work_amd import synth
    from metabuli_work_amd.classifier import Classifier, LocalParameters

    db_dir, _, gen = make_db(db_name)
    r = _reads(gen, 43, n=2300)
    p1, p2 = str(tmp_path / "q1.fq"), str(tmp_path / "q2.fq")
    with open(p1, "wb") as f:
        f.write(synth.fastq_bytes(r.seq1, r.off1, prefix="p"))
    with open(p2, "wb") as f:
        f.write(synth.fastq_bytes(r.seq2, r.off2, prefix="p"))
    par = LocalParameters(seqMode=2, filenames=[p1, p2, db_dir]).load_db_parameters(db_dir)
    one, part = str(tmp_path / "one.tsv"), str(tmp_path / "part.tsv")
    rep1, repp = str(tmp_path / "one_rep.tsv"), str(tmp_path / "part_rep.tsv")
    with Classifier(par, db_dir=db_dir) as whole:
        assert whole.startClassify(one, reads_per_batch=700, report_tsv=rep1) == r.n
    clfs = [Classifier(par, db_dir=db_dir, db_part=(p, parts)) for p in range(parts)]
    try:
        if cap:
            # between a 100-read and a 700-read batch's workspace (a part of the DB, fresh context)
            with Classifier(par, db_dir=db_dir, db_part=(1, parts)) as probe:
                probe.classify_batch(r.seq1, r.off1[:101], r.seq2, r.off2[:101])
                small = probe.workspace_bytes
                probe.classify_batch(r.seq1, r.off1[:701], r.seq2, r.off2[:701])
                big = probe.workspace_bytes
            clfs[1].set_workspace_cap((small + big) // 2)
        with pytest.raises(MtbError, match="one context per DB part"):  # every part must be there
            clfs[0].startClassify(part, peers=[], partitioned=True)
        assert clfs[0].startClassify(part, reads_per_batch=batch, report_tsv=repp, peers=clfs[1:],
                                     partitioned=True) == r.n
        assert (clfs[0].last_run["split_batches"] > 0) == cap
        with pytest.raises(MtbError, match="range-partitioned"):  # parts are refused by the replicated entry
            clfs[0].startClassify(part, peers=clfs[1:])
    finally:
        for c in clfs:
            c.close()
    assert open(part, "rb").read() == open(one, "rb").read()
    assert open(repp, "rb").read() == open(rep1, "rb").read()
    odb = oc.OracleDb(db_dir)
    ores, _ = oc.classify(odb, par.to_c(), r)
    odb.close()
    body = [l.split("\t") for l in open(part).read().split("\n")[1:] if l]
    assert [int(f[2]) for f in body] == [int(o["classification"]) if o["is_classified"] else 0 for o in ores]
