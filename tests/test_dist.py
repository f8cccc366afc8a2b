"""N>1 path on CPU: world_size-2 and -8 gloo processes shard the reads and all-gather the result records
(world 8 as the 8-GPU node runs it, with ranks that hold no reads)."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from metabuli_work_amd._abi import RESULT_DTYPE, TAXCNT_DTYPE
from metabuli_work_amd.dist import append_taxcnt, gather_records, gather_results, shard_bounds, shard_reads


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, seq, off, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bounds = shard_bounds(off, world)
    lo, hi = bounds[rank]
    s, o = shard_reads(seq, off, lo, hi)
    # stand-in per-read record: (global read index, length, checksum of bases) as 3 int64 = 24 bytes
    rec = np.zeros((hi - lo, 3), np.int64)
    for i in range(hi - lo):
        r = s[int(o[i]):int(o[i + 1])]
        rec[i] = (lo + i, len(r), int(r.astype(np.int64).sum()))
    t = torch.from_numpy(rec.view(np.uint8).reshape(hi - lo, 24).copy())
    counts = [b - a for a, b in bounds]
    allrec = gather_records(t, counts)
    if rank == 0:
        q.put(allrec.numpy().copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_reads", [(2, 301), (8, 301), (8, 5)])
def test_shard_and_gather_gloo(world, n_reads):
    """(8, 5): three ranks shard no reads and still take part in the gather."""
    rng = np.random.default_rng(0)
    lens = rng.integers(50, 5000, size=n_reads)
    off = np.zeros(len(lens) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    seq = rng.integers(65, 90, size=int(off[-1])).astype(np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, seq, off, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rec = out.view(np.int64).reshape(-1, 3)
    assert len(rec) == len(lens)
    assert np.array_equal(rec[:, 0], np.arange(len(lens)))
    assert np.array_equal(rec[:, 1], lens)
    sums = [int(seq[int(off[i]):int(off[i + 1])].astype(np.int64).sum()) for i in range(len(lens))]
    assert np.array_equal(rec[:, 2], sums)


def test_shard_bounds_balance():
    off = np.concatenate([[0], np.cumsum(np.full(1000, 150))]).astype(np.uint64)
    b = shard_bounds(off, 8)
    assert b[0][0] == 0 and b[-1][1] == 1000
    sizes = [e - s for s, e in b]
    assert max(sizes) - min(sizes) <= 1
    assert shard_bounds(np.zeros(1, np.uint64), 4) == [(0, 0)] * 4


def _fake_batch(rng, n):
    """Result records with per-read taxID:count lists pooled the way mtb_classify_batch pools them."""
    res = np.zeros(n, RESULT_DTYPE)
    lens = rng.integers(0, 4, n)
    res["taxcnt_len"] = lens
    res["taxcnt_offset"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    res["classification"] = rng.integers(1, 1000, n)
    tc = np.zeros(int(lens.sum()), TAXCNT_DTYPE)
    tc["tax_id"] = rng.integers(1, 1000, len(tc))
    tc["count"] = rng.integers(1, 50, len(tc))
    return res, tc


def _lists(res, tc):
    return [(int(r["classification"]), tc[r["taxcnt_offset"]:r["taxcnt_offset"] + r["taxcnt_len"]].tolist())
            for r in res]


def _results_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(100 + rank)
    # two batches per rank, appended to one step pool as the bench's multi-GPU step does; with 8
    # ranks, ranks 5 and 6 classify no reads at all (an empty owner range)
    pool = torch.zeros((64, 8), dtype=torch.uint8)
    recs, used, want = [], 0, []
    for n in ((0, 0) if rank in (5, 6) else (5 + rank, 0 if rank else 7)):
        res, tc = _fake_batch(rng, n)
        want += _lists(res, tc)
        r = torch.from_numpy(res.view(np.uint8).reshape(-1, 32).copy())
        used = append_taxcnt(r, torch.from_numpy(tc.view(np.uint8).reshape(-1, 8).copy()), pool, used)
        recs.append(r)
    rec, tc = gather_results(torch.cat(recs), pool[:used])
    if rank == 0:
        q.put((rec.numpy().copy(), tc.numpy().copy()))
    q.put(("want", rank, want))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gather_results_rebases_taxcnt_gloo(world):
    """C1 with the taxID:count lists: rank 0 ends up with every rank's (classification, list) in
    rank order, offsets pointing into one gathered pool (world 8: two ranks with no reads)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_results_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    items = [q.get(timeout=120) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {i[1]: i[2] for i in items if isinstance(i[0], str)}
    rec, tc = next(i for i in items if not isinstance(i[0], str))
    res = rec.reshape(-1).view(RESULT_DTYPE)
    tcs = tc.reshape(-1).view(TAXCNT_DTYPE)
    assert _lists(res, tcs) == sum((want[r] for r in range(world)), [])
    assert int(res["taxcnt_len"].sum()) == len(tcs)


class _FakeClf:
    """Stands in for Classifier in bench.ResultGather: hands out one fake batch's records/taxcnt."""

    def __init__(self, res, tc):
        self.res, self.tc = res, tc

    def copy_results(self, dst, on_device=True):
        ctypes.memmove(dst, self.res.ctypes.data, self.res.nbytes)

    def n_taxcnt(self):
        return len(self.tc)

    def copy_taxcnt(self, dst, on_device=True):
        ctypes.memmove(dst, self.tc.ctypes.data, self.tc.nbytes)
        return len(self.tc)


def _bench_gather_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    rng = np.random.default_rng(7 + rank)
    # world 8: rank 3 holds no reads (three empty batches), the last batch is shorter than the rest
    sizes = [0, 0, 0] if rank == 3 else [6, 3 + rank, 2]
    c1 = bench.ResultGather(torch.device("cpu"), 1)
    c1.pool = c1.pool[:2]  # a tiny pool: the adds must grow it
    rec = torch.empty((sum(sizes), 32), dtype=torch.uint8)
    want, a = [], 0
    c1.reset()
    for n in sizes:
        res, tc = _fake_batch(rng, n)
        want += _lists(res, tc)
        c1.add(_FakeClf(res, tc), rec[a:a + n])
        a += n
    r, t = c1.gather(rec)
    q.put((rank, r.numpy().copy(), t.numpy().copy(), want))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_bench_result_gather_gloo(world):
    """bench.py's multi-GPU step (ResultGather: per-batch D2D copies + rebasing, one C1 gather)
    gives every rank all reads' (classification, taxID:count list) in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    items = {i[0]: i[1:] for i in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = sum((items[r][2] for r in range(world)), [])
    for r in range(world):
        res = items[r][0].reshape(-1).view(RESULT_DTYPE)
        assert _lists(res, items[r][1].reshape(-1).view(TAXCNT_DTYPE)) == want


class _FakeBatchClf:
    """Stands in for Classifier.classify_batch: per read (classification = global read index + 1,
    taxcnt list derived from it), pooled the way mtb_classify_batch pools a batch."""

    def classify_batch(self, first, n, *_, device_input=False):
        from metabuli_work_amd.classifier import BatchResult
        res = np.zeros(n, RESULT_DTYPE)
        lens = (np.arange(first, first + n) % 3).astype(np.uint32)
        res["taxcnt_len"] = lens
        res["taxcnt_offset"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
        res["classification"] = np.arange(first, first + n) + 1
        tc = np.zeros(int(lens.sum()), TAXCNT_DTYPE)
        tc["tax_id"] = np.repeat(res["classification"], lens)
        tc["count"] = np.concatenate([np.arange(1, k + 1) for k in lens]) if n else []
        return BatchResult(res, tc, 0, 0, np.zeros(5, np.float32))


def _batch_shard_worker(rank, world, port, sizes, q):
    from metabuli_work_amd.dist import classify_batches_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    starts = np.concatenate([[0], np.cumsum(sizes)]).tolist()
    touched = []

    def batch(k):
        touched.append(k)
        return (starts[k], sizes[k])

    res, tc = classify_batches_sharded(_FakeBatchClf(), [(lambda k=k: batch(k)) for k in range(len(sizes))])
    q.put((rank, touched, res.view(np.uint8).copy(), tc.view(np.uint8).copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_batches_sharded_gloo(world):
    """Batch-index sharding (dist.classify_batches_sharded): rank r materialises only batches
    r, r + N, ...; the gathered records come back in batch order with their taxID:count lists.
    World 8 over 7 batches: rank 7 takes none; the last batch is shorter than the rest."""
    sizes = [4, 0, 7, 3, 5, 6, 1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_shard_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, touched, rec, tcb in got:
        assert touched == list(range(rank, len(sizes), world))
        res = rec.view(RESULT_DTYPE).reshape(-1)
        tc = tcb.view(TAXCNT_DTYPE).reshape(-1)
        n = sum(sizes)
        assert np.array_equal(res["classification"], np.arange(n) + 1)
        for i, r in enumerate(res):
            lst = tc[r["taxcnt_offset"]:r["taxcnt_offset"] + r["taxcnt_len"]]
            assert lst["tax_id"].tolist() == [i + 1] * (i % 3) and lst["count"].tolist() == list(range(1, i % 3 + 1))
