"""N>1 path on CPU: world_size-2 gloo processes shard the reads and all-gather the result records."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from metabuli_work_amd.dist import gather_records, shard_bounds, shard_reads


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


@pytest.mark.parametrize("world", [2])
def test_shard_and_gather_gloo(world):
    rng = np.random.default_rng(0)
    lens = rng.integers(50, 5000, size=301)
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
