"""Multi-GPU read sharding: one process per GPU, reads split across ranks, the DB
replicated in every GPU's HBM, and one collective at the end — an all-gather of the fixed-size
per-read result records (RCCL over xGMI with the "nccl" backend; gloo on CPU for tests).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch
import torch.distributed as dist


def shard_bounds(off: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Split reads [0, n) into `world` contiguous shards of ~equal base count (long reads vary
    500x in length, so equal read counts would not balance the work)."""
    n = len(off) - 1
    if n == 0:
        return [(0, 0)] * world
    total = float(off[-1] - off[0])
    cuts = [0]
    for r in range(1, world):
        target = off[0] + total * r / world
        cuts.append(int(np.searchsorted(off[:-1], target, side="left")))
    cuts.append(n)
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def shard_reads(seq: np.ndarray, off: np.ndarray, lo: int, hi: int) -> Tuple[np.ndarray, np.ndarray]:
    a, b = int(off[lo]), int(off[hi])
    return seq[a:b], (off[lo:hi + 1] - off[lo]).astype(np.uint64)


def gather_records(local: torch.Tensor, counts: List[int], group=None) -> torch.Tensor:
    """All-gather variable-length rows (records of `local.shape[1]` bytes) in rank order."""
    world = dist.get_world_size(group)
    width = local.shape[1]
    cap = max(max(counts), 1)
    pad = torch.zeros((cap, width), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    out = torch.empty((world * cap, width), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out.view(-1), pad.view(-1), group=group)
    parts = [out[r * cap:r * cap + counts[r]] for r in range(world)]
    return torch.cat(parts, 0)


RESULT_BYTES = 32   # mtb_result
TAXCNT_BYTES = 8    # mtb_taxcnt {tax_id, count}
_TC_OFFSET_COL = 4  # mtb_result.taxcnt_offset, as the 5th int32 of the record


def append_taxcnt(results: torch.Tensor, taxcnt: torch.Tensor, pool: torch.Tensor, used: int) -> int:
    """Append one batch's pooled taxID:count entries (taxcnt (T, 8) uint8) to `pool` at `used` and
    rebase the batch's result records (results (n, 32) uint8, in place) onto it. Returns the new fill."""
    t = taxcnt.shape[0]
    if t:
        pool[used:used + t] = taxcnt
        results.view(torch.int32).view(-1, RESULT_BYTES // 4)[:, _TC_OFFSET_COL] += used
    return used + t


def gather_results(results: torch.Tensor, taxcnt: torch.Tensor, group=None):
    """C1: every rank's result records (n_r, 32) uint8 and pooled taxID:count lists
    (T_r, 8) uint8 gathered in rank order, the records' taxcnt offsets rebased onto the gathered
    pool — the same two arrays one GPU would have produced for all reads, so rank 0 can write the
    reference's TSV (Reporter.cpp:38-83, taxID:count per read) and report. Returns
    (results (Σn, 32), taxcnt (ΣT, 8)) on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = results.device
    size = torch.tensor([results.shape[0], taxcnt.shape[0]], dtype=torch.int64, device=dev)
    sizes = torch.empty(world * 2, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes, size, group=group)
    sizes = sizes.view(world, 2).cpu().tolist()
    base = sum(sizes[r][1] for r in range(rank))
    rec = results.clone()
    if base and rec.shape[0]:
        rec.view(torch.int32).view(-1, RESULT_BYTES // 4)[:, _TC_OFFSET_COL] += base
    all_rec = gather_records(rec, [s[0] for s in sizes], group)
    all_tc = gather_records(taxcnt, [s[1] for s in sizes], group)
    return all_rec, all_tc


def classify_sharded(clf, seq1, off1, seq2=None, off2=None, group=None):
    """Replicated DB (configs 2-4): every rank passes the SAME host batch, classifies its shard of
    it (contiguous, about equal bases, shard_bounds) against its own DB replica, and the results
    are gathered (C1). Returns (results (n,) RESULT_DTYPE numpy, taxcnt TAXCNT_DTYPE numpy) for the
    whole batch, in read order, on every rank."""
    from ._abi import RESULT_DTYPE, TAXCNT_DTYPE

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(off1, world)[rank]
    s1, o1 = shard_reads(seq1, off1, lo, hi)
    s2 = o2 = None
    if seq2 is not None:
        s2, o2 = shard_reads(seq2, off2, lo, hi)
    br = clf.classify_batch(s1, o1, s2, o2)
    rec = torch.from_numpy(br.results.view(np.uint8).reshape(-1, RESULT_BYTES).copy())
    tc = torch.from_numpy(br.taxcnt.view(np.uint8).reshape(-1, TAXCNT_BYTES).copy())
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
        rec, tc = rec.to(dev), tc.to(dev)
    all_rec, all_tc = gather_results(rec, tc, group)
    return (all_rec.cpu().numpy().reshape(-1).view(RESULT_DTYPE),
            all_tc.cpu().numpy().reshape(-1).view(TAXCNT_DTYPE))


def classify_batches_sharded(clf, batches, group=None, device_input: bool = False):
    """Replicated DB, sharded by batch index: `batches` yields the run's batches in input order —
    (seq1, off1, seq2, off2) tuples, or callables returning one, so a rank never materialises the
    batches it skips — and rank r classifies batches r, r + N, r + 2N, ... (the reference's
    QuerySplit loop, Classifier.cpp:81-133, dealt round-robin over the GPUs). The result records and
    taxID:count lists are gathered (C1) and put back in batch order. Returns (results
    RESULT_DTYPE numpy, taxcnt TAXCNT_DTYPE numpy) of the whole run on every rank. (For files on one
    node, mtb_start_classify_multi is the native form: one parser feeding every GPU.)"""
    from ._abi import RESULT_DTYPE, TAXCNT_DTYPE

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    recs, pool, sizes, used = [], [], [], 0
    for k, b in enumerate(batches):
        if k % world != rank:
            continue
        b = b() if callable(b) else b
        br = clf.classify_batch(*b, device_input=device_input)
        rec = br.results.view(np.uint8).reshape(-1, RESULT_BYTES).copy()
        rec.view(np.int32).reshape(-1, RESULT_BYTES // 4)[:, _TC_OFFSET_COL] += used  # onto the rank's pool
        used += len(br.taxcnt)
        recs.append(rec)
        pool.append(br.taxcnt.view(np.uint8).reshape(-1, TAXCNT_BYTES))
        sizes.append(len(rec))
    rec = torch.from_numpy(np.concatenate(recs) if recs else np.zeros((0, RESULT_BYTES), np.uint8))
    tc = torch.from_numpy(np.concatenate(pool) if pool else np.zeros((0, TAXCNT_BYTES), np.uint8))
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
        rec, tc = rec.to(dev), tc.to(dev)
    all_rec, all_tc = gather_results(rec, tc, group)
    per_rank = [None] * world
    dist.all_gather_object(per_rank, sizes, group=group)
    # rank-ordered gathered records -> batch order (the taxcnt offsets index the gathered pool, so
    # the records move without rebasing)
    base, start = 0, {}
    for r in range(world):
        for j, n in enumerate(per_rank[r]):
            start[r + j * world] = (base, n)
            base += n
    order = np.concatenate([np.arange(a, a + n) for a, n in (start[k] for k in sorted(start))]) if start else \
        np.zeros(0, np.int64)
    all_rec = all_rec.cpu().numpy()[order]
    return all_rec.reshape(-1).view(RESULT_DTYPE), all_tc.cpu().numpy().reshape(-1).view(TAXCNT_DTYPE)


# ---------------------------------------------------------------------------------------------
# Range-partitioned DB: rank r holds DB part r (AA-aligned k-mer range,
# mtb_partition_bounds) and matches EVERY read of the batch against it; the matches then go
# all-to-all to the rank that owns their read (C2), which sorts and scores them (mtb_assign_chunks);
# the result records are gathered at the end (C1).
# ---------------------------------------------------------------------------------------------
MATCH_BYTES = 24


def owner_bounds(n: int, world: int) -> List[Tuple[int, int]]:
    """Reads [0, n) cut into `world` contiguous owner ranges of equal read count."""
    cuts = [n * r // world for r in range(world + 1)]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def exchange_matches(matches: torch.Tensor, counts: torch.Tensor, bounds: List[Tuple[int, int]], group=None):
    """All-to-all of per-read match segments to the owners of the reads.

    matches: (M, 24) uint8, grouped by read in read order; counts: (n,) int32 matches per read.
    Returns (recv_matches (R, 24) uint8, recv_counts (world * n_own,) int32): one chunk per source
    rank, each grouped by the owner's reads — the layout mtb_assign_chunks takes."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_q = [hi - lo for lo, hi in bounds]
    n_own = n_q[rank]
    recv_cnt = torch.empty(world * n_own, dtype=torch.int32, device=counts.device)
    dist.all_to_all_single(recv_cnt, counts, output_split_sizes=[n_own] * world, input_split_sizes=n_q, group=group)
    csum = torch.zeros(len(counts) + 1, dtype=torch.int64, device=counts.device)
    torch.cumsum(counts.to(torch.int64), 0, out=csum[1:])
    cuts = csum[[lo for lo, _ in bounds] + [bounds[-1][1]]].cpu().tolist()
    send = [cuts[q + 1] - cuts[q] for q in range(world)]
    recv = recv_cnt.view(world, n_own).to(torch.int64).sum(1).cpu().tolist() if n_own else [0] * world
    out = torch.empty((sum(recv), MATCH_BYTES), dtype=torch.uint8, device=matches.device)
    dist.all_to_all_single(out, matches, output_split_sizes=recv, input_split_sizes=send, group=group)
    return out, recv_cnt


def classify_partitioned(clf, seq1, off1, seq2=None, off2=None, group=None, device_input: bool = False,
                         on_device: bool = True):
    """One batch through a range-partitioned DB. Every rank passes the SAME batch; `clf` holds this
    rank's DB part (Classifier(..., db_part=(rank, world))). Returns (owner read range, BatchResult
    of the owned reads, or None with on_device when results stay in HBM). on_device=False stages the
    exchange through host memory (gloo)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = (int(off1.numel()) if device_input else len(off1)) - 1
    clf.classify_batch(seq1, off1, seq2, off2, device_input=device_input, match_only=True)
    _, M = clf.last_counts()
    if on_device:
        dev = torch.device("cuda", torch.cuda.current_device())
        matches = torch.empty((M, MATCH_BYTES), dtype=torch.uint8, device=dev)
        counts = torch.empty(n, dtype=torch.int32, device=dev)
        qlen = torch.empty(n, dtype=torch.int32, device=dev)
        clf.copy_matches(matches, counts, qlen)
    else:
        m_np = np.zeros((M, MATCH_BYTES), np.uint8)
        c_np = np.zeros(n, np.int32)
        q_np = np.zeros(n, np.int32)
        clf.copy_matches(m_np, c_np, q_np)
        matches, counts, qlen = torch.from_numpy(m_np), torch.from_numpy(c_np), torch.from_numpy(q_np)
    bounds = owner_bounds(n, world)
    rm, rc = exchange_matches(matches, counts, bounds, group)
    lo, hi = bounds[rank]
    ql = qlen[lo:hi].contiguous()
    if on_device:
        br = clf.assign_chunks(rm, rm.shape[0], rc, world, ql, hi - lo, fetch=False)
    else:
        br = clf.assign_chunks(rm.numpy(), rm.shape[0], rc.numpy(), world, ql.numpy(), hi - lo)
    return (lo, hi), br
