"""GTDB-scale synthetic reference DB, built in place on the GPU.

Shape: a true-signal part — genomes of `n_true_species` species x 2 strains with
gene blocks, turned into DB k-mers by the GPU builder (mtb_build_db with MTB_BUILD_DEVICE_OUT:
extractTargetKmers, (value, species) dedup with the LCA, IndexCreator.cpp:316-376,
IndexCreator.h:475-629) — plus filler: uniformly random valid metamers (a random AA 8-mer, each
codon a random synonymous one) with the strains of a ~130k-species skeleton taxonomy (GTDB r226 has
129,671 species reps), up to `target_kmers` entries. The two sorted streams are merged by AA-rank
chunk into one resident array of 12-B records (value in the resident rank form, DESIGN.md §3, and
taxID), which a context uses in place (mtb_open_resident). Nothing is written to disk: at 12G k-mers the diffIdx +
info would be ~110 GB.

`encode_into_oracle` writes the same DB in the reference's diffIdx / info / split format
(getDiffIdx, IndexCreator.cpp:868-886; writeTargetFilesAndSplits, :811-861) straight into the
oracle's buffers, for the CPU baseline and its parity sample (test / bench infrastructure).

Bench/test data only: nothing here is on the classify path.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional

import numpy as np
import torch

from . import synth
from ._abi import MtbDbResident, MtbParams, default_params
from ._lib import check, lib
from .dbbuild import HostDb, build_db_device
from .gpu_synth import make_genomes_gpu

AA_RANKS = 21 ** 8
INT64_MIN = -(1 << 63)


def codon_counts() -> np.ndarray:
    """Synonymous codons per AA code (GeneticCode.h, as the library's tables hold them)."""
    base = np.zeros(256, np.uint8)
    aa = np.zeros(64, np.int8)
    num = np.zeros(64, np.int8)
    lib().mtb_debug_tables(base.ctypes.data, aa.ctypes.data, num.ctypes.data)
    cnt = np.ones(21, np.int64)
    for i in range(64):
        if 0 <= aa[i] < 21:
            cnt[aa[i]] = max(cnt[aa[i]], int(num[i]) + 1)
    return cnt


class ResidentDb:
    """A DB resident in HBM as 12-B records {value low 32 bits, value high 32 bits, taxID} (an
    int32 tensor of shape (n + 8, 3), values in the resident rank form; the 8 spare records are the
    context's pad), the layout mtb_open_resident uses in place; `host` carries the taxonomy and
    taxID_list."""

    def __init__(self, records: torch.Tensor, n: int, host: HostDb, n_true: int):
        assert records.dtype == torch.int32 and records.dim() == 2 and records.shape[1] == 3
        assert records.shape[0] >= n + 8 and records.is_contiguous()
        self.records, self.n, self.host, self.n_true = records, n, host, n_true

    @classmethod
    def from_arrays(cls, values: torch.Tensor, info: torch.Tensor, host: HostDb, n_true: Optional[int] = None):
        """Records of sorted resident-form values (int64) and their taxIDs (int32)."""
        n = values.numel()
        rec = torch.empty(n + 8, 3, dtype=torch.int32, device=values.device)
        put_records(rec, 0, values, info)
        return cls(rec, n, host, n if n_true is None else n_true)

    def values(self, a: int = 0, b: Optional[int] = None) -> torch.Tensor:
        """Values [a, b) as int64 (b defaults to n)."""
        b = self.n if b is None else b
        return self.records[a:b, 0:2].clone(memory_format=torch.contiguous_format).view(torch.int64).view(-1)

    def value_at(self, idx: torch.Tensor) -> torch.Tensor:
        return self.records[idx][:, 0:2].clone(memory_format=torch.contiguous_format).view(torch.int64).view(-1)

    def info(self, a: int = 0, b: Optional[int] = None) -> torch.Tensor:
        b = self.n if b is None else b
        return self.records[a:b, 2]

    def c_resident(self) -> MtbDbResident:
        return MtbDbResident(records=self.records.data_ptr(), n_kmers=self.n, rank_form=1)

    @property
    def n_kmers(self) -> int:
        return self.n


def put_records(rec: torch.Tensor, pos: int, values: torch.Tensor, info: torch.Tensor) -> None:
    """rec[pos:pos+m] = records of values (int64) and info (int32); little-endian: the int64 viewed
    as two int32 is (low, high)."""
    m = values.numel()
    rec[pos:pos + m, 0:2] = values.contiguous().view(torch.int32).view(m, 2)
    rec[pos:pos + m, 2] = info


def _filler_chunk(lo: int, hi: int, count: int, g: torch.Generator, cnt_t: torch.Tensor, strain_t: torch.Tensor):
    """`count` random valid metamers with AA ranks in [lo, hi), unique values, sorted; random strains."""
    dev = cnt_t.device
    r = torch.randint(lo, hi, (count,), generator=g, device=dev, dtype=torch.int64)
    dna = torch.zeros_like(r)
    rem = r.clone()
    for k in range(8):  # least significant base-21 digit = the last codon = DNA bits 0..2
        a = rem % 21
        rem = rem // 21
        c = (torch.rand(count, generator=g, device=dev) * cnt_t[a]).long().clamp_(max=7)
        dna |= c << (3 * k)
    del rem
    v = torch.unique((r << 24) | dna)
    del r, dna
    tax = strain_t[torch.randint(0, strain_t.numel(), (v.numel(),), generator=g, device=dev)]
    return v, tax


class GtdbRecipe:
    """The GTDB-scale DB as a recipe that builds any AA-rank range of it on demand: the true-signal
    part (built once, kept sorted in HBM) plus filler generated per chunk of the AA-rank space with a
    per-chunk seed, so a chunk's k-mers do not depend on which other chunks were built. The whole DB
    is chunks [0, n_chunks) (config 3); a range-partitioned DB (config 5: more k-mers than one GPU
    holds) is built one part at a time, each part a run of whole chunks — AA-aligned, as the
    reference's split entries are (IndexCreator.cpp:843-851) — plus its guard k-mer."""

    def __init__(self, dev: torch.device, n_true_species: int = 1000, genome_len: int = 3_000_000,
                 total_species: int = 129_671, target_kmers: int = 12_000_000_000, strains: int = 2, seed: int = 6,
                 n_chunks: int = 64, before_free: Optional[Callable[[torch.Tensor, torch.Tensor], None]] = None,
                 log: Callable[[str], None] = lambda s: None, syncmer: int = 0, smer_len: int = 5,
                 per_genus: int = 1, species_div: float = 0.0, conserved: int = 0, cons_min: int = 100,
                 cons_max: int = 10_000):
        """conserved > 0: that many AA 8-mers of the true-signal genomes are also held by cons_min to
        cons_max filler species each (log-uniform: a heavy tail), as conserved genes' AA 8-mers are
        shared across GTDB's species; their DB runs are long and their reads' queries select among
        thousands of candidates."""
        self.dev, self.seed, self.n_chunks, self.log = dev, seed, n_chunks, log
        taxo = synth.make_taxonomy(total_species, strains, seed=seed,
                                   block_species=n_true_species if per_genus > 1 else 0, block_size=per_genus)
        taxo, gen, seq, off_t, _ = make_genomes_gpu(n_true_species, genome_len, strains, seed, dev, taxo=taxo,
                                                    per_genus=per_genus, species_div=species_div)
        if before_free is not None:
            before_free(seq, off_t)
        par = default_params(kmer_format=2, seq_mode=2, syncmer=syncmer, smer_len=smer_len)
        self.tv, self.ti = build_db_device(gen, taxo, par, device=dev.index or 0, device_seq=(seq, off_t))
        del seq, off_t
        torch.cuda.empty_cache()
        self.n_true = self.tv.numel()
        log(f"true-signal DB part: {self.n_true / 1e9:.3f}G k-mers")
        # filler strains: those of the skeleton species beyond the true-signal ones
        rank = np.array(taxo.rank)
        sp_all = taxo.taxid[rank == "species"]
        self.n_species = len(sp_all)
        filler_sp = set(sp_all[n_true_species:].tolist())
        strains_f = np.array([t for t, p, r in zip(taxo.taxid.tolist(), taxo.parent.tolist(), taxo.rank)
                              if r == "no rank" and p in filler_sp], np.int32)
        self.strain_t = torch.from_numpy(strains_f).to(dev)
        self.cnt_t = torch.from_numpy(codon_counts().astype(np.float32)).to(dev)
        self.edges = [c * AA_RANKS // n_chunks for c in range(n_chunks + 1)]
        e_t = torch.tensor(self.edges, dtype=torch.int64, device=dev)
        self.cut = torch.searchsorted(self.tv, e_t << 24).cpu().tolist()  # true-signal records per chunk
        self.conserved = conserved
        n_cons = 0
        self.cons_cut = [0] * (n_chunks + 1)
        if conserved > 0:
            # the filler species' strains (two per species, consecutive in the taxonomy), and the
            # species of every taxID (for the (value, species) order of the merged records)
            par = taxo.parent.astype(np.int64)
            tid = taxo.taxid.astype(np.int64)
            sp_of = np.zeros(int(tid.max()) + 1, np.int64)
            rk = np.array(taxo.rank)
            sp_of[tid[rk == "species"]] = tid[rk == "species"]
            strain = rk == "no rank"
            sp_of[tid[strain]] = par[strain]
            self.sp_of_t = torch.from_numpy(sp_of).to(dev)
            self.cons_strains = torch.from_numpy(strains_f.reshape(-1, strains).astype(np.int32)).to(dev)
            gc = torch.Generator(device=dev)
            gc.manual_seed(seed * 31337 + 7)
            pick = torch.randint(0, self.n_true, (2 * conserved,), generator=gc, device=dev)
            ranks = torch.unique(self.tv[pick] >> 24)
            ranks = ranks[torch.randperm(ranks.numel(), generator=gc, device=dev)[:conserved]]
            self.cons_rank, _ = torch.sort(ranks)
            u = torch.rand(self.cons_rank.numel(), generator=gc, device=dev, dtype=torch.float64)
            self.cons_k = (cons_min * torch.exp(u * float(np.log(cons_max / cons_min)))).long()
            self.cons_base = torch.randint(0, self.cons_strains.shape[0], (self.cons_rank.numel(),), generator=gc,
                                           device=dev)
            self.cons_cut = torch.searchsorted(self.cons_rank, e_t).cpu().tolist()
            ck = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(self.cons_k, 0)])
            self.cons_kcut = ck[torch.tensor(self.cons_cut, device=dev)].cpu().tolist()  # conserved records per chunk
            n_cons = int(ck[-1].item())
            log(f"conserved AA 8-mers: {self.cons_rank.numel()} x {cons_min}-{cons_max} species "
                f"({n_cons / 1e9:.3f}G k-mers)")
        n_fill = max(0, int(target_kmers) - self.n_true - n_cons)
        self.per = [n_fill // n_chunks + (1 if c < n_fill % n_chunks else 0) for c in range(n_chunks)]
        ids = np.unique(np.concatenate([gen.taxid.astype(np.int32), strains_f]))
        self.host = HostDb(taxo, taxid_list=ids.astype(np.int32))

    def _conserved_chunk(self, c: int, g: torch.Generator):
        """The conserved AA 8-mers of chunk c: per AA rank k consecutive filler species (distinct),
        one strain each, each entry a random synonymous DNA of the AA 8-mer."""
        a, b = self.cons_cut[c], self.cons_cut[c + 1]
        if a == b:
            e = torch.zeros(0, dtype=torch.int64, device=self.dev)
            return e, e.int()
        k = self.cons_k[a:b]
        rr = torch.repeat_interleave(self.cons_rank[a:b], k)
        first = torch.cumsum(k, 0) - k
        j = torch.arange(rr.numel(), device=self.dev) - torch.repeat_interleave(first, k)
        S = self.cons_strains.shape[0]
        sp = (torch.repeat_interleave(self.cons_base[a:b], k) + j) % S
        coin = torch.randint(0, self.cons_strains.shape[1], (rr.numel(),), generator=g, device=self.dev)
        tax = self.cons_strains[sp, coin]
        dna = torch.zeros_like(rr)
        rem = rr.clone()
        for q in range(8):  # least significant base-21 digit = the last codon = DNA bits 0..2
            d = rem % 21
            rem = rem // 21
            cdn = (torch.rand(rr.numel(), generator=g, device=self.dev) * self.cnt_t[d]).long().clamp_(max=7)
            dna |= cdn << (3 * q)
        return (rr << 24) | dna, tax

    def _chunk(self, c: int):
        """Chunk c's records as (sorted values, taxIDs): its true-signal k-mers and its filler
        (+ its conserved AA 8-mers' entries)."""
        g = torch.Generator(device=self.dev)
        g.manual_seed(self.seed * 7919 + 1 + 104729 * c)
        fv, ft = _filler_chunk(self.edges[c], self.edges[c + 1], self.per[c], g, self.cnt_t, self.strain_t)
        a, b = self.cut[c], self.cut[c + 1]
        if self.conserved:
            cv, ct = self._conserved_chunk(c, g)
            v = torch.cat([self.tv[a:b], cv, fv])
            t = torch.cat([self.ti[a:b], ct, ft])
            del fv, ft, cv, ct
            # (value, species) order, one entry per (value, species) (IndexCreator.h:617-624): a
            # conserved entry that meets a filler entry of the same value and species is dropped
            sp = self.sp_of_t[t.long()]
            o1 = torch.argsort(sp, stable=True)
            o2 = torch.argsort(v[o1], stable=True)
            order = o1[o2]
            del o1, o2
            vs, ts, sps = v[order], t[order], sp[order]
            dup = torch.zeros_like(vs, dtype=torch.bool)
            dup[1:] = (vs[1:] == vs[:-1]) & (sps[1:] == sps[:-1])
            keep = ~dup
            return vs[keep], ts[keep]
        v = torch.cat([self.tv[a:b], fv])
        t = torch.cat([self.ti[a:b], ft])
        del fv, ft
        # stable: a value held by a true-signal species and a filler species keeps species order
        # (true-signal species have the smaller taxIDs), as the builder's (value, species) sort does
        vs, order = torch.sort(v, stable=True)
        return vs, t[order]

    def chunk_sizes(self) -> list:
        """Records per chunk (an upper bound with conserved AA 8-mers: a rare duplicate is dropped)."""
        cons = [(self.cons_kcut[c + 1] - self.cons_kcut[c]) if self.conserved else 0 for c in range(self.n_chunks)]
        return [self.cut[c + 1] - self.cut[c] + self.per[c] + cons[c] for c in range(self.n_chunks)]

    def part_chunks(self, parts: int) -> list:
        """Chunk ranges of `parts` parts of about equal k-mer count."""
        cs = np.cumsum([0] + self.chunk_sizes())
        bounds = [0] + [int(np.searchsorted(cs, cs[-1] * p / parts)) for p in range(1, parts)] + [self.n_chunks]
        for i in range(1, len(bounds)):
            bounds[i] = min(max(bounds[i], bounds[i - 1] + 1), self.n_chunks - (len(bounds) - 1 - i))
        return [(bounds[p], bounds[p + 1]) for p in range(parts)]

    def build(self, c0: int = 0, c1: Optional[int] = None, guard: bool = False) -> "ResidentDb":
        """Records of chunks [c0, c1) — with guard and c1 < n_chunks, plus the first k-mer of chunk
        c1: the part's last resident k-mer, never a candidate (the reference's reader stops before
        the DB's last k-mer, KmerMatcher.cpp:363,378), so the next part matches its AA run."""
        c1 = self.n_chunks if c1 is None else c1
        sizes = self.chunk_sizes()
        g_add = 1 if guard and c1 < self.n_chunks else 0
        n = sum(sizes[c0:c1])
        rec = torch.empty(n + g_add + 8, 3, dtype=torch.int32, device=self.dev)
        pos = 0
        for c in range(c0, c1):
            vs, ts = self._chunk(c)
            m = vs.numel()
            put_records(rec, pos, vs, ts)
            pos += m
            del vs, ts
        if g_add:
            vs, ts = self._chunk(c1)
            put_records(rec, pos, vs[:1], ts[:1])
            pos += 1
            del vs, ts
        torch.cuda.empty_cache()
        rdb = ResidentDb(rec, pos, self.host, sum(self.cut[c + 1] - self.cut[c] for c in range(c0, c1)))
        rdb.rank_range = (self.edges[c0], self.edges[c1])
        return rdb

    def free_true(self) -> None:
        del self.tv, self.ti
        torch.cuda.empty_cache()


def build_gtdb_scale(dev: torch.device, n_true_species: int = 1000, genome_len: int = 3_000_000,
                     total_species: int = 129_671, target_kmers: int = 12_000_000_000, strains: int = 2,
                     seed: int = 6, n_chunks: int = 64,
                     before_free: Optional[Callable[[torch.Tensor, torch.Tensor], None]] = None,
                     log: Callable[[str], None] = lambda s: None, syncmer: int = 0, smer_len: int = 5,
                     per_genus: int = 1, species_div: float = 0.0, conserved: int = 0) -> ResidentDb:
    """Build the whole DB on `dev` (GtdbRecipe, all chunks). before_free(seq, off) runs while the
    true-signal genomes are still in HBM (the bench samples its reads there). syncmer: the
    true-signal part holds closed syncmers only (a Syncmer 1 DB, the format of GTDB R226's DB);
    per_genus / species_div: sister species of a genus share a diverged genus genome
    (make_genomes_gpu), so AA runs carry several species."""
    rc = GtdbRecipe(dev, n_true_species, genome_len, total_species, target_kmers, strains, seed, n_chunks,
                    before_free, log, syncmer, smer_len, per_genus, species_div, conserved)
    rdb = rc.build()
    rc.free_true()
    log(f"GTDB-scale DB: {rdb.n / 1e9:.3f}G k-mers ({rdb.n_true / 1e9:.3f}G true signal), "
        f"{rc.n_species} species in the taxonomy")
    return rdb


def run_length_histogram(rdb: ResidentDb, chunk: int = 1 << 27) -> dict:
    """AA runs of a resident DB (k-mers sharing an AA 8-mer: the candidates one query k-mer scans)
    by length, in log2 bins: {"1": runs, "2-3": runs, ...} plus the k-mers in runs of each bin and
    the longest run."""
    dev = rdb.records.device
    edges = torch.tensor([1 << b for b in range(40)], dtype=torch.int64, device=dev)
    runs = torch.zeros(40, dtype=torch.int64, device=dev)
    kmers = torch.zeros(40, dtype=torch.int64, device=dev)
    longest = 0

    def add(lens):
        nonlocal longest
        if lens.numel() == 0:
            return
        b = torch.bucketize(lens, edges, right=True) - 1
        runs.index_add_(0, b, torch.ones_like(lens))
        kmers.index_add_(0, b, lens)
        longest = max(longest, int(lens.max().item()))

    carry, prev = 0, -1
    for a in range(0, rdb.n, chunk):
        r = _lsr(rdb.values(a, min(rdb.n, a + chunk)), 24)
        n = r.numel()
        starts = torch.nonzero(r[1:] != r[:-1]).flatten() + 1
        bounds = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), starts,
                            torch.full((1,), n, dtype=torch.int64, device=dev)])
        lens = bounds[1:] - bounds[:-1]
        if int(r[0].item()) == prev:
            lens[0] += carry
        elif carry:
            add(torch.tensor([carry], dtype=torch.int64, device=dev))
        carry = int(lens[-1].item())
        add(lens[:-1])
        prev = int(r[-1].item())
        del r, starts, bounds, lens
    if carry:
        add(torch.tensor([carry], dtype=torch.int64, device=dev))
    rc, kc = runs.cpu().tolist(), kmers.cpu().tolist()
    out = {}
    for b in range(40):
        if rc[b]:
            lo, hi = 1 << b, (1 << (b + 1)) - 1
            out[str(lo) if lo == hi else f"{lo}-{hi}"] = {"runs": rc[b], "kmers": kc[b]}
    return {"bins": out, "longest_run": longest}


def to_rank_fmt2(v: torch.Tensor) -> torch.Tensor:
    """Format-2 values (int64 bit patterns) -> the resident rank form (the inverse of to_native_fmt2)."""
    aa = _lsr(v, 24)
    r = torch.zeros_like(aa)
    mul = 1
    for k in range(8):
        r += ((aa >> (5 * k)) & 31) * mul
        mul *= 21
    return (r << 24) | (v & 0xFFFFFF)


class SubDb:
    """Parity helper (test / bench infrastructure): the DB runs of a set of AA 8-mers, collected from
    resident DB parts, as a small DB for the oracle. A query k-mer can only match DB k-mers of its own
    AA 8-mer (matchKmers compares AA parts first, KmerMatcher.cpp:381-400), so the oracle classifies
    reads against the runs of their k-mers' AA 8-mers exactly as against the whole DB — provided no
    run is cut and the last k-mer (never a candidate, KmerMatcher.cpp:363,378) is not one of them: a
    sentinel past every collected run closes the DB."""

    def __init__(self, host, ranks: torch.Tensor):
        self.host = host
        self.ranks = torch.unique(ranks)  # sorted AA ranks of the sample's query k-mers
        self.vals, self.infos = [], []

    @classmethod
    def of_kmers(cls, host, kmers: np.ndarray, dev: torch.device) -> "SubDb":
        """kmers: the oracle's extracted query k-mers (format-2 values) of the sample reads; the
        blank slots ({0, 0}) are dropped."""
        kmers = kmers[(kmers["value"] != 0) | (kmers["info"] != 0)]
        v = torch.from_numpy(kmers["value"].view(np.int64).copy()).to(dev)
        return cls(host, _lsr(to_rank_fmt2(v), 24))

    def collect(self, rdb: ResidentDb, rank_lo: int = 0, rank_hi: int = AA_RANKS, db_end: bool = True,
                chunk: int = 1 << 27) -> None:
        """The runs of the sample's AA ranks in [rank_lo, rank_hi) from a resident DB (part).
        db_end: rdb's last record is the DB's last k-mer, which is never a candidate: left out (the
        sentinel takes its place)."""
        rk = self.ranks[(self.ranks >= rank_lo) & (self.ranks < rank_hi)]
        if rk.numel() == 0:
            return
        lo_k, hi_k = rk << 24, (rk + 1) << 24
        lo = torch.zeros_like(rk)
        hi = torch.zeros_like(rk)
        for a in range(0, rdb.n, chunk):  # global lower bounds = sums of the chunks' counts below
            vals = rdb.values(a, min(rdb.n, a + chunk))
            lo += torch.searchsorted(vals, lo_k)
            hi += torch.searchsorted(vals, hi_k)
            del vals
        if db_end:
            hi = torch.clamp(hi, max=rdb.n - 1)
        cnt = hi - lo
        keep = cnt > 0
        lo, cnt = lo[keep], cnt[keep]
        if lo.numel() == 0:
            return
        idx = torch.repeat_interleave(lo, cnt) + (torch.arange(int(cnt.sum().item()), device=lo.device) -
                                                   torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt))
        self.vals.append(rdb.value_at(idx))
        self.infos.append(rdb.records[idx, 2].clone())

    def oracle_db(self, oracle_cls):
        v = torch.cat(self.vals) if self.vals else torch.zeros(0, dtype=torch.int64, device=self.ranks.device)
        t = torch.cat(self.infos) if self.infos else torch.zeros(0, dtype=torch.int32, device=self.ranks.device)
        order = torch.argsort(v, stable=True)  # parts arrive in rank order already; keeps species order
        v, t = v[order], t[order]
        last = int((v[-1] >> 24).item()) if v.numel() else -1
        assert last + 1 < AA_RANKS, "sample hits the last AA 8-mer rank: no room for the sentinel"
        sent = torch.tensor([(last + 1) << 24], dtype=torch.int64, device=v.device)
        v = torch.cat([v, sent])
        t = torch.cat([t, t[:1] if t.numel() else torch.ones(1, dtype=torch.int32, device=v.device)])
        sub = ResidentDb.from_arrays(v, t, self.host)
        return encode_into_oracle(sub, oracle_cls, chunk=1 << 24), sub.n


# ---------------------------------------------------------------------------------------------
# The same DB in the reference's on-disk format, written into the oracle's buffers.
# ---------------------------------------------------------------------------------------------
def _lsr(x: torch.Tensor, s: int) -> torch.Tensor:
    """Logical right shift of int64 bit patterns."""
    return (x >> s) & ((1 << (64 - s)) - 1) if s else x


def to_native_fmt2(v: torch.Tensor) -> torch.Tensor:
    """Resident rank form -> format-2 value (8 x 5-bit AA codes above the 24-bit DNA part), as
    int64 bit patterns."""
    r = v >> 24
    aa = torch.zeros_like(r)
    for k in range(8):
        aa |= (r % 21) << (5 * k)
        r = r // 21
    low = ((aa & ((1 << 39) - 1)) << 24) | (v & 0xFFFFFF)
    return torch.where(aa >= (1 << 39), low | INT64_MIN, low)


def _words(d: torch.Tensor) -> torch.Tensor:
    nw = torch.ones_like(d)
    for gi in range(1, 5):
        nw += (_lsr(d, 15 * gi) != 0).long()
    return nw


def encode_into_oracle(rdb: ResidentDb, oracle_cls, split_num: int = 4096, chunk: int = 1 << 27):
    """Oracle DB (diffIdx / info / split / taxID_list + taxonomy) of the resident DB. The values are
    read from HBM chunk by chunk; diffIdx words are made on the device (getDiffIdx: big-endian
    15-bit groups, the last with 0x8000)."""
    n = rdb.n
    dev = rdb.records.device

    def chunk_deltas(a, b):
        nat = to_native_fmt2(rdb.values(a, b))
        prev = to_native_fmt2(rdb.values(a - 1, a)) if a > 0 else torch.zeros(1, dtype=torch.int64, device=dev)
        return nat - torch.cat([prev, nat[:-1]]), nat

    # pass 1: words per chunk
    bases = [0]
    for a in range(0, n, chunk):
        d, _ = chunk_deltas(a, min(n, a + chunk))
        bases.append(bases[-1] + int(_words(d).sum().item()))
    W = bases[-1]
    # split entries: after every n/(splitNum-1) k-mers, the first later k-mer of a new AA
    size = n // (split_num - 1) if split_num > 1 else 0
    gs = []
    if size:
        idx = torch.arange(1, split_num, dtype=torch.int64, device=dev) * size - 1
        idx = idx[(idx >= 0) & (idx < n)]
        key = ((rdb.value_at(idx) >> 24) + 1) << 24
        g_t = torch.zeros_like(key)  # lower bound over [0, n) = sum over chunks of the chunk's count below
        for a in range(0, n, chunk):
            g_t += torch.searchsorted(rdb.values(a, min(n, a + chunk)), key)
        g_all = g_t.cpu().numpy()
        last = -1
        for gv in g_all.tolist():
            if gv < n and gv != last:
                gs.append(gv)
                last = gv
    db, diff, info, split = oracle_cls.fillable(rdb.host.c_struct(), W, n, split_num)
    split[:] = 0
    gpos = {}  # k-mer index g+1 -> word offset of entry g+1 (start of the next k-mer)
    want = sorted(set(g + 1 for g in gs))
    for ci, a in enumerate(range(0, n, chunk)):
        b = min(n, a + chunk)
        d, _ = chunk_deltas(a, b)
        nw = _words(d)
        off = torch.cumsum(nw, 0) - nw
        out = torch.empty(int(bases[ci + 1] - bases[ci]), dtype=torch.int32, device=dev)
        for gi in range(5):
            sel = nw > gi
            wv = _lsr(d, 15 * gi) & 0x7FFF
            if gi == 0:
                wv = wv | 0x8000
            out[(off + nw - 1 - gi)[sel]] = wv[sel].int()
        out = torch.where(out >= 32768, out - 65536, out).to(torch.int16)
        diff[bases[ci]:bases[ci + 1]] = out.cpu().numpy().view(np.uint16)
        info[a:b] = rdb.info(a, b).cpu().numpy().view(np.uint32)
        for w in want:
            if a <= w < b:
                gpos[w] = bases[ci] + int(off[w - a].item())
            elif w == n and b == n:
                gpos[w] = W
        del d, nw, off, out
    for k, gv in enumerate(gs, start=1):
        if k >= split_num:
            break
        split[3 * k] = np.uint64(int(to_native_fmt2(rdb.values(gv, gv + 1)).item()) & ((1 << 64) - 1))
        split[3 * k + 1] = gpos[gv + 1]
        split[3 * k + 2] = gv + 1
    db.arrays = (diff, info, split)  # the host arrays, for mtb_open_host (bench: the GTDB-scale cold open)
    return db
