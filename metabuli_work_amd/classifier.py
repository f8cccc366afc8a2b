"""Host-side mirror of the reference's Classifier for the `classify` path.

Mirrors the reference interface (names, argument meaning, error behaviour):

* ``LocalParameters`` — the fields of LocalParameters.h:165-190 the path reads, with
  setClassifyDefaults (classify.cpp:10-37) and loadDbParameters (common.cpp:88-133);
* ``Classifier(par)`` — Classifier::Classifier (Classifier.cpp:6-32): loads the DB and makes it
  resident on the GPU through the C-ABI (mtb_open);
* ``Classifier.classify_batch`` — one QuerySplit of Classifier::startClassify (Classifier.cpp:
  81-133): extract, match, sort matches, assign, in one mtb_classify_batch call;
* ``Classifier.startClassify`` — the batch loop over FASTA/FASTQ inputs, writing the per-read
  TSV (Reporter::writeReadClassification, Reporter.cpp:38-83).

All compute runs in libmtbgpu.so (HIP); there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import dataclasses
import gzip
import os
from typing import Iterator, List, Optional, Tuple

import numpy as np

from . import _abi
from ._abi import KMER_DTYPE, MATCH_DTYPE, RESULT_DTYPE, TAXCNT_DTYPE, MtbParams, ptr
from ._lib import MtbError, check, lib


@dataclasses.dataclass
class LocalParameters:
    seqMode: int = 2
    kmerFormat: int = 1
    syncmer: int = 0
    smerLen: int = 5
    reducedAA: int = 0
    skipRedundancy: int = 0
    minScore: float = 0.0
    minSpScore: float = 0.0
    minConsCnt: int = 4
    minConsCntEuk: int = 9
    tieRatio: float = 0.95
    accessionLevel: int = 0
    em: int = 0
    threads: int = 1
    maskMode: int = 0
    maskProb: float = 0.9   # --mask-prob (classify.cpp:32)
    printLineage: int = 0   # --lineage: the TSV's lineage column (Reporter.cpp:41-43,59-61)
    filenames: List[str] = dataclasses.field(default_factory=list)

    def to_c(self) -> MtbParams:
        return MtbParams(seq_mode=self.seqMode, kmer_format=self.kmerFormat, syncmer=self.syncmer,
                         smer_len=self.smerLen, reduced_aa=self.reducedAA, skip_redundancy=self.skipRedundancy,
                         min_score=self.minScore, min_sp_score=self.minSpScore, min_cons_cnt=self.minConsCnt,
                         min_cons_cnt_euk=self.minConsCntEuk, tie_ratio=self.tieRatio,
                         accession_level=self.accessionLevel, em=self.em, threads=self.threads,
                         mask_mode=self.maskMode, mask_prob=self.maskProb)

    def load_db_parameters(self, db_dir: str) -> "LocalParameters":
        p = self.to_c()
        lib().mtb_load_db_parameters(db_dir.encode(), ctypes.byref(p))
        self.reducedAA, self.accessionLevel = p.reduced_aa, p.accession_level
        self.skipRedundancy, self.syncmer, self.smerLen = p.skip_redundancy, p.syncmer, p.smer_len
        self.kmerFormat = p.kmer_format
        return self


def setClassifyDefaults() -> LocalParameters:
    return LocalParameters()


def _after_torch(t) -> None:
    """Device tensors handed to the library were made on torch's current stream (or RCCL's, which
    torch's current stream waits for); the library runs on its own non-blocking stream, so that
    work must be complete before the call."""
    import torch
    torch.cuda.current_stream(t.device).synchronize()


@dataclasses.dataclass
class BatchResult:
    results: np.ndarray   # RESULT_DTYPE per read
    taxcnt: np.ndarray    # TAXCNT_DTYPE pooled
    query_kmers: int
    matches: int
    stage_ms: np.ndarray  # extract, k-mer sort, match, assign, total

    def taxcnt_of(self, i: int) -> List[Tuple[int, int]]:
        r = self.results[i]
        s = int(r["taxcnt_offset"])
        return [(int(t), int(c)) for t, c in self.taxcnt[s:s + int(r["taxcnt_len"])]]


@dataclasses.dataclass
class _DevBatch:
    """A batch classified in halves with its results left in HBM (Classifier._classify_halves_device):
    the assembled device arrays and the halves' work counts and device times."""
    results: object       # (n, 32) uint8 device tensor
    taxcnt: object        # (T, 8) uint8 device tensor
    query_kmers: int
    matches: int
    stats: dict
    stage_ms: np.ndarray
    kernel_ms: np.ndarray


class Classifier:
    """GPU-resident classifier; one instance per device (mirrors Classifier.cpp:6-32)."""

    def __init__(self, par: LocalParameters, db_dir: Optional[str] = None, device: int = 0,
                 db_host: Optional[_abi.MtbDbHost] = None, db_part: Tuple[int, int] = (0, 1), db_resident=None):
        """db_part = (part, parts): hold one AA-aligned k-mer range of a range-partitioned DB
        (see dist.classify_partitioned). db_resident: a DB already in HBM
        (gtdb_synth.ResidentDb), used in place (mtb_open_resident)."""
        self.par = par
        self.device = device
        self.db_part = db_part
        self.handle = ctypes.c_void_p()
        if db_resident is not None:
            self._resident = db_resident
            cp = par.to_c()
            cp.db_part, cp.db_parts = int(db_part[0]), int(db_part[1])  # a resident part of a partitioned DB
            check(lib().mtb_open_resident(ctypes.byref(db_resident.c_resident()),
                                          ctypes.byref(db_resident.host.c_struct()), ctypes.byref(cp), device,
                                          ctypes.byref(self.handle)), "mtb_open_resident")
            return
        if db_host is None and db_dir is None:
            db_dir = par.filenames[1 + (par.seqMode == 2)]
        if db_dir is not None:
            par.load_db_parameters(db_dir)
        cp = par.to_c()
        cp.db_part, cp.db_parts = int(db_part[0]), int(db_part[1])
        if db_host is not None:
            check(lib().mtb_open_host(ctypes.byref(db_host), ctypes.byref(cp), device, ctypes.byref(self.handle)),
                  "mtb_open_host")
        else:
            check(lib().mtb_open(db_dir.encode(), ctypes.byref(cp), device, ctypes.byref(self.handle)), "mtb_open")

    def close(self) -> None:
        self._dev_batch = None
        if self.handle:
            lib().mtb_close(self.handle)
            self.handle = ctypes.c_void_p()

    def clone(self) -> "Classifier":
        """A second classifier over the same DB on the same device (mtb_clone): own stream and batch
        workspace, the DB-derived arrays shared; as a startClassify peer it keeps two batches in
        flight on one GPU."""
        c = Classifier.__new__(Classifier)
        c.par, c.device, c.db_part = self.par, self.device, self.db_part
        c.handle = ctypes.c_void_p()
        if hasattr(self, "_resident"):
            c._resident = self._resident  # the caller-owned records stay alive with every holder
        check(lib().mtb_clone(self.handle, ctypes.byref(c.handle)), "mtb_clone")
        return c

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def db_kmers(self) -> int:
        return int(lib().mtb_db_kmers(self.handle))

    @property
    def workspace_bytes(self) -> int:
        """Device bytes of the batch workspace the context holds (mtb_workspace_bytes)."""
        return int(lib().mtb_workspace_bytes(self.handle))

    OPEN_PHASES = ["read_s", "decode_s", "directory_s", "probe_lines_s", "run_index_s", "taxonomy_s", "total_s",
                   "records_alloc_s"]

    def open_phases(self) -> dict:
        """Seconds of the context's open by phase (mtb_open_phases)."""
        out = (ctypes.c_double * len(self.OPEN_PHASES))()
        lib().mtb_open_phases(self.handle, out, len(self.OPEN_PHASES))
        return {k: round(float(v), 3) for k, v in zip(self.OPEN_PHASES, out)}

    def set_workspace_cap(self, nbytes: int) -> None:
        """Cap the batch workspace (0 = none): a batch past it is classified in pieces."""
        check(lib().mtb_set_workspace_cap(self.handle, int(nbytes)), "mtb_set_workspace_cap")

    def release_workspace(self) -> None:
        """Give the batch workspace back to the device (mtb_release_workspace); an assembled batch
        (_classify_halves_device) goes with it, so every getter sees the empty batch the C getters do."""
        self._dev_batch = None
        check(lib().mtb_release_workspace(self.handle), "mtb_release_workspace")

    def set_stream(self, stream_ptr: int) -> None:
        check(lib().mtb_set_stream(self.handle, ctypes.c_void_p(stream_ptr)), "mtb_set_stream")

    # -- one QuerySplit --------------------------------------------------------------------------
    def classify_batch(self, seq1: np.ndarray, off1: np.ndarray, seq2=None, off2=None, keep_stages: bool = False,
                       device_input: bool = False, fetch: bool = True, match_only: bool = False
                       ) -> Optional[BatchResult]:
        """match_only: stop after the join (MTB_MATCH_ONLY); fetch the per-read match segments with
        copy_matches and score them where the reads are owned (assign_chunks)."""
        n = (len(off1) - 1) if not device_input else int(off1.numel()) - 1
        flags = (_abi.MTB_KEEP_STAGES if keep_stages else 0) | (_abi.MTB_INPUT_DEVICE if device_input else 0)
        if match_only:
            flags |= _abi.MTB_MATCH_ONLY
            fetch = False
        if device_input:
            _after_torch(seq1)
            ptrs = [ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
                    for t in (seq1, off1, seq2, off2)]
        else:
            ptrs = [ptr(np.ascontiguousarray(a)) if a is not None else ctypes.c_void_p(0)
                    for a in (seq1, off1, seq2, off2)]
            self._keep = (seq1, off1, seq2, off2)
        res = np.zeros(n, RESULT_DTYPE) if fetch else None
        self._dev_batch = None  # a new batch: the context's own result buffers again
        rc = check(lib().mtb_classify_batch(self.handle, ptrs[0], ptrs[1], ptrs[2], ptrs[3], n, flags,
                                            ptr(res) if fetch else ctypes.c_void_p(0)), "mtb_classify_batch")
        if rc == _abi.MTB_RETRY:
            # out of HBM for the batch's workspace: Classifier.cpp:127-130 searches the split again
            # with a larger match buffer; here the batch is classified in halves
            if keep_stages or match_only or n < 2:
                raise MtbError(f"mtb_classify_batch: {lib().mtb_last_error().decode()}")
            if not fetch:  # results stay on the device: the halves' records and lists assembled there
                self._classify_halves_device(seq1, off1, seq2, off2, n, device_input)
                return None
            return self._classify_halves(seq1, off1, seq2, off2, n, device_input)
        if not fetch:
            return None
        return BatchResult(res, self.taxcnt(), *self.last_counts(), self.stage_ms())

    def _classify_halves_device(self, seq1, off1, seq2, off2, n, device_input) -> None:
        """classify_batch(fetch=False) past the workspace: the two halves (each split again if it
        still does not fit) are classified in turn and their result records and taxID:count lists
        copied device to device into buffers of this batch (the second half's list offsets rebased
        onto the pooled list), which copy_results / copy_taxcnt / n_taxcnt / last_counts then serve
        — the batch reads as one to the caller, as after an uncapped call."""
        import torch

        dev = torch.device("cuda", self.device)
        mid = n // 2
        recs, pools, qk, mm = [], [], 0, 0
        stats, stage, kern = None, np.zeros(5, np.float32), np.zeros(7, np.float32)
        for lo, hi in ((0, mid), (mid, n)):
            o1 = off1[lo:hi + 1]
            o2 = off2[lo:hi + 1] if off2 is not None else None
            self.classify_batch(seq1, o1, seq2, o2, device_input=device_input, fetch=False)
            rec = torch.empty((hi - lo, _abi.RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            self.copy_results(rec.data_ptr(), on_device=True)
            pool = torch.empty((max(self.n_taxcnt(), 1), _abi.TAXCNT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            nt = self.copy_taxcnt(pool.data_ptr(), on_device=True)
            q, m = self.last_counts()
            recs.append(rec)
            pools.append(pool[:nt])
            qk, mm = qk + q, mm + m
            # the batch's work counts and device times: the halves' summed (a batch maximum stays a
            # maximum, the join path and the unit layout are the last half's)
            st = self.stats()
            stats = st if stats is None else {k: (max(stats[k], v) if k == "max_read_matches" else
                                                  v if k in ("join_path", "uniform_units") else stats[k] + v)
                                              for k, v in st.items()}
            stage += self.stage_ms()
            kern += self.kernel_ms()
        recs[1].view(torch.int32).view(-1, _abi.RESULT_DTYPE.itemsize // 4)[:, 4] += pools[0].shape[0]
        torch.cuda.synchronize(dev)
        self._dev_batch = _DevBatch(torch.cat(recs), torch.cat(pools), qk, mm, stats, stage, kern)

    def _classify_halves(self, seq1, off1, seq2, off2, n, device_input) -> BatchResult:
        """The batch as two read ranges (offsets stay absolute into the same bases), each split
        again if it still does not fit; taxID:count lists concatenated with rebased offsets."""
        mid = n // 2
        parts = []
        for lo, hi in ((0, mid), (mid, n)):
            o1 = off1[lo:hi + 1]
            o2 = off2[lo:hi + 1] if off2 is not None else None
            parts.append(self.classify_batch(seq1, o1, seq2, o2, device_input=device_input))
        a, b = parts
        rb = b.results.copy()
        rb["taxcnt_offset"] += len(a.taxcnt)
        return BatchResult(np.concatenate([a.results, rb]), np.concatenate([a.taxcnt, b.taxcnt]),
                           a.query_kmers + b.query_kmers, a.matches + b.matches, a.stage_ms + b.stage_ms)

    def taxcnt(self) -> np.ndarray:
        if getattr(self, "_dev_batch", None) is not None:
            return self._dev_batch.taxcnt.cpu().numpy().reshape(-1).view(TAXCNT_DTYPE).copy()
        nt = ctypes.c_uint64(0)
        lib().mtb_get_taxcnt(self.handle, ctypes.c_void_p(0), 0, ctypes.byref(nt))
        tc = np.zeros(int(nt.value), TAXCNT_DTYPE)
        check(lib().mtb_get_taxcnt(self.handle, ptr(tc), len(tc), ctypes.byref(nt)), "mtb_get_taxcnt")
        return tc

    def last_counts(self) -> Tuple[int, int]:
        if getattr(self, "_dev_batch", None) is not None:
            return self._dev_batch.query_kmers, self._dev_batch.matches
        q, m = ctypes.c_uint64(0), ctypes.c_uint64(0)
        lib().mtb_last_counts(self.handle, ctypes.byref(q), ctypes.byref(m))
        return int(q.value), int(m.value)

    STATS = ["slots", "query_kmers", "matched_queries", "matches", "max_read_matches", "groups", "groups_ge2",
             "species_runs", "wave_runs", "wave_runs_emulated", "join_path", "live_matches", "gallop_queries",
             "spilled_matches", "long_run_queries", "filter_reruns", "db_records_read", "dup_aa_queries",
             "dup_key_queries", "uniform_units"]

    def stats(self) -> dict:
        """Work counts of the last batch (mtb_last_stats; a batch assembled from halves: their sums)."""
        if getattr(self, "_dev_batch", None) is not None:
            return dict(self._dev_batch.stats)
        out = (ctypes.c_uint64 * len(self.STATS))()
        lib().mtb_last_stats(self.handle, out, len(self.STATS))
        return {k: int(v) for k, v in zip(self.STATS, out)}

    def stage_ms(self) -> np.ndarray:
        if getattr(self, "_dev_batch", None) is not None:
            return self._dev_batch.stage_ms.copy()
        ms = (ctypes.c_float * 5)()
        lib().mtb_last_stage_ms(self.handle, ms, 5)
        return np.array(list(ms), np.float32)

    def kernel_ms(self) -> np.ndarray:
        """[extract, filter, k-mer sort, join, match transpose, match sort, assign] of the last batch
        (HIP events; the sort is 0 on the probe join; a batch assembled from halves: their sums)."""
        if getattr(self, "_dev_batch", None) is not None:
            return self._dev_batch.kernel_ms.copy()
        ms = (ctypes.c_float * 7)()
        lib().mtb_last_kernel_ms(self.handle, ms, 7)
        return np.array(list(ms), np.float32)

    def _copy_dev(self, t, dst_ptr: int, on_device: bool) -> None:
        """A batch assembled from halves (_classify_halves_device): its device tensor to dst."""
        import torch

        del on_device  # the runtime tells host from device pointers (unified addressing)
        if t.numel():
            torch.cuda.synchronize(t.device)
            check(lib().mtb_memcpy(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(t.data_ptr()), t.numel()), "mtb_memcpy")

    def copy_results(self, dst_ptr: int, on_device: bool = True) -> None:
        if getattr(self, "_dev_batch", None) is not None:
            return self._copy_dev(self._dev_batch.results, dst_ptr, on_device)
        check(lib().mtb_copy_results(self.handle, ctypes.c_void_p(dst_ptr), int(on_device)), "mtb_copy_results")

    def n_taxcnt(self) -> int:
        """Pooled taxID:count entries of the last batch."""
        if getattr(self, "_dev_batch", None) is not None:
            return int(self._dev_batch.taxcnt.shape[0])
        nt = ctypes.c_uint64(0)
        lib().mtb_get_taxcnt(self.handle, ctypes.c_void_p(0), 0, ctypes.byref(nt))
        return int(nt.value)

    def copy_taxcnt(self, dst_ptr: int, on_device: bool = True) -> int:
        """The last batch's pooled taxID:count entries to dst (8 B each); returns their number."""
        if getattr(self, "_dev_batch", None) is not None:
            self._copy_dev(self._dev_batch.taxcnt, dst_ptr, on_device)
            return int(self._dev_batch.taxcnt.shape[0])
        nt = ctypes.c_uint64(0)
        check(lib().mtb_copy_taxcnt(self.handle, ctypes.c_void_p(dst_ptr), int(on_device), ctypes.byref(nt)),
              "mtb_copy_taxcnt")
        return int(nt.value)

    def query_kmers(self) -> np.ndarray:
        """The query k-mers K4 consumed (those whose AA 8-mer the DB holds), after MTB_KEEP_STAGES."""
        q = self.stats()["query_kmers"]
        out = np.zeros(q, KMER_DTYPE)
        nq = ctypes.c_uint64(0)
        check(lib().mtb_get_query_kmers(self.handle, ptr(out), q, ctypes.byref(nq)), "mtb_get_query_kmers")
        return out

    def matches(self) -> np.ndarray:
        _, m = self.last_counts()
        out = np.zeros(m, MATCH_DTYPE)
        nm = ctypes.c_uint64(0)
        check(lib().mtb_get_matches(self.handle, ptr(out), m, ctypes.byref(nm)), "mtb_get_matches")
        return out

    def assign_matches(self, matches: np.ndarray, query_len: np.ndarray) -> BatchResult:
        matches = np.ascontiguousarray(matches, MATCH_DTYPE)
        ql = np.ascontiguousarray(query_len, np.uint32)
        res = np.zeros(len(ql), RESULT_DTYPE)
        check(lib().mtb_assign_matches(self.handle, ptr(matches), len(matches), ptr(ql), len(ql), ptr(res)),
              "mtb_assign_matches")
        return BatchResult(res, self.taxcnt(), 0, len(matches), self.stage_ms())

    # -- range-partitioned DB ------------------------------------------------------
    def copy_matches(self, matches=None, read_counts=None, query_len=None) -> None:
        """After classify_batch(match_only=True): per-read match segments, per-read counts and query
        lengths into numpy arrays or device tensors (all of one kind)."""
        arrs = [a for a in (matches, read_counts, query_len) if a is not None]
        on_dev = bool(arrs) and not isinstance(arrs[0], np.ndarray)

        def p(a):
            if a is None:
                return ctypes.c_void_p(0)
            return ctypes.c_void_p(a.data_ptr()) if on_dev else ptr(a)
        check(lib().mtb_copy_matches(self.handle, p(matches), p(read_counts), p(query_len), int(on_dev)),
              "mtb_copy_matches")

    def assign_chunks(self, matches, n_matches: int, chunk_counts, n_chunks: int, query_len, n_reads: int,
                      fetch: bool = True, keep_stages: bool = False) -> Optional[BatchResult]:
        """K5 + K6 on the all-to-all receive layout: n_chunks chunks, each grouped by read, with
        counts chunk_counts[c * n_reads + i]. numpy arrays (host) or device tensors. keep_stages:
        no dead-match pruning, so matches() returns every match afterwards."""
        on_dev = not isinstance(matches, np.ndarray)
        if on_dev:
            _after_torch(matches)
            ps = [ctypes.c_void_p(t.data_ptr()) for t in (matches, chunk_counts, query_len)]
        else:
            self._keep = tuple(np.ascontiguousarray(a) for a in (matches, chunk_counts, query_len))
            ps = [ptr(a) for a in self._keep]
        res = np.zeros(n_reads, RESULT_DTYPE) if fetch else None
        check(lib().mtb_assign_chunks(self.handle, ps[0], n_matches, ps[1], n_chunks, ps[2], n_reads,
                                      (_abi.MTB_INPUT_DEVICE if on_dev else 0) |
                                      (_abi.MTB_KEEP_STAGES if keep_stages else 0),
                                      ptr(res) if fetch else ctypes.c_void_p(0)), "mtb_assign_chunks")
        if not fetch:
            return None
        return BatchResult(res, self.taxcnt(), 0, n_matches, self.stage_ms())

    # -- Classifier::startClassify over files ----------------------------------------------------
    def original_taxid(self, tax_id: int) -> int:
        """TaxonomyWrapper::getOriginalTaxID: results hold internal taxIDs (taxonomyDB)."""
        return int(lib().mtb_original_taxid(self.handle, int(tax_id)))

    def lineage(self, tax_id: int) -> str:
        """TaxonomyWrapper::taxLineage2 of a taxID (the --lineage column)."""
        return lib().mtb_taxon_lineage(self.handle, int(tax_id)).decode()

    def write_report(self, path: str, total_reads: int, tax_counts: dict) -> None:
        """Reporter::writeReportFile (Reporter.cpp:175-190): the per-taxon report of a run from
        tax_counts = {classification taxID: reads} (++taxCounts[classification], Classifier.cpp:201-203)."""
        ids = np.fromiter(tax_counts.keys(), np.int32, len(tax_counts))
        cnt = np.fromiter(tax_counts.values(), np.uint32, len(tax_counts))
        check(lib().mtb_write_report(self.handle, path.encode(), total_reads, ptr(ids), ptr(cnt), len(ids)),
              "mtb_write_report")

    def em_mappings(self, query_offset: int = 0) -> np.ndarray:
        """The last batch's --em mappings (Reporter::writeMappings, Reporter.h:80-92): per classified
        read its <= 10 best species (std::sort order) with score^2, query_id = query_offset + index."""
        n = ctypes.c_uint64(0)
        rc = check(lib().mtb_get_em_mappings(self.handle, int(query_offset), None, 0, ctypes.byref(n)),
                   "mtb_get_em_mappings")
        out = np.zeros(n.value, _abi.EM_MAP_DTYPE)
        if rc == _abi.MTB_RETRY or n.value:
            check(lib().mtb_get_em_mappings(self.handle, int(query_offset), out.ctypes.data, len(out),
                                            ctypes.byref(n)), "mtb_get_em_mappings")
        return out

    def em(self, maps: np.ndarray, total_reads: int):
        """Classifier::em + reclassify (Classifier.cpp:209-386) on the device over all mappings.
        Returns (per-read EM_READ_DTYPE records, {species: (abundance, emTaxCount)}, stats dict)."""
        maps = np.ascontiguousarray(maps, _abi.EM_MAP_DTYPE)
        reads = np.zeros(max(int(total_reads), 1), _abi.EM_READ_DTYPE)
        cap = len(maps) + 1
        ids = np.zeros(cap, np.int32)
        probs = np.zeros(cap, np.float64)
        cnts = np.zeros(cap, np.uint32)
        nsp = ctypes.c_uint64(0)
        st = _abi.MtbEmStats()
        check(lib().mtb_em(self.handle, maps.ctypes.data if len(maps) else None, len(maps), int(total_reads),
                           reads.ctypes.data, ids.ctypes.data, probs.ctypes.data, cnts.ctypes.data, cap,
                           ctypes.byref(nsp), ctypes.byref(st)), "mtb_em")
        k = int(nsp.value)
        sp = {int(ids[i]): (float(probs[i]), int(cnts[i])) for i in range(k)}
        return reads[:int(total_reads)], sp, {f: getattr(st, f) for f, _ in _abi.MtbEmStats._fields_}

    def startClassify(self, out_tsv: str, reads_per_batch: int = 0, report_tsv: Optional[str] = None,
                      max_bases: int = 0, threads: int = 0, em_tsv: Optional[str] = None,
                      em_report_tsv: Optional[str] = None, em_reclassify_report_tsv: Optional[str] = None,
                      peers: Optional[List["Classifier"]] = None, partitioned: bool = False) -> int:
        """Classifier::startClassify (Classifier.cpp:44-164) through the native pipeline
        (mtb_start_classify): FASTA/FASTQ(.gz / BGZF) readers and parsers, pinned batches of at most
        reads_per_batch reads (0: 4M, in practice bounded by max_bases; the first five batches ramping up
        from 1/32 of that) and
        max_bases bases (0: sized from free HBM, the reference's
        RAM-bounded QuerySplits) uploaded on a copy stream, mtb_classify_batch, and the TSV writer
        (+ the per-taxon report, Classifier.cpp:149) overlapping each other; with --em (par.em) the
        EM reassignment after the last batch and its TSV / reports (Classifier.cpp:152-161). Returns
        the reads classified; the run's timings are left in self.last_run.

        peers: more classifiers over the same DB, one per further GPU (mtb_start_classify_multi):
        batch k runs on [self] + peers at k mod (1 + len(peers)), the output is the same files.
        partitioned: [self] + peers hold the parts of a range-partitioned DB (db_part = (p, P) in
        list order); every batch is matched by all of them and scored by the owners of its reads
        (mtb_start_classify_partitioned), the output is still the same files."""
        par = self.par
        opts = _abi.MtbClassifyOpts(
            query1=par.filenames[0].encode(), query2=par.filenames[1].encode() if par.seqMode == 2 else None,
            out_tsv=out_tsv.encode(), report_tsv=report_tsv.encode() if report_tsv else None,
            max_reads=int(reads_per_batch), write_flags=_abi.MTB_WRITE_LINEAGE if par.printLineage else 0,
            max_bases=int(max_bases), threads=int(threads),
            em_tsv=em_tsv.encode() if em_tsv else None, em_report_tsv=em_report_tsv.encode() if em_report_tsv else None,
            em_reclassify_report_tsv=em_reclassify_report_tsv.encode() if em_reclassify_report_tsv else None)
        st = _abi.MtbClassifyStats()
        if partitioned:
            hs = (ctypes.c_void_p * (1 + len(peers or [])))(self.handle, *[c.handle for c in peers or []])
            check(lib().mtb_start_classify_partitioned(hs, len(hs), ctypes.byref(opts), ctypes.byref(st)),
                  "mtb_start_classify_partitioned")
        elif peers:
            hs = (ctypes.c_void_p * (1 + len(peers)))(self.handle, *[c.handle for c in peers])
            check(lib().mtb_start_classify_multi(hs, len(hs), ctypes.byref(opts), ctypes.byref(st)),
                  "mtb_start_classify_multi")
        else:
            check(lib().mtb_start_classify(self.handle, ctypes.byref(opts), ctypes.byref(st)), "mtb_start_classify")
        self.last_run = {f: getattr(st, f) for f, _ in _abi.MtbClassifyStats._fields_}
        return int(st.reads)

    _rank_of = None


# --------------------------------------------------------------------------------------------------
# Host I/O. FastxReader wraps the native reader (mtb_reader_*, mtb_io.cpp) the product path uses;
# read_records / write_classifications below are an independent pure-Python restatement
# (KSeqWrapper semantics: name = header up to first whitespace; Reporter.cpp:38-83) kept for tests.
# --------------------------------------------------------------------------------------------------
class FastxReader:
    """Batches of reads from FASTA/FASTQ(.gz) (one file, or two mates in lock-step)."""

    def __init__(self, path1: str, path2: Optional[str] = None):
        self.h = ctypes.c_void_p()
        check(lib().mtb_reader_open(path1.encode(), path2.encode() if path2 else None, ctypes.byref(self.h)),
              "mtb_reader_open")

    def next(self, max_reads: int, max_bases: int = 1 << 62) -> _abi.MtbReadBatch:
        b = _abi.MtbReadBatch()
        check(lib().mtb_reader_next(self.h, max_reads, max_bases, ctypes.byref(b)), "mtb_reader_next")
        return b

    @staticmethod
    def arrays(b: _abi.MtbReadBatch):
        """Copies of a batch as (names, seq1, off1, seq2, off2) numpy/py objects."""
        n = b.n_reads
        o1 = np.ctypeslib.as_array(b.off1, (n + 1,)).copy()
        s1 = np.frombuffer(ctypes.string_at(b.seq1, int(o1[-1])), np.uint8).copy()
        s2 = o2 = None
        if b.seq2:
            o2 = np.ctypeslib.as_array(b.off2, (n + 1,)).copy()
            s2 = np.frombuffer(ctypes.string_at(b.seq2, int(o2[-1])), np.uint8).copy()
        no = np.ctypeslib.as_array(b.name_off, (n + 1,)).copy()
        raw = ctypes.string_at(b.names, int(no[-1]))
        names = [raw[no[i]:no[i + 1]].decode() for i in range(n)]
        return names, s1, o1, s2, o2

    def close(self):
        if self.h:
            lib().mtb_reader_close(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _open(path: str):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_records(path: str) -> Iterator[Tuple[bytes, bytes]]:
    with _open(path) as f:
        data = f.read()
    if not data:
        return
    if data[:1] == b">":
        for chunk in data[1:].split(b"\n>"):
            lines = chunk.split(b"\n")
            yield lines[0].split()[0] if lines[0].split() else b"", b"".join(l.strip() for l in lines[1:])
    else:
        lines = data.split(b"\n")
        for i in range(0, len(lines) - 3, 4):
            h = lines[i][1:].split()
            yield (h[0] if h else b""), lines[i + 1].strip()


def pack(seqs: List[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(seqs) + 1, np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    return np.frombuffer(b"".join(seqs), np.uint8).copy(), off


def read_batches(q1: str, q2: Optional[str], n: int):
    it1 = read_records(q1)
    it2 = read_records(q2) if q2 else None
    while True:
        names, a, b = [], [], []
        for rec in it1:
            names.append(rec[0].decode())
            a.append(rec[1])
            if it2 is not None:
                r2 = next(it2, None)
                if r2 is None:
                    raise MtbError("paired-end inputs have different read counts (QueryIndexer.cpp:121-124)")
                b.append(r2[1])
            if len(names) == n:
                break
        if not names:
            return
        s1, o1 = pack(a)
        s2, o2 = pack(b) if it2 is not None else (None, None)
        yield names, s1, o1, s2, o2
        if len(names) < n:
            return


def write_classifications(out, names: List[str], br: BatchResult, rank_of=None) -> None:
    res = br.results
    for i, nm in enumerate(names):
        r = res[i]
        score = "%g" % float(r["score"])
        if r["is_classified"]:
            rank = rank_of(int(r["classification"])) if rank_of else "-"
            tc = "".join(f"{t}:{c} " for t, c in br.taxcnt_of(i))
            out.write(f"1\t{nm}\t{int(r['classification'])}\t{int(r['query_length'])}\t{score}\t{rank}\t{tc}\n")
        else:
            out.write(f"0\t{nm}\t0\t{int(r['query_length'])}\t{score}\t-\t-\t\n")
