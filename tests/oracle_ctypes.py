"""ctypes wrapper of the oracle (oracle/liboracle.so) — the parity checker. Test-side only."""
import ctypes
import os
import pathlib
import subprocess

import numpy as np

from metabuli_work_amd._abi import (KMER_DTYPE, MATCH_DTYPE, MTB_OK, MTB_RETRY, RESULT_DTYPE, TAXCNT_DTYPE,
                                    MtbParams, ptr)

ROOT = pathlib.Path(__file__).resolve().parents[1]
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        so = ROOT / "oracle" / "liboracle.so"
        if not so.exists():
            subprocess.run(["make", "-C", str(ROOT / "oracle"), "liboracle.so"], check=True, capture_output=True)
        L = ctypes.CDLL(str(so))
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        L.orc_db_open.restype = vp
        L.orc_db_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, i32]
        L.orc_db_open_host.restype = vp
        L.orc_db_open_host.argtypes = [vp, ctypes.c_char_p, i32]
        L.orc_db_new.restype = vp
        L.orc_db_new.argtypes = [vp, u64, u64, u64, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                 ctypes.c_char_p, i32]
        L.orc_db_close.argtypes = [vp]
        L.orc_db_kmers.restype = u64
        L.orc_db_kmers.argtypes = [vp]
        L.orc_load_db_parameters.argtypes = [ctypes.c_char_p, ctypes.POINTER(MtbParams)]
        L.orc_db_build.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(MtbParams), vp, vp, u32, vp, vp,
                                   vp, vp, vp, u64, i32, ctypes.c_char_p, i32]
        L.orc_extract.argtypes = [ctypes.POINTER(MtbParams), vp, vp, vp, vp, u32, i32, vp, u64,
                                  ctypes.POINTER(u64), vp, vp]
        L.orc_match.argtypes = [vp, ctypes.POINTER(MtbParams), vp, u64, vp, u64, ctypes.POINTER(u64),
                                ctypes.c_char_p, i32]
        L.orc_sort_matches.argtypes = [vp, u64]
        L.orc_assign.argtypes = [vp, ctypes.POINTER(MtbParams), vp, u64, vp, vp, u32, vp, vp, u64,
                                 ctypes.POINTER(u64)]
        L.orc_classify.argtypes = [vp, ctypes.POINTER(MtbParams), vp, vp, vp, vp, u32, vp, vp, u64,
                                   ctypes.POINTER(u64), vp, vp, ctypes.c_char_p, i32]
        L.orc_set_threads.argtypes = [i32]
        L.orc_threads.restype = i32
        L.orc_genetic_tables.argtypes = [vp, vp, vp, vp]
        L.orc_hamming_tables.argtypes = [vp, vp]
        L.orc_hamming_tables.restype = None
        L.orc_hamming.argtypes = [vp, vp, u64, vp, vp, vp]
        L.orc_pin_eval.argtypes = [ctypes.c_int, vp, vp, vp, u64, vp, vp]
        L.orc_pin_write_db.argtypes = [vp, vp, u64, ctypes.c_int, vp, vp, vp, vp]
        L.orc_hamming.restype = None
        L.orc_write_report.argtypes = [vp, ctypes.c_char_p, i32, vp, vp, u64]
        L.orc_write_report.restype = i32
        L.orc_last_em_maps.argtypes = [vp, u64, ctypes.POINTER(u64)]
        L.orc_em.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp, u64, ctypes.POINTER(u64), vp]
        L.orc_tantan.argtypes = [vp, vp, u32, ctypes.c_float, vp, vp]
        L.orc_tantan.restype = None
        _LIB = L
    return _LIB


def tantan(seq: np.ndarray, off: np.ndarray, mask_prob: float = 0.9):
    """SeqIterator::maskLowComplexityRegions of every read (the oracle's tantan restatement): the
    masked bases and tantan's per-letter repeat probabilities."""
    seq = np.ascontiguousarray(seq, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    out = np.zeros(len(seq), np.uint8)
    probs = np.zeros(len(seq), np.float32)
    lib().orc_tantan(ptr(seq), ptr(off), len(off) - 1, float(mask_prob), ptr(out), ptr(probs))
    return out, probs


def load_db_parameters(db_dir: str, par: MtbParams) -> MtbParams:
    lib().orc_load_db_parameters(db_dir.encode(), ctypes.byref(par))
    return par


def build_db(out_dir: str, par: MtbParams, taxo, gen, split_num: int = 4096) -> None:
    """Write a reference-format DB (diffIdx/info/split/taxID_list/db.parameters/taxonomy)."""
    os.makedirs(out_dir, exist_ok=True)
    tax_dir = os.path.join(out_dir, "taxonomy")
    taxo.write_dmp(tax_dir)
    err = ctypes.create_string_buffer(512)
    rc = lib().orc_db_build(out_dir.encode(), tax_dir.encode(), ctypes.byref(par), ptr(gen.seq), ptr(gen.off),
                            gen.n, ptr(gen.taxid), ptr(gen.blk_genome), ptr(gen.blk_start), ptr(gen.blk_end),
                            ptr(gen.blk_strand), len(gen.blk_genome), split_num, err, 512)
    if rc != MTB_OK:
        raise RuntimeError(err.value.decode())


class OracleDb:
    def __init__(self, db_dir: str = None, host_struct=None):
        err = ctypes.create_string_buffer(512)
        if host_struct is not None:
            self.h = lib().orc_db_open_host(ctypes.byref(host_struct), err, 512)
        else:
            self.h = lib().orc_db_open(db_dir.encode(), err, 512)
        if not self.h:
            raise RuntimeError(err.value.decode())

    @classmethod
    def from_host(cls, host_struct):
        return cls(host_struct=host_struct)

    @classmethod
    def fillable(cls, host_struct, n_diff: int, n_info: int, n_split: int):
        """A DB whose diffIdx / info / split the caller writes in place: returns (db, diff, info, split)
        with numpy views of the oracle's own buffers (no second host copy of a large DB)."""
        err = ctypes.create_string_buffer(512)
        pd, pi, ps = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        h = lib().orc_db_new(ctypes.byref(host_struct), n_diff, n_info, n_split, ctypes.byref(pd), ctypes.byref(pi),
                             ctypes.byref(ps), err, 512)
        if not h:
            raise RuntimeError(err.value.decode())
        db = cls.__new__(cls)
        db.h = h

        def view(p, n, t):
            if n == 0:
                return np.zeros(0, t)
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(t))), shape=(n,))
        return db, view(pd, n_diff, np.uint16), view(pi, n_info, np.uint32), view(ps, 3 * n_split, np.uint64)

    @property
    def n_kmers(self) -> int:
        return int(lib().orc_db_kmers(self.h))

    def close(self):
        if self.h:
            lib().orc_db_close(self.h)
            self.h = None

    def __del__(self):
        self.close()


def extract(par: MtbParams, reads, sort: bool = True):
    """Reference query-k-mer buffer (reserved slots, blanks = {0,0}) and per-read queryLength(2)."""
    n = reads.n
    ql1 = np.zeros(n, np.uint32)
    ql2 = np.zeros(n, np.uint32)
    nout = ctypes.c_uint64(0)
    cap = 1
    while True:
        out = np.zeros(cap, KMER_DTYPE)
        rc = lib().orc_extract(ctypes.byref(par), ptr(reads.seq1), ptr(reads.off1), ptr(reads.seq2),
                               ptr(reads.off2), n, int(sort), ptr(out), cap, ctypes.byref(nout), ptr(ql1), ptr(ql2))
        if rc == MTB_RETRY:
            cap = int(nout.value)
            continue
        return out[:nout.value], ql1, ql2


def match(db: OracleDb, par: MtbParams, kmers: np.ndarray, sort: bool = True) -> np.ndarray:
    kmers = np.ascontiguousarray(kmers)
    nout = ctypes.c_uint64(0)
    err = ctypes.create_string_buffer(512)
    cap = max(16, len(kmers))
    while True:
        out = np.zeros(cap, MATCH_DTYPE)
        rc = lib().orc_match(db.h, ctypes.byref(par), ptr(kmers), len(kmers), ptr(out), cap, ctypes.byref(nout),
                             err, 512)
        if rc == MTB_RETRY:
            cap = int(nout.value)
            continue
        if rc != MTB_OK:
            raise RuntimeError(err.value.decode())
        out = out[:nout.value].copy()
        if sort:
            lib().orc_sort_matches(ptr(out), len(out))
        return out


def _results(n_reads, call):
    res = np.zeros(n_reads, RESULT_DTYPE)
    cap = max(16, n_reads * 4)
    ntc = ctypes.c_uint64(0)
    while True:
        tc = np.zeros(cap, TAXCNT_DTYPE)
        rc = call(res, tc, cap, ntc)
        if rc == MTB_RETRY:
            cap = int(ntc.value)
            continue
        if rc != MTB_OK:
            raise RuntimeError(f"oracle returned {rc}")
        return res, tc[:ntc.value].copy()


def assign(db: OracleDb, par: MtbParams, matches: np.ndarray, ql1: np.ndarray, ql2: np.ndarray):
    matches = np.ascontiguousarray(matches)
    n = len(ql1)
    return _results(n, lambda res, tc, cap, ntc: lib().orc_assign(
        db.h, ctypes.byref(par), ptr(matches), len(matches), ptr(ql1), ptr(ql2), n, ptr(res), ptr(tc), cap,
        ctypes.byref(ntc)))


def classify(db: OracleDb, par: MtbParams, reads, stage_s=None, counts=None):
    stage = np.zeros(4, np.float64)
    cnt = np.zeros(2, np.uint64)
    err = ctypes.create_string_buffer(512)
    out = _results(reads.n, lambda res, tc, cap, ntc: lib().orc_classify(
        db.h, ctypes.byref(par), ptr(reads.seq1), ptr(reads.off1), ptr(reads.seq2), ptr(reads.off2), reads.n,
        ptr(res), ptr(tc), cap, ctypes.byref(ntc), ptr(stage), ptr(cnt), err, 512))
    if stage_s is not None:
        stage_s[:] = stage
    if counts is not None:
        counts[:] = cnt
    return out


def write_report(db: OracleDb, path: str, total_reads: int, tax_counts: dict) -> None:
    """Reporter::writeReportFile's per-taxon TSV (oracle/orc_reporter.cpp)."""
    ids = np.fromiter(tax_counts.keys(), np.int32, len(tax_counts))
    cnt = np.fromiter(tax_counts.values(), np.uint32, len(tax_counts))
    if lib().orc_write_report(db.h, path.encode(), total_reads, ids.ctypes.data, cnt.ctypes.data, len(ids)) != 0:
        raise RuntimeError("orc_write_report failed")


def last_em_maps():
    """The last classify/assign call's --em mappings (read indices of that batch)."""
    from metabuli_work_amd import _abi
    n = ctypes.c_uint64(0)
    lib().orc_last_em_maps(None, 0, ctypes.byref(n))
    out = np.zeros(n.value, _abi.EM_MAP_DTYPE)
    if n.value:
        lib().orc_last_em_maps(out.ctypes.data, len(out), ctypes.byref(n))
    return out


def em(db, maps, total_reads):
    """Classifier::em + reclassify restated on one thread (oracle/orc_taxonomer.cpp)."""
    from metabuli_work_amd import _abi
    maps = np.ascontiguousarray(maps, _abi.EM_MAP_DTYPE)
    reads = np.zeros(max(int(total_reads), 1), _abi.EM_READ_DTYPE)
    cap = len(maps) + 1
    ids = np.zeros(cap, np.int32)
    probs = np.zeros(cap, np.float64)
    cnts = np.zeros(cap, np.uint32)
    nsp = ctypes.c_uint64(0)
    st = np.zeros(2, np.uint64)
    rc = lib().orc_em(db.h, maps.ctypes.data if len(maps) else None, len(maps), int(total_reads), reads.ctypes.data,
                      ids.ctypes.data, probs.ctypes.data, cnts.ctypes.data, cap, ctypes.byref(nsp), st.ctypes.data)
    if rc != 0:
        raise RuntimeError("orc_em failed")
    k = int(nsp.value)
    sp = {int(ids[i]): (float(probs[i]), int(cnts[i])) for i in range(k)}
    return reads[:int(total_reads)], sp, {"query_count": int(st[0]), "iterations": int(st[1])}
