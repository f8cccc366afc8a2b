"""Reference-DB construction and in-memory DB handles.

``build_db`` runs the GPU builder (mtb_build_db, csrc/mtb_build.hip): genomes + gene blocks +
taxonomy -> diffIdx / info / split / taxID_list in the reference's on-disk format
(IndexCreator.cpp:316-376,811-886). ``HostDb`` keeps the arrays (and the numpy buffers the C
structs point into) alive, can write them as a DB directory, and yields the ``mtb_db_host``
struct that mtb_open_host / the oracle consume.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from ._abi import MTB_INPUT_DEVICE, MtbDbHost, MtbParams, ptr
from ._lib import check, lib


class MtbBuildInput(ctypes.Structure):
    _fields_ = [("seq", ctypes.c_void_p), ("off", ctypes.c_void_p), ("n_genomes", ctypes.c_uint32),
                ("genome_taxid", ctypes.c_void_p), ("blk_genome", ctypes.c_void_p), ("blk_start", ctypes.c_void_p),
                ("blk_end", ctypes.c_void_p), ("blk_strand", ctypes.c_void_p), ("n_blocks", ctypes.c_uint64),
                ("split_num", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class MtbDbBuilt(ctypes.Structure):
    _fields_ = [("diff_idx", ctypes.c_void_p), ("n_diff_idx", ctypes.c_uint64),
                ("info", ctypes.c_void_p), ("n_info", ctypes.c_uint64),
                ("split", ctypes.c_void_p), ("n_split", ctypes.c_uint64),
                ("taxid_list", ctypes.c_void_p), ("n_taxid_list", ctypes.c_uint64),
                ("dev_values", ctypes.c_void_p), ("dev_info", ctypes.c_void_p)]


MTB_BUILD_DEVICE_OUT = 8


def _pool(strings):
    enc = [s.encode() + b"\0" for s in strings]
    off = np.zeros(len(enc), np.uint64)
    if enc:
        off[1:] = np.cumsum([len(e) for e in enc[:-1]])
    return np.frombuffer(b"".join(enc) or b"\0", np.uint8).copy(), off


class HostDb:
    """A reference DB in host memory (diffIdx, info, split, taxID_list + taxonomy)."""

    def __init__(self, taxo, diff_idx=None, info=None, split=None, taxid_list=None):
        self.taxo = taxo
        self.diff_idx = diff_idx
        self.info = info
        self.split = split
        self.taxid_list = taxid_list
        self._rank_pool, self._rank_off = _pool(taxo.rank)
        self._name_pool, self._name_off = _pool(taxo.name)
        self._node_taxid = np.ascontiguousarray(taxo.taxid, np.int32)
        self._node_parent = np.ascontiguousarray(taxo.parent, np.int32)

    def c_struct(self) -> MtbDbHost:
        h = MtbDbHost()
        h.node_taxid, h.node_parent, h.n_nodes = ptr(self._node_taxid), ptr(self._node_parent), len(self._node_taxid)
        h.rank_pool, h.rank_off = ptr(self._rank_pool), ptr(self._rank_off)
        h.name_pool, h.name_off = ptr(self._name_pool), ptr(self._name_off)
        h.merged_old = h.merged_new = None
        h.n_merged = 0
        if self.diff_idx is not None:
            h.diff_idx, h.n_diff_idx = ptr(self.diff_idx), len(self.diff_idx)
            h.info, h.n_info = ptr(self.info), len(self.info)
            h.split, h.n_split = ptr(self.split), len(self.split) // 3
        if self.taxid_list is not None:
            h.taxid_list, h.n_taxid_list = ptr(self.taxid_list), len(self.taxid_list)
        return h

    @property
    def n_kmers(self) -> int:
        return 0 if self.info is None else len(self.info)

    @property
    def nbytes(self) -> int:
        return int(self.diff_idx.nbytes + self.info.nbytes)

    def write(self, directory: str, par: MtbParams) -> None:
        """Write a DB directory the reference's classify (and mtb_open) can read."""
        os.makedirs(directory, exist_ok=True)
        self.diff_idx.tofile(os.path.join(directory, "diffIdx"))
        self.info.tofile(os.path.join(directory, "info"))
        self.split.tofile(os.path.join(directory, "split"))
        with open(os.path.join(directory, "taxID_list"), "w") as f:
            f.write("".join(f"{t}\n" for t in self.taxid_list.tolist()))
        with open(os.path.join(directory, "db.parameters"), "w") as f:  # writeDbParameters
            f.write("DB_name\tsynthetic\nCreation_date\t1970-01-01\nMetabuli commit used to create the DB\tmtb-gpu\n")
            f.write(f"Reduced_alphabet\t{par.reduced_aa}\nAccession_level\t{par.accession_level}\n")
            f.write("Mask_mode\t0\nMask_prob\t0.900000\nSkip_redundancy\t1\n")
            f.write(f"Syncmer\t{par.syncmer}\n")
            if par.syncmer == 1:
                f.write(f"Syncmer_len\t{par.smer_len}\n")
            f.write(f"Kmer_format\t{par.kmer_format}\n")
        self.taxo.write_dmp(os.path.join(directory, "taxonomy"))


def _build_input(gen, device_seq, split_num, flags):
    inp = MtbBuildInput()
    if device_seq is not None:
        inp.seq, inp.off = device_seq[0].data_ptr(), device_seq[1].data_ptr()
        inp.flags = MTB_INPUT_DEVICE | flags
    else:
        inp.seq, inp.off = ptr(gen.seq).value, ptr(gen.off).value
        inp.flags = flags
    keep = [np.ascontiguousarray(a, np.int32) for a in (gen.taxid, gen.blk_genome, gen.blk_start, gen.blk_end,
                                                         gen.blk_strand)]
    inp.n_genomes = len(gen.taxid)
    inp.genome_taxid, inp.blk_genome, inp.blk_start, inp.blk_end, inp.blk_strand = [a.ctypes.data for a in keep]
    inp.n_blocks = len(keep[1])
    inp.split_num = split_num
    return inp, keep


def _lib_build():
    L = lib()
    L.mtb_build_db.argtypes = [ctypes.POINTER(MtbBuildInput), ctypes.POINTER(MtbDbHost), ctypes.POINTER(MtbParams),
                               ctypes.c_int, ctypes.POINTER(MtbDbBuilt)]
    L.mtb_free_built.argtypes = [ctypes.POINTER(MtbDbBuilt)]
    return L


def build_db(gen, taxo, par: MtbParams, device: int = 0, split_num: int = 4096, device_seq=None) -> HostDb:
    """Build the reference DB on the GPU. ``device_seq`` = (seq, off) torch tensors already in HBM
    (bench path); otherwise ``gen.seq`` / ``gen.off`` are uploaded."""
    hdb = HostDb(taxo)
    inp, keep = _build_input(gen, device_seq, split_num, 0)
    out = MtbDbBuilt()
    L = _lib_build()
    tax_struct = hdb.c_struct()
    check(L.mtb_build_db(ctypes.byref(inp), ctypes.byref(tax_struct), ctypes.byref(par), device, ctypes.byref(out)),
          "mtb_build_db")
    try:
        def arr(p, n, dt):
            if n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(n,)).copy()
        hdb.diff_idx = arr(out.diff_idx, out.n_diff_idx, np.uint16)
        hdb.info = arr(out.info, out.n_info, np.uint32)
        hdb.split = arr(out.split, 3 * out.n_split, np.uint64)
        hdb.taxid_list = arr(out.taxid_list, out.n_taxid_list, np.int32)
    finally:
        L.mtb_free_built(ctypes.byref(out))
    return hdb


_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch (and libmtbgpu) already use
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return _HIP


def build_db_device(gen, taxo, par: MtbParams, device: int = 0, device_seq=None):
    """Build the reference DB on the GPU and keep it there (MTB_BUILD_DEVICE_OUT): returns torch
    tensors (values in resident rank form int64, taxIDs int32), deduplicated and sorted."""
    import torch

    inp, keep = _build_input(gen, device_seq, 4096, MTB_BUILD_DEVICE_OUT)
    out = MtbDbBuilt()
    L = _lib_build()
    htax = HostDb(taxo)  # keeps the arrays the struct points into alive
    tax_struct = htax.c_struct()
    check(L.mtb_build_db(ctypes.byref(inp), ctypes.byref(tax_struct), ctypes.byref(par), device, ctypes.byref(out)),
          "mtb_build_db")
    try:
        n = int(out.n_info)
        dev = torch.device("cuda", device)
        v = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        t = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        if n:
            H = _hip()
            if H.hipMemcpy(v.data_ptr(), out.dev_values, 8 * n, 3) or H.hipMemcpy(t.data_ptr(), out.dev_info, 4 * n, 3):
                raise RuntimeError("hipMemcpy of the built DB failed")
    finally:
        L.mtb_free_built(ctypes.byref(out))
    return v[:n], t[:n]
