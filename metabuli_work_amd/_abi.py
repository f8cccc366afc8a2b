"""ctypes / numpy mirrors of the plain-data structs in include/mtb_gpu.h."""
import ctypes

import numpy as np


class MtbParams(ctypes.Structure):
    _fields_ = [
        ("seq_mode", ctypes.c_int32),
        ("kmer_format", ctypes.c_int32),
        ("syncmer", ctypes.c_int32),
        ("smer_len", ctypes.c_int32),
        ("reduced_aa", ctypes.c_int32),
        ("skip_redundancy", ctypes.c_int32),
        ("min_score", ctypes.c_float),
        ("min_sp_score", ctypes.c_float),
        ("min_cons_cnt", ctypes.c_int32),
        ("min_cons_cnt_euk", ctypes.c_int32),
        ("tie_ratio", ctypes.c_float),
        ("accession_level", ctypes.c_int32),
        ("em", ctypes.c_int32),
        ("threads", ctypes.c_int32),
        ("mask_mode", ctypes.c_int32),
        ("db_part", ctypes.c_int32),
        ("db_parts", ctypes.c_int32),
        ("mask_prob", ctypes.c_float),
    ]


class MtbDbHost(ctypes.Structure):
    _fields_ = [
        ("diff_idx", ctypes.c_void_p), ("n_diff_idx", ctypes.c_uint64),
        ("info", ctypes.c_void_p), ("n_info", ctypes.c_uint64),
        ("split", ctypes.c_void_p), ("n_split", ctypes.c_uint64),
        ("taxid_list", ctypes.c_void_p), ("n_taxid_list", ctypes.c_uint64),
        ("node_taxid", ctypes.c_void_p), ("node_parent", ctypes.c_void_p), ("n_nodes", ctypes.c_uint64),
        ("rank_pool", ctypes.c_void_p), ("rank_off", ctypes.c_void_p),
        ("name_pool", ctypes.c_void_p), ("name_off", ctypes.c_void_p),
        ("merged_old", ctypes.c_void_p), ("merged_new", ctypes.c_void_p), ("n_merged", ctypes.c_uint64),
    ]


class MtbDbResident(ctypes.Structure):
    _fields_ = [("records", ctypes.c_void_p), ("n_kmers", ctypes.c_uint64),
                ("rank_form", ctypes.c_int32), ("reserved", ctypes.c_int32)]


KMER_DTYPE = np.dtype([("value", "<u8"), ("info", "<u8")])
MATCH_DTYPE = np.dtype([("qinfo", "<u8"), ("target_id", "<u4"), ("species_id", "<u4"), ("dna_encoding", "<u4"),
                        ("right_end_hamming", "<u2"), ("hamming", "u1"), ("pad", "u1")])
RESULT_DTYPE = np.dtype([("classification", "<i4"), ("score", "<f4"), ("hamming_dist", "<i4"),
                         ("query_length", "<u4"), ("taxcnt_offset", "<u4"), ("taxcnt_len", "<u4"),
                         ("is_classified", "u1"), ("pad", "u1", (7,))])
TAXCNT_DTYPE = np.dtype([("tax_id", "<i4"), ("count", "<u4")])

assert KMER_DTYPE.itemsize == 16 and MATCH_DTYPE.itemsize == 24
assert RESULT_DTYPE.itemsize == 32 and TAXCNT_DTYPE.itemsize == 8

MTB_OK, MTB_RETRY = 0, 1
MTB_INPUT_DEVICE, MTB_KEEP_STAGES, MTB_MATCH_ONLY = 1, 2, 4
MTB_WRITE_LINEAGE = 1  # mtb_write_classifications flags


def default_params(**kw) -> MtbParams:
    """setClassifyDefaults (classify.cpp:10-37)."""
    p = MtbParams(seq_mode=2, kmer_format=1, syncmer=0, smer_len=5, reduced_aa=0, skip_redundancy=0,
                  min_score=0.0, min_sp_score=0.0, min_cons_cnt=4, min_cons_cnt_euk=9, tie_ratio=0.95,
                  accession_level=0, em=0, threads=1, mask_mode=0, mask_prob=0.9)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def ptr(a) -> ctypes.c_void_p:
    if a is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(a.ctypes.data)


def info_seq(info):
    return (np.asarray(info, np.uint64) >> np.uint64(32)) & np.uint64(0x1FFFFFFF)


def info_frame(info):
    return np.asarray(info, np.uint64) >> np.uint64(61)


def info_pos(info):
    return np.asarray(info, np.uint64) & np.uint64(0xFFFFFFFF)


class MtbReadBatch(ctypes.Structure):
    """mtb_read_batch (include/mtb_gpu.h): one batch from mtb_reader_next."""
    _fields_ = [
        ("n_reads", ctypes.c_uint32),
        ("seq1", ctypes.c_void_p),
        ("off1", ctypes.POINTER(ctypes.c_uint64)),
        ("seq2", ctypes.c_void_p),
        ("off2", ctypes.POINTER(ctypes.c_uint64)),
        ("names", ctypes.c_void_p),
        ("name_off", ctypes.POINTER(ctypes.c_uint64)),
    ]


class MtbClassifyOpts(ctypes.Structure):
    _fields_ = [("query1", ctypes.c_char_p), ("query2", ctypes.c_char_p), ("out_tsv", ctypes.c_char_p),
                ("report_tsv", ctypes.c_char_p), ("max_reads", ctypes.c_uint32), ("write_flags", ctypes.c_uint32),
                ("max_bases", ctypes.c_uint64), ("threads", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("em_tsv", ctypes.c_char_p), ("em_report_tsv", ctypes.c_char_p),
                ("em_reclassify_report_tsv", ctypes.c_char_p)]


class MtbClassifyStats(ctypes.Structure):
    _fields_ = [("reads", ctypes.c_uint64), ("bases", ctypes.c_uint64), ("batches", ctypes.c_uint64),
                ("wall_s", ctypes.c_double), ("gpu_s", ctypes.c_double), ("input_wait_s", ctypes.c_double),
                ("write_s", ctypes.c_double), ("source_s", ctypes.c_double), ("scan_s", ctypes.c_double),
                ("parse_s", ctypes.c_double), ("fill_s", ctypes.c_double), ("first_batch_s", ctypes.c_double),
                ("split_batches", ctypes.c_uint64)]


# --em (include/mtb_gpu.h): MappingRes (common.h:24-28), the reassignment of one read, EM stats
EM_MAP_DTYPE = np.dtype([("query_id", "<u4"), ("species_id", "<i4"), ("score", "<f4")])
EM_READ_DTYPE = np.dtype([("tax_id", "<i4"), ("mapped", "<i4"), ("score", "<f8")])


class MtbEmStats(ctypes.Structure):
    _fields_ = [("query_count", ctypes.c_uint64), ("iterations", ctypes.c_uint32), ("n_species", ctypes.c_uint32),
                ("delta", ctypes.c_double)]
