"""Loader for libmtbgpu.so — the C-ABI of include/mtb_gpu.h.

The product path has no CPU fallback: if the HIP library is missing or fails to load, every
entry point raises. Build it with `python -c "import __graft_entry__ as g; g.build()"` or
`make -C metabuli_work_amd/csrc`.
"""
import ctypes
import pathlib

from ._abi import MtbClassifyOpts, MtbClassifyStats, MtbDbHost, MtbDbResident, MtbEmStats, MtbParams, MtbReadBatch

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = _HERE / "libmtbgpu.so"
_LIB = None

# Every symbol include/mtb_gpu.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "mtb_default_params", "mtb_load_db_parameters", "mtb_open", "mtb_open_host", "mtb_close", "mtb_last_error",
    "mtb_set_stream", "mtb_db_kmers", "mtb_classify_batch", "mtb_get_taxcnt", "mtb_device_results",
    "mtb_clone", "mtb_last_counts", "mtb_last_stats", "mtb_last_stage_ms", "mtb_last_kernel_ms", "mtb_copy_results", "mtb_get_query_kmers",
    "mtb_get_matches", "mtb_assign_matches", "mtb_build_db", "mtb_free_built", "mtb_reader_open", "mtb_reader_next",
    "mtb_reader_close", "mtb_taxon_rank", "mtb_write_classifications", "mtb_partition_bounds", "mtb_copy_matches",
    "mtb_assign_chunks", "mtb_open_resident", "mtb_write_report", "mtb_copy_taxcnt", "mtb_original_taxid",
    "mtb_taxon_lineage", "mtb_start_classify", "mtb_get_em_mappings", "mtb_em", "mtb_write_em_results",
    "mtb_ctx_device", "mtb_start_classify_multi", "mtb_mask_reads", "mtb_workspace_bytes", "mtb_set_workspace_cap",
    "mtb_open_phases", "mtb_start_classify_partitioned", "mtb_release_workspace", "mtb_hamming", "mtb_memcpy",
    "mtb_line_ext_check", "mtb_link_check", "mtb_pin_eval", "mtb_sort_pairs",
]


class MtbError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise MtbError(f"{LIB_PATH} not built: the HIP extension is required (no CPU fallback)")
    L = ctypes.CDLL(str(LIB_PATH))
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    P = ctypes.POINTER
    L.mtb_default_params.argtypes = [P(MtbParams)]
    L.mtb_default_params.restype = None
    L.mtb_load_db_parameters.argtypes = [ctypes.c_char_p, P(MtbParams)]
    L.mtb_open.argtypes = [ctypes.c_char_p, P(MtbParams), i32, P(vp)]
    L.mtb_open_host.argtypes = [P(MtbDbHost), P(MtbParams), i32, P(vp)]
    L.mtb_open_resident.argtypes = [P(MtbDbResident), P(MtbDbHost), P(MtbParams), i32, P(vp)]
    L.mtb_close.argtypes = [vp]
    L.mtb_clone.argtypes = [vp, P(vp)]
    L.mtb_close.restype = None
    L.mtb_last_error.restype = ctypes.c_char_p
    L.mtb_set_stream.argtypes = [vp, vp]
    L.mtb_db_kmers.argtypes = [vp]
    L.mtb_db_kmers.restype = u64
    L.mtb_workspace_bytes.argtypes = [vp]
    L.mtb_workspace_bytes.restype = u64
    L.mtb_set_workspace_cap.argtypes = [vp, u64]
    L.mtb_release_workspace.argtypes = [vp]
    L.mtb_open_phases.argtypes = [vp, P(ctypes.c_double), i32]
    L.mtb_classify_batch.argtypes = [vp, vp, vp, vp, vp, u32, u32, vp]
    L.mtb_get_taxcnt.argtypes = [vp, vp, u64, P(u64)]
    L.mtb_device_results.argtypes = [vp, P(vp), P(vp), P(u64)]
    L.mtb_last_counts.argtypes = [vp, P(u64), P(u64)]
    L.mtb_last_stats.argtypes = [vp, P(u64), i32]
    L.mtb_last_stage_ms.argtypes = [vp, P(ctypes.c_float), i32]
    L.mtb_last_kernel_ms.argtypes = [vp, P(ctypes.c_float), i32]
    L.mtb_copy_results.argtypes = [vp, vp, i32]
    L.mtb_copy_taxcnt.argtypes = [vp, vp, i32, P(u64)]
    L.mtb_get_query_kmers.argtypes = [vp, vp, u64, P(u64)]
    L.mtb_get_matches.argtypes = [vp, vp, u64, P(u64)]
    L.mtb_assign_matches.argtypes = [vp, vp, u64, vp, u32, vp]
    L.mtb_partition_bounds.argtypes = [vp, u64, u64, i32, vp, vp]
    L.mtb_copy_matches.argtypes = [vp, vp, vp, vp, i32]
    L.mtb_assign_chunks.argtypes = [vp, vp, u64, vp, u32, vp, u32, u32, vp]
    L.mtb_reader_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, P(vp)]
    L.mtb_reader_next.argtypes = [vp, u32, u64, P(MtbReadBatch)]
    L.mtb_reader_close.argtypes = [vp]
    L.mtb_reader_close.restype = None
    L.mtb_taxon_rank.argtypes = [vp, ctypes.c_int32]
    L.mtb_taxon_rank.restype = ctypes.c_char_p
    L.mtb_write_classifications.argtypes = [vp, ctypes.c_char_p, i32, P(MtbReadBatch), vp, vp, u32]
    L.mtb_original_taxid.argtypes = [vp, ctypes.c_int32]
    L.mtb_original_taxid.restype = ctypes.c_int32
    L.mtb_taxon_lineage.argtypes = [vp, ctypes.c_int32]
    L.mtb_taxon_lineage.restype = ctypes.c_char_p
    L.mtb_start_classify.argtypes = [vp, P(MtbClassifyOpts), P(MtbClassifyStats)]
    L.mtb_start_classify_multi.argtypes = [P(vp), i32, P(MtbClassifyOpts), P(MtbClassifyStats)]
    L.mtb_start_classify_partitioned.argtypes = [P(vp), i32, P(MtbClassifyOpts), P(MtbClassifyStats)]
    L.mtb_ctx_device.argtypes = [vp]
    L.mtb_mask_reads.argtypes = [vp, vp, vp, u32, vp]
    L.mtb_hamming.argtypes = [i32, vp, vp, u64, vp, vp, vp]
    L.mtb_pin_eval.argtypes = [i32, i32, vp, vp, vp, u64, vp, vp]
    L.mtb_sort_pairs.argtypes = [i32, vp, vp, u64, i32, i32, vp, vp]
    L.mtb_memcpy.argtypes = [vp, vp, u64]
    L.mtb_line_ext_check.argtypes = [vp, vp]
    L.mtb_link_check.argtypes = [vp, vp]
    L.mtb_write_report.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint64, vp, vp, ctypes.c_uint64]
    L.mtb_get_em_mappings.argtypes = [vp, u32, vp, u64, P(u64)]
    L.mtb_em.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp, u64, P(u64), P(MtbEmStats)]
    L.mtb_write_em_results.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, vp, u64, u32]
    L.mtb_debug_tables.argtypes = [vp, vp, vp]
    L.mtb_debug_tables.restype = None
    _LIB = L
    return L


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise MtbError(f"{what} failed ({rc}): {lib().mtb_last_error().decode()}")
    return rc
