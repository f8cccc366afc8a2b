"""The C-ABI library loads on a CPU-only host and exports what include/mtb_gpu.h declares; host-side
parameter logic mirrors the reference (no GPU calls here)."""
import ctypes
import json
import pathlib
import re

import numpy as np
import pytest

from metabuli_work_amd import _abi
from metabuli_work_amd._lib import EXPORTED, lib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "mtb_gpu.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mtb_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = lib()
    decl = declared_symbols()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(L, name), f"{name} declared in include/mtb_gpu.h but not exported"
    assert sorted(EXPORTED) == decl


def test_default_params_are_classify_defaults():
    p = _abi.MtbParams()
    lib().mtb_default_params(ctypes.byref(p))
    # setClassifyDefaults (classify.cpp:10-37)
    assert (p.seq_mode, p.kmer_format, p.syncmer, p.smer_len) == (2, 1, 0, 5)
    assert (p.min_cons_cnt, p.min_cons_cnt_euk, p.accession_level, p.skip_redundancy) == (4, 9, 0, 0)
    assert abs(p.tie_ratio - 0.95) < 1e-7 and p.min_score == 0 and p.min_sp_score == 0
    q = _abi.default_params()
    for f, _ in _abi.MtbParams._fields_:
        if f != "reserved":
            assert getattr(p, f) == getattr(q, f), f


# setClassifyDefaults fields -> mtb_params fields; the rest have no place in the hot path's parameters:
# validateInput / validateDb (the CLI's file checks), verbosity / printLog / ramUsage (the CLI's logging
# and its RAM-bounded query splits: here the batch comes from the caller or free HBM), hammingMargin and
# maxGap (stored by KmerMatcher.cpp:29 / Taxonomer.cpp:27 and read nowhere on the path), matchPerKmer (the
# reference's initial match-buffer factor: here the workspace grows to the batch, MTB_RETRY),
# printLineage (the TSV writer's flag, MTB_WRITE_LINEAGE)
_DEFAULT_FIELDS = {"syncmer": "syncmer", "smerLen": "smer_len", "kmerFormat": "kmer_format", "em": "em",
                   "skipRedundancy": "skip_redundancy", "reducedAA": "reduced_aa", "seqMode": "seq_mode",
                   "minScore": "min_score", "minSpScore": "min_sp_score", "minConsCnt": "min_cons_cnt",
                   "minConsCntEuk": "min_cons_cnt_euk", "maskMode": "mask_mode", "maskProb": "mask_prob",
                   "accessionLevel": "accession_level", "tieRatio": "tie_ratio"}
_DEFAULT_OUTSIDE = {"validateInput", "validateDb", "verbosity", "printLog", "ramUsage", "hammingMargin", "maxGap",
                    "matchPerKmer", "printLineage"}


def test_default_params_pinned_to_reference_text():
    """mtb_default_params against setClassifyDefaults as the reference writes it
    (tests/golden/classify_defaults.json, parsed from src/workflow/classify.cpp:10-37 by
    tests/golden/make_classify_defaults.py): every default the parameters carry is the reference's,
    and every default there is either carried or listed above with the reason it is not."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "classify_defaults.json")))["defaults"]
    assert set(g) == set(_DEFAULT_FIELDS) | _DEFAULT_OUTSIDE
    p = _abi.MtbParams()
    lib().mtb_default_params(ctypes.byref(p))
    for ref, ours in _DEFAULT_FIELDS.items():
        want = g[ref]["value"]
        got = getattr(p, ours)
        if isinstance(want, float):
            assert abs(got - want) < 1e-6, (ref, got, want)
        else:
            assert got == int(want), (ref, got, want)
    assert g["hammingMargin"]["value"] == 0 and g["maxGap"]["value"] == 0


def test_load_db_parameters_quirks(tmp_path):
    d = tmp_path / "db"
    d.mkdir()
    # the writer emits Syncmer_len, which loadDbParameters (common.cpp:117-127) does not read
    (d / "db.parameters").write_text("DB_name\tx\nReduced_alphabet\t0\nAccession_level\t1\nSkip_redundancy\t1\n"
                                     "Syncmer\t1\nSyncmer_len\t6\nKmer_format\t2\n")
    p = _abi.default_params()
    assert lib().mtb_load_db_parameters(str(d).encode(), ctypes.byref(p)) == 1
    assert (p.kmer_format, p.syncmer, p.smer_len, p.skip_redundancy, p.accession_level) == (2, 1, 5, 1, 2)
    (d / "db.parameters").write_text("S-mer_len\t6\nAccession_level\t0\n")
    p = _abi.default_params(accession_level=1)
    lib().mtb_load_db_parameters(str(d).encode(), ctypes.byref(p))
    assert p.smer_len == 6 and p.accession_level == 0
    assert lib().mtb_load_db_parameters(str(tmp_path / "none").encode(), ctypes.byref(p)) == 0


def test_product_genetic_code_matches_reference_tables():
    """The product's restated tables equal the reference GeneticCode.h dump (golden)."""
    g = json.loads((ROOT / "tests" / "golden" / "genetic_code.json").read_text())
    base = np.zeros(256, np.uint8)
    aa = np.zeros(64, np.int8)
    num = np.zeros(64, np.int8)
    lib().mtb_debug_tables(base.ctypes.data, aa.ctypes.data, num.ctypes.data)
    atcg = g["atcg"]
    for c in range(256):
        assert base[c] == (atcg[c] & 14) >> 1
    code = {0: 0, 1: 1, 2: 2, 3: 3}
    for a, b, c, v in g["nuc2aa"]:
        if 7 in (a, b, c):
            assert v == -1
            continue
        assert aa[code[a] << 4 | code[b] << 2 | code[c]] == v
    for a, b, c, v in g["nuc2num"]:
        if 7 in (a, b, c):
            continue
        assert num[a << 4 | b << 2 | c] == v


@pytest.mark.gpu
def test_device_hamming_pinned_to_reference():
    """K4's codon arithmetic on the device (mtb_hamming: hamming_sum_rows / hammings_rows, the forms
    emit_match uses, checked against the plain hamming_sum / hammings in the kernel) equals the
    reference's getHammingDistanceSum / getHammings / getHammings_reverse on the golden pairs
    (tables parsed from KmerMatcher.h:66-158, tests/golden/make_ref_tables.py): every codon pair at
    every field, LUT7's rows 4-5 included, plus 2,048 random pairs."""
    from tests.test_oracle import hamming_golden

    _, a, b, esum, efwd, erev = hamming_golden()
    n = len(a)
    s, f, r = np.zeros(n, np.uint8), np.zeros(n, np.uint16), np.zeros(n, np.uint16)
    rc = lib().mtb_hamming(0, a.ctypes.data, b.ctypes.data, n, s.ctypes.data, f.ctypes.data, r.ctypes.data)
    assert rc == 0, lib().mtb_last_error().decode()
    assert np.array_equal(s, esum)
    assert np.array_equal(f, efwd)
    assert np.array_equal(r, erev)


def test_open_rejects_out_of_scope_params(tmp_path):
    h = ctypes.c_void_p()
    p = _abi.default_params(reduced_aa=1)
    rc = lib().mtb_open(str(tmp_path).encode(), ctypes.byref(p), 0, ctypes.byref(h))
    assert rc < 0


def abi_caller() -> pathlib.Path:
    """tests/_abi_caller: the compiled C caller of include/mtb_gpu.h (built by __graft_entry__.build();
    rebuilt here when missing or older than its source)."""
    import __graft_entry__ as g

    return g.build_abi_caller()


def _mirrors():
    from metabuli_work_amd import dbbuild

    ct = {"mtb_params": _abi.MtbParams, "mtb_db_host": _abi.MtbDbHost, "mtb_db_resident": _abi.MtbDbResident,
          "mtb_read_batch": _abi.MtbReadBatch, "mtb_classify_opts": _abi.MtbClassifyOpts,
          "mtb_classify_stats": _abi.MtbClassifyStats, "mtb_em_stats": _abi.MtbEmStats,
          "mtb_build_input": dbbuild.MtbBuildInput, "mtb_db_built": dbbuild.MtbDbBuilt}
    nd = {"mtb_kmer": _abi.KMER_DTYPE, "mtb_match": _abi.MATCH_DTYPE, "mtb_result": _abi.RESULT_DTYPE,
          "mtb_taxcnt": _abi.TAXCNT_DTYPE, "mtb_em_map": _abi.EM_MAP_DTYPE, "mtb_em_read": _abi.EM_READ_DTYPE}
    return ct, nd


def test_struct_layouts_match_compiled_c():
    """sizeof / offsetof of every public struct as a C compiler lays out include/mtb_gpu.h equal the
    Python mirrors the tests and bench pass through ctypes (a layout drift fails here)."""
    import subprocess

    out = subprocess.run([str(abi_caller()), "--layout"], check=True, capture_output=True, text=True).stdout
    lay = json.loads(out)
    ct, nd = _mirrors()
    assert set(lay) == set(ct) | set(nd)
    for name, cls in ct.items():
        assert lay[name]["size"] == ctypes.sizeof(cls), name
        assert list(lay[name]["fields"]) == [f for f, _ in cls._fields_], name
        for f, off in lay[name]["fields"].items():
            assert getattr(cls, f).offset == off, f"{name}.{f}"
    for name, dt in nd.items():
        assert lay[name]["size"] == dt.itemsize, name
        assert list(lay[name]["fields"]) == list(dt.names), name
        for f, off in lay[name]["fields"].items():
            assert dt.fields[f][1] == off, f"{name}.{f}"
