"""The C-ABI library loads on a CPU-only host and exports what include/mtb_gpu.h declares; host-side
parameter logic mirrors the reference (no GPU calls here)."""
import ctypes
import json
import pathlib
import re

import numpy as np

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


def test_open_rejects_out_of_scope_params(tmp_path):
    h = ctypes.c_void_p()
    p = _abi.default_params(reduced_aa=1)
    rc = lib().mtb_open(str(tmp_path).encode(), ctypes.byref(p), 0, ctypes.byref(h))
    assert rc < 0
