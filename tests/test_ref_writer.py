"""The DB writer pinned to the reference's own code (round 6): tests/golden/ref_writer.npz holds the
diffIdx / info / split files that IndexCreator::writeTargetFilesAndSplits and getDiffIdx
(IndexCreator.cpp:811-886, with WriteBuffer, DiffIdxSplit, MARKER and AminoAcidPart as written)
produce for four sorted unique (value, taxID) lists — 12 to 60,000 k-mers, split counts 4 to 4096,
values repeated across species, deltas of one to five 15-bit groups (tests/golden/make_ref_writer.py).
The oracle's restated writer (oracle/orc_dbwriter.cpp, which the device builder mtb_build_db is
checked against byte for byte in test_gpu_build.py) writes the same bytes."""
import ctypes

import numpy as np
import pytest

from tests import oracle_ctypes as oc

CASES = ["tiny", "small", "mid", "full"]


def golden():
    import pathlib
    return np.load(pathlib.Path(__file__).resolve().parent / "golden" / "ref_writer.npz")


@pytest.mark.parametrize("name", CASES)
def test_oracle_writer_pinned(name):
    g = golden()
    v, ids, sn = g[f"{name}_values"], g[f"{name}_ids"], int(g[f"{name}_split_num"][0])
    n = len(v)
    diff = np.zeros(5 * n + 5, np.uint16)
    nd = ctypes.c_uint64(0)
    info = np.zeros(n, np.uint32)
    split = np.zeros(3 * sn, np.uint64)
    rc = oc.lib().orc_pin_write_db(v.ctypes.data, ids.ctypes.data, n, sn, diff.ctypes.data, ctypes.byref(nd),
                                   info.ctypes.data, split.ctypes.data)
    assert rc == 0
    assert np.array_equal(diff[:nd.value], g[f"{name}_diffIdx"])
    assert np.array_equal(info, g[f"{name}_info"])
    assert np.array_equal(split, g[f"{name}_split"])


def test_writer_golden_decodes_back():
    """The reference's diffIdx decodes (getNextTargetKmer, pinned in test_ref_functions.py) to the
    listed values; every split entry names a k-mer that starts an AA group at its offsets."""
    g = golden()
    for name in CASES:
        w = g[f"{name}_diffIdx"].astype(np.uint64)
        vals = np.zeros(len(w), np.int64)
        n_out = ctypes.c_uint64(0)
        rc = oc.lib().orc_pin_eval(12, np.zeros(len(w), np.int64).ctypes.data, w.ctypes.data,
                                   np.zeros(len(w), np.uint64).ctypes.data, len(w), vals.ctypes.data,
                                   ctypes.byref(n_out))
        assert rc == 0 and np.array_equal(vals[:n_out.value].astype(np.uint64), g[f"{name}_values"])
        sp = g[f"{name}_split"].reshape(-1, 3)
        assert (sp[0] == 0).all()
        used = sp[1:][sp[1:, 1] > 0]
        assert len(used) >= 1 and (np.diff(used[:, 2].astype(np.int64)) > 0).all()
