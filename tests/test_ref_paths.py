"""combineMatchPaths pinned to the reference's own code (round 6): tests/golden/ref_paths.npz holds what
Taxonomer::combineMatchPaths / trimMatchPath / isMatchPathOverlapped (Taxonomer.cpp:410-485, with
MatchPath and Match's partial scores as written) return for 3,000 tie-heavy species runs of 1-65 paths
(tests/golden/make_ref_paths.py): the run's score bits and the kept paths in order, trimmed. The
std::sort inside leaves tied paths in libstdc++'s introsort order, which the device emulates
(mtb_stdsort.h); the oracle's combineMatchPaths (oracle/orc_taxonomer.cpp) is checked here, and the
device's K6 against the oracle in the GPU parity tests (general paths forced, test_general_paths)."""
import ctypes
import pathlib

import numpy as np

from tests import oracle_ctypes as oc


def golden():
    return np.load(pathlib.Path(__file__).resolve().parent / "golden" / "ref_paths.npz")


def test_golden_has_ties_and_trims():
    g = golden()
    p = g["paths"]
    assert len(g["run_len"]) == 3000 and p.shape[1] == 6
    # many runs hold tied (score, hamming, start) paths: the unstable sort's order matters
    ties = 0
    o = 0
    for n in g["run_len"]:
        key = p[o:o + n, [2, 3, 0]]
        ties += len(key) - len(np.unique(key, axis=0))
        o += n
    assert ties > 1000
    kept = g["comb"]
    assert int(g["comb_len"].sum()) == len(kept)
    # trimMatchPath ran: kept paths whose (start, end) no input path has
    spans = {(int(a), int(b)) for a, b in p[:, :2]}
    assert sum((int(a), int(b)) not in spans for a, b in kept[:, :2]) > 100


def test_oracle_combine_pinned():
    g = golden()
    L = oc.lib()
    L.orc_pin_combine.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                                          ctypes.c_void_p, ctypes.c_void_p]
    p, kept = g["paths"], g["comb"]
    o = k = 0
    for r, n in enumerate(g["run_len"]):
        run = p[o:o + n]
        st = np.ascontiguousarray(run[:, 0], np.int32)
        en = np.ascontiguousarray(run[:, 1], np.int32)
        sc = np.ascontiguousarray(run[:, 2], np.uint32).view(np.float32)
        hd = np.ascontiguousarray(run[:, 3], np.int32)
        r0 = np.ascontiguousarray(run[:, 4], np.uint16)
        r1 = np.ascontiguousarray(run[:, 5], np.uint16)
        score = ctypes.c_float(0)
        out = np.zeros(4 * max(n, 1), np.int32)
        nc = ctypes.c_uint64(0)
        assert L.orc_pin_combine(st.ctypes.data, en.ctypes.data, sc.ctypes.data, hd.ctypes.data, r0.ctypes.data,
                                 r1.ctypes.data, n, int(g["read_len"][r]), ctypes.byref(score), out.ctypes.data,
                                 ctypes.byref(nc)) == 0
        c = int(g["comb_len"][r])
        assert np.float32(score.value).view(np.uint32) == g["score_bits"][r], r
        assert nc.value == c, r
        got = out[:4 * c].reshape(-1, 4).astype(np.int64)
        got[:, 3] = got[:, 3].astype(np.int64) & 0xFFFFFFFF
        assert np.array_equal(got, kept[k:k + c]), r
        o += n
        k += c
