"""The dependency-free helper functions on the classify path, pinned to the reference's own function
bodies: tests/golden/ref_functions.json holds what getNextTargetKmer
(KmerMatcher.h:282-297), calScoreIncrement / calHammingDistIncrement / isConsecutive /
isConsecutive2 and the constructor's shape parameters (Taxonomer.cpp:34-58,650-699),
getMaxCoveredLength / getQueryKmerNumber (LocalUtil.h:45-59) and Match::getScore and its partial
scores (Match.h:32-86) compute, as written, on ~75k cases and a ~9k-word diffIdx stream
(tests/golden/make_ref_functions.py cuts the bodies out of /root/reference at generation time and
compiles them with the reference's BitManipulateMacros.h in place). The oracle's restatements (CPU)
and the device's helpers as the kernels call them (mtb_pin_eval, -m gpu) are checked against it."""
import ctypes
import json
import pathlib

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]

PIN = {"score_inc": 0, "ham_inc": 1, "cons": 2, "cons2": 3, "score": 4, "right_score": 5, "left_score": 6,
       "right_ham": 7, "left_ham": 8, "covered": 9, "kmer_num": 10, "shape": 11}
PIN_DECODE = 12
# the reference's shape values are (dnaShift, maxCodonShift, smerLength, denominator, bitsPerCodon,
# totalDnaBits, lastCodonMask); smerLength has no reader on the path (assigned only, Taxonomer.cpp:37,41)
SHAPE_COLS = [0, 1, 3, 4, 5, 6]


def golden():
    return json.loads((ROOT / "tests" / "golden" / "ref_functions.json").read_text())


def cases(g, name):
    f = g["functions"][name]
    p = np.array(f["param"], np.int64)
    a = np.array([int(x) for x in f["a"]], np.uint64)
    b = np.array([int(x) for x in f["b"]], np.uint64)
    exp = np.array(f["out"], np.int64)
    if name == "shape":
        exp = exp[:, SHAPE_COLS]
    return p, a, b, exp


def run(fn_ptr, dev, fn, p, a, b, width=1):
    out = np.zeros(len(a) * width, np.int64)
    n_out = ctypes.c_uint64(0)
    args = ([dev] if dev is not None else []) + [fn, p.ctypes.data, a.ctypes.data, b.ctypes.data, len(a),
                                                  out.ctypes.data, ctypes.byref(n_out)]
    rc = fn_ptr(*args)
    assert rc == 0
    return out[:n_out.value * width].reshape(-1, width) if width > 1 else out[:n_out.value]


def test_golden_sane():
    """The vectors cover what the path feeds these functions: every rightEndHamming byte, shifts and
    ranges 0..8, consecutive pairs by construction (half of them), lengths 0..3000 and beyond, 1-5
    group deltas including zero deltas (one value held by several species)."""
    g = golden()
    f = g["functions"]
    assert len(f["cons"]["out"]) == 3000 and 0.3 < np.mean(f["cons"]["out"]) + np.mean(f["cons2"]["out"]) < 1.2
    assert sorted(set(f["score_inc"]["param"])) == list(range(9))
    assert min(f["covered"]["out"]) < 0 and f["kmer_num"]["out"][150] == (148 // 3 - 7) * 6
    w = np.array(g["decode"]["words"], np.uint32)
    assert ((w & 0x8000) != 0).sum() == len(g["decode"]["values"]) and (w == 0x8000).sum() > 100


@pytest.mark.parametrize("name", list(PIN))
def test_oracle_pinned(name):
    from tests import oracle_ctypes as oc

    p, a, b, exp = cases(golden(), name)
    got = run(oc.lib().orc_pin_eval, None, PIN[name], p, a, b, width=6 if name == "shape" else 1)
    assert np.array_equal(got, exp), name


def test_oracle_decode_pinned():
    from tests import oracle_ctypes as oc

    g = golden()["decode"]
    w = np.array(g["words"], np.uint64)
    got = run(oc.lib().orc_pin_eval, None, PIN_DECODE, np.zeros(len(w), np.int64), w, np.zeros(len(w), np.uint64))
    assert np.array_equal(got.astype(np.uint64), np.array([int(x) for x in g["values"]], np.uint64))


def test_device_shape_pinned():
    """The parameters mtb_open hands the assign kernels (assign_args: dnaShift, maxCodonShift,
    denominator; the kernels' fixed 3-bit codons) — host code, no GPU needed."""
    from metabuli_work_amd._lib import lib

    p, a, b, exp = cases(golden(), "shape")
    assert np.array_equal(run(lib().mtb_pin_eval, 0, PIN["shape"], p, a, b, width=6), exp)


@pytest.mark.gpu
@pytest.mark.parametrize("name", [k for k in PIN if k != "shape"])
def test_device_pinned(name):
    from metabuli_work_amd._lib import lib

    p, a, b, exp = cases(golden(), name)
    assert np.array_equal(run(lib().mtb_pin_eval, 0, PIN[name], p, a, b), exp), name


@pytest.mark.gpu
def test_device_decode_pinned():
    """K3's decode (decode_diff_chunk: terminator flags, scan, per-k-mer deltas, 64-bit scan — the
    code mtb_open runs on every diffIdx chunk) equals getNextTargetKmer's values word for word."""
    from metabuli_work_amd._lib import lib

    g = golden()["decode"]
    w = np.array(g["words"], np.uint64)
    got = run(lib().mtb_pin_eval, 0, PIN_DECODE, np.zeros(len(w), np.int64), w, np.zeros(len(w), np.uint64))
    assert np.array_equal(got.astype(np.uint64), np.array([int(x) for x in g["values"]], np.uint64))
