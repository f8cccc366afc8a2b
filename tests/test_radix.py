"""K2's LSD radix sort is stable: the lane-mask ranking relies on one wave's LDS operations
completing in program order, and every pass after the first must keep equal digits in input order for
the 24-bit prefix order to come out right. Checked directly through mtb_sort_pairs: keys over many
tiles with few distinct sort prefixes (long runs of equal digits in every tile), distinct values = the
input positions, so the output values must be numpy's stable argsort of the prefix exactly. Both tile
sizes (MTB_RADIX_TILE), both rankings (MTB_RADIX_ORRANK), partial last tiles."""
import numpy as np
import pytest

from metabuli_work_amd._lib import lib

LO, HI = 36, 60  # the query sort's prefix (kQuerySortLo / kQuerySortHi)


def sort_pairs(keys, lo=LO, hi=HI):
    n = len(keys)
    vals = np.arange(n, dtype=np.uint32)
    ko = np.zeros(n, np.uint64)
    vo = np.zeros(n, np.uint32)
    rc = lib().mtb_sort_pairs(0, keys.ctypes.data, vals.ctypes.data, n, lo, hi, ko.ctypes.data, vo.ctypes.data)
    assert rc == 0, lib().mtb_last_error().decode()
    return ko, vo


@pytest.mark.gpu
@pytest.mark.parametrize("env", ["", "MTB_RADIX_TILE=4096", "MTB_RADIX_ORRANK=0", "MTB_RADIX_FULLTILE=0"])
@pytest.mark.parametrize("n,distinct", [(8192 * 12 + 77, 5), (100_003, 300), (8191, 2), (4096 * 3, 1)])
def test_radix_sort_stable(monkeypatch, env, n, distinct):
    if env:
        k, v = env.split("=")
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(n + distinct)
    prefixes = rng.integers(0, 1 << (HI - LO), distinct, dtype=np.uint64)
    keys = (prefixes[rng.integers(0, distinct, n)] << np.uint64(LO)) | rng.integers(0, 1 << LO, n, dtype=np.uint64)
    keys |= rng.integers(0, 16, n, dtype=np.uint64) << np.uint64(HI)  # bits above the range: ignored
    ko, vo = sort_pairs(keys)
    order = np.argsort((keys >> np.uint64(LO)) & np.uint64((1 << (HI - LO)) - 1), kind="stable")
    assert np.array_equal(vo, order.astype(np.uint32))
    assert np.array_equal(ko, keys[order])
