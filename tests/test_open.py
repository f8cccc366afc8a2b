"""mtb_open from the DB directory: diffIdx and info go from the files straight into HBM (parallel reads
into pinned buffers, uploads overlapped), checked on the device as validateDatabase.cpp:78-131 checks
them before the decode writes by k-mer index; the context classifies as one opened from host arrays."""
import os
import shutil

import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd._lib import MtbError
from metabuli_work_amd.classifier import Classifier, LocalParameters
from tests import oracle_ctypes as oc


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [None, "999", "65536"])
def test_open_from_files_phases_and_parity(make_db, monkeypatch, chunk):
    """chunk: diffIdx decoded in chunks of that many words (MTB_DECODE_CHUNK_WORDS; the default
    is 2^30, one chunk here): k-mers cut by a chunk's end continue in the next, values carry over."""
    if chunk:
        monkeypatch.setenv("MTB_DECODE_CHUNK_WORDS", chunk)
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 700, paired=True, seed=81)
    par = LocalParameters(seqMode=2)
    par.load_db_parameters(db_dir)
    with Classifier(par, db_dir=db_dir) as clf:
        ph = clf.open_phases()
        got = clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
    assert ph["total_s"] > 0 and ph["read_s"] >= 0 and ph["decode_s"] > 0
    assert ph["total_s"] >= ph["read_s"] + ph["decode_s"] - 1e-6
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), r)
    odb.close()
    assert np.array_equal(got.results["classification"], ores["classification"])
    assert np.array_equal(got.results["score"].view(np.uint32), ores["score"].view(np.uint32))
    assert np.array_equal(got.taxcnt, otc)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [None, "1000"])
@pytest.mark.parametrize("damage", ["info_short", "info_long", "diff_mid_kmer"])
def test_open_rejects_inconsistent_files(make_db, tmp_path, monkeypatch, damage, chunk):
    if chunk:
        monkeypatch.setenv("MTB_DECODE_CHUNK_WORDS", chunk)
    db_dir, _, _ = make_db("fmt2")
    d = str(tmp_path / "db")
    shutil.copytree(db_dir, d)
    if damage == "info_short":
        info = np.fromfile(os.path.join(d, "info"), np.uint32)
        info[:-1].tofile(os.path.join(d, "info"))
        msg = "k-mer count"
    elif damage == "info_long":
        info = np.fromfile(os.path.join(d, "info"), np.uint32)
        np.concatenate([info, info[-1:]]).tofile(os.path.join(d, "info"))
        msg = "k-mer count"
    else:
        diff = np.fromfile(os.path.join(d, "diffIdx"), np.uint16)
        diff[-1] &= 0x7FFF
        diff.tofile(os.path.join(d, "diffIdx"))
        msg = "mid k-mer"
    par = LocalParameters(seqMode=2)
    par.load_db_parameters(d)
    with pytest.raises(MtbError, match=msg):
        Classifier(par, db_dir=d)
