"""Query extraction pinned to the reference's own code (round 6): tests/golden/ref_scanners.npz holds the
k-mers that KmerScanner.h's MetamerScanner / OldMetamerScanner, SyncmerScanner.h's SyncmerScanner
and KmerExtractor::fillQueryKmerBuffer (KmerExtractor.cpp:355-386) emit, as written, for 112 reads
(paired 150 bp, single-end 27-3002 bp of every length residue, N / IUPAC / lower case) in formats
1 and 2 and with closed syncmers (s = 5, 6); tests/golden/make_ref_scanners.py cuts that code out of
/root/reference at generation time and compiles it with GeneticCode.h in place.

CPU: the oracle's restated scanners (oracle/orc_extract.cpp) emit exactly those k-mers, read by read
in emission order (value, seqID, pos, frame). GPU: the device's K1 (every window kept: MTB_FILTER=0,
staged) emits the same multiset."""
import numpy as np
import pytest

from tests import oracle_ctypes as oc
from metabuli_work_amd import synth
from metabuli_work_amd._abi import default_params, info_frame, info_pos, info_seq

CONFIGS = {"fmt2": (2, 0, 5), "fmt1": (1, 0, 5), "fmt2_syncmer5": (2, 1, 5), "fmt2_syncmer6": (2, 1, 6)}


def golden():
    import pathlib
    return np.load(pathlib.Path(__file__).resolve().parent / "golden" / "ref_scanners.npz")


def batches(g):
    """The read set as two batches, the paired reads and the single-end ones: (global read indices,
    synth.Reads)."""
    s1, s2 = [str(x) for x in g["seq1"]], [str(x) for x in g["seq2"]]
    out = []
    for paired in (True, False):
        idx = [i for i in range(len(s1)) if bool(s2[i]) == paired]

        def pack(seqs):
            off = np.zeros(len(seqs) + 1, np.uint64)
            off[1:] = np.cumsum([len(x) for x in seqs])
            return np.frombuffer("".join(seqs).encode(), np.uint8).copy(), off
        a, oa = pack([s1[i] for i in idx])
        if paired:
            b, ob = pack([s2[i] for i in idx])
            out.append((idx, synth.Reads(a, oa, b, ob, np.zeros(len(idx), np.int32))))
        else:
            out.append((idx, synth.Reads(a, oa, None, None, np.zeros(len(idx), np.int32))))
    return out


def expected(g, name, idx):
    """Golden k-mers of the reads idx (global order), seqIDs renumbered to the batch: rows
    (value, seqID, pos, frame) in emission order."""
    v, s, p, f = (g[f"{name}_{k}"] for k in ("value", "seq", "pos", "frame"))
    where = {gi + 1: bi + 1 for bi, gi in enumerate(idx)}
    keep = np.isin(s, np.array(list(where), np.uint32))
    rows = np.stack([v[keep], np.array([where[int(x)] for x in s[keep]], np.uint64),
                     p[keep].astype(np.uint64), f[keep].astype(np.uint64)], 1)
    return rows


def rows_of(kmers):
    info = kmers["info"]
    return np.stack([kmers["value"].astype(np.uint64), info_seq(info).astype(np.uint64),
                     info_pos(info).astype(np.uint64), info_frame(info).astype(np.uint64)], 1)


def test_golden_shape():
    g = golden()
    assert len(g["seq1"]) == 112
    for name, (fmt, syn, smer) in CONFIGS.items():
        n = len(g[f"{name}_value"])
        assert n > 20000, name
        assert set(np.unique(g[f"{name}_frame"]).tolist()) == set(range(6))
    # a syncmer scan keeps a subset of the metamers' windows
    assert len(g["fmt2_syncmer5_value"]) < len(g["fmt2_value"])


@pytest.mark.parametrize("name", list(CONFIGS))
def test_oracle_scanners_pinned(name):
    g = golden()
    fmt, syn, smer = CONFIGS[name]
    for idx, reads in batches(g):
        par = default_params(kmer_format=fmt, syncmer=syn, smer_len=smer, seq_mode=2 if reads.seq2 is not None else 1)
        buf, _, _ = oc.extract(par, reads, sort=False)
        got = rows_of(buf[buf["value"] != 0])
        exp = expected(g, name, idx)
        # per read in buffer order: mate 1's reservation precedes mate 2's (KmerExtractor.cpp:290-300)
        order = np.argsort(got[:, 1], kind="stable")
        assert np.array_equal(got[order], exp), name


@pytest.mark.gpu
@pytest.mark.parametrize("name,db", [("fmt2", "fmt2"), ("fmt1", "fmt1"), ("fmt2_syncmer5", "fmt2_syncmer")])
def test_device_extraction_pinned(make_db, monkeypatch, name, db):
    """K1 on the device, every emitted window kept (no membership filter) and returned by the staged
    getter: the multiset of (value, seqID, pos, frame) equals the reference code's."""
    from metabuli_work_amd.classifier import Classifier, LocalParameters

    monkeypatch.setenv("MTB_FILTER", "0")
    g = golden()
    db_dir, _, _ = make_db(db)
    for idx, reads in batches(g):
        par = LocalParameters(seqMode=2 if reads.seq2 is not None else 1).load_db_parameters(db_dir)
        with Classifier(par, db_dir=db_dir, device=0) as clf:
            clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, keep_stages=True)
            got = rows_of(clf.query_kmers())
        exp = expected(g, name, idx)
        key = lambda a: a[np.lexsort(a.T[::-1])]  # noqa: E731
        assert np.array_equal(key(got), key(exp)), name
