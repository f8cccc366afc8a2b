"""The oracle (CPU restatement) on the CPU: tables pinned to the reference's GeneticCode.h, the
stateful scanners against an independent closed-form restatement, DB-format invariants, the
committed regression fixture, and result sanity on a synthetic workload."""
import ctypes
import json
import os
import pathlib

import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd._abi import default_params, info_frame, info_pos, info_seq
from tests import oracle_ctypes as oc
from tests import pyscan

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_oracle_tables_pinned_to_reference_genetic_code():
    g = json.loads((ROOT / "tests" / "golden" / "genetic_code.json").read_text())
    aa = np.zeros(512, np.int32)
    num = np.zeros(512, np.int32)
    at = np.zeros(256, np.uint8)
    rc = np.zeros(256, np.uint8)
    oc.lib().orc_genetic_tables(aa.ctypes.data, num.ctypes.data, at.ctypes.data, rc.ctypes.data)
    for a, b, c, v in g["nuc2aa"]:
        assert aa[a * 64 + b * 8 + c] == v
    for a, b, c, v in g["nuc2num"]:
        assert num[a * 64 + b * 8 + c] == v
    assert list(at) == g["atcg"] and list(rc) == g["iRCT"]


def hamming_golden():
    """tests/golden/hamming_tables.json: the reference's hammingLookup / HAMMING_LUT0..7 parsed out of
    KmerMatcher.h:66-158 and its GET_3_BITS compiled in place (make_ref_tables.py), with the sums and
    Hamming words its getHammingDistanceSum / getHammings / getHammings_reverse give on 2,560 pairs."""
    g = json.loads((ROOT / "tests" / "golden" / "hamming_tables.json").read_text())
    v = g["vectors"]
    a = np.array([int(x) for x in v["a"]], np.uint64)
    b = np.array([int(x) for x in v["b"]], np.uint64)
    return g, a, b, np.array(v["sum"], np.uint8), np.array(v["fwd"], np.uint16), np.array(v["rev"], np.uint16)


def test_oracle_hamming_tables_pinned_to_reference():
    g, a, b, esum, efwd, erev = hamming_golden()
    assert g["GET_3_BITS"] == [x & 7 for x in range(512)]  # the macro the functions index with
    look = np.zeros(64, np.uint8)
    lut = np.zeros(512, np.uint16)
    oc.lib().orc_hamming_tables(look.ctypes.data, lut.ctypes.data)
    assert look.reshape(8, 8).tolist() == g["hammingLookup"]
    # every field k of every (query codon, target codon): the oracle's codonField, placed at its
    # 2 bits, is the reference's HAMMING_LUTk entry (8 x 8 x 8 cases, LUT7 rows 4-5 included)
    assert lut.reshape(8, 64).tolist() == g["HAMMING_LUT"]
    n = len(a)
    s, f, r = np.zeros(n, np.uint8), np.zeros(n, np.uint16), np.zeros(n, np.uint16)
    oc.lib().orc_hamming(a.ctypes.data, b.ctypes.data, n, s.ctypes.data, f.ctypes.data, r.ctypes.data)
    assert np.array_equal(s, esum) and np.array_equal(f, efwd) and np.array_equal(r, erev)


@pytest.mark.parametrize("fmt,syncmer,smer", [(2, 0, 5), (2, 1, 5), (2, 1, 4), (1, 0, 5)])
@pytest.mark.parametrize("paired", [True, False])
def test_oracle_scanners_vs_closed_form(fmt, syncmer, smer, paired):
    rng = np.random.default_rng(7 + fmt + 3 * syncmer + smer)
    alphabet = np.frombuffer(b"ACGTACGTACGTACGTNacgtRYKM", np.uint8)
    n = 60
    r1, r2 = [], []
    for i in range(n):
        L1 = int(rng.integers(20, 160))
        L2 = int(rng.integers(20, 160))
        r1.append(alphabet[rng.integers(0, len(alphabet), L1)])
        r2.append(alphabet[rng.integers(0, len(alphabet), L2)])
    s1, o1 = synth._pack(r1)
    s2, o2 = synth._pack(r2)
    reads = synth.Reads(s1, o1, s2 if paired else None, o2 if paired else None, np.zeros(n, np.int32))
    par = default_params(kmer_format=fmt, syncmer=syncmer, smer_len=smer, seq_mode=2 if paired else 1)
    kmers, ql1, ql2 = oc.extract(par, reads, sort=False)
    kmers = kmers[info_seq(kmers["info"]) != 0]
    got = sorted(zip(kmers["value"].tolist(), info_seq(kmers["info"]).tolist(), info_pos(kmers["info"]).tolist(),
                     info_frame(kmers["info"]).tolist()))
    want = []
    for i in range(n):
        for v, p, f in pyscan.read_kmers(bytes(r1[i]), bytes(r2[i]) if paired else None, fmt, syncmer, smer):
            want.append((v, i + 1, p, f))
    assert got == sorted(want)
    for i in range(n):
        assert ql1[i] == pyscan.max_cov(len(r1[i]))


def _decode(diff):
    """Vectorised getNextTargetKmer over a whole diffIdx: values and the word index after each."""
    diff = diff.astype(np.uint64)
    term = np.nonzero(diff & np.uint64(0x8000))[0]
    starts = np.concatenate([[0], term[:-1] + 1])
    kidx = np.repeat(np.arange(len(term)), term - starts + 1)
    shift = (term[kidx] - np.arange(len(diff))) * 15
    contrib = (diff & np.uint64(0x7FFF)) << shift.astype(np.uint64)
    deltas = np.add.reduceat(contrib, starts)
    return np.cumsum(deltas, dtype=np.uint64), term + 1


@pytest.mark.parametrize("fmt,syncmer", [(2, 0), (2, 1), (1, 0)])
def test_db_writer_invariants(tmp_path, fmt, syncmer):
    taxo = synth.make_taxonomy(8, 2, seed=5)
    gen = synth.make_genomes(taxo, genome_len=12000, seed=6)
    d = str(tmp_path / "db")
    oc.build_db(d, default_params(kmer_format=fmt, syncmer=syncmer), taxo, gen)
    diff = np.fromfile(os.path.join(d, "diffIdx"), np.uint16)
    info = np.fromfile(os.path.join(d, "info"), np.uint32)
    split = np.fromfile(os.path.join(d, "split"), np.uint64).reshape(-1, 3)
    vals, word_end = _decode(diff)
    assert len(vals) == len(info) > 4095                      # validateDatabase.cpp:78-131
    assert np.all(vals[1:] >= vals[:-1])                      # sorted by value
    assert len(split) == 4096 and not split[0].any()
    used = split[1:][split[1:, 0] != 0]
    assert len(used) > 100
    for ad, doff, ioff in used:
        assert vals[ioff - 1] == ad                           # ADkmer = k-mer at infoIdxOffset-1
        assert word_end[ioff - 1] == doff                     # diffIdxOffset counts words through it
        assert ((vals[ioff - 2] ^ ad) >> np.uint64(24)) != 0  # starts a new AA group
    p = oc.load_db_parameters(d, default_params())
    assert (p.kmer_format, p.syncmer, p.skip_redundancy) == (fmt, syncmer, 1)


def test_oracle_regression_fixture(tmp_path):
    from tests.golden import make_oracle_fixtures as mk
    ref = np.load(ROOT / "tests" / "golden" / "oracle_small.npz")
    for name, fmt, syn in mk.CASES:
        d = str(tmp_path / name)
        res, tc = mk.run_case(fmt, syn, d)
        assert np.array_equal(res, ref[name + "_res"]), name
        assert np.array_equal(tc, ref[name + "_tc"]), name


def test_oracle_classifies_synthetic_reads(make_db):
    d, taxo, gen = make_db("fmt2")
    par = oc.load_db_parameters(d, default_params())
    reads = synth.make_reads(gen, 800, seed=9, random_frac=0.1)
    db = oc.OracleDb(d)
    res, tc = oc.classify(db, par, reads)
    db.close()
    origin = reads.origin
    ok = tot = 0
    for i in range(reads.n):
        if origin[i] < 0 or not res["is_classified"][i]:
            continue
        tot += 1
        c = int(res["classification"][i])
        ok += c in (int(gen.taxid[origin[i]]), int(gen.species[origin[i]]))
    assert tot > 0.7 * (origin >= 0).sum()
    assert ok / tot > 0.95
    rnd = origin < 0
    assert res["is_classified"][rnd].mean() < 0.2


def test_oracle_report_by_hand(make_db, tmp_path):
    """The oracle's per-taxon report (Reporter::writeReportFile, Reporter.cpp:175-244) against a
    report worked out here from the taxonomy: clade counts up the parent chain, unclassified first,
    children by clade count (distinct counts: no ties), two spaces of indent per depth."""
    d, taxo, gen = make_db("fmt2")
    tid = taxo.taxid.tolist()
    par = dict(zip(tid, taxo.parent.tolist()))
    rank = dict(zip(tid, taxo.rank))
    name = dict(zip(tid, taxo.name))
    strains = [int(t) for t in gen.taxid[:3]]
    counts = {0: 7, strains[0]: 5, strains[1]: 3, int(gen.species[2]): 2}
    total = 20
    clade = {}
    for t, c in counts.items():
        clade[t] = clade.get(t, 0) + c
        x = t
        while t and par[x] != x:
            x = par[x]
            clade[x] = clade.get(x, 0) + c
    kids = {}
    for t in tid:
        if par[t] != t:
            kids.setdefault(par[t], []).append(t)
    want = ["#clade_proportion\tclade_count\ttaxon_count\trank\ttaxID\tname",
            "%.4f\t%d\t%d\tno rank\t0\tunclassified" % (100 * 7 / total, 7, 7)]

    def walk(t, depth):
        want.append("%.4f\t%d\t%d\t%s\t%d\t%s%s" % (100 * clade[t] / total, clade[t], counts.get(t, 0), rank[t], t,
                                                     "  " * depth, name[t]))
        for c in sorted((k for k in kids.get(t, []) if k in clade), key=lambda k: -clade[k]):
            walk(c, depth + 1)

    walk(1, 0)
    assert len(set(clade[k] for k in clade)) >= 3
    db = oc.OracleDb(d)
    out = str(tmp_path / "report.tsv")
    oc.write_report(db, out, total, counts)
    db.close()
    assert open(out).read() == "\n".join(want) + "\n"
