"""Native host I/O (mtb_io.cpp): the FASTA/FASTQ(.gz) batch reader against the
independent Python reader and the synthesised reads, its error paths, and (GPU) the end-to-end
startClassify TSV against the oracle's classifications."""
import gzip

import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd._lib import MtbError
from metabuli_work_amd.classifier import Classifier, FastxReader, LocalParameters, read_records
from tests import oracle_ctypes as oc


def _mates(reads, which):
    seq = reads.seq1 if which == 1 else reads.seq2
    off = reads.off1 if which == 1 else reads.off2
    return [bytes(seq[off[i]:off[i + 1]]) for i in range(reads.n)]


def _write_fastq(path, names, seqs):
    data = "".join(f"@{n} some comment\n{s.decode()}\n+\n{'I' * len(s)}\n" for n, s in zip(names, seqs)).encode()
    if path.endswith(".gz"):
        with gzip.open(path, "wb") as f:
            f.write(data)
    else:
        with open(path, "wb") as f:
            f.write(data)


def _write_fasta(path, names, seqs, width=60):
    with open(path, "w") as f:
        for n, s in zip(names, seqs):
            f.write(f">{n}\tdesc\n")
            for i in range(0, len(s), width):
                f.write(s[i:i + width].decode() + "\n")
            if not s:
                f.write("\n")


def _read_all(p1, p2, batch):
    names, m1, m2 = [], [], []
    with FastxReader(p1, p2) as rd:
        while True:
            b = rd.next(batch)
            if b.n_reads == 0:
                break
            nm, s1, o1, s2, o2 = FastxReader.arrays(b)
            assert len(nm) <= batch
            names += nm
            m1 += [bytes(s1[o1[i]:o1[i + 1]]) for i in range(len(nm))]
            if s2 is not None:
                m2 += [bytes(s2[o2[i]:o2[i + 1]]) for i in range(len(nm))]
    return names, m1, m2


@pytest.fixture(scope="module")
def reads():
    taxo = synth.make_taxonomy(6, 2, seed=3)
    gen = synth.make_genomes(taxo, genome_len=8000, seed=4)
    return synth.make_reads(gen, 1000, paired=True, seed=9, short_frac=0.05, rate_n=0.01, rate_lower=0.01)


@pytest.mark.parametrize("gz", [False, True])
def test_fastq_pairs(tmp_path, reads, gz):
    ext = ".fq.gz" if gz else ".fq"
    names = [f"read{i}" for i in range(reads.n)]
    p1, p2 = str(tmp_path / ("r1" + ext)), str(tmp_path / ("r2" + ext))
    _write_fastq(p1, names, _mates(reads, 1))
    _write_fastq(p2, names, _mates(reads, 2))
    got_names, g1, g2 = _read_all(p1, p2, 333)
    assert got_names == names
    assert g1 == _mates(reads, 1) and g2 == _mates(reads, 2)
    assert [s for _, s in read_records(p1)] == g1  # the independent Python reader agrees


def test_fasta_multiline(tmp_path, reads):
    names = [f"contig_{i}" for i in range(reads.n)]
    seqs = _mates(reads, 1)
    p = str(tmp_path / "r.fa")
    _write_fasta(p, names, seqs, width=37)
    got_names, g1, g2 = _read_all(p, None, 1000)
    assert got_names == names and g1 == seqs and g2 == []


def test_fastq_wrapped(tmp_path, reads):
    """Wrapped FASTQ (sequence and quality split over several lines, as kseq accepts) reads the same
    as one-line records."""
    names = [f"w{i}" for i in range(reads.n)]
    seqs = _mates(reads, 1)
    p = str(tmp_path / "wrapped.fq")
    with open(p, "w") as f:
        for nm, sq in zip(names, seqs):
            s = sq.decode()
            f.write(f"@{nm} x\n" + "".join(s[i:i + 37] + "\n" for i in range(0, len(s), 37)) + "+\n" +
                    "".join("I" * len(s[i:i + 41]) + "\n" for i in range(0, len(s), 41)))
    got_names, g1, _ = _read_all(p, None, 257)
    assert got_names == names and g1 == seqs


@pytest.mark.parametrize("mode", ["plain", "gzip", "bgzf", "multi"])
def test_compression_modes(tmp_path, reads, mode):
    """Plain, single-member gzip, BGZF (blocks inflated by a worker pool) and multi-member gzip
    inputs give the same records, for both mates."""
    data1 = synth.fastq_bytes(reads.seq1, reads.off1)
    data2 = synth.fastq_bytes(reads.seq2, reads.off2)
    p1, p2 = str(tmp_path / "a.fq"), str(tmp_path / "b.fq")
    if mode == "multi":  # two gzip members back to back
        cut = len(data1) // 2
        cut = data1.index(b"\n@", cut) + 1
        with open(p1, "wb") as f:
            f.write(gzip.compress(data1[:cut]) + gzip.compress(data1[cut:]))
        synth.write_compressed(p2, data2, "gzip")
    else:
        synth.write_compressed(p1, data1, mode)
        synth.write_compressed(p2, data2, mode)
    names, g1, g2 = _read_all(p1, p2, 300)
    assert names == [f"r{i:09d}" for i in range(reads.n)]
    assert g1 == _mates(reads, 1) and g2 == _mates(reads, 2)


def test_bgzf_empty_and_eof_groups(tmp_path, reads, monkeypatch):
    """A bgzipped file holding only the EOF marker reads as empty input; a file whose last data
    member closes an inflate group (the EOF marker alone in the next group, or every member its own
    group) reads completely (gzread reads both, as the reference's kseq does)."""
    empty = str(tmp_path / "empty.fq.gz")
    synth.write_compressed(empty, b"", "bgzf")
    assert _read_all(empty, None, 100) == ([], [], [])
    data = synth.fastq_bytes(reads.seq1, reads.off1)
    p = str(tmp_path / "a.fq.gz")
    synth.write_compressed(p, data, "bgzf")
    import os
    for group in (1, os.path.getsize(p) - 28):  # 28 B: the EOF marker block
        monkeypatch.setenv("MTB_BGZF_GROUP", str(group))
        names, g1, _ = _read_all(p, None, 300)
        assert names == [f"r{i:09d}" for i in range(reads.n)] and g1 == _mates(reads, 1)


def test_gzip_member_at_buffer_edge(tmp_path, reads, monkeypatch):
    """Multi-member gzip whose second member starts one byte before the end of the input buffer:
    the reader keeps that byte and refills before testing for the next member's magic (all members
    are read, as gzread does)."""
    data = synth.fastq_bytes(reads.seq1, reads.off1)
    cut = data.index(b"\n@", len(data) // 3) + 1
    m1, m2 = gzip.compress(data[:cut]), gzip.compress(data[cut:])
    p = str(tmp_path / "m.fq.gz")
    with open(p, "wb") as f:
        f.write(m1 + m2)
    for extra in (1, 2):
        monkeypatch.setenv("MTB_GZ_BUFFER", str(len(m1) + extra))
        names, g1, _ = _read_all(p, None, 300)
        assert g1 == _mates(reads, 1) and len(names) == reads.n


def test_reader_errors(tmp_path, reads):
    names = [f"r{i}" for i in range(10)]
    seqs = _mates(reads, 1)[:10]
    p1, p2 = str(tmp_path / "a.fq"), str(tmp_path / "b.fq")
    _write_fastq(p1, names, seqs)
    _write_fastq(p2, names[:7], seqs[:7])
    with pytest.raises(MtbError, match="different read counts"):
        _read_all(p1, p2, 4)
    bad = str(tmp_path / "bad.fq")
    with open(bad, "w") as f:
        f.write("not a record\nACGT\n")
    with pytest.raises(MtbError, match="header"):
        _read_all(bad, None, 4)
    with pytest.raises(MtbError, match="cannot open"):
        FastxReader(str(tmp_path / "missing.fq"))


@pytest.mark.gpu
def test_start_classify_tsv(make_db, tmp_path):
    """File in, TSV out (Classifier::startClassify + Reporter::writeReadClassification) against the
    oracle's per-read results for the same reads."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 2500, paired=True, seed=41, short_frac=0.02)
    names = [f"q{i}" for i in range(r.n)]
    p1, p2 = str(tmp_path / "q1.fq.gz"), str(tmp_path / "q2.fq.gz")
    _write_fastq(p1, names, _mates(r, 1))
    _write_fastq(p2, names, _mates(r, 2))
    par = LocalParameters(seqMode=2, filenames=[p1, p2, db_dir])
    par.load_db_parameters(db_dir)
    out = str(tmp_path / "out.tsv")
    rep = str(tmp_path / "report.tsv")
    with Classifier(par, db_dir=db_dir) as clf:
        assert clf.startClassify(out, reads_per_batch=700, report_tsv=rep) == r.n
        assert clf.last_run["batches"] == 4 and clf.last_run["reads"] == r.n
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), r)
    # the per-taxon report (Reporter::writeReportFile) of the oracle's classifications, byte for byte
    cls, cnt = np.unique(np.where(ores["is_classified"] != 0, ores["classification"], 0), return_counts=True)
    orep = str(tmp_path / "oracle_report.tsv")
    oc.write_report(odb, orep, r.n, dict(zip(cls.tolist(), cnt.tolist())))
    odb.close()
    got, want = open(rep).read(), open(orep).read()
    assert got == want
    assert want.startswith("#clade_proportion\tclade_count\ttaxon_count\trank\ttaxID\tname\n")
    assert len(want.splitlines()) > 3
    rank_of = dict(zip(taxo.taxid.tolist(), taxo.rank))
    lines = open(out).read().split("\n")
    assert lines[0] == "#is_classified\tname\ttaxID\tquery_length\tscore\trank\ttaxID:match_count"
    body = [l for l in lines[1:] if l]
    assert len(body) == r.n
    for i, line in enumerate(body):
        f = line.split("\t")
        o = ores[i]
        assert f[0] == ("1" if o["is_classified"] else "0") and f[1] == names[i]
        assert int(f[2]) == (int(o["classification"]) if o["is_classified"] else 0)
        assert int(f[3]) == int(o["query_length"])
        assert f[4] == "%g" % float(o["score"])
        if o["is_classified"]:
            assert f[5] == rank_of.get(int(o["classification"]), "-")
            s = int(o["taxcnt_offset"])
            want = "".join(f"{int(t)}:{int(c)} " for t, c in otc[s:s + int(o["taxcnt_len"])])
            assert f[6] == want
        else:
            assert f[5:] == ["-", "-", ""]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["bgzf", "gzip"])
def test_start_classify_long_reads_batches(make_db, tmp_path, mode):
    """A long-read (seq-mode 3) file larger than one batch: the pipeline cuts batches by bases
    (max_bases, the reference's RAM-bounded QuerySplits) and the TSV is the oracle's, read by read."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_long_reads(gen, 120, n50=3000, min_len=400, seed=44)
    p1 = str(tmp_path / ("long.fq.gz"))
    synth.write_compressed(p1, synth.fastq_bytes(r.seq1, r.off1, prefix="L"), mode)
    par = LocalParameters(seqMode=3, filenames=[p1, db_dir])
    par.load_db_parameters(db_dir)
    out = str(tmp_path / "long.tsv")
    with Classifier(par, db_dir=db_dir) as clf:
        assert clf.startClassify(out, max_bases=40_000, threads=4) == r.n
        assert clf.last_run["batches"] > 5 and clf.last_run["bases"] == int(r.off1[-1])
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), r)
    odb.close()
    body = [l for l in open(out).read().split("\n")[1:] if l]
    assert len(body) == r.n
    for i, line in enumerate(body):
        f = line.split("\t")
        o = ores[i]
        assert f[1] == f"L{i:09d}"
        assert int(f[2]) == (int(o["classification"]) if o["is_classified"] else 0)
        assert f[4] == "%g" % float(o["score"])
        if o["is_classified"]:
            s = int(o["taxcnt_offset"])
            assert f[6] == "".join(f"{int(t)}:{int(c)} " for t, c in otc[s:s + int(o["taxcnt_len"])])


@pytest.mark.gpu
@pytest.mark.parametrize("n_ctx", [2, 3])
def test_start_classify_multi(make_db, tmp_path, n_ctx):
    """mtb_start_classify_multi: the QuerySplit loop spread over several contexts (here all on
    cuda:0; one per GPU in production), batch k on context k mod n. The TSV and the report are
    byte-identical to the one-context run (which test_start_classify_tsv pins to the oracle) and
    the classifications are the oracle's."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 2300, paired=True, seed=47, short_frac=0.02)
    p1, p2 = str(tmp_path / "q1.fq.gz"), str(tmp_path / "q2.fq.gz")
    synth.write_compressed(p1, synth.fastq_bytes(r.seq1, r.off1, prefix="m"), "bgzf")
    synth.write_compressed(p2, synth.fastq_bytes(r.seq2, r.off2, prefix="m"), "bgzf")
    par = LocalParameters(seqMode=2, filenames=[p1, p2, db_dir])
    par.load_db_parameters(db_dir)
    one, many = str(tmp_path / "one.tsv"), str(tmp_path / "many.tsv")
    rep1, repn = str(tmp_path / "one_report.tsv"), str(tmp_path / "many_report.tsv")
    clfs = [Classifier(par, db_dir=db_dir, device=0) for _ in range(n_ctx)]
    try:
        assert clfs[0].startClassify(one, reads_per_batch=257, report_tsv=rep1) == r.n
        assert clfs[0].startClassify(many, reads_per_batch=257, report_tsv=repn, peers=clfs[1:]) == r.n
        assert clfs[0].last_run["batches"] == (r.n + 256) // 257
        # a second run reuses the contexts' pooled slots and parse buffers: the same bytes
        again = str(tmp_path / "again.tsv")
        assert clfs[0].startClassify(again, reads_per_batch=257, peers=clfs[1:]) == r.n
        assert open(again, "rb").read() == open(one, "rb").read()
        with pytest.raises(MtbError, match="listed twice"):
            clfs[0].startClassify(again, peers=[clfs[0]])
    finally:
        for c in clfs:
            c.close()
    assert open(many, "rb").read() == open(one, "rb").read()
    assert open(repn, "rb").read() == open(rep1, "rb").read()
    odb = oc.OracleDb(db_dir)
    ores, _ = oc.classify(odb, par.to_c(), r)
    odb.close()
    body = [l.split("\t") for l in open(many).read().split("\n")[1:] if l]
    assert [int(f[2]) for f in body] == [int(o["classification"]) if o["is_classified"] else 0 for o in ores]


@pytest.mark.gpu
@pytest.mark.parametrize("raw", [150, 600, 7001, 0])
def test_start_classify_parse_buffer_edges(make_db, tmp_path, monkeypatch, raw):
    """The pipeline's record split (splitter + parse workers): raw buffers of a few hundred bytes cut
    records at every kind of position (150: records longer than the buffer's headroom; plain files
    are read through the buffers with MTB_NO_MMAP, raw 0: mapped and split in place), and the two mates (one wrapped, one not) are cut at different
    reads, so the assembler joins blocks that do not line up. The TSV is the default run's byte for
    byte; unequal mate counts still fail (QueryIndexer.cpp:121-124)."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 900, paired=True, seed=53, short_frac=0.02)
    names = [f"e{i}" for i in range(r.n)]
    p1, p2 = str(tmp_path / "q1.fq"), str(tmp_path / "q2.fq")
    with open(p1, "w") as f:
        for nm, sq in zip(names, _mates(r, 1)):
            s = sq.decode()
            f.write(f"@{nm} x\n" + "".join(s[i:i + 29] + "\n" for i in range(0, len(s), 29)) + "+\n" +
                    "".join("I" * len(s[i:i + 31]) + "\n" for i in range(0, len(s), 31)))
    _write_fastq(p2, names, _mates(r, 2))
    par = LocalParameters(seqMode=2, filenames=[p1, p2, db_dir])
    par.load_db_parameters(db_dir)
    ref, got = str(tmp_path / "ref.tsv"), str(tmp_path / "got.tsv")
    with Classifier(par, db_dir=db_dir) as clf:
        monkeypatch.setenv("MTB_NO_MMAP", "1")  # the reference run: default buffers
        assert clf.startClassify(ref, reads_per_batch=301) == r.n
        if raw:
            monkeypatch.setenv("MTB_PARSE_BUFFER", str(raw))
        else:
            monkeypatch.delenv("MTB_NO_MMAP")
        assert clf.startClassify(got, reads_per_batch=301) == r.n
        assert open(got, "rb").read() == open(ref, "rb").read()
        short = str(tmp_path / "short.fq")
        _write_fastq(short, names[:-1], _mates(r, 2)[:-1])
        par2 = LocalParameters(seqMode=2, filenames=[p1, short, db_dir])
        par2.load_db_parameters(db_dir)
        clf.par = par2
        with pytest.raises(MtbError, match="different read counts"):
            clf.startClassify(str(tmp_path / "bad.tsv"), reads_per_batch=301)


@pytest.mark.gpu
@pytest.mark.parametrize("part", [4096, 65536])
def test_start_classify_mapped_parts_prefault(make_db, tmp_path, monkeypatch, part):
    """Plain query files are mapped and given back in parts as the parse jobs finish with them, and a
    helper thread touches the parts up to four ahead of each mate's splitter (round 5). With parts of
    one page or 64 KB (MTB_MAP_PART) the prefaulter, the splitter and the parts' release interleave
    over hundreds of parts: the TSV equals the run read through buffers (MTB_NO_MMAP) and the one
    without prefaulting, byte for byte, and the oracle's taxIDs."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 1200, paired=True, seed=67, short_frac=0.02)
    names = [f"m{i}" for i in range(r.n)]
    p1, p2 = str(tmp_path / "q1.fq"), str(tmp_path / "q2.fq")
    _write_fastq(p1, names, _mates(r, 1))
    _write_fastq(p2, names, _mates(r, 2))
    par = LocalParameters(seqMode=2, filenames=[p1, p2, db_dir])
    par.load_db_parameters(db_dir)
    out = {}
    with Classifier(par, db_dir=db_dir) as clf:
        for name, env in (("buffers", {"MTB_NO_MMAP": "1"}), ("noprefault", {"MTB_PREFAULT": "0"}),
                          ("prefault", {"MTB_PREFAULT": "1"})):
            for k in ("MTB_NO_MMAP", "MTB_PREFAULT"):
                monkeypatch.delenv(k, raising=False)
            monkeypatch.setenv("MTB_MAP_PART", str(part))
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            out[name] = str(tmp_path / f"{name}.tsv")
            assert clf.startClassify(out[name], reads_per_batch=257) == r.n
    ref = open(out["buffers"], "rb").read()
    assert open(out["noprefault"], "rb").read() == ref
    assert open(out["prefault"], "rb").read() == ref
    odb = oc.OracleDb(db_dir)
    ores, _ = oc.classify(odb, par.to_c(), r)
    odb.close()
    body = [l.split("\t") for l in ref.decode().split("\n")[1:] if l]
    assert [int(f[2]) for f in body] == [int(o["classification"]) if o["is_classified"] else 0 for o in ores]


@pytest.mark.gpu
def test_clone_shares_db(make_db, tmp_path):
    """mtb_clone: a second context over the same DB arrays, with its own stream and workspace. Two
    batches in flight on one GPU through mtb_start_classify_multi write the one-context TSV and
    report; the clone keeps working after its parent closed (the shared arrays go with the last
    holder)."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 1500, paired=True, seed=61, short_frac=0.02)
    p1, p2 = str(tmp_path / "c1.fq.gz"), str(tmp_path / "c2.fq.gz")
    synth.write_compressed(p1, synth.fastq_bytes(r.seq1, r.off1, prefix="c"), "bgzf")
    synth.write_compressed(p2, synth.fastq_bytes(r.seq2, r.off2, prefix="c"), "bgzf")
    par = LocalParameters(seqMode=2, filenames=[p1, p2, db_dir])
    par.load_db_parameters(db_dir)
    one, two = str(tmp_path / "one.tsv"), str(tmp_path / "two.tsv")
    rep1, rep2 = str(tmp_path / "one_report.tsv"), str(tmp_path / "two_report.tsv")
    clf = Classifier(par, db_dir=db_dir)
    twin = clf.clone()
    try:
        assert clf.startClassify(one, reads_per_batch=211, report_tsv=rep1) == r.n
        assert clf.startClassify(two, reads_per_batch=211, report_tsv=rep2, peers=[twin]) == r.n
        assert open(two, "rb").read() == open(one, "rb").read()
        assert open(rep2, "rb").read() == open(rep1, "rb").read()
        b1 = clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
        res1, tc1 = b1.results.copy(), b1.taxcnt.copy()
        clf.close()
        b2 = twin.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
        assert np.array_equal(b2.results, res1) and np.array_equal(b2.taxcnt, tc1)
    finally:
        clf.close()
        twin.close()
