"""HBM exhaustion as the reference's retry (KmerMatcher.cpp:474-476 returns false, Classifier.cpp:127-130
searches the split again): a batch whose workspace passes the context's cap (mtb_set_workspace_cap,
MTB_WORKSPACE_CAP) returns MTB_RETRY with the context usable, and the callers classify it in pieces —
Classifier.classify_batch in halves, mtb_start_classify halving down to one read. The results equal the
one-batch run and the oracle's."""
import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd._abi import RESULT_DTYPE, TAXCNT_DTYPE
from metabuli_work_amd.classifier import BatchResult, Classifier, LocalParameters
from tests import oracle_ctypes as oc


def _same(a, b):
    assert np.array_equal(a.results["classification"], b.results["classification"])
    assert np.array_equal(a.results["score"].view(np.uint32), b.results["score"].view(np.uint32))
    assert np.array_equal(a.results["hamming_dist"], b.results["hamming_dist"])
    for i in range(len(a.results)):
        assert a.taxcnt_of(i) == b.taxcnt_of(i)


@pytest.mark.gpu
@pytest.mark.parametrize("frac", [0.6, 0.3])
def test_classify_batch_split_on_retry(make_db, frac):
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 1500, paired=True, seed=61, short_frac=0.03)
    par = LocalParameters(seqMode=2)
    par.load_db_parameters(db_dir)
    with Classifier(par, db_dir=db_dir) as full:
        ref = full.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
        ws = full.workspace_bytes
    assert ws > 0
    with Classifier(par, db_dir=db_dir) as capped:
        capped.set_workspace_cap(int(ws * frac))
        got = capped.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
        assert capped.workspace_bytes <= int(ws * frac)
        _same(got, ref)
        # the context stays usable: a batch that fits runs whole
        small = capped.classify_batch(r.seq1, r.off1[:101], r.seq2, r.off2[:101])
        assert np.array_equal(small.results["classification"], ref.results["classification"][:100])
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), r)
    odb.close()
    assert np.array_equal(got.results["classification"], ores["classification"])
    assert np.array_equal(got.results["score"].view(np.uint32), ores["score"].view(np.uint32))
    assert np.array_equal(got.taxcnt, otc)


@pytest.mark.gpu
def test_classify_batch_retry_raises_when_one_read_does_not_fit(make_db):
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 64, paired=True, seed=62)
    par = LocalParameters(seqMode=2)
    par.load_db_parameters(db_dir)
    from metabuli_work_amd._lib import MtbError
    with Classifier(par, db_dir=db_dir) as clf:
        clf.set_workspace_cap(4096)
        with pytest.raises(MtbError, match="out of HBM"):
            clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
        clf.set_workspace_cap(0)  # usable again once it fits
        assert len(clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2).results) == r.n


@pytest.mark.gpu
def test_start_classify_splits_on_retry(make_db, tmp_path):
    """The file pipeline halves a batch that does not fit and bounds the later batches by the piece
    that did; the TSV and report are byte-identical to the uncapped run."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 2400, paired=True, seed=63, short_frac=0.02)
    p1, p2 = str(tmp_path / "q1.fq"), str(tmp_path / "q2.fq")
    with open(p1, "wb") as f:
        f.write(synth.fastq_bytes(r.seq1, r.off1, prefix="s"))
    with open(p2, "wb") as f:
        f.write(synth.fastq_bytes(r.seq2, r.off2, prefix="s"))
    par = LocalParameters(seqMode=2, filenames=[p1, p2, db_dir])
    par.load_db_parameters(db_dir)
    one, cut = str(tmp_path / "one.tsv"), str(tmp_path / "cut.tsv")
    rep1, repc = str(tmp_path / "one_rep.tsv"), str(tmp_path / "cut_rep.tsv")
    with Classifier(par, db_dir=db_dir) as clf:
        assert clf.startClassify(one, reads_per_batch=800, report_tsv=rep1) == r.n
        assert clf.last_run["split_batches"] == 0
        ws = clf.workspace_bytes
    with Classifier(par, db_dir=db_dir) as clf:
        clf.set_workspace_cap(int(ws * 0.45))
        assert clf.startClassify(cut, reads_per_batch=800, report_tsv=repc) == r.n
        assert clf.last_run["split_batches"] >= 1
    assert open(cut, "rb").read() == open(one, "rb").read()
    assert open(repc, "rb").read() == open(rep1, "rb").read()


@pytest.mark.gpu
def test_release_workspace(make_db):
    """mtb_release_workspace gives the batch workspace back (0 bytes held) and the next batch regrows it
    with the same results."""
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 800, paired=True, seed=62, short_frac=0.03)
    par = LocalParameters(seqMode=2)
    par.load_db_parameters(db_dir)
    with Classifier(par, db_dir=db_dir) as clf:
        a = clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
        assert clf.workspace_bytes > 0
        clf.release_workspace()
        assert clf.workspace_bytes == 0
        b = clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
        assert clf.workspace_bytes > 0
        _same(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("frac", [0.6, 0.3])
def test_device_resident_batch_split_on_retry(make_db, frac):
    """classify_batch(fetch=False) — the bench's device-resident path, inputs and results in HBM — on
    a capped context: the batch is classified in halves (split again where needed) and the halves'
    result records and taxID:count lists assembled on the device, so copy_results / copy_taxcnt /
    n_taxcnt / last_counts read one batch equal to the uncapped run and to the oracle; release of the
    workspace afterwards leaves no stale batch behind (the getters see an empty one)."""
    import torch

    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 1500, paired=True, seed=64, short_frac=0.03)
    par = LocalParameters(seqMode=2)
    par.load_db_parameters(db_dir)
    dev = torch.device("cuda", 0)
    s1, o1 = torch.from_numpy(r.seq1).to(dev), torch.from_numpy(r.off1.astype(np.uint64).view(np.int64)).to(dev)
    s2, o2 = torch.from_numpy(r.seq2).to(dev), torch.from_numpy(r.off2.astype(np.uint64).view(np.int64)).to(dev)

    def run(clf):
        clf.classify_batch(s1, o1, s2, o2, device_input=True, fetch=False)
        rec = torch.zeros((r.n, 32), dtype=torch.uint8, device=dev)
        clf.copy_results(rec.data_ptr(), on_device=True)
        pool = torch.zeros((max(clf.n_taxcnt(), 1), 8), dtype=torch.uint8, device=dev)
        nt = clf.copy_taxcnt(pool.data_ptr(), on_device=True)
        torch.cuda.synchronize()
        res = rec.cpu().numpy().view(RESULT_DTYPE).reshape(-1)
        tc = pool[:nt].cpu().numpy().view(TAXCNT_DTYPE).reshape(-1)
        return BatchResult(res, tc, *clf.last_counts(), None)

    with Classifier(par, db_dir=db_dir) as full:
        ref = run(full)
        ref_stats = full.stats()
        ws = full.workspace_bytes
    with Classifier(par, db_dir=db_dir) as capped:
        capped.set_workspace_cap(int(ws * frac))
        got = run(capped)
        assert capped.workspace_bytes <= int(ws * frac)
        _same(got, ref)
        assert got.query_kmers == ref.query_kmers and got.matches == ref.matches
        # every getter serves the assembled batch: the host taxID:count list, the work
        # counts summed over the pieces, the pieces' device times
        assert np.array_equal(capped.taxcnt(), ref.taxcnt)
        st = capped.stats()
        assert st["query_kmers"] == ref_stats["query_kmers"] and st["matches"] == ref_stats["matches"] == ref.matches
        assert st["max_read_matches"] == ref_stats["max_read_matches"]  # (slots: each piece pads its own units)
        assert capped.stage_ms()[4] > 0 and capped.kernel_ms().sum() > 0
        # a later batch that fits serves the context's own buffers again
        small = capped.classify_batch(r.seq1, r.off1[:101], r.seq2, r.off2[:101])
        assert np.array_equal(small.results["classification"], ref.results["classification"][:100])
        # a second assembled batch, then a release: nothing of it is served afterwards
        run(capped)
        capped.release_workspace()
        assert capped.n_taxcnt() == 0 and capped.last_counts() == (0, 0)
        assert len(capped.taxcnt()) == 0 and capped.stats()["matches"] == 0
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), r)
    odb.close()
    assert np.array_equal(got.results["classification"], ores["classification"])
    assert np.array_equal(got.results["score"].view(np.uint32), ores["score"].view(np.uint32))
    assert np.array_equal(got.taxcnt, otc)
