"""Parity of the HIP path (through the C-ABI) against the oracle, per stage and end to end.

Bar: bit-exact for k-mers, matches, taxIDs and taxID:count lists; per-read float score within
1e-6 (the tolerance north_star states) — in practice the scores are compared bitwise too, since
the device follows the reference's float operations one by one.
"""
import os
import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd._abi import MATCH_DTYPE, info_seq
from metabuli_work_amd.classifier import Classifier, LocalParameters
from tests import oracle_ctypes as oc

pytestmark = pytest.mark.gpu

SCORE_TOL = 1e-6


def _kmer_sorted(k):
    return np.sort(k, order=["value", "info"])


def _match_sorted(m):
    return np.sort(m, order=["qinfo", "species_id", "target_id", "dna_encoding", "right_end_hamming", "hamming"])


def _params(db_dir, seq_mode):
    par = LocalParameters(seqMode=seq_mode)
    par.load_db_parameters(db_dir)
    return par


def _reads(gen, kind, n, seed):
    if kind == "paired":
        return synth.make_reads(gen, n, paired=True, seed=seed, short_frac=0.03, rate_n=0.002, rate_iupac=0.001,
                                rate_lower=0.002)
    if kind == "single":
        return synth.make_reads(gen, n, paired=False, seed=seed, short_frac=0.03, rate_n=0.002)
    if kind == "longbig":  # segments past 2048 matches: thinning + the compact 2049-8192-match sorts
        return synth.make_long_reads(gen, n, n50=12000, min_len=4000, seed=seed)
    return synth.make_long_reads(gen, n, n50=3000, min_len=400, seed=seed)


SEQ_MODE = {"paired": 2, "single": 1, "long": 3, "longbig": 3}


def compare_results(gres, gtc, ores, otc):
    assert len(gres) == len(ores)
    np.testing.assert_array_equal(gres["is_classified"], ores["is_classified"])
    np.testing.assert_array_equal(gres["classification"], ores["classification"])
    np.testing.assert_array_equal(gres["query_length"], ores["query_length"])
    np.testing.assert_allclose(gres["score"], ores["score"], rtol=0, atol=SCORE_TOL)
    assert np.array_equal(gres["score"].view(np.uint32), ores["score"].view(np.uint32)), "scores not bit-identical"
    np.testing.assert_array_equal(gres["taxcnt_len"], ores["taxcnt_len"])
    for i in range(len(gres)):
        a = gtc[gres["taxcnt_offset"][i]:gres["taxcnt_offset"][i] + gres["taxcnt_len"][i]]
        b = otc[ores["taxcnt_offset"][i]:ores["taxcnt_offset"][i] + ores["taxcnt_len"][i]]
        assert np.array_equal(a, b), f"read {i}: taxcnt {a} != {b}"


def _db_aa_ranks(db_dir, fmt):
    """AA ranks of all DB k-mers (diffIdx decoded as getNextTargetKmer does)."""
    diff = np.fromfile(os.path.join(db_dir, "diffIdx"), np.uint16).astype(np.uint64)
    term = np.nonzero(diff & np.uint64(0x8000))[0]
    starts = np.concatenate([[0], term[:-1] + 1])
    kidx = np.repeat(np.arange(len(term)), term - starts + 1)
    shift = (term[kidx] - np.arange(len(diff))) * 15
    vals = np.cumsum(np.add.reduceat((diff & np.uint64(0x7FFF)) << shift.astype(np.uint64), starts), dtype=np.uint64)
    return np.unique(_aa_rank(vals, fmt))


def _aa_rank(values, fmt):
    """Base-21 rank of the 8 AA codes (format 1 stores it directly, format 2 packs 5-bit codes)."""
    aa = values >> np.uint64(24)
    if fmt != 2:
        return aa
    r = np.zeros_like(aa)
    for i in range(7, -1, -1):
        r = r * np.uint64(21) + ((aa >> np.uint64(5 * i)) & np.uint64(31))
    return r


@pytest.mark.parametrize("db_name,kind", [
    ("fmt2", "paired"), ("fmt2", "single"), ("fmt2", "long"),
    ("fmt2_syncmer", "paired"), ("fmt2_syncmer", "long"),
    ("fmt1", "paired"), ("fmt1", "single"),
])
def test_stage_parity(make_db, db_name, kind):
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE[kind])
    reads = _reads(gen, kind, 300 if kind != "long" else 40, seed=5)
    opar = par.to_c()
    odb = oc.OracleDb(db_dir)
    okmers, ql1, ql2 = oc.extract(opar, reads)
    omatches = oc.match(odb, opar, okmers)
    ores, otc = oc.assign(odb, opar, omatches, ql1, ql2)

    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, keep_stages=True)
        # K1 + K2: the multiset of query k-mers (blank reserved slots dropped, and those whose AA
        # 8-mer is absent from the DB: they cannot match, KmerMatcher.cpp compares AA parts first)
        gk = clf.query_kmers()
        ok = okmers_present(okmers, db_dir, par)
        assert len(gk) == len(ok) == clf.stats()["query_kmers"]
        # mtb_last_counts: the reference's "Query k-mer number" (KmerMatcher.cpp:143-152), every
        # non-blank query k-mer before any DB test
        assert br.query_kmers == int((info_seq(okmers["info"]) != 0).sum())
        assert np.array_equal(_kmer_sorted(gk), _kmer_sorted(ok))
        # K2: ordered by the top 24 bits of the 36-bit base-21 AA rank (kQuerySortLo/Hi)
        pre = _aa_rank(gk["value"], par.kmerFormat) >> np.uint64(12)
        assert np.all(pre[1:] >= pre[:-1])
        # K3 + K4: the multiset of matches
        gm = clf.matches()
        assert len(gm) == len(omatches) == br.matches
        assert np.array_equal(_match_sorted(gm), _match_sorted(omatches))
        # K5: matches come back in compareMatches order
        assert np.array_equal(gm, omatches)
        # K6 end to end
        compare_results(br.results, br.taxcnt, ores, otc)
        # K5 + K6 alone on the oracle's matches
        shuffled = omatches[np.random.default_rng(0).permutation(len(omatches))]
        ar = clf.assign_matches(shuffled, ql1 + ql2)
        compare_results(ar.results, ar.taxcnt, ores, otc)
    odb.close()


def okmers_present(okmers, db_dir, par):
    """The oracle's query k-mers K1F keeps: non-blank, AA 8-mer present in the DB."""
    ok = okmers[info_seq(okmers["info"]) != 0]
    return ok[np.isin(_aa_rank(ok["value"], par.kmerFormat), _db_aa_ranks(db_dir, par.kmerFormat))]


def line_ext_check(clf):
    """mtb_line_ext_check: (ranks within reach, resolved by the run-length codes, mismatches)."""
    import ctypes
    from metabuli_work_amd._lib import lib
    out = (ctypes.c_uint64 * 3)()
    rc = lib().mtb_line_ext_check(clf.handle, out)
    assert rc == 0, lib().mtb_last_error().decode()
    return tuple(int(x) for x in out)


@pytest.mark.parametrize("db_name", ["fmt2", "fmt2_syncmer", "fmt1", "fmt2_acc"])
def test_line_ext_matches_run_index(make_db, db_name, monkeypatch):
    """The run-length lines built at open (2-bit run lengths per present AA rank beside each probe
    line) give every present rank within their reach the run the run index holds: the same start
    and length wherever no escape precedes it, and no DB leaves them empty of resolvable ranks. With
    MTB_LINE_EXT=0 (the default) there are none and the entry point says so."""
    db_dir, taxo, gen = make_db(db_name)
    monkeypatch.setenv("MTB_LINE_EXT", "1")
    with Classifier(_params(db_dir, 2), db_dir=db_dir) as clf:
        n, ok, bad = line_ext_check(clf)
        assert bad == 0 and n > 0 and ok > 0
    monkeypatch.setenv("MTB_LINE_EXT", "0")
    with Classifier(_params(db_dir, 2), db_dir=db_dir) as clf:
        import ctypes
        from metabuli_work_amd._lib import lib
        out = (ctypes.c_uint64 * 3)()
        assert lib().mtb_line_ext_check(clf.handle, out) != 0


@pytest.mark.parametrize("db_name", ["fmt2", "fmt2_syncmer", "fmt1", "fmt2_acc"])
def test_link_lines_match_probe_lines(make_db, db_name, monkeypatch):
    """The link lines built at open (round 6: per AA 7-mer the 21 AAs that may follow it and the 21
    that may precede it) hold, for every one of the 21^8 AA ranks, the membership bit of the probe
    lines in both places that stand for it (mtb_link_check, by plain division). Without them
    (MTB_LINK_LINES=0) the entry point says so, and K1F reads the probe lines."""
    import ctypes
    from metabuli_work_amd._lib import lib
    db_dir, taxo, gen = make_db(db_name)
    with Classifier(_params(db_dir, 2), db_dir=db_dir) as clf:
        out = (ctypes.c_uint64 * 3)()
        rc = lib().mtb_link_check(clf.handle, out)
        assert rc == 0, lib().mtb_last_error().decode()
        # (the DB's last k-mer, never a candidate, may or may not leave its rank's bit)
        assert out[0] == 21 ** 8 and out[2] == 0
        assert abs(int(out[1]) - len(_db_aa_ranks(db_dir, clf.par.kmerFormat))) <= 1
    monkeypatch.setenv("MTB_LINK_LINES", "0")
    with Classifier(_params(db_dir, 2), db_dir=db_dir) as clf:
        out = (ctypes.c_uint64 * 3)()
        assert lib().mtb_link_check(clf.handle, out) != 0


@pytest.mark.parametrize("db_name", ["fmt2", "fmt2_syncmer", "fmt1"])
def test_end_to_end_batches(make_db, db_name):
    """Whole path, several batches, against oracle classify."""
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, 2)
    odb = oc.OracleDb(db_dir)
    with Classifier(par, db_dir=db_dir) as clf:
        for seed in (21, 22):
            reads = _reads(gen, "paired", 1500, seed)
            ores, otc = oc.classify(odb, par.to_c(), reads)
            br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
            compare_results(br.results, br.taxcnt, ores, otc)
            assert br.results["is_classified"].mean() > 0.5
    odb.close()


@pytest.mark.parametrize("db_name", ["fmt2", "fmt1"])
@pytest.mark.parametrize("window", ["0", "0:gallop", "0:staged", "0:retry", "0:spill", "0:fine28", "0:unfused",
                                    "0:nodigits", "0:atomiclines", "0:matchxcd", "0:nofast", "0:blockjoin", "0:pipejoin", "0:wave64join", "0:pairjoin", "0:wavepack", "0:nolink", "0:share", "0:bins", "0:binsover", "0:binsnodig", "0:ext", "0:atomicfirst", "0:ballot", "64",
                                    "6144", "6144:staged", "6144:spill", "6144:unfused", "0:nofilter", "6144:nofilter"])
def test_match_window_paths(make_db, db_name, window, monkeypatch):
    """K4's search paths — DB window staged in LDS, or HBM search (the unstaged join: runs from the
    run index, or galloped from the probe line's lower bound with MTB_RUN_INDEX=0) — give the
    oracle's matches whatever the per-block window cap (0 forces the HBM path); and both outputs —
    matches written straight into each read's slot stretch (default), or staged + transposed
    (MTB_DIRECT=0), also when a direct join is rerun staged (MTB_DIRECT=2, the overflow fallback)
    or queries past their read's stretch spill and are scattered after the compaction (MTB_DIRECT=3
    quarters the stretches; the batch then classifies as the oracle does); K1 and K1F fused (the
    default) or apart (MTB_FUSE_FILTER=0: K1 writes every window's key, K1F reads them back);
    and the unstaged join over queries sorted on a 32-bit AA-rank prefix (MTB_SORT_LO_FINE=28, its
    own block line ranges and LDS staging). The unstaged default modes run k_join_uniform (the
    production join: uniform units, run index, direct output); "nofast" the same batch through
    k_match's lean form; "blockjoin" / "pipejoin" through k_join_uniform's block-staged / resident-wave forms; "nolink" K1F through the probe lines alone (no link lines)."""
    window, _, mode = window.partition(":")
    monkeypatch.setenv("MTB_SORT_LO_FINE", "28" if mode == "fine28" else "36")
    monkeypatch.setenv("MTB_MATCH_WINDOW", window)
    monkeypatch.setenv("MTB_RUN_INDEX", "0" if mode == "gallop" else "1")
    monkeypatch.setenv("MTB_DIRECT", {"staged": "0", "retry": "2", "spill": "3"}.get(mode, "1"))
    monkeypatch.setenv("MTB_FUSE_FILTER", "0" if mode == "unfused" else "1")
    monkeypatch.setenv("MTB_FILTER", "0" if mode == "nofilter" else "1")
    monkeypatch.setenv("MTB_RADIX_DIGITS", "0" if mode == "nodigits" else "1")  # K2 histograms from the keys
    # probe lines and run index built by per-k-mer global atomics (round 4's) instead of a wave per line
    monkeypatch.setenv("MTB_LINE_BUILD", "atomic" if mode == "atomiclines" else "wave")
    monkeypatch.setenv("MTB_MATCH_XCD", "1" if mode == "matchxcd" else "0")  # K4 blocks per XCD eighth
    monkeypatch.setenv("MTB_SHARE_RUNS", "1" if mode == "share" else "0")  # same-AA queries share one lookup
    # the production configuration through k_match's lean form instead of k_join_uniform (round 6)
    monkeypatch.setenv("MTB_JOIN_FAST", "0" if mode == "nofast" else "1")
    # k_join_uniform's staging: per wave (the default), per block (round 6's first form), or resident waves
    # with the next tile's lines and keys in flight (A/B)
    monkeypatch.setenv("MTB_JOIN_WAVE", {"blockjoin": "0", "pipejoin": "2", "wave64join": "4", "pairjoin": "7"}.get(mode, "1"))
    # the fused K1F's one probe-line read per window instead of the link lines' one read per window pair
    monkeypatch.setenv("MTB_LINK_LINES", "0" if mode == "nolink" else "1")
    # the fused K1F packing its present windows per wave, no block barrier per group (A/B, round 6)
    monkeypatch.setenv("MTB_K1F_WAVEPACK", "1" if mode == "wavepack" else "0")
    # K1F writing straight into K2's first-pass buckets at any batch size; with 64-slot buckets, which
    # overflow, so the batch reruns through the packed K1F
    monkeypatch.setenv("MTB_K1F_BINS", "2" if mode.startswith("bins") else "0")
    monkeypatch.setenv("MTB_K1F_BINS_RC", "64" if mode == "binsover" else "0")
    monkeypatch.setenv("MTB_K1F_BINS_DIG", "0" if mode == "binsnodig" else "1")  # K2's second pass reads the keys
    monkeypatch.setenv("MTB_LINE_EXT", "1" if mode == "ext" else "0")  # K4's runs from run-length lines (A/B)
    monkeypatch.setenv("MTB_RADIX_ATOMIC_FIRST", "1" if mode == "atomicfirst" else "0")  # K2's first pass ranked by LDS atomics
    monkeypatch.setenv("MTB_RADIX_ORRANK", "0" if mode == "ballot" else "1")  # K2 ranked by ballots, or lane masks
    # warp-specialised resident blocks, resident blocks walking their tiles (the default form), one block per
    # tile; 24-KB tiles for the last two
    monkeypatch.setenv("MTB_SWEEP_PERSIST", {"perblock": "0", "persist": "1"}.get(mode, "2"))
    monkeypatch.setenv("MTB_SWEEP_SMALL", "1" if mode == "small" else "0")  # every window joined, absent AA 8-mers too
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, 2)
    reads = _reads(gen, "paired", 2000, seed=9)
    opar = par.to_c()
    odb = oc.OracleDb(db_dir)
    okmers, ql1, ql2 = oc.extract(opar, reads)
    omatches = oc.match(odb, opar, okmers)
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, keep_stages=True)
        gm = clf.matches()
        assert len(gm) == len(omatches) == br.matches
        assert np.array_equal(gm, omatches)
        if mode.startswith("bins"):  # K2's order after the binned first pass (or its packed rerun)
            gk = clf.query_kmers()
            pre = _aa_rank(gk["value"], par.kmerFormat) >> np.uint64(12)
            assert len(gk) == clf.stats()["query_kmers"] and np.all(pre[1:] >= pre[:-1])
            assert np.array_equal(_kmer_sorted(gk), _kmer_sorted(okmers_present(okmers, db_dir, par)))
            assert clf.stats()["filter_reruns"] == (1 if mode == "binsover" else 0)
        if mode in ("", "ballot"):
            # K2's pair multiset, and its 24-bit prefix order, which the LSD passes after the first give only
            # if they are stable (K1F's packing order, and so the order within a prefix, varies run to run)
            gk = clf.query_kmers()
            pre = _aa_rank(gk["value"], par.kmerFormat) >> np.uint64(12)
            assert np.all(pre[1:] >= pre[:-1])
            assert np.array_equal(_kmer_sorted(gk), _kmer_sorted(okmers_present(okmers, db_dir, par)))
        if mode == "spill":
            assert clf.stats()["spilled_matches"] > 0
            ores, otc = oc.classify(odb, opar, reads)
            br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
            assert clf.stats()["spilled_matches"] > 0
            compare_results(br.results, br.taxcnt, ores, otc)
    odb.close()


@pytest.mark.parametrize("pack", ["", "thread"])
@pytest.mark.parametrize("db_name,kind", [("fmt2", "paired"), ("fmt2_syncmer", "long"), ("fmt1", "paired")])
def test_filter_output_rerun(make_db, db_name, kind, pack, monkeypatch):
    """The fused K1 + K1F writes into a buffer sized from the present share of earlier batches; a
    batch whose present windows outgrow it reruns the filter into a larger one (MTB_PRESENT_SHARE
    starts the share far too small): the k-mers, matches and results stay the oracle's, and the
    next batch fits without a rerun. Both output orders: block-wide (window, wave, lane) (default)
    and thread-major (MTB_FILTER_PACK=thread)."""
    monkeypatch.setenv("MTB_PRESENT_SHARE", "0.001")
    monkeypatch.setenv("MTB_FILTER_PACK", pack)
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE[kind])
    opar = par.to_c()
    odb = oc.OracleDb(db_dir)
    with Classifier(par, db_dir=db_dir) as clf:
        for i, seed in enumerate((31, 32)):
            reads = _reads(gen, kind, 600 if kind != "long" else 40, seed=seed)
            okmers, ql1, ql2 = oc.extract(opar, reads)
            omatches = oc.match(odb, opar, okmers)
            br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, keep_stages=True)
            assert clf.stats()["filter_reruns"] == (1 if i == 0 else 0)
            assert np.array_equal(clf.matches(), omatches)
            ores, otc = oc.classify(odb, opar, reads)
            br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
            compare_results(br.results, br.taxcnt, ores, otc)
    odb.close()


@pytest.mark.parametrize("compact", ["1", "0"])
@pytest.mark.parametrize("db_name,kind,glob,merge", [
    ("fmt2", "paired", "1", "0"), ("fmt2", "long", "1", "0"), ("fmt1", "long", "1", "0"),
    ("fmt2", "paired", "0", "after1"), ("fmt2", "long", "0", "after1"), ("fmt2_syncmer", "long", "0", "after1"),
    ("fmt2", "long", "0", "big0"), ("fmt1", "long", "0", "big0"),
    ("fmt2", "long", "0", "0"), ("fmt2_syncmer", "long", "0", "0"),
    ("fmt2", "long", "0", "512"), ("fmt1", "long", "0", "600"), ("fmt2_syncmer", "long", "0", "512"),
    ("fmt2", "long", "0", "after2"), ("fmt1", "longbig", "0", "after2"), ("fmt2_syncmer", "longbig", "0", "after2"),
    ("fmt2", "longbig", "0", "after2"), ("fmt2", "longbig", "0", "after4"), ("fmt2", "paired", "0", "after2")])
def test_pruned_segment_sorts(make_db, db_name, kind, glob, merge, compact, monkeypatch):
    """Dead-match pruning in every K5 variant, results against the oracle: long reads put segments
    in the 1024-thread LDS sort; MTB_SEGSORT_GLOBAL=1 sends every segment through the global-scratch
    sort; MTB_MERGE_SEG=n sends segments over n matches through the chunked LDS sorts + merge path
    (long reads' path above 8192 matches). Segments over that bound are thinned in place before
    their sort (k_thin_big: lossy LDS counts of the whole segment), or, with MTB_PRUNE_COMPACT=0,
    sorted whole and pruned after the merge. The 129-512-match register sorts prune, then sort the
    live matches (default), or with MTB_PRUNE_AFTER=1 sort whole segments and prune on the sorted
    order; MTB_PRUNE_AFTER=2 (the default) sorts on rank keys and runs the 2049-8192-match sorts on
    compact keys (register runs + merge path), =4 the same on the LDS bitonic network."""
    monkeypatch.setenv("MTB_SEGSORT_GLOBAL", glob)
    monkeypatch.setenv("MTB_PRUNE_AFTER", merge[5:] if merge.startswith("after") else "0")
    monkeypatch.setenv("MTB_MERGE_SEG", "0" if merge.startswith(("after", "big")) else merge)
    # K6: groups of >= 256 matches on a wave each (default) or on a thread (MTB_BIG_GROUPS=0)
    monkeypatch.setenv("MTB_BIG_GROUPS", "0" if merge == "big0" else "1")
    monkeypatch.setenv("MTB_PRUNE_COMPACT", compact)
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE[kind])
    odb = oc.OracleDb(db_dir)
    reads = _reads(gen, kind, {"long": 60, "longbig": 40}.get(kind, 1500), 35)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        assert clf.stats()["live_matches"] < br.matches
        compare_results(br.results, br.taxcnt, ores, otc)
    odb.close()


@pytest.mark.parametrize("db_name", ["fmt2", "fmt2_syncmer", "fmt1"])
def test_general_paths(make_db, db_name, monkeypatch):
    """MTB_FORCE_GENERIC=1 turns off every fast path (LDS DB windows in K4, register and LDS sorts in
    K5, register DP in K6), so the general code the fast paths fall back to is held to the oracle
    too."""
    monkeypatch.setenv("MTB_FORCE_GENERIC", "1")
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, 2)
    odb = oc.OracleDb(db_dir)
    reads = _reads(gen, "paired", 1500, 31)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        compare_results(br.results, br.taxcnt, ores, otc)
    odb.close()


@pytest.mark.parametrize("db_name,kind", [
    ("fmt2", "paired"), ("fmt2", "long"), ("fmt2_syncmer", "paired"), ("fmt2_syncmer", "long"),
    ("fmt1", "paired"), ("fmt1", "single"),
])
@pytest.mark.parametrize("join", ["probe", "sort"])
def test_join_paths(make_db, db_name, kind, join, monkeypatch):
    """Both joins — the probe join (read order, probe lines + DB runs, no query sort) and the
    sort-merge join (radix-sorted queries against LDS windows of the DB) — give the oracle's
    query k-mer count, matches (after K5, in compareMatches order) and classifications."""
    monkeypatch.setenv("MTB_JOIN", join)
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE[kind])
    reads = _reads(gen, kind, 1200 if kind != "long" else 60, seed=77)
    opar = par.to_c()
    odb = oc.OracleDb(db_dir)
    okmers, ql1, ql2 = oc.extract(opar, reads)
    omatches = oc.match(odb, opar, okmers)
    ores, otc = oc.assign(odb, opar, omatches, ql1, ql2)
    ok = okmers[info_seq(okmers["info"]) != 0]
    ok = ok[np.isin(_aa_rank(ok["value"], par.kmerFormat), _db_aa_ranks(db_dir, par.kmerFormat))]
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, keep_stages=True)
        assert clf.stats()["join_path"] == (0 if join == "probe" else 1)
        assert clf.stats()["query_kmers"] == len(ok)
        assert clf.stats()["gallop_queries"] <= len(ok)  # run-index fallbacks (none on lines < 64K k-mers)
        assert br.query_kmers == int((info_seq(okmers["info"]) != 0).sum())
        gm = clf.matches()
        assert len(gm) == len(omatches) == br.matches
        assert np.array_equal(gm, omatches)
        compare_results(br.results, br.taxcnt, ores, otc)
    odb.close()


@pytest.mark.parametrize("db_name,kind", [("fmt2", "paired"), ("fmt2", "long"), ("fmt1", "long"),
                                          ("fmt2_syncmer", "long"), ("fmt2_syncmer", "paired"), ("fmt2", "verylong"),
                                          ("fmt1", "verylong")])
@pytest.mark.parametrize("wave", ["0", "1", "1:emu", "2"])
def test_choose_taxon_kernels(make_db, db_name, kind, wave, monkeypatch):
    """K6's chooseBestTaxon every way — a thread per read (short reads), a wave per read (long
    reads: parallel species scan, per-quotient LDS reduction for filterRedundantMatches) and a
    16-lane group per read (the same reductions per group; reads past its LDS tables take the
    serial filter) — forced on every read kind with MTB_WAVE_TAXON, against the oracle; and k_combine_wave's libstdc++
    introsort emulation forced for every run it takes (MTB_EMULATE_SORT). "verylong": reads of
    12-20 kb, whose quotients take several LDS windows in the wave kernel."""
    wave, _, emu = wave.partition(":")
    monkeypatch.setenv("MTB_WAVE_TAXON", wave)
    # every multi-path species run through k_combine_wave's std::sort emulation (tied paths)
    monkeypatch.setenv("MTB_EMULATE_SORT", "1" if emu else "0")
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE["long" if kind == "verylong" else kind])
    odb = oc.OracleDb(db_dir)
    if kind == "verylong":
        reads = synth.make_long_reads(gen, 10, n50=16000, min_len=12500, seed=57)
    else:
        reads = _reads(gen, kind, 1500 if kind != "long" else 80, 55)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        compare_results(br.results, br.taxcnt, ores, otc)
    odb.close()


@pytest.mark.parametrize("db_name,kind", [("fmt2", "paired"), ("fmt2", "long"), ("fmt2_syncmer", "paired"),
                                          ("fmt1", "paired"), ("fmt1", "single")])
@pytest.mark.parametrize("mode", ["default", "nom64", "hbm", "mixed", "spill", "nofilter", "perblock", "persist",
                                  "small", "retry", "retrynofilter"])
def test_sweep_join(make_db, db_name, kind, mode, monkeypatch):
    """K4S, the DB-sweep join (MTB_JOIN=sweep: DB tiles ending at sort-prefix bucket bounds staged in
    LDS, each tile's queries searched there): the oracle's matches and results with tiles of the
    default size, many small tiles (MTB_SWEEP_NOM=64), every tile searched in HBM (MTB_SWEEP_LDS=0:
    the path of a bucket longer than an LDS tile), a mix (MTB_SWEEP_LDS=80), and queries spilling
    past their read's stretch (MTB_DIRECT=3), and every non-blank window sorted and swept with no
    membership filter (MTB_FILTER=0: no K1F, no probe lines); and the direct join's staged rerun
    (MTB_DIRECT=2), which needs the match windows the sweep does not build, with and
    without the filter."""
    monkeypatch.setenv("MTB_JOIN", "sweep")
    monkeypatch.setenv("MTB_FILTER", "0" if mode.endswith("nofilter") else "1")
    # warp-specialised resident blocks, resident blocks walking their tiles (the default form), one block per
    # tile; 24-KB tiles for the last two
    monkeypatch.setenv("MTB_SWEEP_PERSIST", {"perblock": "0", "persist": "1"}.get(mode, "2"))
    monkeypatch.setenv("MTB_SWEEP_SMALL", "1" if mode == "small" else "0")
    monkeypatch.setenv("MTB_SWEEP_NOM", "64" if mode in ("nom64", "mixed") else "2048")
    monkeypatch.setenv("MTB_SWEEP_LDS", {"hbm": "0", "mixed": "80"}.get(mode, "4096"))
    monkeypatch.setenv("MTB_DIRECT", {"spill": "3", "retry": "2", "retrynofilter": "2"}.get(mode, "1"))
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE[kind])
    reads = _reads(gen, kind, 1500 if kind != "long" else 60, seed=79)
    opar = par.to_c()
    odb = oc.OracleDb(db_dir)
    okmers, ql1, ql2 = oc.extract(opar, reads)
    omatches = oc.match(odb, opar, okmers)
    ores, otc = oc.classify(odb, opar, reads)
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, keep_stages=True)
        gm = clf.matches()
        assert len(gm) == len(omatches) == br.matches
        assert np.array_equal(gm, omatches)
        matched = clf.stats()["matched_queries"]
        assert 0 < matched <= clf.stats()["query_kmers"]
        if mode.endswith("nofilter"):  # every non-blank window went to the join
            assert clf.stats()["query_kmers"] == br.query_kmers == int((info_seq(okmers["info"]) != 0).sum())
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        if mode == "spill" and kind != "long" and db_name != "fmt2_syncmer":  # (long reads, syncmers: few matches per stretch)
            assert clf.stats()["spilled_matches"] > 0
        compare_results(br.results, br.taxcnt, ores, otc)
    odb.close()


@pytest.mark.parametrize("db_name,kind", [("fmt2", "paired"), ("fmt2", "long"), ("fmt1", "long")])
@pytest.mark.parametrize("late", ["glob", "merge512", "nocompact"])
def test_spill_then_late_compaction(make_db, db_name, kind, late, monkeypatch):
    """Spilled queries (MTB_DIRECT=3 quarters the read stretches) with a K5 that compacts every
    segment itself (global-scratch sort, the merge path above 512 matches, or no thinning of big
    segments): the reads that overflowed were compacted with their spills by the join, and the late
    compaction leaves them alone — the results are the oracle's."""
    monkeypatch.setenv("MTB_DIRECT", "3")
    monkeypatch.setenv("MTB_SEGSORT_GLOBAL", "1" if late == "glob" else "0")
    monkeypatch.setenv("MTB_MERGE_SEG", "512" if late == "merge512" else "0")
    monkeypatch.setenv("MTB_PRUNE_COMPACT", "0" if late == "nocompact" else "1")
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE[kind])
    reads = _reads(gen, kind, 1500 if kind != "long" else 60, 83)
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    odb.close()
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        if kind == "paired":  # (long reads keep their matches within a quarter of their stretch)
            assert clf.stats()["spilled_matches"] > 0
        compare_results(br.results, br.taxcnt, ores, otc)


@pytest.mark.parametrize("db_name,kind", [("fmt2", "paired"), ("fmt1", "long")])
def test_dup_stats_counter(make_db, db_name, kind, monkeypatch):
    """MTB_DUP_STATS=1: the repeated AA ranks / whole values per 256-query K4 block (mtb_last_stats
    [17] / [18]: the reference's same-AA and identical-query reuse, KmerMatcher.cpp:277-353, that a
    block could share) equal a host count over the query k-mers in the order K4 consumed them; the
    results are unchanged."""
    monkeypatch.setenv("MTB_DUP_STATS", "1")
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, SEQ_MODE[kind])
    reads = _reads(gen, kind, 1500 if kind == "paired" else 120, seed=91)
    # the same reads twice: identical queries in plenty
    reads = synth.Reads(np.concatenate([reads.seq1, reads.seq1]),
                        np.concatenate([reads.off1[:-1], reads.off1 + reads.off1[-1]]),
                        None if reads.seq2 is None else np.concatenate([reads.seq2, reads.seq2]),
                        None if reads.off2 is None else np.concatenate([reads.off2[:-1], reads.off2 + reads.off2[-1]]),
                        np.concatenate([reads.origin, reads.origin]))
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, keep_stages=True)
        st = clf.stats()
        q = clf.query_kmers()["value"]
    aa, same = 0, 0
    for b in range(0, len(q), 256):
        blk = np.sort(q[b:b + 256])
        aa += int(np.count_nonzero((blk[1:] >> np.uint64(24)) == (blk[:-1] >> np.uint64(24))))
        same += int(np.count_nonzero(blk[1:] == blk[:-1]))
    assert st["dup_aa_queries"] == aa and st["dup_key_queries"] == same
    assert same > 0 and aa >= same
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    odb.close()
    compare_results(br.results, br.taxcnt, ores, otc)
