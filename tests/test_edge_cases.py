"""Edge cases of one batch through the C-ABI against the oracle (empty and ragged
inputs, reads with no k-mer window, windows none of which the DB holds): every batch is classified
by the HIP path and by the oracle on the same reads, results and taxID:count lists compared as in
test_gpu_parity. Each case also runs with K1F writing K2's first-pass buckets at any batch size
(MTB_K1F_BINS=2), whose tile table and sort must survive empty and nearly empty buckets.
"""
import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd.classifier import Classifier
from tests import oracle_ctypes as oc
from tests.test_gpu_parity import _params, compare_results

pytestmark = pytest.mark.gpu


def _pack(seqs):
    """Reads from a list of byte strings: concatenated bases and offsets."""
    off = np.zeros(len(seqs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    return np.frombuffer(b"".join(seqs), dtype=np.uint8).copy(), off


def _reads(first, second=None):
    s1, o1 = _pack(first)
    s2, o2 = _pack(second) if second is not None else (None, None)
    return synth.Reads(s1, o1, s2, o2, np.full(len(first), -1, dtype=np.int32))


def _cases(gen):
    """name -> (seq mode, Reads)."""
    rng = np.random.default_rng(71)
    real = synth.make_reads(gen, 40, paired=True, seed=72)
    m1 = [bytes(real.seq1[real.off1[i]:real.off1[i + 1]]) for i in range(real.n)]
    m2 = [bytes(real.seq2[real.off2[i]:real.off2[i + 1]]) for i in range(real.n)]
    rand = [bytes(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), size=150)) for _ in range(60)]
    return {
        # every read below the shortest window (24 bases): no query k-mer at all
        "too_short": (1, _reads([b"ACGTACGTAC", b"A", b"ACGTACGTACGTACGTACGTACG"] * 5)),
        # bases no codon reads (N and IUPAC codes): no k-mer either
        "all_n": (1, _reads([b"N" * 150, b"RYKMSWN" * 20, b"n" * 60])),
        # one read pair
        "one_pair": (2, _reads(m1[:1], m2[:1])),
        # empty mates beside full ones, and a pair of empty mates
        "empty_mates": (2, _reads([m1[0], b"", m1[2], b""], [b"", m2[1], m2[2], b""])),
        # random sequence against a small DB: next to no query AA 8-mer is present (Q ~ 0)
        "absent": (1, _reads(rand)),
        # ragged: one read of 20 kb among 30-base ones
        "ragged": (1, _reads([m1[3][:30], bytes(gen.seq[:20000]), m1[4][:30], m1[5]])),
    }


@pytest.mark.parametrize("bins", ["0", "2"])
@pytest.mark.parametrize("case", ["too_short", "all_n", "one_pair", "empty_mates", "absent", "ragged"])
def test_edge_case_batches(make_db, monkeypatch, case, bins):
    monkeypatch.setenv("MTB_K1F_BINS", bins)
    db_dir, taxo, gen = make_db("fmt2")
    mode, reads = _cases(gen)[case]
    par = _params(db_dir, mode)
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    odb.close()
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        compare_results(br.results, br.taxcnt, ores, otc)
        if case in ("too_short", "all_n"):
            assert br.query_kmers == 0 and not br.results["is_classified"].any()
        # the context stays usable: the same batch again
        br2 = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        compare_results(br2.results, br2.taxcnt, ores, otc)
