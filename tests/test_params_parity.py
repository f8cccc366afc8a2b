"""Parity over the classify parameter space users actually run (README.md:189-192), against the
oracle: `--min-score 0.15 --min-sp-score 0.5` (Illumina), `--min-score 0.008` with seq-mode 3
(ONT), `--tie-ratio 0.8`, and accession-level DBs classified with `--accession-level 1` or with the
default 0 (which loadDbParameters turns into 2 for a DB built with accessions, common.cpp:100-107).

Branches held to the oracle (Taxonomer.cpp):
* species skipped below minScore (:356-358) and the unclassified test (:149);
* the parent-of-species classification below minSpScore (:178-185);
* the species tie set at bestSpScore * tieRatio and its LCA (:380-401);
* lowerRankClassification with accessionLevel 2: rank "" / "accession" nodes dropped from the BFS
  (:256-266); with accessionLevel 1 the BFS may end on an accession leaf.

The CPU tests check that the fixtures really reach those branches (through the oracle); the GPU
tests compare the HIP path with the oracle end to end and K5+K6 alone on the oracle's matches.
"""
import collections

import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd.classifier import Classifier, LocalParameters
from tests import oracle_ctypes as oc
from tests.test_gpu_parity import compare_results

ILLUMINA = {"minScore": 0.15, "minSpScore": 0.5}
ONT = {"minScore": 0.008}
TIE = {"tieRatio": 0.8}

# (db, read kind, LocalParameters overrides)
CASES = [
    ("fmt2", "paired", ILLUMINA), ("fmt2_syncmer", "paired", ILLUMINA), ("fmt1", "single", ILLUMINA),
    ("fmt2", "long", ONT), ("fmt2_syncmer", "long", ONT), ("fmt1", "long", ONT),
    ("fmt2_acc", "paired", TIE), ("fmt1_acc", "paired", TIE),
    ("fmt2_acc", "paired", {"accessionLevel": 0}), ("fmt2_acc", "paired", {"accessionLevel": 1}),
    ("fmt2_syncmer_acc", "paired", {"accessionLevel": 0}), ("fmt2_syncmer_acc", "paired", {"accessionLevel": 1}),
    ("fmt1_acc", "single", {"accessionLevel": 1}),
    ("fmt2_acc", "paired", dict(ILLUMINA, accessionLevel=1)),
    ("fmt2_acc", "long", dict(ONT, accessionLevel=0)), ("fmt2_acc", "long", dict(ONT, accessionLevel=1)),
    # --min-cons-cnt(-euk): the consecutive-match minimum of a path, and K5's pruning threshold with it
    # (pm = 2, 7 and, with syncmers' codon shift of 3, 3)
    ("fmt2", "paired", {"minConsCnt": 2}), ("fmt2", "long", dict(ONT, minConsCnt=7, minConsCntEuk=7)),
    ("fmt2_syncmer", "paired", {"minConsCnt": 6}),
]
SEQ_MODE = {"paired": 2, "single": 1, "long": 3}


def case_id(c):
    return f"{c[0]}-{c[1]}-" + "-".join(f"{k}={v}" for k, v in c[2].items())


def _params(db_dir, kind, over):
    par = LocalParameters(seqMode=SEQ_MODE[kind], **over)
    par.load_db_parameters(db_dir)
    return par


def mixed_reads(gen, kind, seed):
    """Reads drawn at three divergence levels so scores spread across the minScore / minSpScore
    thresholds (0.5% substitutions score ~0.9, 8% ~0.2-0.4)."""
    if kind == "long":
        return synth.concat_reads([synth.make_long_reads(gen, 12, n50=3000, min_len=400, sub_rate=r, seed=seed + i)
                                   for i, r in enumerate((0.03, 0.08, 0.15))])
    paired = kind == "paired"
    return synth.concat_reads([synth.make_reads(gen, 400, paired=paired, sub_rate=r, seed=seed + i, short_frac=0.02)
                               for i, r in enumerate((0.005, 0.03, 0.08))])


def _outcomes(res, taxo):
    rank = dict(zip(taxo.taxid.tolist(), taxo.rank))
    c = collections.Counter()
    for r in res:
        c[rank.get(int(r["classification"]), "?") if r["is_classified"] else "unclassified"] += 1
    return c


def test_branches_reached(make_db):
    """Oracle side (CPU): the fixtures of the GPU cases reach the branches they are there for."""
    db_dir, taxo, gen = make_db("fmt2")
    odb = oc.OracleDb(db_dir)
    reads = mixed_reads(gen, "paired", 40)
    base = _outcomes(oc.classify(odb, _params(db_dir, "paired", {}).to_c(), reads)[0], taxo)
    ill = _outcomes(oc.classify(odb, _params(db_dir, "paired", ILLUMINA).to_c(), reads)[0], taxo)
    odb.close()
    assert ill["unclassified"] > base["unclassified"]       # species below minScore dropped
    assert ill["genus"] > base["genus"] + 50                 # parent of the species below minSpScore

    db_dir, taxo, gen = make_db("fmt2_acc")
    odb = oc.OracleDb(db_dir)
    reads = mixed_reads(gen, "paired", 40)
    p0 = _params(db_dir, "paired", {"accessionLevel": 0})
    assert p0.accessionLevel == 2                            # common.cpp:104-106
    acc2 = _outcomes(oc.classify(odb, p0.to_c(), reads)[0], taxo)
    acc1 = _outcomes(oc.classify(odb, _params(db_dir, "paired", {"accessionLevel": 1}).to_c(), reads)[0], taxo)
    tie = _outcomes(oc.classify(odb, _params(db_dir, "paired", TIE).to_c(), reads)[0], taxo)
    odb.close()
    assert acc2["accession"] == 0 and acc1["accession"] > 100
    assert acc2["genus"] > 0                                 # related species tie: LCA
    assert tie["genus"] > acc2["genus"]                      # a lower tie ratio widens the tie set


@pytest.mark.gpu
@pytest.mark.parametrize("db_name,kind,over", CASES, ids=[case_id(c) for c in CASES])
def test_params_parity(make_db, db_name, kind, over):
    db_dir, taxo, gen = make_db(db_name)
    par = _params(db_dir, kind, over)
    reads = mixed_reads(gen, kind, 50)
    opar = par.to_c()
    odb = oc.OracleDb(db_dir)
    okmers, ql1, ql2 = oc.extract(opar, reads)
    omatches = oc.match(odb, opar, okmers)
    ores, otc = oc.assign(odb, opar, omatches, ql1, ql2)
    eres, etc = oc.classify(odb, opar, reads)
    compare_results(eres, etc, ores, otc)  # the oracle's staged and whole-path runs agree
    with Classifier(par, db_dir=db_dir) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        compare_results(br.results, br.taxcnt, ores, otc)
        ar = clf.assign_matches(omatches[np.random.default_rng(1).permutation(len(omatches))], ql1 + ql2)
        compare_results(ar.results, ar.taxcnt, ores, otc)
    odb.close()
