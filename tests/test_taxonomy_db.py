"""DBs that ship a taxonomyDB (TaxonomyWrapper::serialize, TaxonomyWrapper.cpp:289-361), as every DB
the reference's `build` writes does (build.cpp:100, IndexCreator.cpp:293), usually with internal
taxIDs (build.cpp:89-92): loadTaxonomy prefers the binary over the dmp files (common.cpp:50-86),
info / taxID_list / results hold internal taxIDs, and the writers print getOriginalTaxID
(TaxonomyWrapper.h:70-79, Reporter.cpp:55,65,72,241).

The file is written by synth.write_taxonomy_db, a restatement of serialize; the TaxonNode and
StringBlock layouts and the serialization version are MMseqs2's (the submodule is absent):
parity unpinned for the byte layout. The oracle restates unserialize (and LCA over the file's own
Euler tour / sparse table); the product reads the same file with its own loader.
"""
import os

import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd._abi import default_params
from metabuli_work_amd.classifier import Classifier, LocalParameters
from tests import oracle_ctypes as oc
from tests.test_gpu_parity import compare_results


def _build(tmp, name, mode):
    """A format-2 DB whose taxonomy is given as: "internal" (taxonomyDB with internal taxIDs, the
    dmp files under taxonomy/ in ORIGINAL IDs, so a loader that reads them gets everything
    wrong), "original" (taxonomyDB without internal IDs), "dmp_internal" (the internal-ID
    taxonomy as dmp files only: the reference answer for "internal"), "old_version" (a taxonomyDB
    of another serialization version: ignored, the dmp files are used)."""
    taxo = synth.make_taxonomy(10, 2, seed=21, accessions=1)
    gen = synth.make_genomes(taxo, genome_len=14000, seed=22, species_div=0.03)
    itaxo, i2o = synth.to_internal_ids(taxo)
    o2i = {int(o): i for i, o in enumerate(i2o)}
    d = str(tmp / name)
    par = default_params(kmer_format=2, accession_level=1)
    internal = mode in ("internal", "dmp_internal")
    if internal:
        igen = synth.Genomes(gen.seq, gen.off, np.array([o2i[int(t)] for t in gen.taxid], np.int32),
                             np.array([o2i[int(t)] for t in gen.species], np.int32), gen.blk_genome,
                             gen.blk_start, gen.blk_end, gen.blk_strand)
        oc.build_db(d, par, itaxo, igen)
    else:
        oc.build_db(d, par, taxo, gen)
    if mode == "internal":
        synth.write_taxonomy_db(itaxo, os.path.join(d, "taxonomyDB"), i2o)
        taxo.write_dmp(os.path.join(d, "taxonomy"))  # stale original-ID dmp files next to it
    elif mode == "original":
        synth.write_taxonomy_db(taxo, os.path.join(d, "taxonomyDB"))
        synth.Taxonomy(taxo.taxid[:1], taxo.parent[:1], taxo.rank[:1], taxo.name[:1]).write_dmp(
            os.path.join(d, "taxonomy"))  # a root-only dmp: only the taxonomyDB can classify
    elif mode == "old_version":
        synth.write_taxonomy_db(taxo, os.path.join(d, "taxonomyDB"))
        with open(os.path.join(d, "taxonomyDB"), "r+b") as f:
            f.write(np.int32(synth.TAXONOMY_DB_VERSION + 1).tobytes())
    return d, taxo, itaxo, i2o, gen


@pytest.fixture(scope="module")
def dbs(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("taxdb")
    return {m: _build(tmp, m, m) for m in ("internal", "original", "dmp_internal", "old_version")}


def _reads(gen):
    return synth.concat_reads([synth.make_reads(gen, 300, seed=61 + i, sub_rate=r) for i, r in enumerate((0.005, 0.04))])


def test_oracle_reads_taxonomy_db(dbs):
    """Oracle (CPU): a taxonomyDB with internal IDs classifies exactly as the same taxonomy given as
    dmp files; one without internal IDs as the original dmp; another version falls back to dmp."""
    d_int, taxo, itaxo, i2o, gen = dbs["internal"]
    reads = _reads(gen)
    par = LocalParameters(seqMode=2).load_db_parameters(d_int).to_c()
    out = {}
    for m in ("internal", "dmp_internal", "original", "old_version"):
        odb = oc.OracleDb(dbs[m][0])
        out[m] = oc.classify(odb, par, reads)
        odb.close()
    compare_results(*out["internal"], *out["dmp_internal"])
    compare_results(*out["original"], *out["old_version"])
    # the internal run, mapped through internal2org, is the original run
    ri, ti = out["internal"]
    ro, to = out["original"]
    assert ri["is_classified"].sum() > 300
    np.testing.assert_array_equal(i2o[ri["classification"]], ro["classification"])
    np.testing.assert_array_equal(ri["score"].view(np.uint32), ro["score"].view(np.uint32))
    np.testing.assert_array_equal(i2o[ti["tax_id"]], to["tax_id"])
    np.testing.assert_array_equal(ti["count"], to["count"])


def test_taxonomy_db_layout(dbs, tmp_path):
    """The writer's header fields land where unserialize reads them (version, internal flag,
    maxNodes, maxTaxID, first TaxonNode)."""
    d, taxo, itaxo, i2o, _ = dbs["internal"]
    raw = open(os.path.join(d, "taxonomyDB"), "rb").read()
    assert np.frombuffer(raw[:4], np.int32)[0] == synth.TAXONOMY_DB_VERSION
    assert np.frombuffer(raw[4:12], np.uint64)[0] == 1
    assert np.frombuffer(raw[12:20], np.uint64)[0] == len(itaxo.taxid)
    assert np.frombuffer(raw[20:24], np.int32)[0] == len(i2o) - 1
    node0 = np.frombuffer(raw[24:56], np.int32)
    assert tuple(node0[:3]) == (0, 1, 1)  # id 0, root taxID 1 (internal 1 = original 1), its own parent


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["internal", "original", "old_version"])
def test_taxonomy_db_parity(dbs, mode, tmp_path):
    """Product vs oracle on taxonomyDB DBs: internal-ID results element by element; the TSV and the
    report print original taxIDs (getOriginalTaxID) and the --lineage column is taxLineage2."""
    d, taxo, itaxo, i2o, gen = dbs[mode]
    reads = _reads(gen)
    par = LocalParameters(seqMode=2).load_db_parameters(d)
    odb = oc.OracleDb(d)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    with Classifier(par, db_dir=d) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        compare_results(br.results, br.taxcnt, ores, otc)
        internal = mode == "internal"
        tmap = (lambda t: int(i2o[t])) if internal else (lambda t: int(t))
        for t in np.unique(ores["classification"]).tolist():
            assert clf.original_taxid(t) == tmap(t)
        # lineage: root-most first, short rank + "_" + name, the root itself left out
        tx = itaxo if internal else taxo
        rank = dict(zip(tx.taxid.tolist(), tx.rank))
        for t in np.unique(ores["classification"][ores["is_classified"] != 0]).tolist():
            assert clf.lineage(t) == clf_lineage_of(tx, t)
        # file -> TSV with lineage, and the report, in original taxIDs
        names = [f"r{i}" for i in range(reads.n)]
        p1, p2 = str(tmp_path / "a.fq"), str(tmp_path / "b.fq")
        for path, seq, off in ((p1, reads.seq1, reads.off1), (p2, reads.seq2, reads.off2)):
            with open(path, "w") as f:
                for i in range(reads.n):
                    s = bytes(seq[off[i]:off[i + 1]]).decode()
                    f.write(f"@{names[i]}\n{s}\n+\n{'I' * len(s)}\n")
        clf.par = LocalParameters(seqMode=2, printLineage=1, filenames=[p1, p2, d]).load_db_parameters(d)
        out, rep = str(tmp_path / "o.tsv"), str(tmp_path / "rep.tsv")
        assert clf.startClassify(out, report_tsv=rep) == reads.n
    lines = open(out).read().splitlines()
    assert lines[0] == "#is_classified\tname\ttaxID\tquery_length\tscore\trank\tlineage\ttaxID:match_count"
    for i, line in enumerate(lines[1:]):
        f = line.split("\t")
        o = ores[i]
        if o["is_classified"]:
            assert int(f[2]) == tmap(int(o["classification"]))
            assert f[5] == rank[int(o["classification"])]
            assert f[6] == clf_lineage_of(tx, int(o["classification"]))
            s = int(o["taxcnt_offset"])
            assert f[7] == "".join(f"{tmap(int(t))}:{int(c)} " for t, c in otc[s:s + int(o["taxcnt_len"])])
        else:
            assert f[2] == "0" and f[5:] == ["-", "-", "-", ""]
    cls, cnt = np.unique(np.where(ores["is_classified"] != 0, ores["classification"], 0), return_counts=True)
    orep = str(tmp_path / "orep.tsv")
    oc.write_report(odb, orep, reads.n, dict(zip(cls.tolist(), cnt.tolist())))
    odb.close()
    assert open(rep).read() == open(orep).read()


def clf_lineage_of(tx, t):
    """taxLineage2 restated over the synthetic taxonomy (TaxonomyWrapper.cpp:431-454)."""
    short = {"subspecies": "ss", "species": "s", "subgenus": "sg", "genus": "g", "subfamily": "sf", "family": "f",
             "suborder": "so", "order": "o", "subclass": "sc", "class": "c", "subphylum": "sp", "phylum": "p",
             "subkingdom": "sk", "kingdom": "k", "superkingdom": "d", "domain": "d", "realm": "r"}
    rank = dict(zip(tx.taxid.tolist(), tx.rank))
    name = dict(zip(tx.taxid.tolist(), tx.name))
    parent = dict(zip(tx.taxid.tolist(), tx.parent.tolist()))
    chain = [t]
    t = parent[t]
    while parent[t] != t:
        chain.append(t)
        t = parent[t]
    return ";".join(f"{short.get(rank[x], '-')}_{name[x]}" for x in chain[::-1])
