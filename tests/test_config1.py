"""Config 1 as SURVEY §8(d) states it (BASELINE.json configs[0], VERDICT r05 missing 5): three random
genomes of 2.0 / 1.5 / 1.0 Mbp (GC 0.5, seed 1) in one genus (root -> genus -> 3 species -> 3
strains), a format-2 DB through the oracle's IndexCreator restatement (splitNum 4096), and 10,000
single-end 150-bp reads (90% sampled with 0.5% substitutions, 10% random; seed 2). Run in format 2
and format 2 + syncmer (s = 5), as §8(d) asks of every config; the GPU path's per-read taxID, score
bits and taxID:count lists equal the oracle's."""
import numpy as np
import pytest

from metabuli_work_amd import synth
from tests import oracle_ctypes as oc


@pytest.fixture(scope="module")
def config1():
    taxo, gen = synth.make_config1()
    return taxo, gen, synth.make_config1_reads(gen)


def test_config1_workload_shape(config1):
    taxo, gen, reads = config1
    assert np.diff(gen.off).tolist() == list(synth.CONFIG1_GENOME_LENS)
    assert taxo.rank.count("species") == 3 and taxo.rank.count("genus") == 1
    par = dict(zip(taxo.taxid.tolist(), taxo.parent.tolist()))
    assert [par[t] for t in gen.taxid.tolist()] == gen.species.tolist() == [3, 4, 5]
    gc = float(np.isin(gen.seq, np.frombuffer(b"GC", np.uint8)).mean())
    assert abs(gc - 0.5) < 0.002
    assert reads.n == 10_000 and reads.seq2 is None
    assert set(np.diff(reads.off1).tolist()) == {150}
    assert abs(float((reads.origin < 0).mean()) - 0.1) < 0.015


@pytest.mark.gpu
@pytest.mark.parametrize("syncmer", [0, 1])
def test_config1_gpu_matches_oracle(config1, tmp_path, syncmer):
    from metabuli_work_amd._abi import default_params
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from tests.test_gpu_parity import compare_results

    taxo, gen, reads = config1
    d = str(tmp_path / "db")
    oc.build_db(d, default_params(kmer_format=2, syncmer=syncmer, smer_len=5), taxo, gen, split_num=4096)
    par = LocalParameters(seqMode=1).load_db_parameters(d)
    assert par.kmerFormat == 2 and par.syncmer == syncmer
    odb = oc.OracleDb(d)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    odb.close()
    with Classifier(par, db_dir=d, device=0) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1)
    compare_results(br.results, br.taxcnt, ores, otc)
    # the workload classifies: most sampled reads reach a taxon, random reads mostly do not
    cls = br.results["is_classified"].astype(bool)
    sampled = reads.origin >= 0
    assert cls[sampled].mean() > 0.8 and cls[~sampled].mean() < 0.2
