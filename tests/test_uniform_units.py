"""Uniform K1 units (round 6): when every frame of a batch fits one chunk (maxW <= 64
windows: mates up to 217 bp) every read gets 6 units per mate and K4 rebuilds a matched query's info
from its slot and the lengths its rank atomic returns. Batches at the threshold on both sides, paired
and single-end, with reads whose mate holds no window, against the oracle and against the same batch
with the layout off (MTB_UNIFORM_UNITS=0)."""
import numpy as np
import pytest

from metabuli_work_amd import synth
from tests import oracle_ctypes as oc


def _reads(gen, n, lens, paired, seed):
    """Reads sampled from the genomes with lengths cycling over `lens` (both mates), 5% of the mates
    cut below one window."""
    rng = np.random.default_rng(seed)
    base = synth.make_reads(gen, n, paired=paired, read_len=max(lens), seed=seed, short_frac=0.05)

    def cut(seq, off):
        out, o = [], [0]
        for i in range(n):
            s = seq[int(off[i]):int(off[i + 1])]
            L = lens[i % len(lens)]
            s = s[:L] if len(s) >= L else s
            out.append(s)
            o.append(o[-1] + len(s))
        return np.concatenate(out).astype(np.uint8), np.array(o, np.uint64)
    s1, o1 = cut(base.seq1, base.off1)
    if not paired:
        return synth.Reads(s1, o1, None, None, base.origin)
    s2, o2 = cut(base.seq2, base.off2)
    return synth.Reads(s1, o1, s2, o2, base.origin)


@pytest.mark.gpu
@pytest.mark.parametrize("window", ["", "0"])
@pytest.mark.parametrize("paired", [True, False])
@pytest.mark.parametrize("lens,uniform", [((150,), True), ((215, 216, 217), True), ((216, 217, 218), False),
                                          ((60, 100, 213), True)])
def test_uniform_units_parity(make_db, monkeypatch, paired, lens, uniform, window):
    """window "0": the unstaged join (k_join_uniform when the layout is on, k_match otherwise)."""
    if window:
        monkeypatch.setenv("MTB_MATCH_WINDOW", window)
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from tests.test_gpu_parity import compare_results

    db_dir, taxo, gen = make_db("fmt2")
    r = _reads(gen, 700, lens, paired, seed=sum(lens) + paired)
    par = LocalParameters(seqMode=2 if paired else 1).load_db_parameters(db_dir)
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), r)
    odb.close()
    got = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("MTB_UNIFORM_UNITS", flag)
        with Classifier(par, db_dir=db_dir, device=0) as clf:
            br = clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2)
            got[flag] = (br, clf.stats())
    br, st = got["1"]
    assert st["uniform_units"] == ((12 if paired else 6) if uniform else 0)
    assert got["0"][1]["uniform_units"] == 0
    compare_results(br.results, br.taxcnt, ores, otc)
    compare_results(got["0"][0].results, got["0"][0].taxcnt, ores, otc)
    assert st["matches"] == got["0"][1]["matches"] > 0
