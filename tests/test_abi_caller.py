"""The boundary driven by a compiled C program (tests/abi_caller.c: mtb_open -> mtb_reader_next ->
mtb_classify_batch -> mtb_get_taxcnt -> mtb_close, no ctypes) gives the oracle's classifications,
score bits and taxID:count lists — also when a workspace cap makes it halve its QuerySplits on
MTB_RETRY (Classifier.cpp:127-130). The caps run from pieces of a few reads (staged join, every
buffer regrown after each retry and each given-back split) to whole 1000-read splits; round 4 saw
one wrong taxID under a 6-MB cap on a work-in-progress build ("Round-4 capped-caller
failure"), so the sweep keeps every regime covered."""
import subprocess

import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd.classifier import LocalParameters
from tests import oracle_ctypes as oc
from tests.test_abi import abi_caller


def _lines(path):
    rows = []
    for line in open(path):
        f = line.rstrip("\n").split("\t")
        rows.append((int(f[1]), int(f[2], 16), int(f[3]), int(f[4]),
                     [tuple(map(int, x.split(":"))) for x in f[5].split()]))
    return rows


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [0, 1_500_000, 3_000_000, 6_000_000, 12_000_000, 40_000_000])
def test_c_caller_matches_oracle(make_db, tmp_path, cap):
    db_dir, taxo, gen = make_db("fmt2")
    r = synth.make_reads(gen, 2100, paired=True, seed=71, short_frac=0.03)
    p1, p2 = tmp_path / "q1.fq", tmp_path / "q2.fq"
    p1.write_bytes(synth.fastq_bytes(r.seq1, r.off1, prefix="c"))
    p2.write_bytes(synth.fastq_bytes(r.seq2, r.off2, prefix="c"))
    out = tmp_path / "c.tsv"
    cmd = [str(abi_caller()), db_dir, "2", str(p1), str(p2), str(out)] + ([str(cap)] if cap else [])
    subprocess.run(cmd, check=True, timeout=120)
    rows = _lines(out)
    assert len(rows) == r.n
    par = LocalParameters(seqMode=2)
    par.load_db_parameters(db_dir)
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par.to_c(), r)
    odb.close()
    ocls = np.where(ores["is_classified"] != 0, ores["classification"], 0)
    assert [x[0] for x in rows] == ocls.tolist()
    assert [x[1] for x in rows] == ores["score"].view(np.uint32).tolist()
    assert [x[2] for x in rows] == ores["hamming_dist"].tolist()
    assert [x[3] for x in rows] == ores["query_length"].tolist()
    for i, x in enumerate(rows):
        s = int(ores[i]["taxcnt_offset"])
        assert x[4] == [(int(t), int(c)) for t, c in otc[s:s + int(ores[i]["taxcnt_len"])]]
