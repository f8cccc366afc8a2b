"""Regenerate tests/golden/oracle_small.npz: oracle results on a small seeded workload.

The reference cannot run here, so this fixture pins the oracle against regressions (it is not an
independent golden vector); the inputs are regenerated from the seeds by the test.
"""
import pathlib
import sys
import tempfile

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

from metabuli_work_amd import synth  # noqa: E402
from metabuli_work_amd._abi import default_params  # noqa: E402
from tests import oracle_ctypes as oc  # noqa: E402

CASES = [("fmt2", 2, 0), ("fmt2_syncmer", 2, 1), ("fmt1", 1, 0)]


def run_case(fmt, syncmer, d):
    taxo = synth.make_taxonomy(9, 2, seed=101)
    gen = synth.make_genomes(taxo, genome_len=12000, seed=102)
    oc.build_db(d, default_params(kmer_format=fmt, syncmer=syncmer), taxo, gen)
    par = oc.load_db_parameters(d, default_params())
    reads = synth.make_reads(gen, 400, seed=103, short_frac=0.03, rate_n=0.002, rate_iupac=0.001)
    db = oc.OracleDb(d)
    res, tc = oc.classify(db, par, reads)
    db.close()
    return res, tc


if __name__ == "__main__":
    out = {}
    for name, fmt, syn in CASES:
        with tempfile.TemporaryDirectory() as d:
            res, tc = run_case(fmt, syn, d)
        out[name + "_res"] = res
        out[name + "_tc"] = tc
    np.savez_compressed(HERE / "oracle_small.npz", **out)
    print("wrote", HERE / "oracle_small.npz")
