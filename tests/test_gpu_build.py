"""GPU reference-DB builder vs the oracle's IndexCreator restatement: byte-identical files."""
import os

import numpy as np
import pytest

from metabuli_work_amd import synth
from metabuli_work_amd._abi import default_params
from metabuli_work_amd.dbbuild import build_db
from tests import oracle_ctypes as oc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fmt,syncmer", [(2, 0), (2, 1), (1, 0)])
def test_builder_matches_oracle_writer(tmp_path, fmt, syncmer):
    taxo = synth.make_taxonomy(12, 3, seed=31)
    gen = synth.make_genomes(taxo, genome_len=15000, strain_div=0.01, seed=32)
    par = default_params(kmer_format=fmt, syncmer=syncmer)
    d = str(tmp_path / "oracle_db")
    oc.build_db(d, par, taxo, gen)
    hdb = build_db(gen, taxo, par, device=0)
    for name, arr in (("diffIdx", hdb.diff_idx), ("info", hdb.info), ("split", hdb.split)):
        ref = np.fromfile(os.path.join(d, name), dtype=arr.dtype)
        assert len(ref) == len(arr), name
        assert np.array_equal(ref, arr), name
    ref_ids = np.loadtxt(os.path.join(d, "taxID_list"), dtype=np.int32, ndmin=1)
    assert np.array_equal(np.sort(ref_ids), np.sort(hdb.taxid_list))
