import os
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmtbgpu.so on cuda:0)")


def _ensure_oracle():
    so = ROOT / "oracle" / "liboracle.so"
    if not so.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle"), "liboracle.so"], check=True, capture_output=True)


@pytest.fixture(scope="session")
def fixture_root(tmp_path_factory):
    _ensure_oracle()
    return tmp_path_factory.mktemp("mtb_fixtures")


# (name, kmer_format, syncmer, n_species, strains, genome_len[, extras])
# "*_acc": an accession-level DB (db.parameters "Accession_level 1"; genomes on rank-"accession"
# leaves, IndexCreator.cpp:640-660), so classify runs with accessionLevel 1 or 2 (common.cpp:100-107);
# its species are diverged copies of a genus genome (species_div), so species ties, LCAs and the
# tie ratio matter
DB_CONFIGS = {
    "fmt2": (2, 0, 14, 2, 24000),
    "fmt2_syncmer": (2, 1, 14, 2, 24000),
    "fmt1": (1, 0, 10, 2, 20000),
    "fmt2_acc": (2, 0, 12, 2, 16000, {"accessions": 2, "species_div": 0.03}),
    "fmt2_syncmer_acc": (2, 1, 12, 2, 16000, {"accessions": 2, "species_div": 0.03}),
    "fmt1_acc": (1, 0, 12, 2, 14000, {"accessions": 2, "species_div": 0.03}),
}


@pytest.fixture(scope="session")
def make_db(fixture_root):
    """Builds (once per session) a synthetic reference DB through the oracle's IndexCreator restatement."""
    from metabuli_work_amd import synth
    from metabuli_work_amd._abi import default_params
    from tests import oracle_ctypes as oc

    cache = {}

    def get(name):
        if name in cache:
            return cache[name]
        fmt, syn, nsp, nst, glen, *ex = DB_CONFIGS[name]
        ex = ex[0] if ex else {}
        acc = ex.get("accessions", 0)
        taxo = synth.make_taxonomy(nsp, nst, seed=11, accessions=acc)
        gen = synth.make_genomes(taxo, genome_len=glen, seed=12, species_div=ex.get("species_div", 0.0))
        d = str(fixture_root / name)
        par = default_params(kmer_format=fmt, syncmer=syn, smer_len=5, accession_level=1 if acc else 0)
        oc.build_db(d, par, taxo, gen)
        cache[name] = (d, taxo, gen)
        return cache[name]

    return get
