"""GTDB-scale DB path at test scale: a DB built in place on the GPU
(true-signal genomes through the device builder + random-metamer filler over a skeleton taxonomy),
classified through mtb_open_resident, against the oracle on the same DB re-encoded in the
reference's diffIdx / info / split format."""
import numpy as np
import pytest
import torch

from metabuli_work_amd import synth
from tests import oracle_ctypes as oc

pytestmark = pytest.mark.gpu


def _host_reads(s1, o1, s2, o2):
    return synth.Reads(s1.cpu().numpy(), o1.cpu().numpy().astype(np.uint64), s2.cpu().numpy(),
                       o2.cpu().numpy().astype(np.uint64), np.zeros(o1.numel() - 1, np.int32))


def test_device_builder_and_encoder_match_the_file_format():
    """MTB_BUILD_DEVICE_OUT + encode_into_oracle reproduce mtb_build_db's diffIdx / info / split."""
    from metabuli_work_amd._abi import default_params
    from metabuli_work_amd.dbbuild import HostDb, build_db, build_db_device
    from metabuli_work_amd.gpu_synth import make_genomes_gpu
    from metabuli_work_amd.gtdb_synth import ResidentDb, encode_into_oracle

    dev = torch.device("cuda", 0)
    taxo, gen, seq, off_t, _ = make_genomes_gpu(12, 40000, 2, 3, dev)
    par = default_params(kmer_format=2, seq_mode=2)
    hdb = build_db(gen, taxo, par, device=0, device_seq=(seq, off_t))
    v, t = build_db_device(gen, taxo, par, device=0, device_seq=(seq, off_t))
    n = v.numel()
    assert n == hdb.n_kmers
    rdb = ResidentDb.from_arrays(v, t, HostDb(taxo, taxid_list=hdb.taxid_list))
    odb = encode_into_oracle(rdb, _Capture, split_num=4096, chunk=1 << 16)
    assert np.array_equal(_Capture.diff, hdb.diff_idx)
    assert np.array_equal(_Capture.info, hdb.info)
    assert np.array_equal(_Capture.split, hdb.split)
    odb.close()


class _Capture(oc.OracleDb):
    """OracleDb.fillable that also keeps the filled views for the comparison."""

    @classmethod
    def fillable(cls, host_struct, n_diff, n_info, n_split):
        db, d, i, s = oc.OracleDb.fillable(host_struct, n_diff, n_info, n_split)
        cls.diff, cls.info, cls.split = d, i, s
        return db, d, i, s


def test_gtdb_shaped_resident_db_parity(monkeypatch):
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from metabuli_work_amd.gpu_synth import make_reads_gpu
    from metabuli_work_amd.gtdb_synth import build_gtdb_scale, encode_into_oracle
    from tests.test_gpu_parity import compare_results

    dev = torch.device("cuda", 0)
    got = {}

    def grab(seq, off):
        got["reads"] = make_reads_gpu(seq, off, 3000, 99, dev)

    rdb = build_gtdb_scale(dev, n_true_species=10, genome_len=30000, total_species=300, target_kmers=3_000_000,
                           n_chunks=4, before_free=grab)
    assert rdb.n > 2_500_000 and rdb.n_true > 50_000
    v = rdb.values()
    assert bool((v[1:] >= v[:-1]).all())
    reads = _host_reads(*got["reads"])
    par = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1)
    from tests.test_gpu_parity import line_ext_check
    monkeypatch.setenv("MTB_LINE_EXT", "1")  # the A/B's run-length lines, checked on a GTDB-shaped DB
    with Classifier(par, db_resident=rdb) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        n, ok, bad = line_ext_check(clf)  # the GTDB-shaped DB's run-length lines against its run index
        assert bad == 0 and ok > 0.5 * n
    odb = encode_into_oracle(rdb, oc.OracleDb, chunk=1 << 20)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    odb.close()
    compare_results(br.results, br.taxcnt, ores, otc)
    assert br.results["is_classified"].mean() > 0.5


def test_partitioned_resident_parts_parity():
    """Config 5's path at test scale: the GTDB-shaped DB built one AA-aligned part at a time
    (GtdbRecipe.build with its guard k-mer), each part opened alone (mtb_open_resident, db_part),
    the reads matched against every part (MTB_MATCH_ONLY), the per-part match segments scored
    together (mtb_assign_chunks, the all-to-all receive layout). Results equal the oracle's on the
    whole DB, and the oracle on the sub-DB of the reads' AA runs (gtdb_synth.SubDb, the bench's
    config-5 parity check) gives the same results too."""
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from metabuli_work_amd.gpu_synth import make_reads_gpu
    from metabuli_work_amd.gtdb_synth import GtdbRecipe, SubDb, encode_into_oracle
    from tests.test_gpu_parity import compare_results

    dev = torch.device("cuda", 0)
    got = {}

    def grab(seq, off):
        got["reads"] = make_reads_gpu(seq, off, 2500, 77, dev)

    rc = GtdbRecipe(dev, n_true_species=10, genome_len=30000, total_species=300, target_kmers=4_000_000,
                    n_chunks=12, before_free=grab)
    reads = _host_reads(*got["reads"])
    n = reads.n
    par = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1)
    ext, _, _ = oc.extract(par.to_c(), reads)
    sub = SubDb.of_kmers(rc.host, ext, dev)
    P = 3
    parts = rc.part_chunks(P)
    assert parts[0][0] == 0 and parts[-1][1] == rc.n_chunks
    chunks, counts, ql = [], [], None
    for p, (c0, c1) in enumerate(parts):
        part = rc.build(c0, c1, guard=True)
        lo_r, hi_r = part.rank_range
        sub.collect(part, lo_r, hi_r, db_end=(p == P - 1))
        with Classifier(par, db_resident=part, db_part=(p, P)) as clf:
            clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2, match_only=True)
            _, m = clf.last_counts()
            mt = np.zeros((m, 24), np.uint8)
            ct = np.zeros(n, np.uint32)
            qt = np.zeros(n, np.uint32)
            clf.copy_matches(mt, ct, qt)
        chunks.append(mt)
        counts.append(ct)
        ql = qt
        del part
        torch.cuda.empty_cache()
    allm = np.concatenate(chunks)
    whole = rc.build()
    with Classifier(par, db_resident=whole) as clf:
        br = clf.assign_chunks(allm, len(allm), np.concatenate(counts), P, ql, n)
        full = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
    assert np.array_equal(br.results, full.results) and np.array_equal(br.taxcnt, full.taxcnt)
    odb = encode_into_oracle(whole, oc.OracleDb, chunk=1 << 20)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    odb.close()
    compare_results(br.results, br.taxcnt, ores, otc)
    sdb, sub_n = sub.oracle_db(oc.OracleDb)
    assert sub_n < whole.n
    sres, stc = oc.classify(sdb, par.to_c(), reads)
    sdb.close()
    compare_results(sres, stc, ores, otc)
    assert br.results["is_classified"].mean() > 0.5


def test_conserved_heavy_tail_parity():
    """The heavy-tailed variant at test scale: AA 8-mers of the true-signal genomes shared by 20 to
    2000 filler species each (long DB runs: the join's long-run selection path, many matches per
    query), classified through the resident DB against the oracle on the same DB; the run-length
    histogram accounts for every k-mer."""
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from metabuli_work_amd.gpu_synth import make_reads_gpu
    from metabuli_work_amd.gtdb_synth import GtdbRecipe, encode_into_oracle, run_length_histogram
    from tests.test_gpu_parity import compare_results

    dev = torch.device("cuda", 0)
    got = {}

    def grab(seq, off):
        got["reads"] = make_reads_gpu(seq, off, 2000, 91, dev)

    rc = GtdbRecipe(dev, n_true_species=10, genome_len=30000, total_species=3000, target_kmers=4_000_000,
                    n_chunks=4, before_free=grab, conserved=400, cons_min=20, cons_max=2000)
    rdb = rc.build()
    v = rdb.values()
    assert bool((v[1:] >= v[:-1]).all())
    h = run_length_histogram(rdb, chunk=1 << 20)
    assert sum(b["kmers"] for b in h["bins"].values()) == rdb.n
    assert h["longest_run"] >= 500
    reads = _host_reads(*got["reads"])
    par = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1)
    with Classifier(par, db_resident=rdb) as clf:
        br = clf.classify_batch(reads.seq1, reads.off1, reads.seq2, reads.off2)
        st = clf.stats()
    odb = encode_into_oracle(rdb, oc.OracleDb, chunk=1 << 20)
    ores, otc = oc.classify(odb, par.to_c(), reads)
    odb.close()
    compare_results(br.results, br.taxcnt, ores, otc)
    assert st["max_read_matches"] > 50
