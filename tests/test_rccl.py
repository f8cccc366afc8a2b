"""The RCCL (backend "nccl") branches of the multi-GPU paths, run for real on the one GPU a box has
(VERDICT r05 item 1): a world-1 "nccl" process group on cuda:0, so every collective of
dist.gather_results / classify_sharded / classify_batches_sharded / exchange_matches /
classify_partitioned and the bench's ResultGather runs through RCCL on device tensors — the code the
8-GPU scaling run takes, which until now only gloo had executed. World 1 is what one GPU allows (RCCL
refuses two ranks on one device); the N > 1 layouts (rebasing, rank order, empty ranks) are covered
by the gloo tests in test_dist.py / test_partition.py. Every result is compared with the oracle.
"""
import importlib.util
import os
import pathlib
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import oracle_ctypes as oc

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reads(gen, seed, n=1200):
    from metabuli_work_amd import synth
    return synth.make_reads(gen, n, paired=True, seed=seed, short_frac=0.03, rate_n=0.002)


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _rccl_worker(port, db_dir, seed, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist

    from metabuli_work_amd import synth
    from metabuli_work_amd.classifier import Classifier, LocalParameters
    from metabuli_work_amd.dist import (classify_batches_sharded, classify_partitioned, classify_sharded,
                                        exchange_matches, gather_results, owner_bounds, shard_reads)

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out = {"backend": dist.get_backend()}
    taxo = synth.make_taxonomy(14, 2, seed=11)
    gen = synth.make_genomes(taxo, genome_len=24000, seed=12)
    r = _reads(gen, seed)
    par = LocalParameters(seqMode=2).load_db_parameters(db_dir)

    def host(rec, tc):
        return rec.cpu().numpy().reshape(-1).copy(), tc.cpu().numpy().reshape(-1).copy()

    with Classifier(par, db_dir=db_dir, device=0) as clf:
        # C1 of the replicated DB: the host batch's shard, its records moved to HBM, RCCL all-gathers
        res, tc = classify_sharded(clf, r.seq1, r.off1, r.seq2, r.off2)
        out["sharded"] = (res.view(np.uint8).copy(), tc.view(np.uint8).copy())
        # batches dealt by index (config 4's form), gathered over RCCL and put back in batch order
        cuts = [(a, min(r.n, a + 500)) for a in range(0, r.n, 500)]
        batches = [shard_reads(r.seq1, r.off1, a, b) + shard_reads(r.seq2, r.off2, a, b) for a, b in cuts]
        res, tc = classify_batches_sharded(clf, batches)
        out["batches"] = (res.view(np.uint8).copy(), tc.view(np.uint8).copy())
        # the bench's C1: device-resident batches, records and lists copied device to device into the
        # step buffers (offsets rebased), then gathered through RCCL
        s1, s2 = torch.from_numpy(r.seq1).to(dev), torch.from_numpy(r.seq2).to(dev)
        o1 = torch.from_numpy(r.off1.astype(np.uint64).view(np.int64)).to(dev)
        o2 = torch.from_numpy(r.off2.astype(np.uint64).view(np.int64)).to(dev)
        rg = _bench().ResultGather(dev, r.n)
        rec_all = torch.empty((r.n, 32), dtype=torch.uint8, device=dev)
        for step in range(2):  # reset() between steps, as the bench's timed loop does
            rg.reset()
            for a, b in cuts:
                clf.classify_batch(s1, o1[a:b + 1], s2, o2[a:b + 1], device_input=True, fetch=False)
                rg.add(clf, rec_all[a:b])
            grec, gtc = rg.gather(rec_all)
            assert grec.device == dev and gtc.device == dev
        out["result_gather"] = host(grec, gtc)
    # config 5's exchange: match-only pass, per-read segments all-to-all (RCCL) on device tensors,
    # K5 + K6 on the receive layout, C1
    with Classifier(par, db_dir=db_dir, device=0, db_part=(0, 1)) as clf:
        (lo, hi), br = classify_partitioned(clf, r.seq1, r.off1, r.seq2, r.off2, on_device=True)
        assert br is None and (lo, hi) == (0, r.n)
        rec = torch.empty((r.n, 32), dtype=torch.uint8, device=dev)
        clf.copy_results(rec.data_ptr(), on_device=True)
        pool = torch.empty((max(clf.n_taxcnt(), 1), 8), dtype=torch.uint8, device=dev)
        nt = clf.copy_taxcnt(pool.data_ptr(), on_device=True)
        out["partitioned"] = host(*gather_results(rec, pool[:nt]))
        # exchange_matches alone on device tensors: the segments come back unchanged at world 1
        clf.classify_batch(r.seq1, r.off1, r.seq2, r.off2, match_only=True)
        _, M = clf.last_counts()
        m = torch.empty((M, 24), dtype=torch.uint8, device=dev)
        cnt = torch.empty(r.n, dtype=torch.int32, device=dev)
        ql = torch.empty(r.n, dtype=torch.int32, device=dev)
        clf.copy_matches(m, cnt, ql)
        rm, rc = exchange_matches(m, cnt, owner_bounds(r.n, 1))
        out["exchange_same"] = bool(torch.equal(rm, m) and torch.equal(rc, cnt))
        out["exchange_m"] = int(M)
    dist.destroy_process_group()
    q.put(out)


@pytest.mark.gpu
def test_rccl_world1_paths_match_oracle(make_db):
    from metabuli_work_amd._abi import RESULT_DTYPE, TAXCNT_DTYPE
    from metabuli_work_amd.classifier import LocalParameters
    from tests.test_gpu_parity import compare_results

    db_dir, taxo, gen = make_db("fmt2")
    r = _reads(gen, 43)
    par_c = LocalParameters(seqMode=2).load_db_parameters(db_dir).to_c()
    odb = oc.OracleDb(db_dir)
    ores, otc = oc.classify(odb, par_c, r)
    odb.close()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), db_dir, 43, q))
    p.start()
    got = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert got["backend"] == "nccl"
    for k in ("sharded", "batches", "result_gather", "partitioned"):
        rec, tc = got[k]
        res, tcs = rec.view(RESULT_DTYPE).reshape(-1), tc.view(TAXCNT_DTYPE).reshape(-1)
        assert len(res) == len(ores), k
        assert int(res["taxcnt_len"].sum()) == len(tcs), k
        compare_results(res, tcs, ores, otc)
    assert got["exchange_same"] and got["exchange_m"] > 0
