"""Builds the bench workload twice (genomes, reads, DB) and classifies it twice; prints hashes of
every stage so run-to-run nondeterminism can be located. GPU only."""
import os
import sys

import numpy as np
import torch
import xxhash

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from metabuli_work_amd._abi import default_params  # noqa: E402
from metabuli_work_amd.classifier import Classifier, LocalParameters  # noqa: E402
from metabuli_work_amd.dbbuild import build_db  # noqa: E402


def h(x):
    if isinstance(x, torch.Tensor):
        x = x.cpu().numpy()
    return xxhash.xxh64(np.ascontiguousarray(x).view(np.uint8)).hexdigest()


def main():
    species = int(sys.argv[1]) if len(sys.argv) > 1 else 25000
    pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    dev = torch.device("cuda", 0)
    par = default_params(kmer_format=2, seq_mode=2)
    for trial in range(2):
        taxo, gen, seq, off_t, lens = bench.make_genomes_gpu(species, 75000, 2, 5, dev)
        s1, o1, s2, o2 = bench.make_reads_gpu(seq, off_t, pairs, 5001, dev)
        print(f"trial {trial}: genomes {h(seq)} reads {h(s1)} {h(s2)} blocks {h(gen.blk_start)}", flush=True)
        hdb = build_db(gen, taxo, par, device=0, device_seq=(seq, off_t))
        print(f"trial {trial}: db kmers {hdb.n_kmers} diff {h(hdb.diff_idx)} info {h(hdb.info)} "
              f"split {h(hdb.split)}", flush=True)
        del seq
        torch.cuda.empty_cache()
        lp = LocalParameters(seqMode=2, kmerFormat=2, skipRedundancy=1)
        with Classifier(lp, db_host=hdb.c_struct(), device=0) as clf:
            for rep in range(2):
                br = clf.classify_batch(s1, o1, s2, o2, device_input=True)
                print(f"trial {trial} rep {rep}: Q {br.query_kmers} M {br.matches} results {h(br.results)} "
                      f"taxcnt {h(br.taxcnt)}", flush=True)
        del hdb


if __name__ == "__main__":
    main()
