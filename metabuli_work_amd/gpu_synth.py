"""Synthetic workloads generated on the GPU (torch): genomes with gene blocks, Illumina-style
read pairs, ONT-style long reads (bench.py and the GTDB-scale DB of gtdb_synth.py). Bench/test data
only: nothing here is on the classify path.
"""
import numpy as np
import torch

from . import synth


# ---------------------------------------------------------------------------------------------
def make_genomes_gpu(n_species, mean_len, strains, seed, dev, taxo=None, per_genus=1, species_div=0.0):
    """Genomes of the first n_species species of `taxo` (made here when None), `strains` 2%-diverged
    strains each, with gene blocks shared by a species' strains. per_genus > 1: species come in
    groups of per_genus (the genera of make_taxonomy(block_species=..., block_size=per_genus)) whose
    genomes are species_div-diverged copies of one genus genome (GTDB-like: sister species share
    most of their AA 8-mers, so a DB AA run holds several species)."""
    rng = np.random.default_rng(seed)
    if taxo is None:
        taxo = synth.make_taxonomy(n_species, strains, seed=seed)
    per_genus = max(1, int(per_genus))
    n_gen = (n_species + per_genus - 1) // per_genus
    glens = rng.integers(int(mean_len * 0.3), int(mean_len * 1.7), size=n_gen).astype(np.int64)
    lens = glens[np.arange(n_species) // per_genus]
    base_off = np.zeros(n_species + 1, np.int64)
    base_off[1:] = np.cumsum(lens)
    total = int(base_off[-1])
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    lut = torch.tensor([65, 67, 71, 84], dtype=torch.uint8, device=dev)
    if per_genus == 1:
        base = torch.randint(0, 4, (total,), dtype=torch.uint8, device=dev, generator=g)
    else:  # each species: its genus genome with species_div substitutions
        base = torch.empty(total, dtype=torch.uint8, device=dev)
        for gi in range(n_gen):
            L = int(glens[gi])
            gb = torch.randint(0, 4, (L,), dtype=torch.uint8, device=dev, generator=g)
            for s in range(gi * per_genus, min(n_species, (gi + 1) * per_genus)):
                m = torch.rand(L, device=dev, generator=g) < species_div
                sh = torch.randint(1, 4, (L,), dtype=torch.uint8, device=dev, generator=g)
                base[int(base_off[s]):int(base_off[s + 1])] = torch.where(m, (gb + sh) % 4, gb)
    seq = torch.empty(total * strains, dtype=torch.uint8, device=dev)
    chunk = 1 << 28
    for k in range(strains):
        for a in range(0, total, chunk):
            b = min(total, a + chunk)
            x = base[a:b]
            m = torch.rand(b - a, device=dev, generator=g) < 0.02
            sh = torch.randint(1, 4, (b - a,), dtype=torch.uint8, device=dev, generator=g)
            x = torch.where(m, (x + sh) % 4, x)
            seq[k * total + a:k * total + b] = lut[x.long()]
    del base
    # genome k*n_species + s = strain k of species s; taxIDs: the strain nodes of each species
    rank = np.array(taxo.rank)
    sp_ids = taxo.taxid[rank == "species"][:n_species]
    strain_of = {}
    for t, p, r in zip(taxo.taxid.tolist(), taxo.parent.tolist(), taxo.rank):
        if r == "no rank" and t != 1:
            strain_of.setdefault(p, []).append(t)
    gtax = np.zeros(n_species * strains, np.int32)
    for s, sp in enumerate(sp_ids.tolist()):
        for k in range(strains):
            gtax[k * n_species + s] = strain_of[sp][k]
    off = np.zeros(n_species * strains + 1, np.int64)
    off[1:] = np.concatenate([np.cumsum(np.tile(lens, strains))])
    # gene blocks per species, shared by its strains (same coordinates)
    bg, bs, be, bst = [], [], [], []
    for s in range(n_species):
        L = int(lens[s])
        n_est = L // 300 + 2
        ln = rng.integers(300, 3000, size=n_est)
        gap = rng.integers(0, 60, size=n_est)
        starts = np.concatenate([[int(rng.integers(0, 50))], np.cumsum(ln + gap)[:-1] + int(rng.integers(0, 50))])
        ends = starts + ln - 1
        keep = starts + 300 < L
        starts, ends = starts[keep], np.minimum(ends[keep], L - 1)
        strand = np.where(rng.random(len(starts)) < 0.5, 1, -1)
        for k in range(strains):
            bg.append(np.full(len(starts), k * n_species + s, np.int32))
            bs.append(starts.astype(np.int32))
            be.append(ends.astype(np.int32))
            bst.append(strand.astype(np.int32))
    gen = synth.Genomes(seq=None, off=off.astype(np.uint64), taxid=gtax,
                        species=np.repeat(sp_ids, 1)[np.tile(np.arange(n_species), strains)],
                        blk_genome=np.concatenate(bg), blk_start=np.concatenate(bs), blk_end=np.concatenate(be),
                        blk_strand=np.concatenate(bst))
    off_t = torch.from_numpy(off).to(dev)
    return taxo, gen, seq, off_t, lens


def make_reads_gpu(seq, off_t, n_pairs, seed, dev, read_len=150, sub_rate=0.005, random_frac=0.1,
                   abundance_sigma=0.0):
    """abundance_sigma > 0: a skewed sample — genome g drawn with weight length_g * A_g, A_g log-normal
    (mu 0, sigma abundance_sigma, seeded), so a few genomes take tens of x the coverage of the rest
    (real samples); 0: proportional to length."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    # genome chosen proportionally to its (weighted) length (searchsorted on the cumulative weights:
    # torch.multinomial is not run-to-run deterministic on this device)
    glen_all = (off_t[1:] - off_t[:-1]).double()
    if abundance_sigma > 0:
        ab = np.random.default_rng(seed).lognormal(0.0, abundance_sigma, off_t.numel() - 1)
        w = glen_all * torch.from_numpy(ab).to(dev)
    else:
        w = glen_all
    cw = torch.cumsum(w, 0)
    u = torch.rand(n_pairs, device=dev, generator=g, dtype=torch.float64) * float(cw[-1].item())
    gsel = torch.searchsorted(cw, u, right=True).clamp(max=off_t.numel() - 2)
    gl = (off_t[1:] - off_t[:-1])[gsel]
    ins = (torch.randn(n_pairs, device=dev, generator=g) * 30 + 300).round().long().clamp(min=read_len)
    ins = torch.minimum(ins, gl)
    start = (torch.rand(n_pairs, device=dev, generator=g) * (gl - ins + 1).float()).long()
    start = torch.minimum(start, gl - ins)
    p0 = off_t[gsel] + start
    ar = torch.arange(read_len, device=dev)
    A = seq[p0[:, None] + ar]
    comp = torch.zeros(256, dtype=torch.uint8, device=dev)
    comp[torch.tensor([65, 67, 71, 84], device=dev)] = torch.tensor([84, 71, 67, 65], dtype=torch.uint8, device=dev)
    B = comp[seq[(p0 + ins - read_len)[:, None] + ar].long()].flip(1)
    flip = (torch.rand(n_pairs, device=dev, generator=g) < 0.5)[:, None]
    m1 = torch.where(flip, B, A)
    m2 = torch.where(flip, A, B)
    lut = torch.tensor([65, 67, 71, 84], dtype=torch.uint8, device=dev)
    out = []
    rnd = torch.rand(n_pairs, device=dev, generator=g) < random_frac
    for m in (m1, m2):
        sub = torch.rand(m.shape, device=dev, generator=g) < sub_rate
        repl = lut[torch.randint(0, 4, m.shape, device=dev, generator=g)]
        m = torch.where(sub, repl, m)
        rr = lut[torch.randint(0, 4, m.shape, device=dev, generator=g)]
        m = torch.where(rnd[:, None], rr, m)
        out.append(m.contiguous().view(-1))
    off = torch.arange(0, (n_pairs + 1) * read_len, read_len, dtype=torch.int64, device=dev)
    return out[0], off, out[1], off.clone()


def make_long_reads_gpu(seq, off_t, n_reads, seed, dev, n50=10000, min_len=1000, sub_rate=0.05, indel_rate=0.01):
    """ONT-style single-end reads (SURVEY §8(d) config 4 shape): lognormal lengths (N50 ~10 kb,
    >= 1 kb), random strand, 5% substitutions, 1% indels (half deletions, half insertions)."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    rng = np.random.default_rng(seed)
    glen = (off_t[1:] - off_t[:-1]).cpu().numpy()
    cum = np.cumsum(glen)
    gsel = np.searchsorted(cum, rng.random(n_reads) * cum[-1], side="right").clip(max=len(glen) - 1)
    L = np.minimum(glen[gsel], np.maximum(min_len, rng.lognormal(np.log(n50 * 0.8), 0.5, n_reads))).astype(np.int64)
    st = (rng.random(n_reads) * (glen[gsel] - L + 1)).astype(np.int64)
    p0 = off_t.cpu().numpy()[gsel] + st
    lens = torch.from_numpy(L).to(dev)
    roff = torch.zeros(n_reads + 1, dtype=torch.int64, device=dev)
    roff[1:] = torch.cumsum(lens, 0)
    tot = int(roff[-1].item())
    rid = torch.repeat_interleave(torch.arange(n_reads, device=dev), lens)
    within = torch.arange(tot, device=dev) - roff[rid]
    rev = torch.from_numpy(rng.random(n_reads) < 0.5).to(dev)
    pos = torch.where(rev[rid], torch.from_numpy(p0).to(dev)[rid] + lens[rid] - 1 - within,
                      torch.from_numpy(p0).to(dev)[rid] + within)
    b = seq[pos]
    comp = torch.zeros(256, dtype=torch.uint8, device=dev)
    comp[torch.tensor([65, 67, 71, 84], device=dev)] = torch.tensor([84, 71, 67, 65], dtype=torch.uint8, device=dev)
    b = torch.where(rev[rid], comp[b.long()], b)
    lut = torch.tensor([65, 67, 71, 84], dtype=torch.uint8, device=dev)
    sub = torch.rand(tot, device=dev, generator=g) < sub_rate
    b = torch.where(sub, lut[torch.randint(0, 4, (tot,), device=dev, generator=g)], b)
    # indels: each base is kept 0 (deleted), 1 or 2 times (a random base inserted after it)
    u = torch.rand(tot, device=dev, generator=g)
    copies = torch.ones(tot, dtype=torch.int64, device=dev)
    copies[u < indel_rate / 2] = 0
    copies[(u >= indel_rate / 2) & (u < indel_rate)] = 2
    idx = torch.repeat_interleave(torch.arange(tot, device=dev), copies)
    first = torch.ones(idx.numel(), dtype=torch.bool, device=dev)
    first[1:] = idx[1:] != idx[:-1]
    out = torch.where(first, b[idx], lut[torch.randint(0, 4, (idx.numel(),), device=dev, generator=g)])
    new_len = torch.zeros(n_reads, dtype=torch.int64, device=dev).index_add_(0, rid, copies)
    off = torch.zeros(n_reads + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(new_len, 0)
    ls = np.sort(new_len.cpu().numpy())[::-1]
    n50_obs = int(ls[np.searchsorted(np.cumsum(ls), ls.sum() / 2)])
    return out.contiguous(), off, n50_obs
