"""Synthetic inputs for tests and the benchmark (SURVEY.md §8(d) "Synthetic inputs").

There is no network, so the reference genomes, taxonomy and read sets are generated here from
fixed seeds:

* a taxonomy tree in NCBI dmp form (root 1 -> superkingdom -> ... -> genus -> species -> strain);
* genomes: one random base genome per species, strains as substituted copies of it;
* gene blocks: contiguous segments with a random strand, the analogue of the Prodigal ORFs the
  reference's DB builder extracts target k-mers from (IndexCreator.cpp:1087-1240);
* reads: fragments sampled from the genomes (paired 150 bp, or ONT-like long reads) with
  substitutions, a share of random reads, and sprinkled N / IUPAC / lower-case characters.

Everything is numpy and deterministic in its seed.
"""
from __future__ import annotations

import dataclasses
import os
import struct
from typing import List, Optional

import numpy as np

_BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ACGTNacgtn", b"TGCANtgcan"):
    _COMP[_a] = _b


@dataclasses.dataclass
class Taxonomy:
    taxid: np.ndarray      # int32, nodes.dmp row order (root first)
    parent: np.ndarray     # int32
    rank: List[str]
    name: List[str]

    def write_dmp(self, directory: str) -> None:
        os.makedirs(directory, exist_ok=True)
        with open(os.path.join(directory, "nodes.dmp"), "w") as f:
            for t, p, r in zip(self.taxid.tolist(), self.parent.tolist(), self.rank):
                f.write(f"{t}\t|\t{p}\t|\t{r}\t|\t\t|\n")
        with open(os.path.join(directory, "names.dmp"), "w") as f:
            for t, n in zip(self.taxid.tolist(), self.name):
                f.write(f"{t}\t|\t{n}\t|\t\t|\tscientific name\t|\n")
        with open(os.path.join(directory, "merged.dmp"), "w") as f:
            pass


@dataclasses.dataclass
class Genomes:
    seq: np.ndarray        # uint8, concatenated
    off: np.ndarray        # uint64, n+1
    taxid: np.ndarray      # int32 per genome (strain or species node)
    species: np.ndarray    # int32 species taxID per genome
    blk_genome: np.ndarray  # int32 gene blocks
    blk_start: np.ndarray
    blk_end: np.ndarray
    blk_strand: np.ndarray

    @property
    def n(self) -> int:
        return len(self.off) - 1


@dataclasses.dataclass
class Reads:
    seq1: np.ndarray
    off1: np.ndarray
    seq2: Optional[np.ndarray]
    off2: Optional[np.ndarray]
    origin: np.ndarray     # int32 genome index per read, -1 for random reads

    @property
    def n(self) -> int:
        return len(self.off1) - 1

    def names(self) -> List[str]:
        return [f"read{i}" for i in range(self.n)]


def make_taxonomy(n_species: int, strains_per_species: int, seed: int = 1, n_genera: Optional[int] = None,
                  with_eukaryota: bool = True, accessions: int = 0, block_species: int = 0,
                  block_size: int = 1) -> Taxonomy:
    """Root 1 -> {Bacteria, Eukaryota} -> phylum -> class -> order -> family -> genus -> species
    -> strain ("no rank"). Species are spread over genera; the last 1/8 of the genera sit under
    Eukaryota so that the minConsCntEuk branch (Taxonomer.cpp:497-500) is exercised.

    accessions > 0: every strain (or strainless species) gets that many leaves of rank
    "accession", as an accession-level DB build adds them (IndexCreator.cpp:640-660: one new taxon
    per genome accession, child of the genome's taxID); genomes are then made per accession.
    block_species > 0: the first block_species species sit in genera of block_size species each
    (species s in genus s // block_size), so sister species of a genus can share genomes' k-mers."""
    rng = np.random.default_rng(seed)
    n_genera = n_genera or max(1, n_species // 3)
    tax, par, rank, name = [1], [1], ["no rank"], ["root"]
    nxt = [2]

    def add(p: int, r: str, nm: Optional[str] = None) -> int:
        t = nxt[0]
        nxt[0] += 1
        tax.append(t); par.append(p); rank.append(r); name.append(nm or f"{r}_{t}")
        return t

    bact = add(1, "superkingdom", "Bacteria")
    euk = add(1, "superkingdom", "Eukaryota") if with_eukaryota else bact
    genera = []
    n_euk = n_genera // 8 if with_eukaryota else 0
    for g in range(n_genera):
        dom = euk if g >= n_genera - n_euk else bact
        p = add(dom, "phylum")
        c = add(p, "class")
        o = add(c, "order")
        fam = add(o, "family")
        genera.append(add(fam, "genus"))
    for s in range(n_species):
        if s < block_species:
            g = genera[(s // max(1, block_size)) % n_genera]
        else:
            g = genera[int(rng.integers(0, n_genera))] if s >= n_genera else genera[s]
        sp = add(g, "species")
        leaves = [add(sp, "no rank") for _ in range(strains_per_species)] or [sp]
        for lf in leaves:
            for _ in range(accessions):
                add(lf, "accession", f"GCF_{nxt[0]:09d}.1")
    return Taxonomy(np.array(tax, np.int32), np.array(par, np.int32), rank, name)


def _random_dna(rng, n: int, gc: float = 0.5) -> np.ndarray:
    p = np.array([(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2])
    return _BASES[rng.choice(4, size=n, p=p)]


def _mutate(rng, s: np.ndarray, rate: float) -> np.ndarray:
    out = s.copy()
    m = rng.random(len(s)) < rate
    k = int(m.sum())
    if k:
        shift = rng.integers(1, 4, size=k)
        idx = np.searchsorted(_BASES, out[m])
        idx = np.where(_BASES[np.clip(idx, 0, 3)] == out[m], idx, 0)
        out[m] = _BASES[(idx + shift) % 4]
    return out


def make_genomes(taxo: Taxonomy, genome_len: int = 20000, strain_div: float = 0.02, seed: int = 1,
                 len_jitter: float = 0.3, min_block: int = 300, max_block: int = 3000,
                 accession_div: float = 0.004, species_div: float = 0.0) -> Genomes:
    """One genome per strain node (or per species when the species has no strain child); with
    accession leaves, one genome per accession instead (accession_div from its strain's).
    species_div > 0: the species of a genus are diverged copies of one genus genome (GTDB-like
    sharing: related species hold the same AA 8-mers, so species ties and LCAs occur), instead of
    independent random genomes."""
    rng = np.random.default_rng(seed)
    rank = np.array(taxo.rank)
    species_ids = taxo.taxid[rank == "species"]
    children, accs = {}, {}
    for t, p, r in zip(taxo.taxid.tolist(), taxo.parent.tolist(), taxo.rank):
        if r == "no rank" and t != 1:
            children.setdefault(p, []).append(t)
        elif r == "accession":
            accs.setdefault(p, []).append(t)
    seqs, taxids, species = [], [], []

    def emit(g, t, sp):
        if t in accs:
            for a in accs[t]:
                seqs.append(_mutate(rng, g, accession_div)); taxids.append(a); species.append(sp)
        else:
            seqs.append(g); taxids.append(t); species.append(sp)
    parent_of = dict(zip(taxo.taxid.tolist(), taxo.parent.tolist()))
    genus_base = {}
    for sp in species_ids.tolist():
        if species_div > 0:
            gb = genus_base.get(parent_of[sp])
            if gb is None:
                L = max(600, int(genome_len * (1 + len_jitter * (rng.random() * 2 - 1))))
                gb = genus_base[parent_of[sp]] = _random_dna(rng, L, gc=float(rng.uniform(0.35, 0.65)))
            base = _mutate(rng, gb, species_div)
        else:
            L = max(600, int(genome_len * (1 + len_jitter * (rng.random() * 2 - 1))))
            base = _random_dna(rng, L, gc=float(rng.uniform(0.35, 0.65)))
        kids = children.get(sp, [])
        if not kids:
            emit(base, sp, sp)
        for k in kids:
            emit(_mutate(rng, base, strain_div), k, sp)
    return _with_blocks(rng, seqs, taxids, species, min_block, max_block)


def _with_blocks(rng, seqs, taxids, species, min_block: int = 300, max_block: int = 3000) -> Genomes:
    """Genomes with gene blocks (the stand-in for Prodigal's gene calls that the DB writer extracts
    k-mers from): consecutive blocks of min_block..max_block bases on a random strand, short gaps
    between them."""
    off = np.zeros(len(seqs) + 1, np.uint64)
    off[1:] = np.cumsum([len(s) for s in seqs])
    bg, bs, be, bst = [], [], [], []
    for gi, s in enumerate(seqs):
        pos = int(rng.integers(0, 50))
        L = len(s)
        while pos + min_block < L:
            ln = int(rng.integers(min_block, max_block))
            end = min(L - 1, pos + ln - 1)
            bg.append(gi); bs.append(pos); be.append(end); bst.append(1 if rng.random() < 0.5 else -1)
            pos = end + 1 + int(rng.integers(0, 60))
    return Genomes(np.concatenate(seqs), off, np.array(taxids, np.int32), np.array(species, np.int32),
                   np.array(bg, np.int32), np.array(bs, np.int32), np.array(be, np.int32), np.array(bst, np.int32))


CONFIG1_GENOME_LENS = (2_000_000, 1_500_000, 1_000_000)


def make_config1(seed: int = 1):
    """SURVEY §8(d) config 1 (BASELINE.json configs[0], the reference's CPU-runnable case): three
    random genomes (GC 0.5; 2.0 / 1.5 / 1.0 Mbp; seed 1), each its own species in one genus —
    root 1 -> genus 2 -> species 3, 4, 5 -> strains 6, 7, 8 (a genome per strain). Returns
    (Taxonomy, Genomes)."""
    rng = np.random.default_rng(seed)
    taxo = Taxonomy(np.array([1, 2, 3, 4, 5, 6, 7, 8], np.int32), np.array([1, 1, 2, 2, 2, 3, 4, 5], np.int32),
                    ["no rank", "genus", "species", "species", "species", "no rank", "no rank", "no rank"],
                    ["root", "genus_2", "species_3", "species_4", "species_5", "strain_6", "strain_7", "strain_8"])
    seqs = [_random_dna(rng, L, gc=0.5) for L in CONFIG1_GENOME_LENS]
    return taxo, _with_blocks(rng, seqs, [6, 7, 8], [3, 4, 5])


def make_config1_reads(gen: Genomes, n_reads: int = 10_000, seed: int = 2) -> Reads:
    """Config 1's reads: single-end 150 bp, 90% sampled from the genomes with 0.5% substitutions,
    10% random; seed 2."""
    return make_reads(gen, n_reads, paired=False, read_len=150, sub_rate=0.005, random_frac=0.1, seed=seed)


def concat_reads(parts: List["Reads"]) -> "Reads":
    """One read set from several (e.g. drawn at different substitution rates)."""
    def cat(seqs, offs):
        out, base = [np.zeros(1, np.uint64)], 0
        for o in offs:
            out.append(o[1:] + np.uint64(base))
            base += int(o[-1])
        return np.concatenate(seqs).astype(np.uint8), np.concatenate(out)
    s1, o1 = cat([p.seq1 for p in parts], [p.off1 for p in parts])
    s2 = o2 = None
    if parts[0].seq2 is not None:
        s2, o2 = cat([p.seq2 for p in parts], [p.off2 for p in parts])
    return Reads(s1, o1, s2, o2, np.concatenate([p.origin for p in parts]))


def _revcomp(s: np.ndarray) -> np.ndarray:
    return _COMP[s[::-1]]


def _sprinkle(rng, s: np.ndarray, rate_n: float, rate_iupac: float, rate_lower: float) -> np.ndarray:
    if rate_n > 0:
        s[rng.random(len(s)) < rate_n] = ord("N")
    if rate_iupac > 0:
        m = rng.random(len(s)) < rate_iupac
        s[m] = np.frombuffer(b"RYKMSWBDHVU", np.uint8)[rng.integers(0, 11, int(m.sum()))]
    if rate_lower > 0:
        m = (rng.random(len(s)) < rate_lower) & (s >= 65) & (s <= 90)
        s[m] = s[m] + 32
    return s


def _pack(reads: List[np.ndarray]):
    off = np.zeros(len(reads) + 1, np.uint64)
    off[1:] = np.cumsum([len(r) for r in reads])
    seq = np.concatenate(reads) if reads else np.zeros(0, np.uint8)
    return seq.astype(np.uint8), off


def make_reads(gen: Genomes, n_reads: int, paired: bool = True, read_len: int = 150, insert: int = 300,
               insert_sd: int = 30, sub_rate: float = 0.005, random_frac: float = 0.1, seed: int = 2,
               rate_n: float = 0.0005, rate_iupac: float = 0.0002, rate_lower: float = 0.0005,
               short_frac: float = 0.0) -> Reads:
    """Illumina-style reads. short_frac of the reads get a mate shorter than one k-mer window so
    the shared empty-read rule (KmerExtractor.cpp:451-494) is exercised."""
    rng = np.random.default_rng(seed)
    lens = np.diff(gen.off).astype(np.int64)
    w = lens / lens.sum()
    r1, r2, origin = [], [], np.full(n_reads, -1, np.int32)
    for i in range(n_reads):
        if rng.random() < random_frac:
            a = _random_dna(rng, read_len)
            b = _random_dna(rng, read_len)
        else:
            g = int(rng.choice(len(lens), p=w))
            origin[i] = g
            G = gen.seq[int(gen.off[g]):int(gen.off[g + 1])]
            frag = int(max(read_len, min(len(G), rng.normal(insert, insert_sd))))
            st = int(rng.integers(0, max(1, len(G) - frag + 1)))
            f = G[st:st + frag]
            if rng.random() < 0.5:
                f = _revcomp(f)
            a = _mutate(rng, f[:read_len], sub_rate)
            b = _mutate(rng, _revcomp(f)[:read_len], sub_rate)
        if short_frac > 0 and rng.random() < short_frac:
            cut = int(rng.integers(5, 26))
            if rng.random() < 0.5:
                a = a[:cut]
            else:
                b = b[:cut]
        r1.append(_sprinkle(rng, a.copy(), rate_n, rate_iupac, rate_lower))
        r2.append(_sprinkle(rng, b.copy(), rate_n, rate_iupac, rate_lower))
    s1, o1 = _pack(r1)
    if paired:
        s2, o2 = _pack(r2)
        return Reads(s1, o1, s2, o2, origin)
    return Reads(s1, o1, None, None, origin)


def make_long_reads(gen: Genomes, n_reads: int, n50: int = 10000, min_len: int = 1000, sub_rate: float = 0.05,
                    indel_rate: float = 0.01, seed: int = 7) -> Reads:
    """ONT-like single-end reads: lognormal lengths, substitutions and indels."""
    rng = np.random.default_rng(seed)
    lens = np.diff(gen.off).astype(np.int64)
    w = lens / lens.sum()
    out, origin = [], np.zeros(n_reads, np.int32)
    for i in range(n_reads):
        g = int(rng.choice(len(lens), p=w))
        origin[i] = g
        G = gen.seq[int(gen.off[g]):int(gen.off[g + 1])]
        L = int(min(len(G), max(min_len, rng.lognormal(np.log(n50 * 0.8), 0.5))))
        st = int(rng.integers(0, max(1, len(G) - L + 1)))
        f = G[st:st + L]
        if rng.random() < 0.5:
            f = _revcomp(f)
        f = _mutate(rng, f, sub_rate)
        if indel_rate > 0:
            keep = rng.random(len(f)) >= indel_rate / 2
            f = f[keep]
            ins = rng.random(len(f)) < indel_rate / 2
            f = np.insert(f, np.nonzero(ins)[0], _BASES[rng.integers(0, 4, int(ins.sum()))])
        out.append(f.astype(np.uint8))
    s, o = _pack(out)
    return Reads(s, o, None, None, origin)


def to_internal_ids(taxo: Taxonomy):
    """Internal taxIDs as TaxonomyWrapper's dmp loader assigns them with useInternalTaxID
    (TaxonomyWrapper.cpp:147-185: 1, 2, ... in order of first appearance scanning nodes.dmp rows,
    each row's taxID then its parent; internal 0 stays unused). Returns (the taxonomy in internal
    IDs, internal2org as an int32 array with internal2org[0] = 0)."""
    o2i, i2o = {}, [0]
    for t, p in zip(taxo.taxid.tolist(), taxo.parent.tolist()):
        for x in (t, p):
            if x not in o2i:
                o2i[x] = len(i2o)
                i2o.append(x)
    tax = np.array([o2i[t] for t in taxo.taxid.tolist()], np.int32)
    par = np.array([o2i[p] for p in taxo.parent.tolist()], np.int32)
    return Taxonomy(tax, par, list(taxo.rank), list(taxo.name)), np.array(i2o, np.int32)


TAXONOMY_DB_VERSION = 2  # NcbiTaxonomy::SERIALIZATION_VERSION (MMseqs2; the submodule is absent: unpinned)


def write_taxonomy_db(taxo: Taxonomy, path: str, internal2org: Optional[np.ndarray] = None) -> None:
    """A taxonomyDB file as TaxonomyWrapper::serialize writes it (TaxonomyWrapper.cpp:289-361):
    version int, [size_t 1 when internal taxIDs are used], size_t maxNodes, int maxTaxID,
    TaxonNode[maxNodes] (MMseqs2 layout: int id, taxId, parentTaxId, 4 pad bytes, size_t rankIdx,
    nameIdx), int D[maxTaxID + 1], [int internal2orgTaxId[maxTaxID + 1]], int E[2 maxNodes],
    L[2 maxNodes], H[maxNodes], the sparse table M[2 maxNodes][flog2(2 maxNodes) + 1] (initTaxonomy,
    :115-146), then StringBlock<unsigned int> {byteCapacity, entryCapacity, entryCount, bytes,
    offsets}. `taxo` is in the IDs the DB uses (internal ones when internal2org is given)."""
    n = len(taxo.taxid)
    max_tax = int(max(taxo.taxid.max(), taxo.parent.max()))
    if internal2org is not None:
        max_tax = max(max_tax, len(internal2org) - 1)
    D = np.full(max_tax + 1, -1, np.int32)
    D[taxo.taxid] = np.arange(n, dtype=np.int32)
    # string block: each node's rank appended in node order (loadNodes), then the names (loadNames)
    strings, rank_idx, name_idx = [], [], []
    for r in taxo.rank:
        rank_idx.append(len(strings)); strings.append(r)
    for nm in taxo.name:
        name_idx.append(len(strings)); strings.append(nm)
    enc = [s.encode() + b"\0" for s in strings]
    offs = np.zeros(len(enc), np.uint32)
    offs[1:] = np.cumsum([len(e) for e in enc])[:-1]
    blob = b"".join(enc)
    # Euler tour from taxID 1 (NcbiTaxonomy::elh), iterative
    children = [[] for _ in range(n)]
    for i in range(n):
        if taxo.parent[i] != taxo.taxid[i]:
            children[D[taxo.parent[i]]].append(int(taxo.taxid[i]))
    E, L, H = [], [], np.zeros(n, np.int32)
    stack = [(1, 0, 0)]  # (taxID, level, next child)
    while stack:
        t, lvl, k = stack.pop()
        i = int(D[t])
        if k == 0:
            if H[i] == 0:
                H[i] = len(E)
            E.append(i); L.append(lvl)
        if k < len(children[i]):
            stack.append((t, lvl, k + 1))
            stack.append((children[i][k], lvl + 1, 0))
        else:
            E.append(int(D[taxo.parent[i]])); L.append(lvl - 1)
    N = 2 * n
    E = np.array((E + [0] * N)[:N], np.int32)
    L = np.array((L + [0] * N)[:N], np.int32)
    K = int(np.floor(np.log2(N))) + 1
    M = np.zeros((N, K), np.int32)
    M[:, 0] = np.arange(N)
    j = 1
    while (1 << j) <= N:  # NcbiTaxonomy::computeSparseTable
        h = 1 << (j - 1)
        m = N - (1 << j) + 1
        a, b = M[:m, j - 1], M[h:h + m, j - 1]
        M[:m, j] = np.where(L[a] < L[b], a, b)
        j += 1
    node = np.zeros(n, np.dtype([("id", "<i4"), ("taxId", "<i4"), ("parentTaxId", "<i4"), ("pad", "<i4"),
                                 ("rankIdx", "<u8"), ("nameIdx", "<u8")]))
    node["id"] = np.arange(n)
    node["taxId"] = taxo.taxid
    node["parentTaxId"] = taxo.parent
    node["rankIdx"] = rank_idx
    node["nameIdx"] = name_idx
    with open(path, "wb") as f:
        f.write(np.int32(TAXONOMY_DB_VERSION).tobytes())
        if internal2org is not None:
            f.write(np.uint64(1).tobytes())
        f.write(np.uint64(n).tobytes())
        f.write(np.int32(max_tax).tobytes())
        f.write(node.tobytes())
        f.write(D.tobytes())
        if internal2org is not None:
            i2o = np.zeros(max_tax + 1, np.int32)
            i2o[:len(internal2org)] = internal2org
            f.write(i2o.tobytes())
        f.write(E.tobytes()); f.write(L.tobytes()); f.write(H.tobytes()); f.write(M.tobytes())
        f.write(np.array([len(blob), len(enc), len(enc)], np.uint32).tobytes())
        f.write(blob)
        f.write(offs.tobytes())


# ---- FASTQ files of synthetic reads (tests, end-to-end bench) ------------------------------------
def fastq_bytes(seq: np.ndarray, off: np.ndarray, prefix: str = "r", qual: int = ord("I")) -> bytes:
    """FASTQ text of reads (seq, off): "@<prefix><9-digit index>" headers, one sequence and one
    quality line each. Vectorised for fixed-length reads, a loop otherwise."""
    n = len(off) - 1
    lens = np.diff(off.astype(np.int64))
    if n and (lens == lens[0]).all():
        L = int(lens[0])
        hl = 1 + len(prefix) + 9 + 1
        rec = hl + (L + 1) + 2 + (L + 1)
        out = np.empty((n, rec), np.uint8)
        out[:, 0] = ord("@")
        out[:, 1:1 + len(prefix)] = np.frombuffer(prefix.encode(), np.uint8)
        idx = np.arange(n, dtype=np.int64)
        for k in range(9):
            out[:, 1 + len(prefix) + k] = ord("0") + (idx // 10 ** (8 - k)) % 10
        out[:, hl - 1] = ord("\n")
        out[:, hl:hl + L] = seq[:n * L].reshape(n, L)
        out[:, hl + L] = ord("\n")
        out[:, hl + L + 1] = ord("+")
        out[:, hl + L + 2] = ord("\n")
        out[:, hl + L + 3:hl + 2 * L + 3] = qual
        out[:, rec - 1] = ord("\n")
        return out.tobytes()
    parts = []
    for i in range(n):
        s = bytes(seq[int(off[i]):int(off[i + 1])])
        parts.append(b"@%s%09d\n%s\n+\n%s\n" % (prefix.encode(), i, s, bytes([qual]) * len(s)))
    return b"".join(parts)


def _bgzf_block(data: bytes, level: int) -> bytes:
    import struct
    import zlib
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    cdata = c.compress(data) + c.flush()
    bsize = 18 + len(cdata) + 8 - 1
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff\x06\x00BC\x02\x00" + struct.pack("<H", bsize)
    return hdr + cdata + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def write_compressed(path: str, data: bytes, mode: str = "bgzf", level: int = 1, threads: int = 16) -> None:
    """data to path: mode "plain", "gzip" (one member) or "bgzf" (64 KB members with their size in a
    BC extra field, as bgzip writes; compressed by a thread pool: zlib releases the GIL)."""
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    if mode == "plain":
        with open(path, "wb") as f:
            f.write(data)
        return
    if mode == "gzip":
        # one gzip member, its deflate stream compressed in 64 MB segments by a thread pool (as pigz
        # does: each segment ends with a sync flush, the last one finishes the stream)
        seg = 1 << 26
        mv = memoryview(data)
        starts = list(range(0, len(data), seg)) or [0]

        def deflate(i):
            c = zlib.compressobj(level, zlib.DEFLATED, -15)
            out = c.compress(mv[i:i + seg])
            return out + c.flush(zlib.Z_FINISH if i == starts[-1] else zlib.Z_SYNC_FLUSH)
        with ThreadPoolExecutor(threads) as ex, open(path, "wb") as f:
            f.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\xff")  # no flags, no mtime, OS unknown
            for part in ex.map(deflate, starts):
                f.write(part)
            crc = 0
            for i in range(0, len(data), seg):
                crc = zlib.crc32(mv[i:i + seg], crc)
            f.write(struct.pack("<II", crc & 0xFFFFFFFF, len(data) & 0xFFFFFFFF))
        return
    blk = 65280
    mv = memoryview(data)
    with ThreadPoolExecutor(threads) as ex, open(path, "wb") as f:
        for part in ex.map(lambda i: _bgzf_block(bytes(mv[i:i + blk]), level), range(0, len(data), blk)):
            f.write(part)
        f.write(_bgzf_block(b"", level))  # the BGZF end-of-file marker block
