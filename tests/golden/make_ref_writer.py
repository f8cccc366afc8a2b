"""Regenerate tests/golden/ref_writer.npz: the diffIdx / info / split files the reference's OWN DB writer
produces for fixed sorted unique (value, taxID) lists (round 6).

Runs in this container only; as in make_ref_functions.py, the code is cut out of /root/reference at
run time into a throw-away C++ file next to minimal declarations (a `Kmer` of value / id, a `Buffer`,
an `IndexCreator` with the members the cut code reads), compiled with BitManipulateMacros.h in place,
run in a temporary directory (the writer writes its files there) and deleted. The cut code:
* `WriteBuffer` (common.h:284-330) and `DiffIdxSplit` (Kmer.h:111-119), whole
* the constructor's `MARKER` choice (IndexCreator.cpp:31-37) and `AminoAcidPart` (IndexCreator.h:209-214)
* `IndexCreator::writeTargetFilesAndSplits` and `IndexCreator::getDiffIdx` (IndexCreator.cpp:811-886)
The lists stand for what filterKmers<DB_CREATION> hands the writer (IndexCreator.cpp:368): sorted by
value, one entry per (value, species), so a value repeats across species (a zero delta); AA parts
are drawn from a small set so AA groups straddle the split offsets.
"""
import pathlib
import subprocess
import tempfile

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REF = pathlib.Path("/root/reference/src/commons")

from make_ref_functions import definitions, if_else  # noqa: E402
from make_ref_scanners import class_text  # noqa: E402


def program() -> str:
    cm = (REF / "common.h").read_text()
    km = (REF / "Kmer.h").read_text()
    ih = (REF / "IndexCreator.h").read_text()
    ic = (REF / "IndexCreator.cpp").read_text()
    wb = "template<typename T>\n" + class_text(cm, "struct WriteBuffer {")
    ds = class_text(km, "struct DiffIdxSplit{")
    aa = definitions(ih, r"size_t AminoAcidPart\(size_t kmer\)")
    assert len(aa) == 1
    marker = if_else(ic, "par.reducedAA == 1")
    defs = definitions(ic, r"void IndexCreator::writeTargetFilesAndSplits\(") + \
        definitions(ic, r"void IndexCreator::getDiffIdx\(\s*uint64_t & lastKmer")
    assert len(defs) == 2, len(defs)
    return "\n".join([
        "#include <cstdint>", "#include <cstdio>", "#include <cstdlib>", "#include <cstring>", "#include <iostream>",
        "#include <string>", "#include <utility>", "#include <vector>", '#include "BitManipulateMacros.h"',
        "using namespace std;",
        wb, ds,
        "struct Kmer { uint64_t value; uint32_t id; };",
        "template <typename T> struct Buffer { T *buffer; size_t startIndexOfReserve; };",
        "struct Par { int splitNum; int reducedAA; };",
        "struct IndexCreator {",
        "  Par par; string dbDir; int numOfFlush = 0; int kmerFormat = 2; uint64_t MARKER;",
        "  void setMarker() {", marker, "  }",
        *aa,
        "  void writeTargetFilesAndSplits(Buffer<Kmer> &kmerBuffer, const size_t *uniqKmerIdx, size_t &uniqKmerCnt,"
        " const vector<pair<size_t, size_t>> &uniqKmerIdxRanges);",
        "  void getDiffIdx(uint64_t &lastKmer, uint64_t entryToWrite, WriteBuffer<uint16_t> &diffBuffer);",
        "};", *defs, DRIVER])


# argv: dbDir splitNum; stdin: n, then n lines "value id"
DRIVER = r"""
int main(int argc, char **argv) {
  IndexCreator ic; ic.dbDir = argv[1]; ic.par = Par{atoi(argv[2]), 0}; ic.setMarker();
  size_t n; if (scanf("%zu", &n) != 1) return 1;
  std::vector<Kmer> k(n); std::vector<size_t> idx(n);
  for (size_t i = 0; i < n; i++) {
    unsigned long long v; unsigned id;
    if (scanf("%llu %u", &v, &id) != 2) return 2;
    k[i] = Kmer{(uint64_t)v, id}; idx[i] = i;
  }
  Buffer<Kmer> b{k.data(), 0};
  vector<pair<size_t, size_t>> ranges{{0, n}};
  size_t cnt = n;
  ic.writeTargetFilesAndSplits(b, idx.data(), cnt, ranges);
  return 0;
}
"""

CASES = [("tiny", 12, 4), ("small", 1000, 16), ("mid", 20000, 64), ("full", 60000, 4096)]


def kmer_list(rng, n):
    """Sorted (value, taxID) entries: AA parts from a small pool (runs of several k-mers), DNA parts
    random, some values repeated across species, deltas of 1 to 5 15-bit groups."""
    pool = np.sort(rng.integers(0, 21 ** 8, max(4, n // 3), dtype=np.uint64))
    aa = pool[rng.integers(0, len(pool), n)]
    v = (aa << np.uint64(24)) | rng.integers(0, 1 << 24, n, dtype=np.uint64)
    v[: n // 50] = rng.integers(0, 1 << 62, n // 50, dtype=np.uint64)  # some far-apart values (long deltas)
    v = np.sort(v)
    rep = rng.random(n) < 0.1
    v[1:][rep[1:]] = v[:-1][rep[1:]]  # the same value again: another species
    v = np.sort(v)
    ids = rng.integers(1, 1 << 20, n, dtype=np.uint64).astype(np.uint32)
    return v, ids


if __name__ == "__main__":
    rng = np.random.default_rng(20261020)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        src = pathlib.Path(d) / "ref_writer.cpp"
        exe = pathlib.Path(d) / "ref_writer"
        src.write_text(program())
        subprocess.run(["g++", "-O1", "-std=c++17", f"-I{REF}", str(src), "-o", str(exe)], check=True)
        for name, n, split_num in CASES:
            v, ids = kmer_list(rng, n)
            db = pathlib.Path(d) / name
            db.mkdir()
            inp = f"{n}\n" + "\n".join(f"{int(a)} {int(b)}" for a, b in zip(v, ids)) + "\n"
            subprocess.run([str(exe), str(db), str(split_num)], input=inp, capture_output=True, text=True, check=True)
            out[f"{name}_values"] = v
            out[f"{name}_ids"] = ids
            out[f"{name}_split_num"] = np.array([split_num])
            out[f"{name}_diffIdx"] = np.fromfile(db / "diffIdx", np.uint16)
            out[f"{name}_info"] = np.fromfile(db / "info", np.uint32)
            out[f"{name}_split"] = np.fromfile(db / "split", np.uint64)
            print(name, n, "k-mers:", len(out[f"{name}_diffIdx"]), "words,",
                  int((out[f"{name}_split"].reshape(-1, 3)[:, 1] > 0).sum()), "split entries")
    np.savez_compressed(HERE / "ref_writer.npz", **out)
    print("wrote", HERE / "ref_writer.npz")
