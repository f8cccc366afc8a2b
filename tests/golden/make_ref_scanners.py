"""Regenerate tests/golden/ref_scanners.npz: the query k-mers the reference's OWN extraction code emits
for a fixed read set, in emission order (round 6: the scanners were "parity unpinned" until now).

Runs in this container only (it reads /root/reference); the committed .npz is what the tests read.
As in make_ref_functions.py nothing of the reference enters the repository: the code below is cut out
of the reference's files at run time, pasted into a throw-away C++ file in a temporary directory next
to minimal declarations (the fields and constructors the cut code uses: a `Kmer` of value / pos /
seqID / frame, a `Buffer`, the `KmerExtractor` member array of scanners), compiled with the
reference's own GeneticCode.h in place (-I src/commons), run and deleted. The cut code:
* `class KmerScanner`, `class MetamerScanner`, `class OldMetamerScanner` (KmerScanner.h:11-181) and
  `class SyncmerScanner` (SyncmerScanner.h:9-102), whole, as written
* the `atcg` / `iRCT` tables (common.cpp:13-23)
* `LocalUtil::getMaxCoveredLength` (LocalUtil.h:50-59)
* `KmerExtractor::fillQueryKmerBuffer` (KmerExtractor.cpp:355-386): the six frames of one mate
The driver calls them the way the reference's callers do: the scanner per KmerExtractor's
constructor (KmerExtractor.cpp:8-30: format 1 -> OldMetamerScanner, format 2 -> SyncmerScanner with
--syncmer, else MetamerScanner) and per read processSequence's calls (KmerExtractor.cpp:311-353:
seqID = read index + 1; mate 2 offset by queryLength + 3, queryLength = getMaxCoveredLength of mate 1,
KmerExtractor.cpp:478). Reads whose mates cannot hold a k-mer (the shared empty-read rule,
KmerExtractor.cpp:451-494) are not in the set; the GPU tests cover that rule against the oracle.
"""
import pathlib
import re
import subprocess
import tempfile

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REF = pathlib.Path("/root/reference/src/commons")

from make_ref_functions import _block_end, definitions  # noqa: E402


def class_text(text: str, head: str) -> str:
    i = text.index(head)
    e = _block_end(text, text.index("{", i))
    assert text[e] == ";"
    return text[i:e + 1]


def program() -> str:
    ks = (REF / "KmerScanner.h").read_text()
    ss = (REF / "SyncmerScanner.h").read_text()
    cc = (REF / "common.cpp").read_text()
    lu = (REF / "LocalUtil.h").read_text()
    ke = (REF / "KmerExtractor.cpp").read_text()
    classes = [class_text(ks, "class KmerScanner {"), class_text(ks, "class MetamerScanner : public KmerScanner {"),
               class_text(ks, "class OldMetamerScanner : public MetamerScanner {"),
               class_text(ss, "class SyncmerScanner : public MetamerScanner {")]
    tables = [cc[m.start():cc.index(";", m.start()) + 1] for m in re.finditer(r"const std::string (atcg|iRCT) =", cc)]
    assert len(tables) == 2
    covered = definitions(lu, r"template\s*<typename T>\s*T LocalUtil::getMaxCoveredLength\(")
    fill = definitions(ke, r"void KmerExtractor::fillQueryKmerBuffer\(")
    assert len(covered) == 1 and len(fill) == 1
    return "\n".join([
        "#include <cstdint>", "#include <cstdio>", "#include <deque>", "#include <iostream>", "#include <string>",
        "#include <vector>", '#include "GeneticCode.h"',
        "typedef int TaxID;",
        "struct Kmer {",
        "  uint64_t value; uint32_t pos; uint32_t seqID; uint8_t frame;",
        "  Kmer() : value(0), pos(0), seqID(0), frame(0) {}",
        "  Kmer(uint64_t v, TaxID t) : value(v), pos((uint32_t)t), seqID(0), frame(0) {}",
        "  Kmer(uint64_t v, uint32_t p) : value(v), pos(p), seqID(0), frame(0) {}",
        "  Kmer(uint64_t v, uint32_t s, uint32_t p, uint8_t f) : value(v), pos(p), seqID(s), frame(f) {}",
        "};",
        *tables, *classes,
        "struct LocalUtil { template<typename T> static T getMaxCoveredLength(T queryLength); };", *covered,
        "template <typename T> struct Buffer { T *buffer; };",
        "struct KmerExtractor {",
        "  KmerScanner **kmerScanners;",
        "  void fillQueryKmerBuffer(const char *seq, int seqLen, Buffer<Kmer> &kmerBuffer, size_t &posToWrite,"
        " uint32_t seqID, uint32_t offset);",
        "};", *fill, DRIVER])


# stdin: "<kmerFormat> <syncmer> <smerLen> <nReads>", then per read "<len1> <len2>" and the mates' bases on
# their own lines (len2 = 0: single-end). stdout: per emitted k-mer "value seqID pos frame".
DRIVER = r"""
int main() {
  int fmt, syncmer, smerLen; long n;
  if (scanf("%d %d %d %ld", &fmt, &syncmer, &smerLen, &n) != 4) return 1;
  GeneticCode gc(false);
  KmerScanner *sc = fmt == 1 ? (KmerScanner *)new OldMetamerScanner(gc)
                  : syncmer ? (KmerScanner *)new SyncmerScanner(smerLen, gc) : (KmerScanner *)new MetamerScanner(gc);
  KmerExtractor ex; ex.kmerScanners = &sc;
  std::vector<Kmer> buf(1 << 22);
  Buffer<Kmer> kb{buf.data()};
  static char s1[1 << 20], s2[1 << 20];
  for (long i = 0; i < n; i++) {
    int l1, l2;
    if (scanf("%d %d", &l1, &l2) != 2) return 2;
    if (scanf("%s", s1) != 1) return 3;
    if (l2 && scanf("%s", s2) != 1) return 4;
    size_t pos = 0;
    ex.fillQueryKmerBuffer(s1, l1, kb, pos, (uint32_t)i + 1, 0);
    if (l2) ex.fillQueryKmerBuffer(s2, l2, kb, pos, (uint32_t)i + 1, (uint32_t)LocalUtil::getMaxCoveredLength(l1) + 3);
    for (size_t k = 0; k < pos; k++)
      printf("%llu %u %u %u\n", (unsigned long long)buf[k].value, buf[k].seqID, buf[k].pos, (unsigned)buf[k].frame);
  }
  return 0;
}
"""

CONFIGS = [("fmt2", 2, 0, 5), ("fmt1", 1, 0, 5), ("fmt2_syncmer5", 2, 1, 5), ("fmt2_syncmer6", 2, 1, 6)]


def reads(rng):
    """Paired 150-bp and single-end reads of every length residue mod 3, with N, IUPAC codes and
    lower case sprinkled in (atcg / iRCT map them), plus a few long reads."""
    alpha = np.frombuffer(b"ACGT", np.uint8)
    iupac = np.frombuffer(b"NRYKMSWBDHVUn", np.uint8)

    def one(L):
        s = alpha[rng.integers(0, 4, L)].copy()
        m = rng.random(L)
        s[m < 0.004] = iupac[rng.integers(0, len(iupac), int((m < 0.004).sum()))]
        low = (m > 0.995)
        s[low] = s[low] + 32 * ((s[low] >= 65) & (s[low] <= 90))
        return s.tobytes().decode()

    out = []
    for _ in range(60):
        out.append((one(150), one(150)))
    for L in list(range(27, 60)) + [100, 101, 102, 250, 251, 252]:
        out.append((one(L), ""))
    for L in (1200, 2501, 3002):
        out.append((one(L), ""))
    for _ in range(10):  # mates of unequal lengths
        out.append((one(int(rng.integers(40, 300))), one(int(rng.integers(40, 300)))))
    return out


if __name__ == "__main__":
    rng = np.random.default_rng(20261019)
    rs = reads(rng)
    arrays = {"seq1": np.array([a for a, _ in rs]), "seq2": np.array([b for _, b in rs])}
    with tempfile.TemporaryDirectory() as d:
        src = pathlib.Path(d) / "ref_scanners.cpp"
        exe = pathlib.Path(d) / "ref_scanners"
        src.write_text(program())
        subprocess.run(["g++", "-O1", "-std=c++17", f"-I{REF}", str(src), "-o", str(exe)], check=True)
        for name, fmt, syn, smer in CONFIGS:
            inp = [f"{fmt} {syn} {smer} {len(rs)}"]
            for a, b in rs:
                inp.append(f"{len(a)} {len(b)}")
                inp.append(a)
                if b:
                    inp.append(b)
            got = subprocess.run([str(exe)], input="\n".join(inp) + "\n", capture_output=True, text=True,
                                 check=True).stdout.split()
            v = np.array(got, dtype=np.uint64).reshape(-1, 4)
            arrays[f"{name}_value"] = v[:, 0]
            arrays[f"{name}_seq"] = v[:, 1].astype(np.uint32)
            arrays[f"{name}_pos"] = v[:, 2].astype(np.uint32)
            arrays[f"{name}_frame"] = v[:, 3].astype(np.uint8)
            print(name, len(v), "k-mers")
    np.savez_compressed(HERE / "ref_scanners.npz", **arrays)
    print("wrote", HERE / "ref_scanners.npz")
