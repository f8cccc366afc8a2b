"""Regenerate tests/golden/ref_functions.json: golden vectors of the dependency-free helper functions on
the classify path, computed by the reference's OWN function bodies.

Runs in this container only (it reads /root/reference, which the GPU box does not have); the committed
JSON is what the tests read. Nothing of the reference is copied into the repository: the function
definitions are cut out of the reference's files at run time (the text between each definition's
signature and its closing brace, as written), pasted into a throw-away C++ file in a temporary
directory next to minimal declarations of their classes (only the fields the bodies read), compiled
with g++ against the reference's own BitManipulateMacros.h where it lies (-I src/commons), run on the
vectors below and deleted. No MMseqs2 stand-ins are involved: none of these bodies needs one.

Functions (reference file:line):
* KmerMatcher::getNextTargetKmer, the index form classify's matchKmers calls (KmerMatcher.h:282-297;
  call sites KmerMatcher.cpp:269,368,403), and the pointer form (:299-314) as a cross-check
* Taxonomer::calScoreIncrement / calHammingDistIncrement (Taxonomer.cpp:650-669)
* Taxonomer::isConsecutive / isConsecutive2, with and without a shift (Taxonomer.cpp:671-699)
* the Taxonomer constructor's shape parameters: dnaShift / maxCodonShift / smerLength,
  denominator, bitsPerCodon / totalDnaBits / lastCodonMask (Taxonomer.cpp:34-58)
* LocalUtil::getQueryKmerNumber / getMaxCoveredLength (LocalUtil.h:45-59), T = int as every classify
  caller instantiates them (KmerExtractor.cpp:363,454-481; QueryIndexer.cpp:56,101,116)
* Match::getScore / getRightPartScore / getLeftPartScore / getRightPartHammingDist /
  getLeftPartHammingDist (Match.h:32-86)
"""
import json
import pathlib
import random
import re
import subprocess
import tempfile

HERE = pathlib.Path(__file__).resolve().parent
REF = pathlib.Path("/root/reference/src/commons")


def _block_end(text: str, open_brace: int) -> int:
    """Index just past the brace that closes the one at open_brace (no braces in strings here)."""
    depth = 0
    for i in range(open_brace, len(text)):
        if text[i] == "{":
            depth += 1
        elif text[i] == "}":
            depth -= 1
            if depth == 0:
                return i + 1
    raise ValueError("unbalanced braces")


def definitions(text: str, head: str):
    """Every definition whose signature starts with `head` (a regex), signature through body."""
    out = []
    for m in re.finditer(head, text):
        ob = text.index("{", m.end())
        out.append(text[m.start():_block_end(text, ob)])
    return out


def if_else(text: str, cond: str) -> str:
    """`if (<cond>) {...} else {...}` as written."""
    i = text.index(f"if ({cond})")
    e1 = _block_end(text, text.index("{", i))
    m = re.compile(r"\s*else\s*").match(text, e1)
    return text[i:_block_end(text, text.index("{", m.end()))]


def program() -> str:
    km = (REF / "KmerMatcher.h").read_text()
    tx = (REF / "Taxonomer.cpp").read_text()
    lu = (REF / "LocalUtil.h").read_text()
    mh = (REF / "Match.h").read_text()
    next_idx = [d for d in definitions(km, r"inline uint64_t KmerMatcher::getNextTargetKmer\(")
                if "diffBufferIdx" in d and "totalPos" in d]
    next_ptr = [d for d in definitions(km, r"inline uint64_t KmerMatcher::getNextTargetKmer\(")
                if "*&diffIdxBuffer" in d and "totalPos" in d]
    assert len(next_idx) == 1 and len(next_ptr) == 1
    tax_defs = (definitions(tx, r"float Taxonomer::calScoreIncrement\(") +
                definitions(tx, r"int Taxonomer::calHammingDistIncrement\(") +
                definitions(tx, r"bool Taxonomer::isConsecutive\(") +
                definitions(tx, r"bool Taxonomer::isConsecutive2\("))
    assert len(tax_defs) == 6, len(tax_defs)
    shape = "\n".join(if_else(tx, c) for c in ("par.syncmer", "par.seqMode == 1 || par.seqMode == 2",
                                                "par.reducedAA == 1"))
    lu_defs = definitions(lu, r"template\s*<typename T>\s*T LocalUtil::get(QueryKmerNumber|MaxCoveredLength)\(")
    assert len(lu_defs) == 2
    m_struct = mh[mh.index("struct Match {"):]
    m_defs = []
    for h in (r"float getScore\(", r"virtual float getRightPartScore\(", r"virtual float getLeftPartScore\(",
              r"virtual int getRightPartHammingDist\(", r"virtual int getLeftPartHammingDist\("):
        d = definitions(m_struct, h)
        assert d, h
        m_defs.append(d[0])
    return "\n".join([
        "#include <cstdint>", "#include <cstddef>", "#include <cstdio>", "#include <cstring>",
        '#include "BitManipulateMacros.h"',
        "struct Match {", "  uint32_t dnaEncoding = 0;", "  uint16_t rightEndHamming = 0;", *m_defs, "};",
        "struct KmerMatcher {",
        "  static uint64_t getNextTargetKmer(uint64_t lookingTarget, const uint16_t *diffIdxBuffer,"
        " size_t &diffBufferIdx, size_t &totalPos);",
        "  static uint64_t getNextTargetKmer(uint64_t lookingTarget, uint16_t *&diffIdxBuffer, size_t &totalPos);",
        "};", next_idx[0], next_ptr[0],
        "struct Par { int syncmer, smerLen, seqMode, reducedAA; };",
        "struct Taxonomer {",
        "  int dnaShift = 0, maxCodonShift = 0, smerLength = 0, denominator = 0, bitsPerCodon = 0, totalDnaBits = 0;",
        "  uint32_t lastCodonMask = 0;",
        "  void shape(const Par &par) {", shape, "  }",
        "  float calScoreIncrement(uint16_t hammings, int shift);",
        "  int calHammingDistIncrement(uint16_t hammings, int shift);",
        "  bool isConsecutive(const Match *match1, const Match *match2);",
        "  bool isConsecutive(const Match *match1, const Match *match2, int shift);",
        "  bool isConsecutive2(const Match *match1, const Match *match2);",
        "  bool isConsecutive2(const Match *match1, const Match *match2, int shift);",
        "};", *tax_defs,
        "struct LocalUtil {",
        "  template<typename T> static T getQueryKmerNumber(T queryLength, int spaceNum, int kLength = 8);",
        "  template<typename T> static T getMaxCoveredLength(T queryLength);",
        "};", *lu_defs,
        DRIVER])


# Reads "<fn> <param> <a> <b>" lines, prints one result per line (floats as their bit pattern).
DRIVER = r"""
static unsigned fbits(float f) { unsigned u; memcpy(&u, &f, 4); return u; }
int main() {
  char fn[32]; long long param; unsigned long long a, b;
  Taxonomer t; Par p{0, 5, 2, 0}; t.shape(p);
  static uint16_t words[1 << 20]; size_t nw = 0;
  while (scanf("%31s %lld %llu %llu", fn, &param, &a, &b) == 4) {
    Match m1, m2; m1.dnaEncoding = (uint32_t)a; m2.dnaEncoding = (uint32_t)b;
    m1.rightEndHamming = (uint16_t)a;
    if (!strcmp(fn, "score_inc")) printf("%u\n", fbits(t.calScoreIncrement((uint16_t)a, (int)param)));
    else if (!strcmp(fn, "ham_inc")) printf("%d\n", t.calHammingDistIncrement((uint16_t)a, (int)param));
    else if (!strcmp(fn, "cons")) printf("%d\n", param ? t.isConsecutive(&m1, &m2, (int)param) : t.isConsecutive(&m1, &m2));
    else if (!strcmp(fn, "cons2")) printf("%d\n", param ? t.isConsecutive2(&m1, &m2, (int)param) : t.isConsecutive2(&m1, &m2));
    else if (!strcmp(fn, "score")) printf("%u\n", fbits(m1.getScore()));
    else if (!strcmp(fn, "right_score")) printf("%u\n", fbits(m1.getRightPartScore((int)param)));
    else if (!strcmp(fn, "left_score")) printf("%u\n", fbits(m1.getLeftPartScore((int)param)));
    else if (!strcmp(fn, "right_ham")) printf("%d\n", m1.getRightPartHammingDist((int)param));
    else if (!strcmp(fn, "left_ham")) printf("%d\n", m1.getLeftPartHammingDist((int)param));
    else if (!strcmp(fn, "covered")) printf("%d\n", LocalUtil::getMaxCoveredLength<int>((int)a));
    else if (!strcmp(fn, "kmer_num")) printf("%d\n", LocalUtil::getQueryKmerNumber<int>((int)a, (int)param));
    else if (!strcmp(fn, "word")) words[nw++] = (uint16_t)a;
    else if (!strcmp(fn, "decode")) {  // the words so far: every value, both overloads, and totalPos
      size_t idx = 0, pos = 0, pos2 = 0; uint64_t v = 0, v2 = 0; uint16_t *ptr = words;
      printf("%zu", nw);
      while (idx < nw) {
        v = KmerMatcher::getNextTargetKmer(v, words, idx, pos);
        v2 = KmerMatcher::getNextTargetKmer(v2, ptr, pos2);
        printf(" %llu", (unsigned long long)v);
        if (v != v2 || pos != pos2 || pos != idx || ptr != words + idx) { printf(" MISMATCH"); break; }
      }
      printf("\n");
    } else if (!strcmp(fn, "shape")) {
      Taxonomer s; Par q{(int)(a >> 16), (int)(a & 0xFF), (int)b, (int)param}; s.shape(q);
      printf("%d %d %d %d %d %d %u\n", s.dnaShift, s.maxCodonShift, s.smerLength, s.denominator, s.bitsPerCodon,
             s.totalDnaBits, s.lastCodonMask);
    } else { printf("?\n"); }
  }
  return 0;
}
"""


def encode_delta(d: int):
    """A delta as diffIdx words: 15-bit groups, most significant first, bit 15 on the last
    (IndexCreator.cpp:868-886)."""
    groups = []
    while True:
        groups.append(d & 0x7FFF)
        d >>= 15
        if not d:
            break
    groups.reverse()
    groups[-1] |= 0x8000
    return groups


def vectors(rng):
    v = {}
    hams = list(range(256)) + [rng.getrandbits(16) for _ in range(1024)] + [0xFFFF, 0xAAAA, 0x5555]
    v["score_inc"] = v["ham_inc"] = [(s, h, 0) for h in hams for s in range(0, 9)]
    pairs = []
    for _ in range(3000):
        sh = rng.randrange(0, 8)
        a = rng.getrandbits(32) if rng.random() < 0.2 else rng.getrandbits(24)
        k = 3 * max(sh, 1)
        if rng.random() < 0.5:  # consecutive by construction, for isConsecutive2 or isConsecutive
            lo = (1 << (24 - k)) - 1
            b = (((a & lo) << k) | rng.getrandbits(k)) if rng.random() < 0.5 else \
                (((a >> k) & lo) | (rng.getrandbits(k) << (24 - k)))
        else:
            b = rng.getrandbits(24)
        pairs.append((sh, a, b))
    v["cons"] = v["cons2"] = pairs
    rehs = list(range(256)) + [rng.getrandbits(16) for _ in range(768)] + [0xFFFF]
    v["score"] = [(0, h, 0) for h in rehs]
    for fn in ("right_score", "left_score", "right_ham", "left_ham"):
        v[fn] = [(r, h, 0) for h in rehs for r in range(0, 9)]
    lens = list(range(0, 3001)) + [rng.randrange(3001, 1 << 22) for _ in range(1000)]
    v["covered"] = [(0, L, 0) for L in lens]
    v["kmer_num"] = [(0, L, 0) for L in lens] + [(s, L, 0) for L in lens[:400:7] for s in (1, 2)]
    # (reducedAA, syncmer << 16 | smerLen, seqMode)
    v["shape"] = [(0, (syn << 16) | smer, mode) for syn in (0, 1) for smer in (4, 5, 6, 7) for mode in (1, 2, 3)]
    return v


def deltas(rng, n=6000):
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.1:
            out.append(0)  # the same value again (another species): a lone 0x8000
        elif r < 0.6:
            out.append(rng.getrandbits(rng.randrange(1, 16)))   # one group
        elif r < 0.9:
            out.append(rng.getrandbits(rng.randrange(16, 31)))  # two groups
        else:
            out.append(rng.getrandbits(rng.randrange(31, 46)))  # three groups
    # a few of four and five groups (a sparse DB's first k-mers)
    out += [(1 << 45) + rng.getrandbits(44), (1 << 59) + 12345, 1 << 60]
    return out


if __name__ == "__main__":
    rng = random.Random(20261019)
    vec = vectors(rng)
    ds = deltas(rng)
    words = [w for d in ds for w in encode_delta(d)]
    lines = []
    order = []
    for fn, rows in vec.items():
        for p, a, b in rows:
            lines.append(f"{fn} {p} {a} {b}")
            order.append(fn)
    lines += [f"word 0 {w} 0" for w in words] + ["decode 0 0 0"]
    with tempfile.TemporaryDirectory() as d:
        src = pathlib.Path(d) / "ref_functions.cpp"
        exe = pathlib.Path(d) / "ref_functions"
        src.write_text(program())
        subprocess.run(["g++", "-O1", "-std=c++17", f"-I{REF}", str(src), "-o", str(exe)], check=True)
        got = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.splitlines()
    assert len(got) == len(order) + 1, (len(got), len(order))
    res = {fn: [] for fn in vec}
    for fn, g in zip(order, got):
        res[fn].append([int(x) for x in g.split()] if fn == "shape" else int(g))
    dec = got[-1].split()
    assert "MISMATCH" not in dec and int(dec[0]) == len(words)
    values = [int(x) for x in dec[1:]]
    assert len(values) == len(ds)
    out = {"source": "function bodies cut from /root/reference/src/commons {KmerMatcher.h:282-314, "
                     "Taxonomer.cpp:34-58,650-699, LocalUtil.h:45-59, Match.h:32-86} at generation time, compiled "
                     "with the reference's BitManipulateMacros.h in place (tests/golden/make_ref_functions.py)",
           "functions": {fn: {"param": [p for p, _, _ in vec[fn]], "a": [str(a) for _, a, _ in vec[fn]],
                              "b": [str(b) for _, _, b in vec[fn]], "out": res[fn]} for fn in vec},
           "decode": {"words": words, "values": [str(x) for x in values]}}
    (HERE / "ref_functions.json").write_text(json.dumps(out, separators=(",", ":")) + "\n")
    print("wrote", HERE / "ref_functions.json", sum(len(r) for r in vec.values()), "cases,", len(words), "words")
