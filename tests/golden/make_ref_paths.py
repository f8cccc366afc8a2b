"""Regenerate tests/golden/ref_paths.npz: what the reference's OWN combineMatchPaths computes for fixed
sets of match paths (round 6). combineMatchPaths (Taxonomer.cpp:410-468) sorts one species' paths with
std::sort on a comparator that leaves ties (equal score, hamming distance and start) in the order
libstdc++'s introsort leaves them, then keeps them greedily, trimming overlaps under 24 bases
(trimMatchPath, :475-485, through Match's partial scores, Match.h:46-86). The device's K6 emulates
that std::sort (mtb_stdsort.h); the oracle calls it.

Runs in this container only; as in make_ref_functions.py the code is cut out of /root/reference at
run time into a throw-away C++ file next to minimal declarations (a `Match` with the fields MatchPath
and the partial scores read, a `Taxonomer` declaring the three members), compiled with
BitManipulateMacros.h in place, run and deleted. The cut code: `struct MatchPath`
(Taxonomer.h:35-59), Match's score methods (Match.h:32-86), `Taxonomer::combineMatchPaths`,
`isMatchPathOverlapped` and `trimMatchPath` (Taxonomer.cpp:410-485). The runs are tie-heavy: scores
on a coarse grid of multiples of 0.5, few hamming distances, starts on a few codon positions.
"""
import pathlib
import struct
import subprocess
import tempfile

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REF = pathlib.Path("/root/reference/src/commons")

from make_ref_functions import definitions  # noqa: E402
from make_ref_scanners import class_text  # noqa: E402


def program() -> str:
    th = (REF / "Taxonomer.h").read_text()
    tx = (REF / "Taxonomer.cpp").read_text()
    mh = (REF / "Match.h").read_text()
    mp = class_text(th, "struct MatchPath {")
    m_struct = mh[mh.index("struct Match {"):]
    m_defs = []
    for h in (r"float getScore\(", r"virtual float getRightPartScore\(", r"virtual float getLeftPartScore\(",
              r"virtual int getRightPartHammingDist\(", r"virtual int getLeftPartHammingDist\("):
        m_defs.append(definitions(m_struct, h)[0])
    defs = (definitions(tx, r"float Taxonomer::combineMatchPaths\(") +
            definitions(tx, r"bool Taxonomer::isMatchPathOverlapped\(") +
            definitions(tx, r"void Taxonomer::trimMatchPath\("))
    assert len(defs) == 3
    return "\n".join([
        "#include <algorithm>", "#include <cstdint>", "#include <cstdio>", "#include <cstring>", "#include <iostream>",
        "#include <vector>", '#include "BitManipulateMacros.h"', "using namespace std;",
        "struct QInfo { uint32_t pos; };",
        "struct Match {", "  QInfo qInfo{}; uint16_t rightEndHamming = 0; uint8_t hamming = 0;", *m_defs, "};",
        mp,
        "struct Taxonomer {",
        "  float combineMatchPaths(vector<MatchPath> &matchPaths, size_t matchPathStart,"
        " vector<MatchPath> &combinedMatchPaths, size_t combMatchPathStart, int readLength);",
        "  bool isMatchPathOverlapped(const MatchPath &matchPath1, const MatchPath &matchPath2);",
        "  void trimMatchPath(MatchPath &path1, const MatchPath &path2, int overlapLength);",
        "};", *defs, DRIVER])


# stdin: per run "<readLength> <n>" then n lines "start end scoreBits hd rehStart rehEnd";
# stdout: per run "scoreBits k" then k lines "start end hd scoreBits"
DRIVER = r"""
static unsigned fb(float f) { unsigned u; memcpy(&u, &f, 4); return u; }
int main() {
  int L; size_t n;
  Taxonomer t;
  while (scanf("%d %zu", &L, &n) == 2) {
    vector<Match> ms(2 * n);
    vector<MatchPath> paths;
    for (size_t i = 0; i < n; i++) {
      int s, e, hd; unsigned sb, r0, r1; float sc;
      if (scanf("%d %d %u %d %u %u", &s, &e, &sb, &hd, &r0, &r1) != 6) return 2;
      memcpy(&sc, &sb, 4);
      ms[2 * i].rightEndHamming = (uint16_t)r0; ms[2 * i + 1].rightEndHamming = (uint16_t)r1;
      paths.emplace_back(s, e, sc, hd, 1, &ms[2 * i], &ms[2 * i + 1]);
    }
    vector<MatchPath> comb;
    float score = t.combineMatchPaths(paths, 0, comb, 0, L);
    printf("%u %zu\n", fb(score), comb.size());
    for (auto &p : comb) printf("%d %d %d %u\n", p.start, p.end, p.hammingDist, fb(p.score));
  }
  return 0;
}
"""


def runs(rng, n_runs=3000):
    out = []
    for _ in range(n_runs):
        n = int(rng.choice([1, 2, 3, 5, 8, 16, 17, 30, 64, 65]))
        L = int(rng.choice([147, 294, 300, 2000]))
        starts = rng.integers(0, 8, n) * 3 * int(rng.choice([1, 4, 12]))
        lens = 24 + 3 * rng.integers(0, int(rng.choice([1, 3, 12])), n)
        scores = 0.5 * rng.integers(40, 48 if rng.random() < 0.7 else 200, n)  # coarse: many ties
        hd = rng.integers(0, 2 if rng.random() < 0.7 else 6, n)
        r0 = rng.integers(0, 1 << 16, n)
        r1 = rng.integers(0, 1 << 16, n)
        out.append((L, [(int(s), int(s + ln - 1), float(sc), int(h), int(a), int(b))
                        for s, ln, sc, h, a, b in zip(starts, lens, scores, hd, r0, r1)]))
    return out


def fbits(x: float) -> int:
    return struct.unpack("<I", struct.pack("<f", x))[0]


if __name__ == "__main__":
    rng = np.random.default_rng(20261021)
    rs = runs(rng)
    lines = []
    for L, ps in rs:
        lines.append(f"{L} {len(ps)}")
        lines += [f"{s} {e} {fbits(sc)} {h} {a} {b}" for s, e, sc, h, a, b in ps]
    with tempfile.TemporaryDirectory() as d:
        src = pathlib.Path(d) / "ref_paths.cpp"
        exe = pathlib.Path(d) / "ref_paths"
        src.write_text(program())
        subprocess.run(["g++", "-O1", "-std=c++17", f"-I{REF}", str(src), "-o", str(exe)], check=True)
        got = subprocess.run([str(exe)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                             check=True).stdout.split("\n")
    it = iter(got)
    run_len, run_rl, paths, score, comb_len, comb = [], [], [], [], [], []
    for L, ps in rs:
        sb, k = (int(x) for x in next(it).split())
        run_len.append(len(ps))
        run_rl.append(L)
        paths += [(s, e, fbits(sc), h, a, b) for s, e, sc, h, a, b in ps]
        score.append(sb)
        comb_len.append(k)
        comb += [tuple(int(x) for x in next(it).split()) for _ in range(k)]
    np.savez_compressed(HERE / "ref_paths.npz", run_len=np.array(run_len, np.int32),
                        read_len=np.array(run_rl, np.int32), paths=np.array(paths, np.int64),
                        score_bits=np.array(score, np.uint32), comb_len=np.array(comb_len, np.int32),
                        comb=np.array(comb, np.int64))
    print("wrote", HERE / "ref_paths.npz", len(rs), "runs,", len(paths), "paths,", len(comb), "kept")
