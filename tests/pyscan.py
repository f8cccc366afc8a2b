"""Pure-Python closed-form restatement of the query scanners (small inputs only), independent of
the oracle's stateful C++ scanners: a window is emitted iff its 8 codons translate and (syncmer)
its earliest-minimum s-mer is at either end (KmerScanner.h:82-181, SyncmerScanner.h:36-102)."""
import json
import pathlib

_G = json.loads((pathlib.Path(__file__).resolve().parent / "golden" / "genetic_code.json").read_text())
AA = {(a, b, c): v for a, b, c, v in _G["nuc2aa"]}
NUM = {(a, b, c): v for a, b, c, v in _G["nuc2num"]}
ATCG = _G["atcg"]
IRCT = _G["iRCT"]


def code(ch):
    return (ch & 14) >> 1


def max_cov(n):
    return n - 2 if n % 3 == 2 else (n - 4 if n % 3 == 1 else n - 3)


def frame_windows(seq: bytes, frame: int, fmt: int, syncmer: int, smer: int):
    n = len(seq)
    used = max_cov(n)
    fwd = frame < 3
    begin = frame if fwd else ((n % 3) - (frame % 3)) % 3
    s, e = begin, begin + used - 1
    aalen = used // 3
    cods = []
    for j in range(aalen):
        if fmt == 2:
            if fwd:
                t = [ATCG[seq[s + 3 * j + k]] for k in range(3)]
            else:
                t = [IRCT[ATCG[seq[e - 3 * j - k]]] for k in range(3)]
        else:
            if fwd:
                t = [ATCG[seq[e - 3 * j - 2 + k]] for k in range(3)]
            else:
                t = [IRCT[ATCG[seq[s + 3 * j + 2 - k]]] for k in range(3)]
        key = tuple(code(x) for x in t)
        cods.append((AA[key], NUM[key]))
    out = []
    for p in range(aalen - 7):
        w = cods[p:p + 8]
        if any(a < 0 for a, _ in w):
            continue
        if syncmer:
            sm = []
            for q in range(8 - smer + 1):
                v = 0
                for a, _ in w[q:q + smer]:
                    v = (v << 5) | a
                sm.append(v)
            best = min(range(len(sm)), key=lambda i: (sm[i], i))
            if best not in (0, len(sm) - 1):
                continue
        dna = 0
        for _, c in w:
            dna = (dna << 3) | c
        if fmt == 2:
            aa = 0
            for a, _ in w:
                aa = (aa << 5) | a
        else:
            aa = 0
            for a, _ in w:
                aa = aa * 21 + a
        pos = s + 3 * p if (fwd == (fmt == 2)) else e - 3 * (p + 8) + 1
        out.append(((aa << 24) | dna, pos, frame))
    return out


def read_kmers(seq1: bytes, seq2, fmt, syncmer=0, smer=5):
    """(value, pos, frame) of both mates, mate-2 positions offset by queryLength+3; [] if either
    mate is shorter than one window (shared empty flag)."""
    mates = [seq1] + ([seq2] if seq2 is not None else [])
    if any(max_cov(len(m)) // 3 - 7 < 1 for m in mates):
        return []
    out = []
    for f in range(6):
        out += frame_windows(seq1, f, fmt, syncmer, smer)
    if seq2 is not None:
        off = max_cov(len(seq1)) + 3
        for f in range(6):
            out += [(v, p + off, fr) for v, p, fr in frame_windows(seq2, f, fmt, syncmer, smer)]
    return out
