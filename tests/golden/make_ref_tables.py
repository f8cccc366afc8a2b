"""Regenerate tests/golden/hamming_tables.json from the reference's own text.

Runs in this container only (it reads /root/reference, which the GPU box does not have); the
committed JSON is what the tests read.

* `hammingLookup[8][8]` and `HAMMING_LUT0..7[64]` are parsed out of
  /root/reference/src/commons/KmerMatcher.h:66-158 (the numbers only, comments stripped).
* `GET_3_BITS` (the codon extraction every Hamming function applies, KmerMatcher.h:348-416) comes
  from oracle/_ref/refbits, which `make -C oracle ref` compiles against the reference's own
  BitManipulateMacros.h where it lies.
* Golden vectors: for a fixed set of (query, target) DNA parts — every codon pair at every one of
  the 8 codon positions, plus seeded random pairs — the sum, forward and reverse Hamming words the
  reference's getHammingDistanceSum / getHammings / getHammings_reverse compute, evaluated here
  literally as those functions are written (table lookups at GET_3_BITS(x >> 3i)).
"""
import json
import pathlib
import random
import re
import subprocess

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]
REF = pathlib.Path("/root/reference/src/commons/KmerMatcher.h")


def _numbers(block: str):
    block = re.sub(r"/\*.*?\*/", " ", block, flags=re.S)
    block = re.sub(r"//[^\n]*", " ", block)
    return [int(x) for x in re.findall(r"\d+", block)]


def parse_tables(text: str):
    m = re.search(r"uint8_t\s+hammingLookup\s*\[8\]\s*\[8\]\s*=\s*\{(.*?)\};", text, re.S)
    look = _numbers(m.group(1))
    assert len(look) == 64, len(look)
    luts = []
    for k in range(8):
        m = re.search(r"HAMMING_LUT%d\s*\[64\]\s*=\s*\{(.*?)\};" % k, text, re.S)
        v = _numbers(m.group(1))
        assert len(v) == 64, (k, len(v))
        luts.append(v)
    return [look[8 * i:8 * i + 8] for i in range(8)], luts


def ref_sum(look, get3, a, b):  # KmerMatcher.h:348-360
    return sum(look[get3[(a >> (3 * i)) & 511]][get3[(b >> (3 * i)) & 511]] for i in range(8))


def ref_hammings(luts, get3, a, b, reverse):  # KmerMatcher.h:386-416
    h = 0
    for i in range(8):
        lut = luts[7 - i] if reverse else luts[i]
        h |= lut[get3[(a >> (3 * i)) & 511] << 3 | get3[(b >> (3 * i)) & 511]]
    return h


if __name__ == "__main__":
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True)
    bits = json.loads(subprocess.run([str(ROOT / "oracle" / "_ref" / "refbits")], check=True, capture_output=True,
                                     text=True).stdout)
    look, luts = parse_tables(REF.read_text())
    get3 = bits["get3"]
    pairs = []
    for pos in range(8):  # every codon pair at every position, the other codons equal (0..7 cycling)
        for q in range(8):
            for t in range(8):
                base = sum(((pos + j) % 8) << (3 * j) for j in range(8))
                a = (base & ~(7 << (3 * pos))) | q << (3 * pos)
                b = (base & ~(7 << (3 * pos))) | t << (3 * pos)
                pairs.append((a, b))
    rng = random.Random(20261018)
    for _ in range(2048):  # random 24-bit DNA parts (high bits set too: only the low 24 are read)
        pairs.append((rng.getrandbits(64), rng.getrandbits(64)))
    vec = {"a": [str(a) for a, _ in pairs], "b": [str(b) for _, b in pairs],
           "sum": [ref_sum(look, get3, a, b) for a, b in pairs],
           "fwd": [ref_hammings(luts, get3, a, b, False) for a, b in pairs],
           "rev": [ref_hammings(luts, get3, a, b, True) for a, b in pairs]}
    out = {"source": "KmerMatcher.h:66-158 (tables), BitManipulateMacros.h compiled in place (GET_3_BITS)",
           "hammingLookup": look, "HAMMING_LUT": luts, "GET_3_BITS": get3, "GET_2_BITS": bits["get2"],
           "vectors": vec}
    (HERE / "hamming_tables.json").write_text(json.dumps(out, separators=(",", ":")) + "\n")
    print("wrote", HERE / "hamming_tables.json", len(pairs), "pairs")
