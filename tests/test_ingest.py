"""Host ingest on the CPU:
* the pipeline's parallel record split (scan_records + parse_records, mtb_pipeline.cpp MateReader)
  against the serial record reader (next_record, kseq semantics, KmerExtractor.cpp:442-494): the
  same records, names and errors for wrapped / CRLF / blank-line / truncated inputs, cut at raw
  buffer sizes down to a few bytes so records straddle buffer ends (tools/ingest_check.cpp);
* the parallel gzip inflate (mtb_gunzip.cpp) against Python's zlib and the one-thread zlib source,
  byte for byte: compression levels 0/1/9, several members, empty members, trailing garbage,
  truncation anywhere, CRC-32 / ISIZE errors, chunks down to 4 KB (tools/gunzip_check.cpp)."""
import os
import pathlib
import subprocess

import numpy as np
import pytest

from metabuli_work_amd import synth

ROOT = pathlib.Path(__file__).resolve().parents[1]
LIB = ROOT / "metabuli_work_amd"


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if not (LIB / "libmtbgpu.so").exists():
        pytest.skip("libmtbgpu.so not built")
    exe = tmp_path_factory.mktemp("ingest") / "ingest_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), str(ROOT / "tools" / "ingest_check.cpp"),
                    f"-L{LIB}", "-lmtbgpu", f"-Wl,-rpath,{LIB}"], check=True, capture_output=True)
    return exe


@pytest.fixture(scope="module")
def gunzip(tmp_path_factory):
    if not (LIB / "libmtbgpu.so").exists():
        pytest.skip("libmtbgpu.so not built")
    exe = tmp_path_factory.mktemp("gunzip") / "gunzip_check"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe), str(ROOT / "tools" / "gunzip_check.cpp"),
                    f"-L{LIB}", "-lmtbgpu", f"-Wl,-rpath,{LIB}"], check=True, capture_output=True)
    return exe


def _run(exe, path, buf, recs=8192, env=None):
    r = subprocess.run([str(exe), str(path), str(buf), str(recs)], capture_output=True, text=True, timeout=120,
                       env=None if env is None else {**os.environ, **env})
    return r.returncode, r.stdout.strip()


def _fastq(rng, n, wrap=0, crlf=False, qual_at=False):
    nl = "\r\n" if crlf else "\n"
    out = []
    for i in range(n):
        L = int(rng.integers(0, 60))
        s = "".join(rng.choice(list("ACGTN"), L)) if L else ""
        q = "".join(rng.choice(list("@+!#IJ"), L)) if L else ""
        if qual_at and L:
            q = "@" + q[1:]
        head = f"@r{i} extra words{nl}"
        if wrap and L:
            sl = nl.join(s[k:k + wrap] for k in range(0, L, wrap))
            ql = nl.join(q[k:k + wrap] for k in range(0, L, wrap))
        else:
            sl, ql = s, q
        out.append(f"{head}{sl}{nl}+{nl}{ql}{nl}")
    return "".join(out)


def _fasta(rng, n, wrap=13, blanks=True):
    out = []
    for i in range(n):
        L = int(rng.integers(1, 80))
        s = "".join(rng.choice(list("ACGTacgtN"), L))
        out.append(f">s{i}\tdesc\n" + "\n".join(s[k:k + wrap] for k in range(0, L, wrap)) + "\n")
        if blanks and i % 3 == 0:
            out.append("\n\n")
    return "".join(out)


CASES = {
    "fastq": lambda rng: _fastq(rng, 300),
    "fastq_wrapped": lambda rng: _fastq(rng, 200, wrap=7),
    "fastq_crlf": lambda rng: _fastq(rng, 200, crlf=True),
    "fastq_qual_at": lambda rng: _fastq(rng, 200, qual_at=True),
    "fasta": lambda rng: _fasta(rng, 300),
    "fasta_no_final_newline": lambda rng: _fasta(rng, 50, blanks=False).rstrip("\n"),
    "fastq_no_final_newline": lambda rng: _fastq(rng, 50).rstrip("\n"),
    "leading_blank_lines": lambda rng: "\n\r\n\n" + _fastq(rng, 20) + "\n\n",
}


@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("buf,recs", [(5, 8192), (97, 3), (4096, 1), (1 << 20, 8192)])
def test_split_matches_serial(checker, tmp_path, case, buf, recs):
    rng = np.random.default_rng(len(case) * 131 + buf)
    p = tmp_path / "in.fq"
    p.write_bytes(CASES[case](rng).encode())
    rc, out = _run(checker, p, buf, recs)
    assert rc == 0 and "same=1" in out, out
    assert "records=0 " not in out


@pytest.mark.parametrize("mode,env", [("gzip", None), ("bgzf", None), ("bgzf", {"MTB_NO_LIBDEFLATE": "1"})])
def test_split_compressed(checker, tmp_path, mode, env):
    """BGZF members inflate through libdeflate when it loads, through zlib otherwise: both read the same."""
    rng = np.random.default_rng(5)
    p = tmp_path / "in.fq.gz"
    synth.write_compressed(str(p), _fastq(rng, 3000, wrap=11).encode(), mode)
    rc, out = _run(checker, p, 1000, 17, env)
    assert rc == 0 and "same=1" in out and "records=3000 " in out, out


@pytest.mark.parametrize("text,msg", [
    ("@r1\nACGT\n+\nIIII\n@r2\nACGT\n", "truncated FASTQ record"),
    ("@r1\nACGT\n+\nIIII\n@r2\nACGT\n+\nII\n", "truncated FASTQ record"),
    ("@r1\nACGT\n+\nIIII\nxr2\nACGT\n+\nIIII\n", "not a FASTA/FASTQ record header"),
])
@pytest.mark.parametrize("buf", [3, 1 << 16])
def test_split_errors_match(checker, tmp_path, text, msg, buf):
    p = tmp_path / "bad.fq"
    p.write_bytes(text.encode())
    rc, out = _run(checker, p, buf, 1)
    assert rc == 0 and "same=1" in out and f'err="{msg}"' in out, out


def _gz(data, level=6):
    import zlib
    c = zlib.compressobj(level, zlib.DEFLATED, 31)
    return c.compress(data) + c.flush()


@pytest.fixture(scope="module")
def fastq_bytes():
    rng = np.random.default_rng(11)
    return _fastq(rng, 6000, wrap=0).encode() + _fastq(rng, 2000, wrap=9).encode()


def _gz_cases(b):
    g = _gz(b, 1)
    bad_crc, bad_len = bytearray(g), bytearray(g)
    bad_crc[-6] ^= 1
    bad_len[-2] ^= 1
    empty = _gz(b"")
    third = len(b) // 3
    return {
        "level0": _gz(b, 0), "level1": g, "level9": _gz(b, 9),
        "members": _gz(b[:third], 1) + _gz(b[third:2 * third], 9) + _gz(b[2 * third:], 6),
        "empty_members": empty + g + empty + empty,
        "garbage_after": g + b"\x00\x01 not gzip",
        "truncated_mid": g[:len(g) // 2 + 777],
        "truncated_trailer": g[:-3],
        "truncated_at_trailer": g[:-8],
        "bad_crc": bytes(bad_crc), "bad_isize": bytes(bad_len),
    }


@pytest.mark.parametrize("chunk,threads", [(4096, 3), (65536, 2), (1 << 20, 4)])
def test_parallel_gunzip_matches_zlib(gunzip, tmp_path, fastq_bytes, chunk, threads):
    import zlib
    for name, data in _gz_cases(fastq_bytes).items():
        p = tmp_path / f"{name}.gz"
        p.write_bytes(data)
        got = {}
        for mode in ("par", "ser"):
            out = tmp_path / f"{name}.{mode}"
            env = dict(os.environ, SERIAL="1") if mode == "ser" else None
            r = subprocess.run([str(gunzip), str(p), str(threads), str(chunk), str(out)], capture_output=True,
                               text=True, timeout=120, env=env)
            got[mode] = (r.stdout.strip(), out.read_bytes())
        assert got["par"] == got["ser"], (name, got["par"][0], got["ser"][0])
        if name.startswith("bad"):
            assert "rc=-1" in got["par"][0] and "check" in got["par"][0], (name, got["par"][0])
        elif not name.startswith("truncated"):
            d = zlib.decompressobj(31)
            want, rest = b"", data
            while rest[:2] == b"\x1f\x8b":  # members in sequence, as gzip.decompress (without its garbage check)
                d = zlib.decompressobj(31)
                want += d.decompress(rest)
                rest = d.unused_data
            assert got["par"][1] == want, name
