"""mtb_stdsort.h (device emulation of libstdc++ std::sort) vs the host's libstdc++ std::sort on
non-total comparators: the permutations of tied elements must be identical."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]

SRC = r'''
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "mtb_stdsort.h"
struct P { float score; int hd; int start; int id; };
int main() {
    std::mt19937 rng(12345);
    long checked = 0;
    for (int trial = 0; trial < 4000; trial++) {
        int n = trial < 200 ? trial : (int)(rng() % (trial < 3000 ? 300 : 5000));
        int keyRange = 1 + (int)(rng() % 6);
        std::vector<P> a(n);
        for (int i = 0; i < n; i++) {
            a[i].score = 0.5f * (float)(rng() % keyRange);
            a[i].hd = (int)(rng() % 2);
            a[i].start = (int)(rng() % keyRange);
            a[i].id = i;
        }
        if (trial % 7 == 0) std::sort(a.begin(), a.end(), [](const P& x, const P& y) { return x.id > y.id; });
        auto comp = [](const P& x, const P& y) {
            if (x.score != y.score) return x.score > y.score;
            if (x.hd != y.hd) return x.hd < y.hd;
            return x.start > y.start;
        };
        std::vector<P> b = a;
        std::sort(a.begin(), a.end(), comp);
        mtb::stdsort::sort(b.data(), b.data() + n, comp);
        for (int i = 0; i < n; i++)
            if (a[i].id != b[i].id) { printf("MISMATCH trial %d n %d at %d\n", trial, n, i); return 1; }
        checked += n;
    }
    // depth-limit (heapsort) path: many equal keys with an ordering that defeats median-of-3
    for (int n : {1000, 4096, 20000}) {
        std::vector<P> a(n);
        for (int i = 0; i < n; i++) { a[i].score = (float)((i % 2) ? i : n - i); a[i].hd = 0; a[i].start = i % 3; a[i].id = i; }
        auto comp = [](const P& x, const P& y) { return x.score < y.score; };
        std::vector<P> b = a;
        std::sort(a.begin(), a.end(), comp);
        mtb::stdsort::sort(b.data(), b.data() + n, comp);
        for (int i = 0; i < n; i++) if (a[i].id != b[i].id) { printf("MISMATCH adversarial n %d\n", n); return 1; }
    }
    printf("OK %ld\n", checked);
    return 0;
}
'''


def test_stdsort_emulation_matches_libstdcxx(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(SRC)
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'metabuli_work_amd' / 'csrc'}", str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert out.stdout.startswith("OK")
