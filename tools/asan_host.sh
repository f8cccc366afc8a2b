#!/bin/bash
# Host-code sanitizer pass (AddressSanitizer + UBSan, CPU only): the record split (scan_records /
# parse_records), the byte sources and the parallel gzip inflate, built from their sources with g++
# around tools/ingest_check.cpp and tools/gunzip_check.cpp (the C-ABI entry points the TSV formatter
# calls are stubbed: the checkers never format). Runs the test_ingest cases and the gzip edge cases.
set -e
cd "$(dirname "$0")/.."
T=${TMPDIR:-/tmp}/mtb_asan
mkdir -p $T
cat > $T/stubs.cpp <<'CPP'
#include <string>
#include "metabuli_work_amd/csrc/mtb_host.h"
namespace mtb {
void set_error(const std::string&) {}
const TaxText& tax_text(const mtb_ctx*) { static TaxText t; return t; }
}
extern "C" {
int32_t mtb_original_taxid(const mtb_ctx*, int32_t t) { return t; }
const char* mtb_taxon_rank(const mtb_ctx*, int32_t) { return "-"; }
const char* mtb_taxon_lineage(const mtb_ctx*, int32_t) { return "-"; }
}
CPP
F="-g -O1 -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I. -Imetabuli_work_amd/csrc"
S="metabuli_work_amd/csrc/mtb_io.cpp metabuli_work_amd/csrc/mtb_gunzip.cpp metabuli_work_amd/csrc/mtb_source.cpp"
g++ $F -o $T/ingest_check tools/ingest_check.cpp $S $T/stubs.cpp -lz -lpthread -ldl
g++ $F -o $T/gunzip_check tools/gunzip_check.cpp metabuli_work_amd/csrc/mtb_gunzip.cpp metabuli_work_amd/csrc/mtb_source.cpp -lz -lpthread -ldl
python3 - "$T" <<'PY'
import os, subprocess, sys, zlib
import numpy as np
sys.path.insert(0, os.getcwd())
from tests.test_ingest import CASES, _gz_cases, _fastq
T = sys.argv[1]
bad = 0
def run(args):
    global bad
    r = subprocess.run(args, capture_output=True, text=True)
    if r.returncode not in (0, 3) or "ERROR: AddressSanitizer" in r.stderr or "runtime error" in r.stderr:
        bad += 1
        print(" ".join(args), r.returncode, r.stderr[-1500:])
for case, fn in CASES.items():
    open(f"{T}/in.fq", "wb").write(fn(np.random.default_rng(7)).encode())
    for buf, recs in ((5, 8192), (97, 3), (1 << 20, 8192)):
        run([f"{T}/ingest_check", f"{T}/in.fq", str(buf), str(recs)])
b = _fastq(np.random.default_rng(11), 6000).encode()
for name, data in _gz_cases(b).items():
    open(f"{T}/{name}.gz", "wb").write(data)
    for chunk in (4096, 65536):
        run([f"{T}/gunzip_check", f"{T}/{name}.gz", "3", str(chunk), f"{T}/out"])
print("sanitizer findings:", bad)
sys.exit(1 if bad else 0)
PY
