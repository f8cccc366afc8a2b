// Parallel gzip inflate check (tests/test_ingest.py): decompresses FILE with the parallel source
// (open_parallel_gzip: THREADS workers, CHUNK compressed bytes per chunk) or, with SERIAL set, with
// the one-thread zlib source, and writes the bytes to OUT.
//   gunzip_check FILE THREADS CHUNK OUT
// prints: bytes=N rc=R err="..."
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../metabuli_work_amd/csrc/mtb_io.h"

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: gunzip_check FILE THREADS CHUNK OUT\n");
        return 2;
    }
    std::string e;
    auto src = getenv("SERIAL") ? mtb::open_source(argv[1], 1, false, e)
                                : mtb::open_parallel_gzip(argv[1], atoi(argv[2]), strtoull(argv[3], nullptr, 10), e);
    if (!src) {
        printf("bytes=0 rc=-1 err=\"%s\"\n", e.c_str());
        return 1;
    }
    FILE* o = fopen(argv[4], "wb");
    if (!o) return 1;
    std::vector<char> buf(1u << 20);
    long g;
    size_t total = 0;
    while ((g = src->read(buf.data(), buf.size())) > 0) {
        fwrite(buf.data(), 1, (size_t)g, o);
        total += (size_t)g;
    }
    fclose(o);
    printf("bytes=%zu rc=%ld err=\"%s\"\n", total, g, src->err.c_str());
    return 0;
}
