// Host ingest check and timing (tests/test_ingest.py): parses one FASTA/FASTQ file
// (plain, gzip or BGZF) with the serial record reader (next_record, the synchronous mtb_reader path)
// and with the pipeline's two passes (scan_records cutting raw buffers of `buf` bytes at record
// boundaries, parse_records on each cut, the unfinished record carried into the next buffer, as
// MateReader::run does), and checks that both give the same records, names and errors.
//   ingest_check FILE BUF_BYTES [MAX_RECS_PER_CUT]
// prints: records=N bytes=B serial_s=.. scan_s=.. parse_s=.. same=1|0 err=".."
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../metabuli_work_amd/csrc/mtb_io.h"

using Clock = std::chrono::steady_clock;
static double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }

struct Out {
    std::string seq, names, err;
    std::vector<uint64_t> off{0}, noff{0};
};

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: ingest_check FILE BUF_BYTES [MAX_RECS_PER_CUT]\n");
        return 2;
    }
    const size_t bufBytes = strtoull(argv[2], nullptr, 10);
    const uint32_t maxRecs = argc > 3 ? (uint32_t)strtoul(argv[3], nullptr, 10) : 8192u;
    // serial reader
    Out a;
    auto t0 = Clock::now();
    {
        mtb::FastxStream st;
        if (!st.open(argv[1], 4, true)) {
            printf("open failed: %s\n", st.err.c_str());
            return 1;
        }
        while (mtb::next_record(st, a.seq, a.off, a.names, a.noff, a.err)) {
        }
    }
    const double serialS = secs(t0);
    // the whole decompressed input in memory, then cut and parsed as the pipeline does
    std::string all;
    const int srcThreads = getenv("INGEST_THREADS") ? atoi(getenv("INGEST_THREADS")) : 4;
    auto ts = Clock::now();
    {
        std::string e;
        // INGEST_PGZ=<chunk bytes>: the parallel gzip source at any thread count (timing)
        auto src = getenv("INGEST_PGZ") ? mtb::open_parallel_gzip(argv[1], srcThreads, strtoull(getenv("INGEST_PGZ"), nullptr, 10), e)
                                        : mtb::open_source(argv[1], srcThreads, true, e);
        if (!src) {
            printf("open failed: %s\n", e.c_str());
            return 1;
        }
        std::vector<char> tmp(1u << 24);
        long got;
        all.reserve(1u << 28);
        while ((got = src->read(tmp.data(), tmp.size())) > 0) all.append(tmp.data(), (size_t)got);
    }
    const double sourceS = secs(ts);
    Out b;
    double scanS = 0, parseS = 0;
    size_t fed = 0;  // bytes of `all` moved into buffers so far
    std::vector<char> buf(std::max<size_t>(bufBytes, 1));
    size_t have = 0;
    std::vector<std::string> chunks;  // the raw buffers the cuts point into
    while (b.err.empty()) {
        const size_t k = std::min(buf.size() - have, all.size() - fed);
        memcpy(buf.data() + have, all.data() + fed, k);
        have += k;
        fed += k;
        const bool eof = fed == all.size();
        size_t pos = 0;
        while (true) {
            uint32_t recs = 0;
            auto t1 = Clock::now();
            const size_t used = mtb::scan_records(buf.data() + pos, have - pos, eof, maxRecs, &recs, b.err);
            scanS += secs(t1);
            if (recs) chunks.emplace_back(buf.data() + pos, used);
            pos += used;
            if (!b.err.empty() || recs < maxRecs) break;
        }
        if (!b.err.empty() || eof) break;
        const size_t rest = have - pos;
        if (rest > buf.size() / 2) {
            std::vector<char> nb(buf.size() * 2);
            memcpy(nb.data(), buf.data() + pos, rest);
            buf.swap(nb);
        } else {
            memmove(buf.data(), buf.data() + pos, rest);
        }
        have = rest;
    }
    auto t2 = Clock::now();
    for (auto& c : chunks) {
        std::string e;
        mtb::parse_records(c.data(), c.size(), b.seq, b.off, b.names, b.noff, e);
        if (!e.empty() && b.err.empty()) b.err = e;
    }
    parseS = secs(t2);
    // next_record leaves a failing record's name (and part of its sequence) behind: compare whole records
    a.noff.resize(a.off.size());
    a.names.resize(a.noff.back());
    a.seq.resize(a.off.back());
    const bool same = a.seq == b.seq && a.names == b.names && a.off == b.off && a.noff == b.noff && a.err == b.err;
    printf("records=%zu bytes=%zu serial_s=%.4f source_s=%.4f scan_s=%.4f parse_s=%.4f same=%d err=\"%s\" err2=\"%s\"\n",
           a.off.size() - 1, all.size(), serialS, sourceS, scanS, parseS, same ? 1 : 0, a.err.c_str(), b.err.c_str());
    return same ? 0 : 3;
}
