// Host input around the device path: decompressed byte sources for FASTA/FASTQ
// files (plain, gzip, or BGZF with its blocks inflated by a thread pool) and the record parser with
// kseq's semantics, shared by the synchronous reader (mtb_reader_*) and the threaded pipeline
// (mtb_start_classify, mtb_pipeline.cpp).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/mtb_gpu.h"

namespace mtb {

// Decompressed bytes of one input file, in order.
struct ByteSource {
    virtual ~ByteSource() {}
    // Up to cap bytes into dst; 0 at end of input, -1 on error (err set).
    virtual long read(char* dst, size_t cap) = 0;
    std::string err;
};

// Plain files pass through; gzip (one or several members) inflates on one thread; BGZF (gzip
// members carrying their block size in a "BC" extra field, as bgzip writes them) inflates up to
// `threads` blocks at once. With prefetch, a thread of its own keeps the next chunks ready.
std::unique_ptr<ByteSource> open_source(const std::string& path, int threads, bool prefetch, std::string& err);

// Ordinary (non-BGZF) gzip inflated by `threads` workers at once (mtb_gunzip.cpp): the file is
// cut into chunks of chunkBytes compressed bytes, each decoded from the first block boundary found
// in it, and checked against the true boundaries, CRC-32 and ISIZE in stream order.
std::unique_ptr<ByteSource> open_parallel_gzip(const std::string& path, int threads, size_t chunkBytes,
                                               std::string& err);

// With MTB_NICE set, helper threads of the input path (inflate, read-ahead, record split, parse,
// batch fill, TSV formatting) run five nice levels below the caller's threads, so the threads that
// feed and drain the GPU are scheduled first when the host's cores are all busy (off by default:
// the same-box A/B, profiles/r03/e2e_ab.json, measured no gain).
void background_thread();

// The per-read classification TSV (Reporter::writeReadClassification, Reporter.cpp:38-83): its
// header line, and one batch's lines formatted by `threads` threads into part[0..) in read order.
const char* classification_header(bool lineage);
void format_classifications(const mtb_ctx* ctx, const mtb_read_batch& batch, const mtb_result* res,
                            const mtb_taxcnt* taxcnt, uint32_t flags, std::vector<std::string>& part,
                            unsigned threads);

// gzip's CRC-32 (libdeflate's folded carry-less multiply when it loads, zlib's otherwise).
uint32_t crc32_bytes(uint32_t crc, const uint8_t* p, size_t n);

// Buffered line access over a ByteSource.
struct FastxStream {
    std::unique_ptr<ByteSource> src;
    std::vector<char> buf;  // unread bytes live in [pos, end)
    size_t pos = 0, end = 0;
    bool eof = false;
    std::string err;
    bool open(const std::string& path, int threads, bool prefetch);
    size_t fill(size_t want);
    bool line(const char*& p, size_t& n);
    int peek();
};

// One record appended to (seq, off) and (names, noff): kseq semantics — the name is the header up
// to the first space or tab; FASTA sequence lines run to the next '>' header; FASTQ sequence lines
// run to the '+' line, and quality lines follow until they are as long as the sequence (wrapped
// records). false at the end of the input, or with err set on malformed input.
bool next_record(FastxStream& s, std::string& seq, std::vector<uint64_t>& off, std::string& names,
                 std::vector<uint64_t>& noff, std::string& err);

// The same semantics over an in-memory range, split in two passes so records can be parsed in
// parallel: scan_records counts up to maxRecs whole records at the front of p[0, n) (eof: the
// range ends the input) and returns the bytes they span — a record the range does not complete
// is left for the next range; parse_records appends every record of a range scan_records cut.
// err is set on malformed input.
size_t scan_records(const char* p, size_t n, bool eof, uint32_t maxRecs, uint32_t* recs, std::string& err);
uint32_t parse_records(const char* p, size_t n, std::string& seq, std::vector<uint64_t>& off, std::string& names,
                       std::vector<uint64_t>& noff, std::string& err);

}  // namespace mtb
