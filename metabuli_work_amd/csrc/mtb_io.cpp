// Host I/O around the device path: a FASTA/FASTQ(.gz) batch reader that fills
// the flat buffers mtb_classify_batch takes, and the per-read classification TSV writer.
//
// Reader: replaces QueryIndexer's counting pass plus KmerExtractor::loadChunkOfReads'
// serial kseq loop (QueryIndexer.cpp:30-147, KmerExtractor.cpp:442-494): one streaming pass over
// a decompressed byte source (mtb_source.cpp: plain / gzip / BGZF inflated by a worker pool, read
// ahead on a thread of its own), records split with memchr with kseq's semantics (names cut at the
// first whitespace, wrapped FASTA and FASTQ). Mates are read in lock-step; unequal read counts are
// an error, as in QueryIndexer.cpp:121-124. The threaded classify pipeline is mtb_pipeline.cpp.
//
// Writer: Reporter::writeReadClassification (Reporter.cpp:38-83), formatted by several threads
// into per-thread strings and written in read order. Scores print as ostream << float (%g).
#include <zlib.h>

#include <algorithm>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "mtb_host.h"
#include "mtb_io.h"

namespace mtb {

bool FastxStream::open(const std::string& path, int threads, bool prefetch) {
    src = open_source(path, threads, prefetch, err);
    if (!src) return false;
    buf.resize(64u << 20);
    return true;
}

// Make at least `want` bytes available from pos (or everything left). Returns bytes available.
size_t FastxStream::fill(size_t want) {
    if (end - pos >= want || eof) return end - pos;
    if (pos > 0) {
        memmove(buf.data(), buf.data() + pos, end - pos);
        end -= pos;
        pos = 0;
    }
    if (buf.size() < want + (1u << 20)) buf.resize(want + (1u << 20));
    while (end < buf.size() && !eof) {
        const long got = src->read(buf.data() + end, std::min<size_t>(buf.size() - end, 1u << 30));
        if (got < 0) err = src->err;
        if (got <= 0) {
            eof = true;
            break;
        }
        end += (size_t)got;
        if (end - pos >= want) break;
    }
    return end - pos;
}

// Next line (without '\n' / '\r'); false at end of input.
bool FastxStream::line(const char*& p, size_t& n) {
    for (size_t want = 1u << 16;; want *= 2) {
        const size_t avail = fill(want);
        if (avail == 0) return false;
        const char* s = buf.data() + pos;
        const char* nl = (const char*)memchr(s, '\n', avail);
        if (nl || eof) {
            size_t len = nl ? (size_t)(nl - s) : avail;
            pos += len + (nl ? 1 : 0);
            if (len && s[len - 1] == '\r') len--;
            p = s;
            n = len;
            return true;
        }
        if (avail < want) return false;
    }
}

int FastxStream::peek() {
    if (fill(1) == 0) return -1;
    return (unsigned char)buf[pos];
}

bool next_record(FastxStream& s, std::string& seq, std::vector<uint64_t>& off, std::string& names,
                 std::vector<uint64_t>& noff, std::string& err) {
    const char* p;
    size_t n;
    while (true) {  // skip blank lines before a header
        const int c = s.peek();
        if (c < 0) {
            if (!s.err.empty()) err = s.err;
            return false;
        }
        if (c == '\n' || c == '\r') {
            s.line(p, n);
            continue;
        }
        break;
    }
    if (!s.line(p, n)) return false;
    if (n == 0 || (p[0] != '>' && p[0] != '@')) {
        err = "not a FASTA/FASTQ record header";
        return false;
    }
    const bool fastq = p[0] == '@';
    size_t nameLen = 1;
    while (nameLen < n && p[nameLen] != ' ' && p[nameLen] != '\t') nameLen++;
    names.append(p + 1, nameLen - 1);
    noff.push_back(names.size());
    const size_t seqStart = seq.size();
    if (fastq) {  // sequence lines up to the '+' line, then quality lines until as long (kseq)
        bool plus = false;
        while (s.line(p, n)) {
            if (n && p[0] == '+') {
                plus = true;
                break;
            }
            seq.append(p, n);
        }
        if (!plus) {
            err = "truncated FASTQ record";
            return false;
        }
        const size_t slen = seq.size() - seqStart;
        size_t qlen = 0;
        while (qlen < slen) {
            if (!s.line(p, n)) {
                err = "truncated FASTQ record";
                return false;
            }
            qlen += n;
        }
    } else {
        while (true) {
            const int c = s.peek();
            if (c < 0 || c == '>') break;
            s.line(p, n);
            seq.append(p, n);
        }
    }
    if (!s.err.empty()) {
        err = s.err;
        return false;
    }
    off.push_back(seq.size());
    return true;
}

namespace {

// Lines of an in-memory range: next() gives the line at `pos` without '\n' / '\r'. kIncomplete
// when the range holds no '\n' after pos and is not the end of the input.
enum LineRc { kLine, kEnd, kIncomplete };

struct MemLines {
    const char* p;
    size_t n, pos;
    bool eof;
    LineRc next(const char*& s, size_t& len) {
        if (pos == n) return eof ? kEnd : kIncomplete;
        s = p + pos;
        const char* nl = (const char*)memchr(s, '\n', n - pos);
        if (!nl && !eof) return kIncomplete;
        len = nl ? (size_t)(nl - s) : n - pos;
        pos += len + (nl ? 1 : 0);
        if (len && s[len - 1] == '\r') len--;
        return kLine;
    }
};

// next_record's semantics over p[0, n): whole records only, at most maxRecs of them. kParse
// appends them to the block buffers; without it the records are only counted (the splitter's
// boundary pass). Returns the bytes the whole records (and blank lines before them) span.
template <bool kParse>
size_t walk_records(const char* p, size_t n, bool eof, uint32_t maxRecs, uint32_t* recs, std::string* seq,
                    std::vector<uint64_t>* off, std::string* names, std::vector<uint64_t>* noff, std::string& err) {
    MemLines m{p, n, 0, eof};
    size_t done = 0;
    uint32_t k = 0;
    const char* s;
    size_t len;
    while (k < maxRecs) {
        // blank lines before a header (a line starting with '\r' counts as blank, as in next_record)
        while (m.pos < n && (p[m.pos] == '\n' || p[m.pos] == '\r')) {
            if (m.next(s, len) == kIncomplete) break;
        }
        if (m.pos == n || (m.pos < n && (p[m.pos] == '\n' || p[m.pos] == '\r'))) {
            if (m.pos == n && eof) done = n;  // trailing blank lines end the input
            break;
        }
        const LineRc h = m.next(s, len);
        if (h != kLine) break;
        if (len == 0 || (s[0] != '>' && s[0] != '@')) {
            err = "not a FASTA/FASTQ record header";
            break;
        }
        const bool fastq = s[0] == '@';
        const char* name = s + 1;
        size_t nameLen = 1;
        while (nameLen < len && s[nameLen] != ' ' && s[nameLen] != '\t') nameLen++;
        nameLen--;
        const size_t seqStart = kParse ? seq->size() : 0;
        bool complete = true;
        if (fastq) {
            size_t slen = 0;
            LineRc rc;
            while ((rc = m.next(s, len)) == kLine && !(len && s[0] == '+')) {
                if (kParse) seq->append(s, len);
                slen += len;
            }
            if (rc != kLine) {
                if (rc == kEnd) err = "truncated FASTQ record";
                complete = false;
            }
            for (size_t qlen = 0; complete && qlen < slen;) {
                rc = m.next(s, len);
                if (rc != kLine) {
                    if (rc == kEnd) err = "truncated FASTQ record";
                    complete = false;
                }
                qlen += len;
            }
        } else {
            while (true) {  // sequence lines up to the next '>' (a record at the input's end is whole)
                if (m.pos == n) {
                    complete = eof;
                    break;
                }
                if (p[m.pos] == '>') break;
                if (m.next(s, len) != kLine) {
                    complete = false;
                    break;
                }
                if (kParse) seq->append(s, len);
            }
        }
        if (!complete) {
            if (kParse) seq->resize(seqStart);
            break;
        }
        if (kParse) {
            names->append(name, nameLen);
            noff->push_back(names->size());
            off->push_back(seq->size());
        }
        k++;
        done = m.pos;
    }
    *recs = k;
    return done;
}

}  // namespace

size_t scan_records(const char* p, size_t n, bool eof, uint32_t maxRecs, uint32_t* recs, std::string& err) {
    return walk_records<false>(p, n, eof, maxRecs, recs, nullptr, nullptr, nullptr, nullptr, err);
}

uint32_t parse_records(const char* p, size_t n, std::string& seq, std::vector<uint64_t>& off, std::string& names,
                       std::vector<uint64_t>& noff, std::string& err) {
    uint32_t k = 0;
    walk_records<true>(p, n, true, 0xFFFFFFFFu, &k, &seq, &off, &names, &noff, err);
    return k;
}

}  // namespace mtb

using mtb::FastxStream;
using mtb::next_record;

namespace mtb {

const char* classification_header(bool lineage) {
    return lineage ? "#is_classified\tname\ttaxID\tquery_length\tscore\trank\tlineage\ttaxID:match_count\n"
                   : "#is_classified\tname\ttaxID\tquery_length\tscore\trank\ttaxID:match_count\n";
}

namespace {

// ostream << float text (%g, 6 significant digits) of the scores a thread has seen: a read's score
// is a sum of multiples of 0.5 over its length, so a batch holds few distinct values.
struct ScoreText {
    struct Entry {
        uint32_t bits = 0xFFFFFFFFu;  // a NaN pattern no score has
        uint8_t len = 0;              // kLong: the text did not fit (formatted in place instead)
        char s[12];
    };
    static constexpr uint8_t kLong = 0xFF;
    Entry e[4096];
    const Entry& get(float v) {
        uint32_t b;
        memcpy(&b, &v, 4);
        Entry& x = e[(b ^ (b >> 12) ^ (b >> 24)) & 4095u];
        if (x.bits != b) {
            char tmp[32];
            const auto r = std::to_chars(tmp, tmp + sizeof tmp, (double)v, std::chars_format::general, 6);
            const size_t len = (size_t)(r.ptr - tmp);
            x.bits = b;
            x.len = len <= sizeof x.s ? (uint8_t)len : kLong;
            if (x.len != kLong) memcpy(x.s, tmp, len);
        }
        return x;
    }
};

}  // namespace

void format_classifications(const mtb_ctx* ctx, const mtb_read_batch& batch, const mtb_result* res,
                            const mtb_taxcnt* taxcnt, uint32_t flags, std::vector<std::string>& part,
                            unsigned threads) {
    const uint32_t n = batch.n_reads;
    const char* names = batch.names;
    const uint64_t* name_off = batch.name_off;
    const bool lineage = (flags & MTB_WRITE_LINEAGE) != 0;
    if (lineage && n) mtb_taxon_lineage(ctx, 1);  // build the per-node lineages before the threads
    const TaxText& tt = tax_text(ctx);
    const unsigned nt = std::max(1u, std::min(threads, std::thread::hardware_concurrency()));
    const uint32_t per = (n + nt - 1) / nt;
    part.resize(nt);
    auto work = [&](unsigned t) {
        std::string& o = part[t];
        const uint32_t lo = t * per, hi = std::min<uint32_t>(n, lo + per);
        static thread_local std::unique_ptr<ScoreText> scores;
        if (!scores) scores.reset(new ScoreText());
        // the lines go through a raw cursor into o (grown by doubling, cut to size at the end):
        // per field a memcpy of precomputed text (taxIDs' original IDs, ranks, scores) instead of a
        // conversion, the integers left through std::to_chars
        size_t pos = 0;
        o.resize(std::max<size_t>(o.capacity(), (size_t)(hi > lo ? hi - lo : 0) * 64 + 256));
        char* w = &o[0];
        auto room = [&](size_t need) {
            if (pos + need > o.size()) {
                o.resize(std::max(2 * o.size(), pos + need));
                w = &o[0];
            }
        };
        auto put = [&](const char* p, size_t len) {
            memcpy(w + pos, p, len);
            pos += len;
        };
        auto num = [&](auto v) { pos = (size_t)(std::to_chars(w + pos, w + pos + 24, v).ptr - w); };
        auto taxid = [&](int32_t x) {  // getOriginalTaxID (Reporter.cpp:55,65,72)
            if (x >= 0 && (uint32_t)x < tt.n) put(tt.buf.data() + tt.idOff[x], tt.idOff[x + 1] - tt.idOff[x]);
            else num(mtb_original_taxid(ctx, x));
        };
        for (uint32_t i = lo; i < hi; i++) {
            const mtb_result& r = res[i];
            const size_t nameLen = name_off[i + 1] - name_off[i];
            const char* lin = r.is_classified && lineage ? mtb_taxon_lineage(ctx, r.classification) : nullptr;
            const size_t linLen = lin ? strlen(lin) : 0;
            const int32_t cls = r.is_classified ? r.classification : 0;
            const size_t rankLen = cls >= 0 && (uint32_t)cls < tt.n ? tt.rankOff[cls + 1] - tt.rankOff[cls] : 64;
            room(nameLen + linLen + rankLen + 96 + (size_t)(r.is_classified ? r.taxcnt_len : 0) * 24);
            w[pos++] = r.is_classified ? '1' : '0';
            w[pos++] = '\t';
            put(names + name_off[i], nameLen);
            // the std::map order of the taxID:count list is the internal one, as the reference's
            w[pos++] = '\t';
            taxid(cls);
            w[pos++] = '\t';
            num(r.query_length);
            w[pos++] = '\t';
            const ScoreText::Entry& sc = scores->get(r.score);
            if (sc.len != ScoreText::kLong) {
                put(sc.s, sc.len);
            } else {
                room(64);
                pos = (size_t)(std::to_chars(w + pos, w + pos + 32, (double)r.score, std::chars_format::general, 6).ptr - w);
            }
            w[pos++] = '\t';
            if (r.is_classified) {
                if ((uint32_t)cls < tt.n) {
                    put(tt.buf.data() + tt.rankOff[cls], rankLen);
                } else {
                    const char* rk = mtb_taxon_rank(ctx, cls);
                    room(strlen(rk) + 64 + (size_t)r.taxcnt_len * 24);
                    put(rk, strlen(rk));
                }
                w[pos++] = '\t';
                if (lineage) {
                    put(lin, linLen);
                    w[pos++] = '\t';
                }
                for (uint32_t k = 0; k < r.taxcnt_len; k++) {
                    const mtb_taxcnt& c = taxcnt[r.taxcnt_offset + k];
                    taxid(c.tax_id);
                    w[pos++] = ':';
                    num(c.count);
                    w[pos++] = ' ';
                }
                w[pos++] = '\n';
            } else {
                lineage ? put("-\t-\t-\t\n", 7) : put("-\t-\t\n", 5);
            }
        }
        o.resize(pos);
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++)
        th.emplace_back([&, t] {
            background_thread();  // helpers of the calling thread
            work(t);
        });
    work(0);
    for (auto& x : th) x.join();
}

}  // namespace mtb

static constexpr int kReaderThreads = 4;  // BGZF inflate workers per file

struct mtb_reader {
    FastxStream a, b;
    bool paired = false;
    std::string seq1, seq2, names, err;
    std::vector<uint64_t> off1, off2, noff;
};

extern "C" {

int mtb_reader_open(const char* path1, const char* path2, mtb_reader** out) {
    if (!path1 || !out) return MTB_ERR_ARG;
    mtb_reader* r = new mtb_reader();
    if (!r->a.open(path1, kReaderThreads, true)) {
        mtb::set_error(r->a.err);
        delete r;
        return MTB_ERR_IO;
    }
    if (path2) {
        r->paired = true;
        if (!r->b.open(path2, kReaderThreads, true)) {
            mtb::set_error(r->b.err);
            delete r;
            return MTB_ERR_IO;
        }
    }
    *out = r;
    return MTB_OK;
}

int mtb_reader_next(mtb_reader* r, uint32_t max_reads, uint64_t max_bases, mtb_read_batch* batch) {
    if (!r || !batch || max_reads == 0) return MTB_ERR_ARG;
    r->seq1.clear();
    r->seq2.clear();
    r->names.clear();
    r->off1.assign(1, 0);
    r->off2.assign(1, 0);
    r->noff.assign(1, 0);
    std::string dummyNames;
    std::vector<uint64_t> dummyOff(1, 0);
    uint32_t n = 0;
    while (n < max_reads && r->seq1.size() + r->seq2.size() < max_bases) {
        if (!next_record(r->a, r->seq1, r->off1, r->names, r->noff, r->err)) break;
        if (r->paired) {
            dummyNames.clear();
            dummyOff.assign(1, 0);
            if (!next_record(r->b, r->seq2, r->off2, dummyNames, dummyOff, r->err)) {
                if (r->err.empty()) r->err = "paired-end inputs have different read counts (QueryIndexer.cpp:121-124)";
                break;
            }
        }
        n++;
    }
    if (!r->err.empty()) {
        mtb::set_error(r->err);
        return MTB_ERR_IO;
    }
    if (r->paired && n == 0 && r->b.peek() >= 0 && r->b.peek() != '\n') {
        mtb::set_error("paired-end inputs have different read counts (QueryIndexer.cpp:121-124)");
        return MTB_ERR_IO;
    }
    batch->n_reads = n;
    batch->seq1 = r->seq1.data();
    batch->off1 = r->off1.data();
    batch->seq2 = r->paired ? r->seq2.data() : nullptr;
    batch->off2 = r->paired ? r->off2.data() : nullptr;
    batch->names = r->names.data();
    batch->name_off = r->noff.data();
    return MTB_OK;
}

void mtb_reader_close(mtb_reader* r) { delete r; }

int mtb_write_classifications(const mtb_ctx* ctx, const char* path, int append, const mtb_read_batch* batch,
                              const mtb_result* res, const mtb_taxcnt* taxcnt, uint32_t flags) {
    if (!ctx || !path || !batch || (!res && batch->n_reads)) return MTB_ERR_ARG;
    FILE* f = fopen(path, append ? "ab" : "wb");
    if (!f) {
        mtb::set_error(std::string("cannot write ") + path);
        return MTB_ERR_IO;
    }
    if (!append) fputs(mtb::classification_header((flags & MTB_WRITE_LINEAGE) != 0), f);
    // the formatted parts stay allocated per calling thread: repeated calls reuse warm memory
    static thread_local std::vector<std::string> part;
    mtb::format_classifications(ctx, *batch, res, taxcnt, flags, part, 8);
    for (auto& s : part) fwrite(s.data(), 1, s.size(), f);
    const bool ok = fclose(f) == 0;
    if (!ok) {
        mtb::set_error(std::string("write failed: ") + path);
        return MTB_ERR_IO;
    }
    return MTB_OK;
}

int mtb_write_em_results(mtb_ctx* ctx, const char* path, const char* classification_tsv, const mtb_em_read* reads,
                         uint64_t n_reads, uint32_t flags) {
    if (!ctx || !path || !classification_tsv || (!reads && n_reads)) return MTB_ERR_ARG;
    // Classifier::loadOriginalResults (Classifier.cpp:450-480): name = column 2, query_length =
    // column 4 of each non-comment line of the classification TSV
    FILE* in = fopen(classification_tsv, "rb");
    if (!in) {
        mtb::set_error(std::string("cannot read ") + classification_tsv);
        return MTB_ERR_IO;
    }
    FILE* f = fopen(path, "wb");
    if (!f) {
        fclose(in);
        mtb::set_error(std::string("cannot write ") + path);
        return MTB_ERR_IO;
    }
    const bool lineage = (flags & MTB_WRITE_LINEAGE) != 0;
    fputs(lineage ? "#is_classified\tname\ttaxID\tquery_length\tscore\trank\tlineage\n"
                  : "#is_classified\tname\ttaxID\tquery_length\tscore\trank\n", f);
    std::string o;
    char* line = nullptr;
    size_t cap = 0;
    ssize_t len;
    uint64_t i = 0;
    char tmp[96];
    while ((len = getline(&line, &cap, in)) >= 0) {
        if (len && line[len - 1] == '\n') line[--len] = 0;
        if (len == 0 || line[0] == '#') continue;
        const char* c0 = line;
        const char* t1 = strchr(c0, '\t');
        const char* t2 = t1 ? strchr(t1 + 1, '\t') : nullptr;
        const char* t3 = t2 ? strchr(t2 + 1, '\t') : nullptr;
        if (!t3) continue;  // "Invalid line format" (fewer than 4 columns): skipped
        const std::string name(t1 + 1, t2);
        const int length = atoi(t3 + 1);
        const mtb_em_read r = i < n_reads ? reads[i] : mtb_em_read{0, 0, 0.0};
        i++;
        o += r.tax_id != 0 ? "1\t" : "0\t";
        o += name;
        snprintf(tmp, sizeof tmp, "\t%d\t%d\t%g\t", mtb_original_taxid(ctx, r.tax_id), length, r.score);
        o += tmp;
        if (r.tax_id != 0) {
            o += mtb_taxon_rank(ctx, r.tax_id);
            if (lineage) {
                o += '\t';
                o += mtb_taxon_lineage(ctx, r.tax_id);
            }
        } else {
            o += lineage ? "-\t-" : "-";
        }
        o += '\n';
        if (o.size() > (1u << 22)) {
            fwrite(o.data(), 1, o.size(), f);
            o.clear();
        }
    }
    free(line);
    fclose(in);
    fwrite(o.data(), 1, o.size(), f);
    if (fclose(f) != 0) {
        mtb::set_error(std::string("write failed: ") + path);
        return MTB_ERR_IO;
    }
    return MTB_OK;
}

}  // extern "C"
