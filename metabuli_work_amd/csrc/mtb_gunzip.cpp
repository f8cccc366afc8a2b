// Parallel inflate of ordinary (single- or multi-member, non-BGZF) gzip query files: the format
// most .fastq.gz files come in, which zlib inflates on one thread (the reference reads it through
// kseq/gzread, QueryIndexer.cpp:30-147 and KmerExtractor.cpp:442-494).
//
// The compressed file (memory-mapped) is cut into chunks of kChunk bytes. A pool of workers
// decodes the chunks at once:
//   * chunk j > 0 starts at the first dynamic-Huffman block header found at or after its first bit
//     (a header whose code-length, literal/length and distance codes are all complete prefix codes,
//     and whose first block then decodes);
//   * a chunk decodes whole blocks until a block starts at or after the next chunk's first bit;
//   * the 32 KB window before a chunk's start is unknown while it decodes: a back-reference into it
//     is written as a marker (256 + its index in the window) in 16-bit output symbols.
// A coordinator takes the chunks in order: chunk j is accepted only if it started exactly where
// the previous piece stopped (a false block header, or a stored / fixed block at the boundary,
// makes the coordinator decode that range itself from the true boundary), so every byte comes from
// a decode that started at a real block boundary. The window of each piece is the last 32 KB of the
// previous piece's bytes; the workers then turn markers into bytes and compute CRC-32 per member
// segment, and read() checks each member's CRC-32 and ISIZE (as zlib does at a member's end).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <type_traits>

#include "mtb_io.h"

namespace mtb {
namespace {

constexpr uint32_t kWin = 32768;

constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// LSB-first bit input over an in-memory buffer (bits past the end read as 0 and are counted).
struct BitIn {
    const uint8_t* base = nullptr;
    const uint8_t* in = nullptr;
    const uint8_t* end = nullptr;
    uint64_t buf = 0;
    uint32_t cnt = 0;  // valid bits in buf
    uint64_t pad = 0;  // zero bytes supplied past the end
    void init(const uint8_t* b, size_t n, uint64_t bit) {
        base = b;
        end = b + n;
        in = b + std::min<uint64_t>(bit >> 3, n);
        buf = 0;
        cnt = 0;
        pad = 0;
        refill();
        drop(bit & 7);
    }
    inline void refill() {
        if (end - in >= 8) {
            uint64_t w;
            memcpy(&w, in, 8);
            buf |= w << cnt;
            in += (63 - cnt) >> 3;
            cnt |= 56;
        } else {
            while (cnt <= 56) {
                if (in < end) {
                    buf |= (uint64_t)*in++ << cnt;
                } else {
                    pad++;
                }
                cnt += 8;
            }
        }
    }
    inline uint32_t peek(uint32_t n) const { return (uint32_t)(buf & ((1ull << n) - 1)); }
    inline void drop(uint32_t n) {
        buf >>= n;
        cnt -= n;
    }
    inline uint32_t take(uint32_t n) {
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
    uint64_t bitpos() const { return ((uint64_t)(in - base) + pad) * 8 - cnt; }
    bool overrun() const { return bitpos() > (uint64_t)(end - base) * 8; }
    void align() { drop(cnt & 7); }
};

// Canonical Huffman decode table: 2^bits primary entries, then subtables for longer codes.
// Entry: bits 0-3 code length (0 with no flag: an unused code), bit 4 subtable link (bits 5-7 its
// index bits, bits 16-31 its offset); for symbols bits 8-11 the extra bits, bit 12 a literal, bit 13
// end of block, bit 14 a symbol deflate does not allow, bits 16-31 the literal, the length or
// distance base, or the plain symbol.
constexpr uint32_t kSub = 1u << 4, kLit = 1u << 12, kEob = 1u << 13, kBad = 1u << 14;
enum class Alphabet { kPlain, kLitLen, kDist };

struct Huff {
    std::vector<uint32_t> t;
    uint32_t bits = 0;
    static uint32_t entry(Alphabet a, uint32_t s, uint32_t L) {
        if (a == Alphabet::kPlain) return L | s << 16;
        if (a == Alphabet::kLitLen) {
            if (s < 256) return L | kLit | s << 16;
            if (s == 256) return L | kEob;
            if (s > 285) return L | kBad;
            return L | (uint32_t)kLenExtra[s - 257] << 8 | (uint32_t)kLenBase[s - 257] << 16;
        }
        if (s > 29) return L | kBad;
        return L | (uint32_t)kDistExtra[s] << 8 | (uint32_t)kDistBase[s] << 16;
    }
    // zlib's rules (inflate_table): over-subscribed sets are errors; an incomplete set is accepted
    // only for a code of one length-1 symbol, and never for the code-length code; an empty
    // distance code is accepted.
    bool build(const uint8_t* lens, int n, uint32_t primaryBits, Alphabet a, bool allowEmpty) {
        bits = primaryBits;
        uint16_t count[16] = {0};
        for (int i = 0; i < n; i++) count[lens[i]]++;
        count[0] = 0;
        int maxLen = 0;
        for (int L = 1; L <= 15; L++)
            if (count[L]) maxLen = L;
        t.assign((size_t)1 << bits, 0u);
        if (maxLen == 0) return allowEmpty;
        int left = 1;
        for (int L = 1; L <= 15; L++) {
            left = (left << 1) - count[L];
            if (left < 0) return false;
        }
        if (left > 0 && (a == Alphabet::kPlain || maxLen != 1)) return false;
        uint32_t next[16];
        uint32_t code = 0;
        for (int L = 1; L <= 15; L++) {
            code = (code + count[L - 1]) << 1;
            next[L] = code;
        }
        const uint32_t subBits = maxLen > (int)bits ? (uint32_t)maxLen - bits : 0;
        for (int s = 0; s < n; s++) {
            const uint32_t L = lens[s];
            if (!L) continue;
            const uint32_t c = next[L]++;
            uint32_t r = 0;  // the code bit-reversed: deflate packs codes MSB first into an LSB-first stream
            for (uint32_t k = 0; k < L; k++) r |= ((c >> k) & 1u) << (L - 1 - k);
            const uint32_t e = entry(a, (uint32_t)s, L);
            if (L <= bits) {
                for (uint32_t k = r; k < (1u << bits); k += 1u << L) t[k] = e;
            } else {
                const uint32_t p = r & ((1u << bits) - 1);
                if (!(t[p] & kSub)) {
                    const size_t off = t.size();
                    t.resize(off + ((size_t)1 << subBits), 0u);
                    t[p] = kSub | (subBits << 5) | ((uint32_t)off << 16);
                }
                const uint32_t off = t[p] >> 16, hi = r >> bits;
                for (uint32_t k = hi; k < (1u << subBits); k += 1u << (L - bits)) t[off + k] = e;
            }
        }
        return true;
    }
    inline uint32_t decode(uint64_t b) const {
        uint32_t e = t[b & ((1u << bits) - 1)];
        if (e & kSub) e = t[(e >> 16) + ((b >> bits) & ((1u << ((e >> 5) & 7u)) - 1))];
        return e;
    }
};

const Huff& fixed_lit() {
    static const Huff h = [] {
        uint8_t l[288];
        for (int i = 0; i < 288; i++) l[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
        Huff x;
        x.build(l, 288, 10, Alphabet::kLitLen, false);
        return x;
    }();
    return h;
}

const Huff& fixed_dist() {
    static const Huff h = [] {
        uint8_t l[32];  // 30 and 31 complete the code and are invalid distances
        for (int i = 0; i < 32; i++) l[i] = 5;
        Huff x;
        x.build(l, 32, 8, Alphabet::kDist, false);
        return x;
    }();
    return h;
}

// A dynamic block's header after BFINAL/BTYPE: the code-length code and both codes.
bool read_dynamic(BitIn& b, Huff& lit, Huff& dist) {
    b.refill();
    const uint32_t hlit = b.take(5) + 257, hdist = b.take(5) + 1, hclen = b.take(4) + 4;
    if (hlit > 286 || hdist > 30) return false;
    uint8_t cl[19] = {0};
    b.refill();
    for (uint32_t i = 0; i < hclen; i++) {
        if (i == 12) b.refill();
        cl[kClOrder[i]] = (uint8_t)b.take(3);
    }
    Huff clh;
    if (!clh.build(cl, 19, 7, Alphabet::kPlain, false)) return false;
    uint8_t lens[286 + 30];
    uint32_t i = 0;
    while (i < hlit + hdist) {
        b.refill();
        const uint32_t e = clh.decode(b.buf);
        const uint32_t L = e & 15u;
        if (!L) return false;
        b.drop(L);
        const uint32_t s = e >> 16;
        if (s < 16) {
            lens[i++] = (uint8_t)s;
            continue;
        }
        uint32_t rep;
        uint8_t v = 0;
        if (s == 16) {
            if (i == 0) return false;
            v = lens[i - 1];
            rep = 3 + b.take(2);
        } else if (s == 17) {
            rep = 3 + b.take(3);
        } else {
            rep = 11 + b.take(7);
        }
        if (i + rep > hlit + hdist) return false;
        while (rep--) lens[i++] = v;
    }
    if (lens[256] == 0) return false;
    return lit.build(lens, (int)hlit, 10, Alphabet::kLitLen, false) &&
           dist.build(lens + hlit, (int)hdist, 8, Alphabet::kDist, true) && !b.overrun();
}

// The gzip member header at byte `at`; returns the first deflate byte, or 0 if not a header.
size_t gzip_header(const uint8_t* d, size_t n, size_t at) {
    if (at + 10 > n || d[at] != 0x1f || d[at + 1] != 0x8b || d[at + 2] != 8) return 0;
    const uint8_t flg = d[at + 3];
    size_t p = at + 10;
    if (flg & 4) {  // FEXTRA
        if (p + 2 > n) return 0;
        p += 2 + (size_t)(d[p] | (d[p + 1] << 8));
    }
    for (int f : {8, 16})  // FNAME, FCOMMENT: zero-terminated
        if (flg & f) {
            while (p < n && d[p]) p++;
            p++;
        }
    if (flg & 2) p += 2;  // FHCRC
    return p <= n ? p : 0;
}

struct Trailer {
    uint64_t at;  // output index (in the piece) where the member ends
    uint32_t crc, isize;
};

// A grow-only array that is not zero-filled.
template <typename T>
struct Buf {
    std::unique_ptr<T[]> p;
    size_t cap = 0;
    void reserve(size_t want, size_t lo, size_t hi) {  // keeps [lo, hi)
        if (want <= cap) return;
        const size_t c = std::max(want, cap * 2);
        std::unique_ptr<T[]> o(new T[c]);
        if (hi > lo) memcpy(o.get() + lo, p.get() + lo, (hi - lo) * sizeof(T));
        p.swap(o);
        cap = c;
    }
    void release() {
        p.reset();
        cap = 0;
    }
};

// The output of one range of the compressed stream, indexed 0..n. While the window before the
// piece is unknown, symbols are 16-bit (a byte, or 256 + an index into the window); once the last
// 32 KB decoded hold no marker, no later symbol can reference the window and decoding continues in
// bytes: [0, n16) are symbols, [off8, n) bytes (the 32 KB [off8, n16) in both).
struct Piece {
    uint64_t startBits = 0, endBits = 0;
    Buf<uint16_t> s16;
    Buf<uint8_t> b8;
    size_t n = 0, n16 = 0, off8 = 0;
    bool bytes = false;  // decoding into b8
    std::vector<Trailer> trailers;
    bool streamEnd = false;          // the last member ended inside this piece (or the input did)
    bool endsAtMemberStart = false;  // endBits is the first block of a member
    bool ok = false;
    std::string err;
    uint8_t byte_at(size_t k, const uint8_t* window) const {  // with the window before the piece
        if (bytes && k >= off8) return b8.p[k];
        const uint16_t v = s16.p[k];
        return v < 256 ? (uint8_t)v : window[v - 256];
    }
};

enum { kBlockDone = 0, kSwitch = 1, kTruncated = 2, kError = -1 };

// The symbols of one Huffman-coded block (after its header) from the bit input, into the piece's
// current buffer: 16-bit symbols (kBytes false) or bytes. mStart: piece index where the current
// member began (-1: before the piece). kSwitch: the last 32 KB are free of markers (16-bit mode).
template <bool kBytes>
int decode_block(BitIn& b, const Huff* lit, const Huff* dist, Piece& r, int64_t mStart, int64_t& lastMarker,
                 size_t estimate, bool canSwitch) {
    using Sym = typename std::conditional<kBytes, uint8_t, uint16_t>::type;
    Buf<Sym>& buf = *[&] {
        if constexpr (kBytes) return &r.b8;
        else return &r.s16;
    }();
    const size_t lo = kBytes ? r.off8 : 0;  // the buffer's valid range starts here
    size_t k = r.n, kSafe = k;
    Sym* o = buf.p.get();
    size_t cap = buf.cap;
    auto fail = [&](const char* m) {
        r.err = m;
        r.n = k;
        return kError;
    };
    while (true) {
        // the input ended inside the last symbol: keep what came before it (zlib's output for a
        // truncated stream)
        if (b.pad && b.overrun()) {
            r.n = kSafe;
            return kTruncated;
        }
        kSafe = k;
        if (k + 264 > cap) {  // a match writes up to 7 symbols past its end
            buf.reserve(std::max(k + 264, estimate), lo, k);
            o = buf.p.get();
            cap = buf.cap;
        }
        // one refill covers a length/distance pair: 15 + 5 + 15 + 13 <= 56 bits
        b.refill();
        uint32_t e = lit->decode(b.buf);
        if (e & kLit) {
            b.drop(e & 15u);
            o[k++] = (Sym)(e >> 16);
            if (b.pad) continue;     // near the end: one symbol per overrun check
            e = lit->decode(b.buf);  // a second literal without a refill (>= 41 bits left)
            if (e & kLit) {
                b.drop(e & 15u);
                o[k++] = (Sym)(e >> 16);
                continue;
            }
            b.refill();
        }
        if (!(e & 15u) || (e & kBad)) return fail("gzip data error: invalid literal/length code");
        b.drop(e & 15u);
        if (e & kEob) {
            if (b.pad && b.overrun()) {
                r.n = k;
                return kTruncated;
            }
            break;
        }
        const uint32_t len = (e >> 16) + b.take((e >> 8) & 15u);
        const uint32_t de = dist->decode(b.buf);
        if (!(de & 15u) || (de & kBad)) return fail("gzip data error: invalid distance code");
        b.drop(de & 15u);
        const uint32_t dd = (de >> 16) + b.take((de >> 8) & 15u);
        const int64_t from = (int64_t)k - dd;
        if (from < (int64_t)lo || (mStart > 0 && from < mStart)) {
            if (kBytes || from >= 0 || mStart >= 0) return fail("gzip data error: invalid distance too far back");
            // 16-bit mode, into the unknown window before the piece (from >= -32768: dd <= 32768)
            for (uint32_t q = 0; q < len; q++) {
                const int64_t at = from + q;
                o[k + q] = at >= 0 ? o[at] : (Sym)(256 + kWin + at);
            }
            lastMarker = (int64_t)(k + len);
        } else {
            const Sym* src = o + from;
            Sym* dst = o + k;
            if (!kBytes && from < lastMarker) {  // the source may hold markers: copy and look
                uint32_t any = 0;
                for (uint32_t q = 0; q < len; q++) any |= (dst[q] = src[q]);
                if (any >= 256) lastMarker = (int64_t)(k + len);
            } else if (dd >= 8) {
                for (uint32_t q = 0; q < len; q += 8) memcpy(dst + q, src + q, 8 * sizeof(Sym));  // 8 per step
            } else if (dd == 1) {
                const Sym v = src[0];
                for (uint32_t q = 0; q < len; q++) dst[q] = v;
            } else {
                for (uint32_t q = 0; q < len; q++) dst[q] = src[q];
            }
        }
        k += len;
        if (!kBytes && canSwitch && (int64_t)k - lastMarker >= (int64_t)kWin) {
            r.n = k;
            return kSwitch;
        }
    }
    r.n = k;
    return kBlockDone;
}

// Continue in bytes: the last 32 KB of symbols (all bytes) start the byte buffer.
void switch_to_bytes(Piece& r, size_t estimate) {
    r.n16 = r.n;
    r.off8 = r.n - kWin;
    r.b8.reserve(std::max(estimate, r.n + (1u << 16)), 0, 0);
    for (size_t k = r.off8; k < r.n; k++) r.b8.p[k] = (uint8_t)r.s16.p[k];
    r.bytes = true;
}

// Decode whole blocks from `start` (a block boundary) until a block starts at or after stopBits
// (after at least one block), or the stream ends. memberStart: the piece begins a member (no
// window before it: bytes from the start), else back-references before the piece become markers.
bool inflate_piece(const uint8_t* d, size_t n, uint64_t start, uint64_t stopBits, bool memberStart, Piece& r,
                   bool firstBlockOnly = false) {
    BitIn b;
    b.init(d, n, start);
    r.startBits = start;
    r.n = r.n16 = r.off8 = 0;
    r.bytes = memberStart;
    r.trailers.clear();
    r.streamEnd = r.endsAtMemberStart = r.ok = false;
    r.err.clear();
    // about 5 output bytes per compressed byte for FASTQ: the estimate is 8
    const uint64_t span = stopBits == UINT64_MAX ? (uint64_t)n * 8 - std::min<uint64_t>(start, (uint64_t)n * 8)
                                                 : (stopBits > start ? stopBits - start : 0);
    const size_t estimate = firstBlockOnly ? (1u << 17) : (size_t)std::min<uint64_t>(span, 1ull << 26) + (1u << 16);
    int64_t mStart = memberStart ? 0 : -1;  // output index where the current member began
    int64_t lastMarker = 0;
    Huff dynLit, dynDist;
    bool first = true;
    auto truncated = [&] {
        r.streamEnd = true;
        r.endBits = (uint64_t)n * 8;
        r.ok = !firstBlockOnly;
        return r.ok;
    };
    auto fail = [&](const char* m) {
        if (b.overrun()) return truncated();  // the input ended: not an error (GzSource's rule)
        r.err = m;
        return false;
    };
    while (true) {
        if (!first && (b.bitpos() >= stopBits || firstBlockOnly)) break;
        first = false;
        b.refill();
        const uint32_t hdr = b.take(3);
        const bool final = hdr & 1;
        const uint32_t type = hdr >> 1;
        if (type == 0) {  // stored
            b.align();
            b.refill();
            const uint32_t len = b.take(16), nlen = b.take(16);
            if ((len ^ 0xFFFFu) != nlen) return fail("gzip data error: invalid stored block lengths");
            if (r.bytes)
                r.b8.reserve(r.n + len, r.off8, r.n);
            else
                r.s16.reserve(r.n + len, 0, r.n);
            for (uint32_t k = 0; k < len; k++) {
                b.refill();
                const uint32_t v = b.take(8);
                if (b.overrun()) return truncated();  // the bytes the input holds are output
                if (r.bytes)
                    r.b8.p[r.n++] = (uint8_t)v;
                else
                    r.s16.p[r.n++] = (uint16_t)v;
            }
        } else {
            const Huff* lit;
            const Huff* dist;
            if (type == 1) {
                lit = &fixed_lit();
                dist = &fixed_dist();
            } else if (type == 2) {
                if (!read_dynamic(b, dynLit, dynDist)) return fail("gzip data error: invalid block header");
                lit = &dynLit;
                dist = &dynDist;
            } else {
                return fail("gzip data error: invalid block type");
            }
            int rc;
            if (!r.bytes) {
                rc = decode_block<false>(b, lit, dist, r, mStart, lastMarker, estimate, !firstBlockOnly);
                if (rc == kSwitch) switch_to_bytes(r, estimate);
            }
            if (r.bytes) rc = decode_block<true>(b, lit, dist, r, mStart, lastMarker, estimate, false);
            if (rc == kError) return b.overrun() ? truncated() : false;
            if (rc == kTruncated) return truncated();
        }
        if (final) {  // the member's trailer, then another member or the end of the input
            b.align();
            const uint64_t at = b.bitpos() >> 3;
            if (at + 8 > n) return truncated();  // no trailer to check
            Trailer t;
            t.at = r.n;
            t.crc = (uint32_t)d[at] | (uint32_t)d[at + 1] << 8 | (uint32_t)d[at + 2] << 16 | (uint32_t)d[at + 3] << 24;
            t.isize = (uint32_t)d[at + 4] | (uint32_t)d[at + 5] << 8 | (uint32_t)d[at + 6] << 16 |
                      (uint32_t)d[at + 7] << 24;
            r.trailers.push_back(t);
            const size_t next = gzip_header(d, n, at + 8);
            if (!next) {  // anything but another gzip member ends the input (GzSource's rule)
                r.streamEnd = true;
                r.endBits = (at + 8) * 8;
                r.ok = true;
                return true;
            }
            b.init(d, n, (uint64_t)next * 8);
            mStart = (int64_t)r.n;
            if (b.bitpos() >= stopBits) {
                r.endsAtMemberStart = true;
                break;
            }
        }
    }
    r.endBits = b.bitpos();
    r.ok = true;
    return true;
}

// The first bit at or after `from` (and before `limit`) where a dynamic block header is complete
// and its first block decodes; UINT64_MAX if none.
uint64_t find_block(const uint8_t* d, size_t n, uint64_t from, uint64_t limit, Piece& scratch) {
    for (uint64_t p = from; p < limit; p++) {
        const size_t byte = p >> 3;
        if (byte + 8 > n) return UINT64_MAX;
        uint64_t w;
        memcpy(&w, d + byte, 8);
        w >>= (p & 7);
        // BFINAL 0, BTYPE 2 (bits 100), HLIT <= 29, HDIST <= 29
        if ((w & 7u) != 4u || ((w >> 3) & 31u) > 29u || ((w >> 8) & 31u) > 29u) continue;
        BitIn b;
        b.init(d, n, p + 3);
        Huff lit, dist;
        if (!read_dynamic(b, lit, dist)) continue;
        if (inflate_piece(d, n, p, UINT64_MAX, false, scratch, true)) return p;
    }
    return UINT64_MAX;
}

struct ParallelGzSource : ByteSource {
    const uint8_t* d = nullptr;
    size_t n = 0;
    uint64_t chunkBytes = 1u << 20;
    int nThreads = 2;
    uint64_t nChunks = 0;
    size_t deflateStart = 0;

    struct Task {
        uint64_t j;
        std::shared_ptr<Piece> piece;
        bool done = false;
    };
    struct Out {  // a resolved piece; its bytes (piece->b8) once the workers translated it
        std::shared_ptr<Piece> piece;
        std::vector<uint8_t> window;  // the 32 KB before the piece
        std::vector<uint64_t> segLen;  // segments split at the member ends
        std::vector<uint32_t> segCrc;
        bool done = false;
    };

    std::mutex mu;
    std::condition_variable cv;
    std::map<uint64_t, std::shared_ptr<Task>> decodes;  // chunk -> speculative decode
    std::deque<uint64_t> decodeQ;
    std::deque<std::shared_ptr<Out>> translateQ;
    std::deque<std::shared_ptr<Out>> ready;  // in stream order
    uint64_t nextChunk = 0;                  // the next chunk to queue for decoding
    bool stop = false, finished = false;
    std::string failure;
    std::vector<std::thread> workers;
    std::thread coord;
    std::vector<std::shared_ptr<Piece>> spare;  // consumed pieces, buffers kept (no fresh pages per chunk)

    std::shared_ptr<Piece> new_piece() {  // holds mu
        if (spare.empty()) return std::make_shared<Piece>();
        auto p = spare.back();
        spare.pop_back();
        return p;
    }

    // read() state
    std::shared_ptr<Out> cur;
    size_t curPos = 0;
    uint32_t memberCrc = 0;
    uint64_t memberLen = 0;

    ~ParallelGzSource() override {
        {
            std::lock_guard<std::mutex> l(mu);
            stop = true;
        }
        cv.notify_all();
        if (coord.joinable()) coord.join();
        for (auto& t : workers) t.join();
        if (d) munmap((void*)d, n);
    }

    size_t lookahead() const { return (size_t)nThreads * 2; }

    void start() {
        nChunks = (n + chunkBytes - 1) / chunkBytes;
        for (int i = 0; i < nThreads; i++)
            workers.emplace_back([this] {
                background_thread();
                work();
            });
        coord = std::thread([this] {
            background_thread();
            coordinate();
        });
    }

    void queue_decodes(uint64_t upTo) {  // holds mu
        while (nextChunk < nChunks && nextChunk < upTo) {
            if (nextChunk > 0) {  // chunk 0 is the coordinator's
                auto t = std::make_shared<Task>();
                t->j = nextChunk;
                t->piece = new_piece();
                decodes[nextChunk] = t;
                decodeQ.push_back(nextChunk);
            }
            nextChunk++;
        }
        cv.notify_all();
    }

    void work() {
        Piece scratch;
        while (true) {
            std::shared_ptr<Out> tr;
            std::shared_ptr<Task> dt;
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return stop || !translateQ.empty() || !decodeQ.empty(); });
                if (stop) return;
                if (!translateQ.empty()) {  // translations first: they feed the reader
                    tr = translateQ.front();
                    translateQ.pop_front();
                } else {
                    const uint64_t j = decodeQ.front();
                    decodeQ.pop_front();
                    auto it = decodes.find(j);
                    if (it == decodes.end()) continue;  // the coordinator is past this chunk
                    dt = it->second;
                }
            }
            if (tr) {
                translate(*tr);
                std::lock_guard<std::mutex> l(mu);
                tr->done = true;
                cv.notify_all();
                continue;
            }
            const uint64_t lo = dt->j * chunkBytes * 8, hi = (dt->j + 1) * chunkBytes * 8;
            const uint64_t p = find_block(d, n, lo, hi, scratch);
            if (p != UINT64_MAX) inflate_piece(d, n, p, hi, false, *dt->piece);
            std::lock_guard<std::mutex> l(mu);
            dt->done = true;
            cv.notify_all();
        }
    }

    // markers -> bytes with the piece's window, then CRC-32 per member segment
    void translate(Out& o) {
        Piece& p = *o.piece;
        const size_t sym = p.bytes ? p.off8 : p.n;  // [0, sym) are 16-bit symbols only
        if (!p.bytes) p.b8.reserve(p.n + 1, 0, 0);
        const uint16_t* s = p.s16.p.get();
        uint8_t* b = p.b8.p.get();
        const uint8_t* w = o.window.data();
        size_t i = 0;
        for (; i + 32 <= sym; i += 32) {  // runs without markers narrow in SIMD
            uint16_t any = 0;
            for (int q = 0; q < 32; q++) any |= s[i + q];
            if (any < 256) {
                for (int q = 0; q < 32; q++) b[i + q] = (uint8_t)s[i + q];
            } else {
                for (int q = 0; q < 32; q++) {
                    const uint16_t v = s[i + q];
                    b[i + q] = v < 256 ? (uint8_t)v : w[v - 256];
                }
            }
        }
        for (; i < sym; i++) {
            const uint16_t v = s[i];
            b[i] = v < 256 ? (uint8_t)v : w[v - 256];
        }
        uint64_t at = 0;
        for (size_t t = 0; t <= p.trailers.size(); t++) {
            const uint64_t e = t < p.trailers.size() ? p.trailers[t].at : p.n;
            o.segLen.push_back(e - at);
            o.segCrc.push_back(crc32_bytes(0, b + at, (size_t)(e - at)));
            at = e;
        }
    }

    void fail_all(const std::string& m) {
        std::lock_guard<std::mutex> l(mu);
        if (failure.empty()) failure = m;
        finished = true;
        cv.notify_all();
    }

    void coordinate() {
        uint64_t expected = (uint64_t)deflateStart * 8;
        bool atMember = true;
        std::vector<uint8_t> window(kWin, 0);
        while (true) {
            const uint64_t j = expected / (chunkBytes * 8);
            const uint64_t stopBits = (j + 1) * chunkBytes * 8;
            std::shared_ptr<Piece> piece;
            {
                std::unique_lock<std::mutex> l(mu);
                // keep the workers `lookahead` chunks ahead, without outrunning the reader
                cv.wait(l, [&] { return stop || ready.size() < lookahead(); });
                if (stop) return;
                queue_decodes(j + 1 + lookahead());
                for (auto it = decodes.begin(); it != decodes.end() && it->first < j;) it = decodes.erase(it);
                auto it = decodes.find(j);
                if (it != decodes.end()) {
                    auto t = it->second;
                    cv.wait(l, [&] { return stop || t->done; });
                    if (stop) return;
                    if (t->piece->ok && t->piece->startBits == expected) piece = t->piece;
                    decodes.erase(it);
                }
            }
            if (!piece) {  // chunk 0, or the speculative decode did not start at the true boundary
                {
                    std::lock_guard<std::mutex> l(mu);
                    piece = new_piece();
                }
                if (!inflate_piece(d, n, expected, stopBits, atMember, *piece)) {
                    fail_all(piece->err);
                    return;
                }
            }
            auto o = std::make_shared<Out>();
            o->piece = piece;
            o->window = window;
            // the next piece's window: the last kWin bytes of window + this piece
            std::vector<uint8_t> next(kWin);
            const size_t m = piece->n;
            const size_t fromPiece = std::min<size_t>(m, kWin);
            const size_t keep = kWin - fromPiece;
            memcpy(next.data(), window.data() + kWin - keep, keep);
            for (size_t i = 0; i < fromPiece; i++) next[keep + i] = piece->byte_at(m - fromPiece + i, window.data());
            window.swap(next);
            {
                std::lock_guard<std::mutex> l(mu);
                ready.push_back(o);
                translateQ.push_back(o);
                cv.notify_all();
            }
            if (piece->streamEnd) break;
            expected = piece->endBits;
            atMember = piece->endsAtMemberStart;
            if (expected >= (uint64_t)n * 8) break;  // the input ends at a block boundary: its end (GzSource's rule)
        }
        std::lock_guard<std::mutex> l(mu);
        finished = true;
        cv.notify_all();
    }

    long read(char* dst, size_t cap) override {
        size_t got = 0;
        while (got < cap) {
            if (!cur || curPos == cur->piece->n) {
                if (cur && !finish_piece()) return -1;
                std::unique_lock<std::mutex> l(mu);
                cur.reset();
                cv.wait(l, [&] { return !ready.empty() || finished; });
                if (ready.empty()) {
                    if (!failure.empty()) {
                        err = failure;
                        return -1;
                    }
                    break;
                }
                auto o = ready.front();
                cv.wait(l, [&] { return o->done; });
                ready.pop_front();
                cv.notify_all();
                cur = o;
                curPos = 0;
                continue;
            }
            const size_t k = std::min(cap - got, cur->piece->n - curPos);
            memcpy(dst + got, cur->piece->b8.p.get() + curPos, k);
            got += k;
            curPos += k;
        }
        return (long)got;
    }

    // A consumed piece's member checks: CRC-32 and ISIZE at each member end (zlib's gzip checks).
    bool finish_piece() {
        const Piece& p = *cur->piece;
        for (size_t s = 0; s < cur->segLen.size(); s++) {
            memberCrc = (uint32_t)crc32_combine(memberCrc, cur->segCrc[s], (z_off_t)cur->segLen[s]);
            memberLen += cur->segLen[s];
            if (s < p.trailers.size()) {
                if (p.trailers[s].crc != memberCrc) {
                    err = "gzip data error: incorrect data check";
                    return false;
                }
                if (p.trailers[s].isize != (uint32_t)memberLen) {
                    err = "gzip data error: incorrect length check";
                    return false;
                }
                memberCrc = 0;
                memberLen = 0;
            }
        }
        std::lock_guard<std::mutex> l(mu);
        if (spare.size() < lookahead()) spare.push_back(cur->piece);
        return true;
    }
};

}  // namespace

std::unique_ptr<ByteSource> open_parallel_gzip(const std::string& path, int threads, size_t chunkBytes,
                                               std::string& err) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) {
        err = "cannot open " + path;
        return nullptr;
    }
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size <= 0) {
        ::close(fd);
        err = "cannot read " + path;
        return nullptr;
    }
    void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) {
        err = "cannot map " + path;
        return nullptr;
    }
    madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
    auto s = std::make_unique<ParallelGzSource>();
    s->d = (const uint8_t*)m;
    s->n = (size_t)st.st_size;
    s->deflateStart = gzip_header(s->d, s->n, 0);
    if (!s->deflateStart) {
        err = "not a gzip file: " + path;
        return nullptr;
    }
    s->chunkBytes = std::max<size_t>(chunkBytes, 64);
    s->nThreads = std::max(1, threads);
    s->start();
    return s;
}

}  // namespace mtb
