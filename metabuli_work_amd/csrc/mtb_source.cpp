// Decompressed byte sources for the query files (mtb_io.h): plain, gzip (one thread, members in
// sequence) and BGZF (blocks inflated by a worker pool, returned in order), each optionally behind a
// prefetch thread. Replaces the serial kseq/gzread input of QueryIndexer.cpp:30-147 and
// KmerExtractor::loadChunkOfReads (KmerExtractor.cpp:442-494).
#include <dlfcn.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <zlib.h>

#include <condition_variable>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

#include "mtb_io.h"

namespace mtb {
namespace {

// libdeflate (the image's libdeflate.so.0, 1.10: whole-buffer inflate, ~2x zlib's rate) when it can
// be loaded, for BGZF members, which are whole gzip streams of known output size; zlib otherwise.
struct Libdeflate {
    void* (*alloc)() = nullptr;
    void (*free_)(void*) = nullptr;
    int (*gunzip)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
    uint32_t (*crc)(uint32_t, const void*, size_t) = nullptr;  // carry-less-multiply CRC-32
    Libdeflate() {
        if (getenv("MTB_NO_LIBDEFLATE")) return;  // A/B and the zlib path's tests
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (void* (*)())dlsym(h, "libdeflate_alloc_decompressor");
        free_ = (void (*)(void*))dlsym(h, "libdeflate_free_decompressor");
        gunzip = (int (*)(void*, const void*, size_t, void*, size_t, size_t*))dlsym(h, "libdeflate_gzip_decompress");
        crc = (uint32_t(*)(uint32_t, const void*, size_t))dlsym(h, "libdeflate_crc32");
        if (!alloc || !free_ || !gunzip) alloc = nullptr;
    }
    bool ok() const { return alloc != nullptr; }
};

const Libdeflate& libdeflate() {
    static const Libdeflate l;
    return l;
}

struct PlainSource : ByteSource {
    FILE* f = nullptr;
    ~PlainSource() override {
        if (f) fclose(f);
    }
    long read(char* dst, size_t cap) override {
        const size_t got = fread(dst, 1, cap, f);
        if (got == 0 && ferror(f)) {
            err = "read error";
            return -1;
        }
        return (long)got;
    }
};

// gzip / zlib streams, concatenated members included (inflateReset at each member's end).
struct GzSource : ByteSource {
    FILE* f = nullptr;
    z_stream zs{};
    bool init = false, done = false;
    std::vector<unsigned char> in;
    explicit GzSource(size_t bufBytes) : in(std::max<size_t>(bufBytes, 16)) {}
    ~GzSource() override {
        if (init) inflateEnd(&zs);
        if (f) fclose(f);
    }
    bool refill() {
        if (zs.avail_in > 0) return true;
        const size_t got = fread(in.data(), 1, in.size(), f);
        zs.next_in = in.data();
        zs.avail_in = (uInt)got;
        return got > 0;
    }
    // at least `k` input bytes buffered (the leftover moved to the front), unless the file ends first
    bool need(uInt k) {
        if (zs.avail_in >= k) return true;
        const uInt have = zs.avail_in;
        memmove(in.data(), zs.next_in, have);
        const size_t got = fread(in.data() + have, 1, in.size() - have, f);
        zs.next_in = in.data();
        zs.avail_in = (uInt)(have + got);
        return zs.avail_in >= k;
    }
    long read(char* dst, size_t cap) override {
        if (done) return 0;
        zs.next_out = reinterpret_cast<unsigned char*>(dst);
        zs.avail_out = (uInt)std::min<size_t>(cap, 1u << 30);
        const uInt want = zs.avail_out;
        while (zs.avail_out > 0) {
            if (!refill()) {
                done = true;  // end of file (a truncated member ends the input here, as gzread does)
                break;
            }
            const int rc = inflate(&zs, Z_NO_FLUSH);
            if (rc == Z_STREAM_END) {
                // another member may follow (multi-member gzip); anything else ends the input
                if (!need(2) || zs.next_in[0] != 0x1f || zs.next_in[1] != 0x8b) {
                    done = true;
                    break;
                }
                inflateReset(&zs);
            } else if (rc != Z_OK && rc != Z_BUF_ERROR) {
                err = std::string("gzip data error: ") + (zs.msg ? zs.msg : "inflate failed");
                return -1;
            }
        }
        return (long)(want - zs.avail_out);
    }
};

// BGZF: every member carries BSIZE (member length - 1) in a "BC" extra subfield and its
// uncompressed length in ISIZE, so members can be cut out of the file without inflating and
// inflated independently. A reader thread cuts groups of members, a pool inflates them, read()
// hands the groups' output back in file order.
struct BgzfSource : ByteSource {
    struct Group {
        std::vector<unsigned char> comp;
        std::vector<uint32_t> memberEnd;  // offsets into comp
        std::vector<char> out;
        bool ready = false;
        std::string err;
    };
    FILE* f = nullptr;
    int nThreads = 1;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::shared_ptr<Group>> pending;  // in file order, inflated or not
    std::deque<std::shared_ptr<Group>> work;     // not yet picked by a worker
    bool readerDone = false, stop = false;
    std::string readErr;
    std::vector<std::thread> threads;
    std::shared_ptr<Group> cur;
    size_t curPos = 0;

    size_t kGroupBytes = 4u << 20;  // compressed bytes per group (MTB_BGZF_GROUP: tests)
    size_t maxPending() const { return (size_t)nThreads * 3; }

    ~BgzfSource() override {
        {
            std::lock_guard<std::mutex> l(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : threads) t.join();
        if (f) fclose(f);
    }
    void start(int n) {
        nThreads = n < 1 ? 1 : n;
        threads.emplace_back([this] {
            background_thread();
            reader();
        });
        for (int i = 0; i < nThreads; i++)
            threads.emplace_back([this] {
                background_thread();
                worker();
            });
    }
    void reader() {
        std::vector<unsigned char> hdr(18);
        while (true) {
            auto g = std::make_shared<Group>();
            while (g->comp.size() < kGroupBytes) {
                const size_t got = fread(hdr.data(), 1, 18, f);
                if (got == 0) break;
                if (got < 18 || hdr[0] != 0x1f || hdr[1] != 0x8b || !(hdr[3] & 4) || hdr[12] != 'B' || hdr[13] != 'C') {
                    readErr = "malformed BGZF block";
                    break;
                }
                const uint32_t bsize = (uint32_t)hdr[16] | ((uint32_t)hdr[17] << 8);
                const size_t at = g->comp.size();
                g->comp.resize(at + bsize + 1);
                memcpy(g->comp.data() + at, hdr.data(), 18);
                if (fread(g->comp.data() + at + 18, 1, bsize + 1 - 18, f) != bsize + 1 - 18) {
                    readErr = "truncated BGZF block";
                    break;
                }
                g->memberEnd.push_back((uint32_t)g->comp.size());
            }
            std::unique_lock<std::mutex> l(mu);
            if (!g->memberEnd.empty()) {
                cv.wait(l, [&] { return stop || pending.size() < maxPending(); });
                if (stop) return;
                pending.push_back(g);
                work.push_back(g);
                cv.notify_all();
            }
            if (g->comp.size() < kGroupBytes || !readErr.empty()) {
                readerDone = true;
                cv.notify_all();
                return;
            }
        }
    }
    void worker() {
        z_stream zs{};
        inflateInit2(&zs, 16 + MAX_WBITS);
        const Libdeflate& ld = libdeflate();
        void* dec = ld.ok() ? ld.alloc() : nullptr;
        while (true) {
            std::shared_ptr<Group> g;
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return stop || !work.empty() || readerDone; });
                if (stop || (work.empty() && readerDone)) break;
                g = work.front();
                work.pop_front();
            }
            size_t total = 0, beg = 0;
            for (uint32_t e : g->memberEnd) {  // ISIZE: the member's last 4 bytes
                const unsigned char* t = g->comp.data() + e - 4;
                total += (size_t)t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
            }
            g->out.resize(total);
            size_t o = 0;
            for (uint32_t e : g->memberEnd) {
                const unsigned char* t = g->comp.data() + e - 4;
                if ((t[0] | t[1] | t[2] | t[3]) == 0) {  // ISIZE 0 (e.g. the EOF marker): no output to make
                    beg = e;
                    continue;
                }
                if (dec) {  // the member's output is exactly its ISIZE
                    const size_t isize = (size_t)t[0] | ((size_t)t[1] << 8) | ((size_t)t[2] << 16) | ((size_t)t[3] << 24);
                    size_t got = 0;
                    if (ld.gunzip(dec, g->comp.data() + beg, e - beg, g->out.data() + o, isize, &got) != 0 ||
                        got != isize) {
                        g->err = "BGZF block does not inflate";
                        break;
                    }
                    o += got;
                    beg = e;
                    continue;
                }
                inflateReset(&zs);
                zs.next_in = g->comp.data() + beg;
                zs.avail_in = (uInt)(e - beg);
                zs.next_out = reinterpret_cast<unsigned char*>(g->out.data() + o);
                zs.avail_out = (uInt)(total - o);
                const int rc = inflate(&zs, Z_FINISH);
                if (rc != Z_STREAM_END) {
                    g->err = "BGZF block does not inflate";
                    break;
                }
                o = total - zs.avail_out;
                beg = e;
            }
            g->out.resize(o);
            g->comp = std::vector<unsigned char>();
            {
                std::lock_guard<std::mutex> l(mu);
                g->ready = true;
            }
            cv.notify_all();
        }
        inflateEnd(&zs);
        if (dec) ld.free_(dec);
    }
    long read(char* dst, size_t cap) override {
        size_t n = 0;
        while (n < cap) {
            if (!cur || curPos == cur->out.size()) {
                std::unique_lock<std::mutex> l(mu);
                if (cur) {
                    pending.pop_front();
                    cv.notify_all();
                }
                cur.reset();
                curPos = 0;
                cv.wait(l, [&] { return !pending.empty() || readerDone; });
                if (pending.empty()) {
                    if (!readErr.empty()) {
                        err = readErr;
                        return -1;
                    }
                    break;
                }
                auto g = pending.front();
                cv.wait(l, [&] { return g->ready; });
                if (!g->err.empty()) {
                    err = g->err;
                    return -1;
                }
                cur = g;
                continue;
            }
            const size_t k = std::min(cap - n, cur->out.size() - curPos);
            memcpy(dst + n, cur->out.data() + curPos, k);
            n += k;
            curPos += k;
        }
        return (long)n;
    }
};

// A thread of its own reads ahead from the wrapped source in chunks (decompression overlaps the
// parsing that consumes them).
struct PrefetchSource : ByteSource {
    std::unique_ptr<ByteSource> inner;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::vector<char>> q;
    bool done = false, stop = false;
    std::string innerErr;
    std::thread t;
    std::vector<char> cur;
    size_t curPos = 0;
    static constexpr size_t kChunk = 16u << 20;
    static constexpr size_t kDepth = 4;

    explicit PrefetchSource(std::unique_ptr<ByteSource> s) : inner(std::move(s)) {
        t = std::thread([this] {
            background_thread();
            while (true) {
                std::vector<char> c(kChunk);
                const long got = inner->read(c.data(), c.size());
                std::unique_lock<std::mutex> l(mu);
                if (got < 0) innerErr = inner->err.empty() ? "read error" : inner->err;
                if (got <= 0) {
                    done = true;
                    cv.notify_all();
                    return;
                }
                c.resize((size_t)got);
                cv.wait(l, [&] { return stop || q.size() < kDepth; });
                if (stop) return;
                q.push_back(std::move(c));
                cv.notify_all();
            }
        });
    }
    ~PrefetchSource() override {
        {
            std::lock_guard<std::mutex> l(mu);
            stop = true;
        }
        cv.notify_all();
        t.join();
    }
    long read(char* dst, size_t cap) override {
        size_t n = 0;
        while (n < cap) {
            if (curPos == cur.size()) {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return !q.empty() || done; });
                if (q.empty()) {
                    if (!innerErr.empty()) {
                        err = innerErr;
                        return -1;
                    }
                    break;
                }
                cur = std::move(q.front());
                q.pop_front();
                curPos = 0;
                cv.notify_all();
                continue;
            }
            const size_t k = std::min(cap - n, cur.size() - curPos);
            memcpy(dst + n, cur.data() + curPos, k);
            n += k;
            curPos += k;
        }
        return (long)n;
    }
};

}  // namespace

void background_thread() {
    static const bool on = getenv("MTB_NICE") != nullptr;  // opt-in: not better in the e2e A/B
    if (!on) return;
    const id_t tid = (id_t)syscall(SYS_gettid);
    errno = 0;
    const int now = getpriority(PRIO_PROCESS, tid);
    if (errno == 0 && now < 19) setpriority(PRIO_PROCESS, tid, now + 5 > 19 ? 19 : now + 5);  // best effort
}

uint32_t crc32_bytes(uint32_t crc, const uint8_t* p, size_t n) {
    const Libdeflate& ld = libdeflate();
    if (ld.crc) return ld.crc(crc, p, n);
    return (uint32_t)crc32_z(crc, p, n);
}

std::unique_ptr<ByteSource> open_source(const std::string& path, int threads, bool prefetch, std::string& err) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) {
        err = "cannot open " + path;
        return nullptr;
    }
    unsigned char h[18] = {0};
    const size_t got = fread(h, 1, sizeof h, f);
    rewind(f);
    std::unique_ptr<ByteSource> s;
    const bool gz = got >= 2 && h[0] == 0x1f && h[1] == 0x8b;
    const bool bgzf = gz && got >= 18 && (h[3] & 4) && h[12] == 'B' && h[13] == 'C' && h[14] == 2;
    // test knobs: the gzip input buffer and the BGZF group size, so member / group boundaries can be
    // placed at buffer edges
    const char* gzBuf = getenv("MTB_GZ_BUFFER");
    const char* bgzfGroup = getenv("MTB_BGZF_GROUP");
    if (bgzf) {
        auto b = std::make_unique<BgzfSource>();
        b->f = f;
        if (bgzfGroup) b->kGroupBytes = std::max<size_t>(1, strtoull(bgzfGroup, nullptr, 10));
        b->start(threads);
        return b;  // the pool reads ahead already
    }
    if (gz) {
        // a file of several chunks with threads to spare inflates in parallel (MTB_GZ_SERIAL: the
        // one-thread zlib path; MTB_GZ_CHUNK: the chunk size, tests)
        const char* gzChunk = getenv("MTB_GZ_CHUNK");
        const size_t chunk = gzChunk ? strtoull(gzChunk, nullptr, 10) : (1u << 20);
        fseek(f, 0, SEEK_END);
        const long size = ftell(f);
        rewind(f);
        if (threads >= 2 && !getenv("MTB_GZ_SERIAL") && size > 0 && (size_t)size >= 4 * chunk) {
            fclose(f);
            return open_parallel_gzip(path, threads, chunk, err);
        }
        auto g = std::make_unique<GzSource>(gzBuf ? strtoull(gzBuf, nullptr, 10) : (4u << 20));
        g->f = f;
        if (inflateInit2(&g->zs, 15 + 32) != Z_OK) {
            err = "zlib init failed";
            return nullptr;
        }
        g->init = true;
        s = std::move(g);
    } else {
        auto p = std::make_unique<PlainSource>();
        p->f = f;
        s = std::move(p);
    }
    if (prefetch) return std::make_unique<PrefetchSource>(std::move(s));
    return s;
}

}  // namespace mtb
