// Classifier::startClassify (Classifier.cpp:44-164) as a native pipeline over files (SURVEY
// §8(f)1-2): the reference indexes the input in one serial pass (QueryIndexer.cpp:30-147), then
// re-reads it chunk by chunk on one thread (KmerExtractor.cpp:442-494) while the compute waits.
// Here four kinds of threads overlap:
//   * per mate file, a byte source (BGZF blocks inflated by a worker pool; gzip / plain read ahead),
//     a splitter cutting the bytes at record boundaries and a pool of parse workers turning each
//     cut into a block of up to kBlockReads records;
//   * an assembler filling pinned host batches (the copies split over kCopyThreads threads) (<= max_reads reads, <= max_bases bases: the
//     reference's RAM-bounded QuerySplits, QueryIndexer.cpp:62-67,132-137) and uploading each to
//     its device's buffers on that device's copy stream;
//   * per context (one per GPU) a worker running mtb_classify_batch on the uploaded batches
//     (MTB_INPUT_DEVICE): batch k goes to context k mod n — the reference's QuerySplit loop
//     (Classifier.cpp:81-133) spread over the GPUs of one node;
//   * a writer taking the classified batches back in batch order, formatting the per-read TSV
//     (Reporter.cpp:38-83) and counting reads per taxon for the report (Classifier.cpp:149,
//     Reporter.cpp:175-190), so the output is the one a single context writes.
// Batches rotate through kSlots slots per context, so on every GPU batch k+n is parsed and uploaded
// and batch k-n written while batch k runs.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>

#include "mtb_host.h"
#include "mtb_io.h"

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

template <typename T>
struct BoundedQueue {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<T> q;
    size_t cap;
    bool closed = false;
    explicit BoundedQueue(size_t c) : cap(c) {}
    bool push(T v) {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return closed || q.size() < cap; });
        if (closed) return false;
        q.push_back(std::move(v));
        cv.notify_all();
        return true;
    }
    bool pop(T& v) {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return closed || !q.empty(); });
        if (q.empty()) return false;
        v = std::move(q.front());
        q.pop_front();
        cv.notify_all();
        return true;
    }
    void close() {
        std::lock_guard<std::mutex> l(mu);
        closed = true;
        cv.notify_all();
    }
};

// First error of any thread (the C-ABI's error string is per thread: the caller's is set at the end).
struct ErrorBox {
    std::mutex mu;
    std::string msg;
    int code = MTB_OK;
    std::atomic<bool> failed{false};
    void set(int c, const std::string& m) {
        std::lock_guard<std::mutex> l(mu);
        if (code == MTB_OK) {
            code = c;
            msg = m;
        }
        failed = true;
    }
};

constexpr uint32_t kBlockReads = 8192;
// parsed jobs a mate may hold ahead of the assembler: two full batches (a batch of up to 2.6M
// 150-bp pairs is ~320 jobs of kBlockReads), so the splitter and the parsers run a batch ahead while
// the assembler fills and uploads one (160 — less than one 1.55M-pair batch — held the splitter in
// lockstep with the assembler: DESIGN §5 round 5). MTB_JOBS_AHEAD overrides it (A/B).
constexpr size_t kJobsAhead = 640;
static size_t jobs_ahead() {
    const char* e = getenv("MTB_JOBS_AHEAD");
    const long v = e ? atol(e) : 0;
    return v > 0 ? (size_t)v : kJobsAhead;
}
// and at most this many raw bytes per job (long reads: 8192 records would be ~80 MB a job)
constexpr size_t kJobBytes = 4u << 20;
constexpr int kSlots = 3;
constexpr uint64_t kRamp = 5;  // default batch size: the first kRamp batches ramp up from 1/32 of it
constexpr size_t kCopyThreads = 4;     // threads filling one pinned batch
constexpr unsigned kFormatThreads = 8;  // threads formatting one batch's TSV lines (MTB_FORMAT_THREADS)

struct RecordBlock {
    std::string names, seq;
    std::vector<uint64_t> noff{0}, off{0};
    uint32_t n = 0;
};

// A raw byte range of the input in memory, shared by the parse jobs cut from it.
struct RawBuf {
    std::unique_ptr<char[]> p;
    size_t cap;
    explicit RawBuf(size_t c) : p(new char[c]), cap(c) {}
};

// Whole records p[b, e) of a raw buffer, parsed into blk by a parse worker.
struct Mapping;

struct ParseJob {
    std::shared_ptr<void> raw;  // keeps the bytes alive: a raw buffer, or the file's mapping
    Mapping* map = nullptr;     // the mapping whose parts [b, e) this job holds (released after the parse)
    const char* data = nullptr;  // the job's records, [data, data + (e - b))
    size_t b = 0, e = 0;
    uint32_t recs = 0;  // as counted by the splitter
    RecordBlock blk;
    std::string err;
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    void reset() {
        raw.reset();
        map = nullptr;
        data = nullptr;
        b = e = 0;
        recs = 0;
        blk.n = 0;
        blk.seq.clear();  // the capacities stay: a recycled job's parse writes into warm memory
        blk.names.clear();
        blk.off.assign(1, 0);
        blk.noff.assign(1, 0);
        err.clear();
        done = false;
    }
    void finish() {
        {
            std::lock_guard<std::mutex> l(mu);
            done = true;
        }
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return done; });
    }
};

// A plain (uncompressed) query file mapped whole: the splitter cuts records in the page cache's
// own pages, with no read copy and no carried records. The mapping is given back in parts of partBytes
// bytes as soon as the splitter is past a part and the parse jobs reading it are done (their
// records are copied into blocks): the page-table teardown of a multi-GB mapping then runs on the
// parse workers during the run, not as one munmap after the last batch.
struct Mapping {
    // parts of 64 MB (MTB_MAP_PART=<bytes>, whole pages: tests cut small files into many parts)
    size_t partBytes = 64u << 20;
    const char* p = nullptr;
    size_t n = 0, parts = 0;
    std::unique_ptr<std::atomic<int>[]> refs;   // per part: its jobs + 1 while the splitter is not past it
    std::unique_ptr<std::atomic<bool>[]> gone;  // per part: unmapped
    void init() {
        if (const char* e = getenv("MTB_MAP_PART")) {
            const size_t page = (size_t)sysconf(_SC_PAGESIZE), v = strtoull(e, nullptr, 10);
            if (v) partBytes = (v + page - 1) / page * page;
        }
        parts = (n + partBytes - 1) / partBytes;
        refs.reset(new std::atomic<int>[parts]);
        gone.reset(new std::atomic<bool>[parts]);
        for (size_t c = 0; c < parts; c++) {
            refs[c] = 1;
            gone[c] = false;
        }
    }
    void drop(size_t c) {
        if (!gone[c].exchange(true)) munmap((void*)(p + c * partBytes), std::min(partBytes, n - c * partBytes));
    }
    void hold(size_t b, size_t e) {  // a job's bytes [b, e)
        for (size_t c = b / partBytes; c < parts && c * partBytes < e; c++) refs[c]++;
    }
    void release(size_t b, size_t e) {
        for (size_t c = b / partBytes; c < parts && c * partBytes < e; c++)
            if (--refs[c] == 0) drop(c);
    }
    void release_part(size_t c) {  // the splitter is past part c
        if (--refs[c] == 0) drop(c);
    }
    // a hold on part c only while it is still mapped (refs > 0), for the prefaulter
    bool try_hold(size_t c) {
        int r = refs[c].load();
        while (r > 0 && !refs[c].compare_exchange_weak(r, r + 1)) {
        }
        return r > 0;
    }
    ~Mapping() {
        for (size_t c = 0; c < parts; c++)
            if (!gone[c]) munmap((void*)(p + c * partBytes), std::min(partBytes, n - c * partBytes));
    }
};

// The mapping of a plain file; nullptr for gzip / BGZF (or a file that cannot be mapped).
std::shared_ptr<Mapping> map_plain(const char* path) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return nullptr;
    struct stat st;
    unsigned char magic[2] = {0, 0};
    std::shared_ptr<Mapping> m;
    if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && (st.st_size < 2 || pread(fd, magic, 2, 0) == 2) &&
        !(magic[0] == 0x1f && magic[1] == 0x8b)) {
        m = std::make_shared<Mapping>();
        m->n = (size_t)st.st_size;
        if (m->n) {
            void* p = mmap(nullptr, m->n, PROT_READ, MAP_PRIVATE, fd, 0);
            if (p == MAP_FAILED) {
                m.reset();
            } else {
                m->p = (const char*)p;
                m->init();
                madvise(p, m->n, MADV_SEQUENTIAL);
                madvise(p, m->n, MADV_WILLNEED);
            }
        }
    }
    close(fd);
    return m;
}

// What an idle object must not keep: a parse job that was never parsed (a stopped or failed run)
// still holds its raw buffer or the file's mapping, and its hold on the mapping's parts.
inline void on_idle(RawBuf&) {}
inline void on_idle(ParseJob& j) {
    if (j.map) j.map->release(j.b, j.e);
    j.map = nullptr;
    j.raw.reset();
}

// A free list of T: objects come back when their last shared_ptr goes, so the input's bytes flow
// through the same few buffers instead of freshly mapped (page-faulting) ones per chunk.
template <typename T>
struct Recycler : std::enable_shared_from_this<Recycler<T>> {
    std::mutex mu;
    std::vector<std::unique_ptr<T>> idle;
    // an idle object `fits` accepts (others are dropped: e.g. raw buffers of a smaller size kept
    // from an earlier run), else make()
    template <typename Make, typename Fits>
    std::shared_ptr<T> get(Make make, Fits fits) {
        std::unique_ptr<T> x;
        {
            std::lock_guard<std::mutex> l(mu);
            while (!idle.empty() && !x) {
                x = std::move(idle.back());
                idle.pop_back();
                if (!fits(*x)) x.reset();
            }
        }
        if (!x) x.reset(make());
        auto self = this->shared_from_this();
        return std::shared_ptr<T>(x.release(), [self](T* t) {
            on_idle(*t);
            std::lock_guard<std::mutex> l(self->mu);
            self->idle.emplace_back(t);
        });
    }
};

// One mate file, three stages:
//   * a reader thread filling recycled raw buffers from the byte source, past `head` bytes of
//     headroom at the front;
//   * a splitter moving the previous buffer's unfinished record into that headroom and cutting the
//     bytes at record boundaries into jobs of kBlockReads records (scan_records: a boundary pass
//     with next_record's semantics, no copying);
//   * a pool of parse workers filling the jobs' blocks (parse_records).
// `out` hands the jobs on in file order, each to be waited for. The reference parses every record
// on one thread (KmerExtractor.cpp:442-494).
struct MateReader {
    size_t head = 1u << 20;       // headroom for the unfinished record of the previous buffer
    size_t rawBytes = 32u << 20;  // raw buffer (MTB_PARSE_BUFFER: tests cut records at buffer ends)
    std::unique_ptr<mtb::ByteSource> src;
    BoundedQueue<std::shared_ptr<ParseJob>> out{jobs_ahead()}, work{jobs_ahead()};
    struct Chunk {
        std::shared_ptr<RawBuf> buf;
        size_t got = 0;  // bytes at buf->p + head
        bool eof = false;
    };
    BoundedQueue<Chunk> chunks{3};
    std::shared_ptr<Recycler<RawBuf>> raws = std::make_shared<Recycler<RawBuf>>();
    std::shared_ptr<Recycler<ParseJob>> jobs = std::make_shared<Recycler<ParseJob>>();
    std::thread t, reader;
    std::vector<std::thread> parsers;
    double sourceS = 0, scanS = 0;
    std::atomic<uint64_t> parseNs{0};
    std::string readErr;

    void read_loop(ErrorBox* eb) {
        while (!eb->failed) {
            Chunk c;
            c.buf = raws->get([&] { return new RawBuf(head + rawBytes); },
                              [&](const RawBuf& b) { return b.cap == head + rawBytes; });
            const auto r0 = Clock::now();
            while (c.got < rawBytes) {
                const long got = src->read(c.buf->p.get() + head + c.got, rawBytes - c.got);
                if (got < 0) {
                    readErr = src->err.empty() ? "read error" : src->err;
                    break;
                }
                if (got == 0) {
                    c.eof = true;
                    break;
                }
                c.got += (size_t)got;
            }
            sourceS += secs(r0, Clock::now());
            const bool last = c.eof;
            if (!readErr.empty() || !chunks.push(std::move(c)) || last) break;
        }
        chunks.close();
    }

    std::shared_ptr<Mapping> mapped;  // a plain file: split in place

    // The mapped file's page tables filled ahead of the splitter by a helper thread: on a fresh
    // mapping half of the splitter's scan time was page faults (a 1.25-GB tmpfs FASTQ: scan 0.151 s
    // cold, 0.079 s prefaulted). Parts of partBytes bytes, at most kAhead parts ahead of the splitter,
    // each under a hold so it cannot be unmapped while touched. MTB_PREFAULT=0 turns it off (A/B).
    static constexpr size_t kAhead = 4;
    std::atomic<size_t> splitPos{0};
    std::atomic<bool> splitDone{false};
    void prefault_loop() {
        const char* p = mapped->p;
        const size_t n = mapped->n;
        for (size_t c = 1; c < mapped->parts && !splitDone; c++) {  // part 0: the splitter's own first faults
            while (!splitDone && c > splitPos.load() / mapped->partBytes + kAhead) std::this_thread::sleep_for(std::chrono::microseconds(200));
            if (splitDone || (c + 1) * mapped->partBytes <= splitPos.load() || !mapped->try_hold(c)) continue;
            // page by page: MADV_POPULATE_READ over a part held the mapping's lock long enough to slow the
            // parsers, the batch assembly and the first batch (e2e plain 16.8-19.2 -> 14.4-15.8M pairs/s)
            const size_t b = c * mapped->partBytes, e = std::min(n, b + mapped->partBytes);
            volatile char sink = 0;
            for (size_t i = b; i < e; i += 4096) sink = sink + p[i];
            mapped->release(b, b + 1);
        }
    }

    // The mapped file's records cut into jobs (the whole file is in view: no carries).
    void split_mapped(ErrorBox* eb, std::string& err) {
        const char* p = mapped->p;
        const size_t n = mapped->n;
        size_t pos = 0, passed = 0;  // parts the splitter is past
        const char* pf = getenv("MTB_PREFAULT");
        std::thread prefaulter;
        if (!(pf && atoi(pf) == 0) && mapped->parts > 1)
            prefaulter = std::thread([this] {
                mtb::background_thread();
                prefault_loop();
            });
        struct Join {  // the prefaulter ends with the split, on every path out
            MateReader* r;
            std::thread& t;
            ~Join() {
                r->splitDone = true;
                if (t.joinable()) t.join();
            }
        } join{this, prefaulter};
        while (!eb->failed && pos < n) {
            splitPos = pos;
            uint32_t recs = 0;
            const auto s0 = Clock::now();
            const bool capped = n - pos > kJobBytes;
            size_t used = mtb::scan_records(p + pos, capped ? kJobBytes : n - pos, !capped, kBlockReads, &recs, err);
            if (recs == 0 && capped && err.empty())  // a record longer than the cap: the rest of the file
                used = mtb::scan_records(p + pos, n - pos, true, kBlockReads, &recs, err);
            scanS += secs(s0, Clock::now());
            if (!err.empty() || recs == 0) break;  // trailing blank lines (or an error)
            auto j = jobs->get([] { return new ParseJob(); }, [](const ParseJob&) { return true; });
            j->reset();
            j->raw = mapped;
            j->map = mapped.get();
            j->data = p + pos;
            j->b = pos;
            j->e = pos + used;
            j->recs = recs;
            mapped->hold(j->b, j->e);
            pos += used;
            for (; passed < mapped->parts && (passed + 1) * mapped->partBytes <= pos; passed++) mapped->release_part(passed);
            if (!out.push(j)) break;
            if (!work.push(j)) {
                j->err = "input stopped";
                j->finish();
                break;
            }
        }
        for (; passed < mapped->parts; passed++) mapped->release_part(passed);
    }

    void run(ErrorBox* eb, int nParsers) {
        mtb::background_thread();  // the splitter
        if (!mapped)
            reader = std::thread([this, eb] {
                mtb::background_thread();
                read_loop(eb);
            });
        for (int i = 0; i < nParsers; i++)
            parsers.emplace_back([this, eb] {
                mtb::background_thread();
                std::shared_ptr<ParseJob> j;
                while (work.pop(j)) {
                    const auto p0 = Clock::now();
                    if (!eb->failed) {
                        RecordBlock& b = j->blk;  // a record's sequence is under half its FASTQ bytes
                        b.seq.reserve((j->e - j->b) / 2 + 64);
                        b.off.reserve(j->recs + 1);
                        b.noff.reserve(j->recs + 1);
                        b.n = mtb::parse_records(j->data, j->e - j->b, b.seq, b.off, b.names, b.noff,
                                                 j->err);
                    }
                    if (j->map) j->map->release(j->b, j->e);  // its parts may be unmapped now
                    j->map = nullptr;
                    j->raw.reset();
                    parseNs += (uint64_t)(secs(p0, Clock::now()) * 1e9);
                    j->finish();
                }
            });
        std::string err;
        if (mapped) {
            split_mapped(eb, err);
            if (!err.empty()) eb->set(MTB_ERR_IO, err);
            work.close();
            for (auto& p : parsers) p.join();
            out.close();
            return;
        }
        std::shared_ptr<RawBuf> prev;  // holds the unfinished record [pos, end)
        size_t pos = 0, end = 0;
        bool stopped = false;
        Chunk c;
        while (!eb->failed && !stopped && chunks.pop(c)) {
            // the unfinished record goes in front of the new bytes: in the headroom, or (a record
            // longer than the headroom) into a buffer of its own
            const size_t rest = end - pos;
            std::shared_ptr<RawBuf> buf;
            size_t beg;
            if (rest <= head) {
                buf = c.buf;
                beg = head - rest;
                if (rest) memcpy(buf->p.get() + beg, prev->p.get() + pos, rest);
            } else {
                buf = std::make_shared<RawBuf>(rest + c.got + 1);
                beg = 0;
                memcpy(buf->p.get(), prev->p.get() + pos, rest);
                memcpy(buf->p.get() + rest, c.buf->p.get() + head, c.got);
                c.buf.reset();
            }
            prev.reset();
            pos = beg;
            end = beg + rest + c.got;
            while (!stopped) {
                uint32_t recs = 0;
                const auto s0 = Clock::now();
                bool capped = end - pos > kJobBytes;
                size_t used = mtb::scan_records(buf->p.get() + pos, capped ? kJobBytes : end - pos, c.eof && !capped,
                                                kBlockReads, &recs, err);
                if (recs == 0 && capped && err.empty()) {  // a record longer than the cap: the whole buffer
                    used = mtb::scan_records(buf->p.get() + pos, end - pos, c.eof, kBlockReads, &recs, err);
                    capped = false;
                }
                scanS += secs(s0, Clock::now());
                if (!err.empty() || recs == 0) {
                    pos += used;  // trailing blank lines at the end of the input
                    break;
                }
                auto j = jobs->get([] { return new ParseJob(); }, [](const ParseJob&) { return true; });
                j->reset();
                j->raw = buf;
                j->data = buf->p.get() + pos;
                j->b = pos;
                j->e = pos + used;
                j->recs = recs;
                pos += used;
                if (!out.push(j)) {
                    stopped = true;
                } else if (!work.push(j)) {
                    j->err = "input stopped";
                    j->finish();
                    stopped = true;
                }
                if (!capped && recs < kBlockReads) break;  // the buffer ends inside a record (or the input ends)
            }
            if (!err.empty() || c.eof) break;
            prev = buf;
        }
        prev.reset();
        chunks.close();  // a stopped splitter releases the reader
        reader.join();
        if (err.empty()) err = readErr;
        if (!err.empty()) eb->set(MTB_ERR_IO, err);
        work.close();
        for (auto& p : parsers) p.join();
        out.close();
    }
};

template <typename T>
struct Pinned {  // grow-only pinned host buffer
    T* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = n + n / 4 + 1024;
        hipError_t e = hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocPortable);
        if (e == hipSuccess) cap = want;
        return e;
    }
    ~Pinned() {
        if (p) hipHostFree(p);
    }
};

struct DevMem {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = bytes + bytes / 4 + 1024;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    ~DevMem() {
        if (p) hipFree(p);
    }
};

// A range-partitioned run's copy of a batch on a further context's device.
struct PeerIn {
    DevMem dseq1, dseq2, doff1, doff2;
    hipEvent_t uploaded = nullptr;
    int device = 0;
    ~PeerIn() {
        hipSetDevice(device);
        if (uploaded) hipEventDestroy(uploaded);
    }
};

struct Slot {
    int ctx = 0;             // the context (GPU) the slot's batches run on
    uint64_t index = 0;      // batch number in input order
    uint64_t firstRead = 0;  // run-wide index of the batch's first read (--em query IDs)
    int rc = MTB_OK;         // the batch's classify status
    std::string err;
    double gpuS = 0;
    double tReady = 0, tGpu0 = 0, tGpu1 = 0, tW0 = 0, tW1 = 0;  // MTB_PIPE_TRACE: seconds since the start
    float devMs = 0;     // MTB_PIPE_TRACE: the batch's device time (HIP events)
    uint64_t ws = 0;     // MTB_PIPE_TRACE: the context's workspace bytes after the batch
    std::vector<mtb_em_map> em;
    Pinned<uint64_t> off1, off2;
    std::string names;
    std::vector<uint64_t> noff;
    uint32_t n = 0;
    uint64_t bases = 0;
    DevMem dseq1, dseq2, doff1, doff2;
    hipEvent_t uploaded = nullptr;
    Pinned<mtb_result> res;  // pinned: the device-to-host copies run at full PCIe rate
    Pinned<mtb_taxcnt> tc;
    std::vector<std::unique_ptr<PeerIn>> peers;  // range-partitioned run: the batch on contexts 1..P-1
};

// Device-to-device copies of a range-partitioned run (the batch to the further parts' devices, the
// owners' match segments): hipMemcpyPeerAsync over xGMI where the two devices have peer access, else
// staged through a pinned host buffer, chunk by chunk and synchronously (a node without peer access
// between some pair still runs; MTB_PEER_COPY=host forces the staging for every pair, same device
// included: the GPU tests exercise it on cuda:0). Decided once per run, logged once per pair.
struct PeerLinks {
    int n = 0;
    std::vector<int> dev;
    std::vector<char> direct;  // [a * n + b]: a copy from context b's device to context a's is a peer copy
    bool forced = false;
    void init(mtb_ctx* const* ctxs, int nCtx) {
        n = nCtx;
        dev.resize(n);
        for (int a = 0; a < n; a++) dev[a] = mtb_ctx_device(ctxs[a]);
        const char* e = getenv("MTB_PEER_COPY");
        forced = e && !strcmp(e, "host");
        direct.assign((size_t)n * n, 1);
        for (int a = 0; a < n; a++)
            for (int b = 0; b < n; b++) {
                if (forced) { direct[a * n + b] = 0; continue; }
                if (dev[a] == dev[b]) continue;  // a device copy on one GPU
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, dev[a], dev[b]) != hipSuccess) can = 0;
                if (can) {
                    hipSetDevice(dev[a]);
                    const hipError_t r = hipDeviceEnablePeerAccess(dev[b], 0);
                    if (r != hipSuccess && r != hipErrorPeerAccessAlreadyEnabled) can = 0;
                    (void)hipGetLastError();
                }
                direct[a * n + b] = (char)can;
                if (!can)
                    fprintf(stderr, "[mtb] no peer access from GPU %d to GPU %d: their copies are staged through host "
                                    "memory\n", dev[a], dev[b]);
            }
        if (forced) fprintf(stderr, "[mtb] MTB_PEER_COPY=host: every device-to-device copy staged through host memory\n");
    }
    // bytes from context b's device memory to context a's; st: a stream of a's device (peer copies
    // are queued on it; the staged path returns with the copy done)
    bool copy(int a, void* dst, int b, const void* src, size_t bytes, hipStream_t st) const {
        if (!bytes) return true;
        if (direct[a * n + b]) return hipMemcpyPeerAsync(dst, dev[a], src, dev[b], bytes, st) == hipSuccess;
        constexpr size_t kBounce = 64u << 20;
        // one pinned buffer per copying thread, freed when the thread ends (a run's workers end with it;
        // thread-storage objects of the main thread go before the runtime's static teardown)
        struct Bounce {
            char* p = nullptr;
            ~Bounce() {
                if (p) (void)hipHostFree(p);
            }
        };
        thread_local Bounce tb;
        if (!tb.p && hipHostMalloc((void**)&tb.p, kBounce, hipHostMallocDefault) != hipSuccess) {
            tb.p = nullptr;
            return false;
        }
        char* const bounce = tb.p;
        if (hipStreamSynchronize(st) != hipSuccess) return false;  // earlier work on st first
        for (size_t off = 0; off < bytes; off += kBounce) {
            const size_t len = std::min(kBounce, bytes - off);
            if (hipSetDevice(dev[b]) != hipSuccess ||
                hipMemcpy(bounce, (const char*)src + off, len, hipMemcpyDeviceToHost) != hipSuccess ||
                hipSetDevice(dev[a]) != hipSuccess ||
                hipMemcpyAsync((char*)dst + off, bounce, len, hipMemcpyHostToDevice, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return false;
        }
        return true;
    }
};

// Threads of a range-partitioned run meeting once per step of a batch (C++17: no std::barrier).
struct Barrier {
    std::mutex mu;
    std::condition_variable cv;
    int n, waiting = 0;
    uint64_t gen = 0;
    explicit Barrier(int k) : n(k) {}
    void wait() {
        std::unique_lock<std::mutex> l(mu);
        const uint64_t g = gen;
        if (++waiting == n) {
            waiting = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(l, [&] { return gen != g; });
        }
    }
};

// One batch of a range-partitioned run, shared by the P partition
// workers: every context matches the whole piece against its DB part (MTB_MATCH_ONLY), the
// per-read match segments go to the owner of their reads (owner p: reads [lo + k p / P, lo + k (p+1) / P)
// of a k-read piece) by device-to-device / peer copies, and each owner scores its reads with
// mtb_assign_chunks. Pieces halve when a context runs out of HBM, as whole batches do.
struct PartBatch {
    explicit PartBatch(int P) : bar(P), rc(P), err(P), mOff(P), m(P), cnt(P), ql(P), tc(P) {}
    Barrier bar;
    std::deque<std::pair<uint32_t, uint32_t>> pieces;
    std::vector<int> rc;
    std::vector<std::string> err;
    std::vector<std::vector<uint64_t>> mOff;
    std::vector<const mtb_match*> m;
    std::vector<const uint32_t*> cnt, ql;
    std::vector<std::vector<mtb_taxcnt>> tc;
    std::vector<mtb_taxcnt> all;
    uint32_t cap = 0;  // the piece size that fitted (bounds later batches)
    bool split = false;
    int fail = MTB_OK;
    std::string failMsg;
};

// An owner's staging on its device: the chunks of its reads' matches from every part, their
// per-read counts, its reads' query lengths.
struct OwnerStage {
    DevMem m, cnt, ql;
    hipStream_t st = nullptr;
};

// One assembler copy thread's staging towards a context's device: two pinned chunks (one filled
// while the other uploads) on a stream of its own. A batch's bases go to HBM through these chunks
// instead of a pinned copy of the whole batch, so a run pins kCopyThreads x 2 x kStageChunk bytes
// once per context (a whole-batch pinned slot was ~1.2 GB per mate at 3.5M-pair batches, pinned
// step by step through the batch-size ramp of a context's first run).
constexpr size_t kStageChunk = 8u << 20;
struct Stager {
    int device = 0;
    char* buf[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    hipStream_t st = nullptr;
    int k = 0;  // the buffer filled next
    bool init(int dev) {
        if (st) return true;
        device = dev;
        if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return false;
        for (int i = 0; i < 2; i++)
            if (hipHostMalloc((void**)&buf[i], kStageChunk, hipHostMallocDefault) != hipSuccess ||
                hipEventCreateWithFlags(&done[i], hipEventDisableTiming) != hipSuccess)
                return false;
        return true;
    }
    ~Stager() {
        hipSetDevice(device);
        if (st) hipStreamSynchronize(st);
        for (int i = 0; i < 2; i++) {
            if (buf[i]) hipHostFree(buf[i]);
            if (done[i]) hipEventDestroy(done[i]);
        }
        if (st) hipStreamDestroy(st);
    }
};

// A context's slots, kept between runs (mtb::ctx_pipeline_cache): their pinned host buffers and
// device input buffers are grown once, not re-pinned (hipHostMalloc) batch by batch every run.
struct SlotPool {
    int device = 0;
    std::vector<std::unique_ptr<Slot>> slots;
    std::unique_ptr<Stager> stagers[kCopyThreads];  // the assembler's copy threads towards this device
    // the mates' raw buffers and parse jobs (warm host memory instead of freshly faulted pages)
    std::shared_ptr<Recycler<RawBuf>> raws[2] = {std::make_shared<Recycler<RawBuf>>(),
                                                 std::make_shared<Recycler<RawBuf>>()};
    std::shared_ptr<Recycler<ParseJob>> jobs[2] = {std::make_shared<Recycler<ParseJob>>(),
                                                   std::make_shared<Recycler<ParseJob>>()};
    ~SlotPool() {
        hipSetDevice(device);
        for (auto& s : slots)
            if (s->uploaded) hipEventDestroy(s->uploaded);
        slots.clear();  // the buffers are freed on the context's device
        for (auto& g : stagers) g.reset();
    }
};

// Reads of one mate's current block, consumed from `at`.
struct Cursor {
    std::shared_ptr<RecordBlock> b;
    uint32_t at = 0;
    bool next(MateReader& m, ErrorBox& eb) {
        if (b && at < b->n) return true;
        at = 0;
        std::shared_ptr<ParseJob> j;
        while (m.out.pop(j)) {
            j->wait();
            if (!j->err.empty()) {
                eb.set(MTB_ERR_IO, j->err);
                return false;
            }
            if (!j->blk.n) continue;
            b = std::shared_ptr<RecordBlock>(j, &j->blk);
            return true;
        }
        b.reset();
        return false;
    }
};

// One uploaded batch on its context: results into s->res, its taxID:count lists into s->tc, its
// --em mappings into s->em. A batch whose workspace does not fit (MTB_RETRY: out of HBM) is
// classified in halves, recursively down to one read, as the reference searches a split again
// after its match buffer ran out (Classifier.cpp:127-130); the piece size that fitted bounds the
// context's later batches (cap, as matchPerKmer stays raised). Pieces are read ranges of the
// uploaded batch (the offsets stay absolute), their lists appended with rebased offsets.
static int classify_piece(mtb_ctx* c, Slot* s, bool paired, uint32_t lo, uint32_t hi) {
    return mtb_classify_batch(c, (const char*)s->dseq1.p, (const uint64_t*)s->doff1.p + lo,
                              paired ? (const char*)s->dseq2.p : nullptr,
                              paired ? (const uint64_t*)s->doff2.p + lo : nullptr, hi - lo, MTB_INPUT_DEVICE,
                              s->res.p + lo);
}

static int piece_mappings(mtb_ctx* c, Slot* s, uint32_t lo) {
    uint64_t nm = 0;
    int rc = mtb_get_em_mappings(c, (uint32_t)(s->firstRead + lo), nullptr, 0, &nm);
    if (rc == MTB_RETRY || (rc == MTB_OK && nm)) {
        const size_t at = s->em.size();
        s->em.resize(at + nm);
        rc = mtb_get_em_mappings(c, (uint32_t)(s->firstRead + lo), s->em.data() + at, nm, &nm);
    }
    return rc;
}

static int classify_slot(mtb_ctx* c, Slot* s, bool paired, bool em, uint32_t& cap, std::atomic<uint64_t>& split) {
    if (!cap || s->n <= cap) {  // the whole batch at once (the usual case)
        int rc = classify_piece(c, s, paired, 0, s->n);
        if (rc == MTB_OK) {
            uint64_t nt = 0;
            mtb_get_taxcnt(c, nullptr, 0, &nt);
            rc = s->tc.ensure(std::max<uint64_t>(nt, 1)) == hipSuccess ? mtb_get_taxcnt(c, s->tc.p, s->tc.cap, &nt)
                                                                     : MTB_ERR_OOM;
            if (rc == MTB_OK && em) rc = piece_mappings(c, s, 0);
            return rc;
        }
        if (rc != MTB_RETRY || s->n < 2) return rc == MTB_RETRY ? MTB_ERR_OOM : rc;
        cap = s->n / 2;
        fprintf(stderr, "[mtb] batch %llu: %s; classifying it in pieces of <= %u reads\n",
                (unsigned long long)s->index, mtb_last_error(), cap);
    }
    split++;
    std::deque<std::pair<uint32_t, uint32_t>> todo;
    for (uint32_t lo = 0; lo < s->n; lo += cap) todo.push_back({lo, std::min<uint32_t>(s->n, lo + cap)});
    std::vector<mtb_taxcnt> tc;
    while (!todo.empty()) {
        const uint32_t lo = todo.front().first, hi = todo.front().second;
        int rc = classify_piece(c, s, paired, lo, hi);
        if (rc == MTB_RETRY && hi - lo > 1) {  // halve the piece, and every later one
            const uint32_t mid = lo + (hi - lo) / 2;
            todo.pop_front();
            todo.push_front({mid, hi});
            todo.push_front({lo, mid});
            if (mid - lo < cap) {
                cap = mid - lo;
                fprintf(stderr, "[mtb] batch %llu: %s; pieces of <= %u reads\n", (unsigned long long)s->index,
                        mtb_last_error(), cap);
            }
            continue;
        }
        if (rc != MTB_OK) return rc == MTB_RETRY ? MTB_ERR_OOM : rc;
        todo.pop_front();
        uint64_t nt = 0;
        mtb_get_taxcnt(c, nullptr, 0, &nt);
        const size_t at = tc.size();
        tc.resize(at + nt);
        rc = mtb_get_taxcnt(c, tc.data() + at, nt, &nt);
        if (rc != MTB_OK) return rc;
        for (uint32_t i = lo; i < hi; i++) s->res.p[i].taxcnt_offset += (uint32_t)at;
        if (em && (rc = piece_mappings(c, s, lo)) != MTB_OK) return rc;
    }
    if (s->tc.ensure(std::max<size_t>(tc.size(), 1)) != hipSuccess) return MTB_ERR_OOM;
    std::copy(tc.begin(), tc.end(), s->tc.p);
    return MTB_OK;
}

}  // namespace

static int start_classify(mtb_ctx* const* ctxs, int nCtx, const mtb_classify_opts* opt, mtb_classify_stats* stats,
                          bool partitioned);

extern "C" int mtb_start_classify(mtb_ctx* ctx, const mtb_classify_opts* opt, mtb_classify_stats* stats) {
    return start_classify(&ctx, 1, opt, stats, false);
}

extern "C" int mtb_start_classify_multi(mtb_ctx* const* ctxs, int nCtx, const mtb_classify_opts* opt,
                                        mtb_classify_stats* stats) {
    return start_classify(ctxs, nCtx, opt, stats, false);
}

extern "C" int mtb_start_classify_partitioned(mtb_ctx* const* ctxs, int nCtx, const mtb_classify_opts* opt,
                                              mtb_classify_stats* stats) {
    return start_classify(ctxs, nCtx, opt, stats, true);
}

static int start_classify(mtb_ctx* const* ctxs, int nCtx, const mtb_classify_opts* opt, mtb_classify_stats* stats,
                          bool partitioned) {
    using mtb::set_error;
    if (!ctxs || nCtx < 1 || !opt || !opt->query1 || !opt->out_tsv) {
        set_error("null argument");
        return MTB_ERR_ARG;
    }
    for (int d = 0; d < nCtx; d++)
        if (!ctxs[d]) {
            set_error("null context");
            return MTB_ERR_ARG;
        }
    for (int d = 0; d < nCtx; d++)
        for (int e = 0; e < d; e++)
            if (ctxs[d] == ctxs[e]) {
                set_error("a context is listed twice");
                return MTB_ERR_ARG;
            }
    mtb_ctx* const ctx0 = ctxs[0];  // the writers' taxonomy, the report and --em
    // every context must classify a batch as ctx0 would: the same parameters (host threads aside)
    // over the whole of the same DB
    std::vector<bool> partSeen(nCtx, false);
    for (int d = 0; d < nCtx; d++) {
        mtb_params a = mtb::ctx_params(ctxs[d]), b = mtb::ctx_params(ctx0);
        if (!partitioned && a.db_parts > 1) {
            set_error("a context holds one part of a range-partitioned DB: use mtb_start_classify_partitioned");
            return MTB_ERR_ARG;
        }
        if (partitioned) {  // one context per part, each part once
            if (a.db_parts != nCtx || a.db_part < 0 || a.db_part >= nCtx || partSeen[a.db_part]) {
                set_error("mtb_start_classify_partitioned needs one context per DB part (db_parts = n_ctx)");
                return MTB_ERR_ARG;
            }
            partSeen[a.db_part] = true;
            a.db_part = b.db_part = 0;
        }
        a.threads = b.threads = 0;
        if (memcmp(&a, &b, sizeof a) != 0 || (!partitioned && mtb_db_kmers(ctxs[d]) != mtb_db_kmers(ctx0))) {
            set_error("the contexts differ in their parameters or DB: batches would be classified differently");
            return MTB_ERR_ARG;
        }
    }
    if (partitioned && nCtx < 2) {
        set_error("a range-partitioned run needs >= 2 contexts");
        return MTB_ERR_ARG;
    }
    const auto t0 = Clock::now();
    const bool paired = opt->query2 != nullptr;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int threads = opt->threads > 0 ? opt->threads : (int)std::min(16u, hw);
    // default: up to 4M reads a batch, in practice bounded by max_bases (from free HBM: ~2M pairs
    // beside a GTDB-scale DB), reached through a ramp of kRamp batches from 1/32 of it
    const uint32_t maxReads = opt->max_reads ? opt->max_reads : 4000000u;
    uint64_t maxBases = opt->max_bases;
    if (!maxBases) {  // ~90 device bytes of workspace per base at GTDB scale; slots < 2^31
        // per device: its free HBM plus what its contexts' grow-only workspaces already hold (their
        // next batches reuse it), shared by those contexts; 3/4 of a share for a context's batch
        std::map<int, std::pair<uint64_t, int>> avail;  // device -> (bytes, contexts)
        for (int d = 0; d < nCtx; d++) {
            const int dev = mtb_ctx_device(ctxs[d]);
            if (!avail.count(dev)) {
                size_t freeB = 0, totalB = 0;
                if (hipSetDevice(dev) != hipSuccess || hipMemGetInfo(&freeB, &totalB) != hipSuccess) {
                    set_error("cannot query device memory");
                    return MTB_ERR_HIP;
                }
                avail[dev] = {freeB, 0};
            }
            avail[dev].first += mtb::ctx_workspace_bytes(ctxs[d]);
            avail[dev].second++;
        }
        maxBases = 1ull << 30;
        for (auto& kv : avail)
            maxBases = std::min<uint64_t>(maxBases, (uint64_t)(0.75 * (double)kv.second.first / kv.second.second / 95.0));
        maxBases = std::max<uint64_t>(maxBases, 1ull << 20);
        // a context holding more than its share (e.g. grown by larger batches before) gives it back
        for (int d = 0; d < nCtx; d++) {
            const auto& a = avail[mtb_ctx_device(ctxs[d])];
            if (a.second > 1 && mtb::ctx_workspace_bytes(ctxs[d]) > a.first / a.second) mtb::ctx_release_workspace(ctxs[d]);
        }
    }
    ErrorBox eb;
    MateReader m1, m2;
    const int srcThreads = std::max(1, paired ? threads / 2 : threads);
    const int parseThreads = std::max(2, srcThreads / 2);  // per mate
    {
        std::string err;
        // plain files are mapped and split in place; compressed ones read through a byte source (no
        // prefetch thread: the reader thread of each MateReader reads ahead into recycled buffers)
        if (!getenv("MTB_NO_MMAP")) {
            m1.mapped = map_plain(opt->query1);
            if (paired) m2.mapped = map_plain(opt->query2);
        }
        if ((!m1.mapped && !(m1.src = mtb::open_source(opt->query1, srcThreads, false, err))) ||
            (paired && !m2.mapped && !(m2.src = mtb::open_source(opt->query2, srcThreads, false, err)))) {
            set_error(err);
            return MTB_ERR_IO;
        }
    }
    // per context: kSlots slots (kept in the context between runs), a copy stream on its device,
    // free and ready queues
    std::vector<Slot*> slotMem;
    PeerLinks links;  // range-partitioned run: peer copies or host-staged ones, per pair of contexts
    if (partitioned) links.init(ctxs, nCtx);
    std::vector<hipStream_t> up(nCtx, nullptr);
    std::vector<std::unique_ptr<BoundedQueue<Slot*>>> freeQ, readyQ;
    for (int d = 0; d < nCtx; d++) {
        if (hipSetDevice(mtb_ctx_device(ctxs[d])) != hipSuccess ||
            hipStreamCreateWithFlags(&up[d], hipStreamNonBlocking) != hipSuccess) {
            for (int e = 0; e < d; e++) hipStreamDestroy(up[e]);
            set_error("cannot create the upload stream");
            return MTB_ERR_HIP;
        }
        freeQ.emplace_back(new BoundedQueue<Slot*>(kSlots));
        readyQ.emplace_back(new BoundedQueue<Slot*>(kSlots));
        std::shared_ptr<void>& cache = mtb::ctx_pipeline_cache(ctxs[d]);
        if (!cache) {
            auto pool = std::make_shared<SlotPool>();
            pool->device = mtb_ctx_device(ctxs[d]);
            for (int k = 0; k < kSlots; k++) {
                pool->slots.emplace_back(new Slot());
                hipEventCreateWithFlags(&pool->slots.back()->uploaded, hipEventDisableTiming);
            }
            cache = pool;
        }
        for (auto& x : std::static_pointer_cast<SlotPool>(cache)->slots) {
            Slot* s = x.get();
            s->ctx = d;
            slotMem.push_back(s);
            freeQ[d]->push(s);
        }
    }
    BoundedQueue<Slot*> writeQ(slotMem.size() + 1);
    std::map<int, std::unique_ptr<std::mutex>> growMu;  // per device: workspace growth runs alone
    for (int d = 0; d < nCtx; d++)
        if (!growMu.count(mtb_ctx_device(ctxs[d]))) growMu[mtb_ctx_device(ctxs[d])].reset(new std::mutex());

    {  // the mates' buffers come from the first context's pool
        auto pool = std::static_pointer_cast<SlotPool>(mtb::ctx_pipeline_cache(ctx0));
        m1.raws = pool->raws[0];
        m1.jobs = pool->jobs[0];
        m2.raws = pool->raws[1];
        m2.jobs = pool->jobs[1];
    }
    if (const char* e = getenv("MTB_PARSE_BUFFER")) {  // tests: records straddle buffers and outgrow the headroom
        m1.rawBytes = m2.rawBytes = std::max<size_t>(1, strtoull(e, nullptr, 10));
        m1.head = m2.head = std::min(m1.head, m1.rawBytes);
    }
    m1.t = std::thread([&] { m1.run(&eb, parseThreads); });
    if (paired) m2.t = std::thread([&] { m2.run(&eb, parseThreads); });

    // MTB_PIPE_TRACE=<file> (experiments): one line per batch with its stage times
    FILE* trace = getenv("MTB_PIPE_TRACE") ? fopen(getenv("MTB_PIPE_TRACE"), "a") : nullptr;
    // assembler: blocks -> pinned batches -> device buffers of context (batch mod n)
    double fillS = 0, firstBatchS = 0;
    std::thread assembler([&] {
        Cursor c1, c2;
        bool end = false;
        uint64_t index = 0, firstRead = 0;
        while (!end && !eb.failed) {
            const int d = partitioned ? 0 : (int)(index % (uint64_t)nCtx);  // partitioned: every context, via ctx0's slots
            Slot* s = nullptr;
            if (!freeQ[d]->pop(s)) break;
            s->n = 0;
            s->bases = 0;
            s->names.clear();
            s->noff.assign(1, 0);
            uint64_t b1 = 0, b2 = 0;
            std::vector<std::pair<std::shared_ptr<RecordBlock>, std::pair<uint32_t, uint32_t>>> take1, take2;
            // which reads go in: whole block stretches until max_reads / max_bases
            static const char* kUnequal = "paired-end inputs have different read counts (QueryIndexer.cpp:121-124)";
            // with the default batch size the first batches ramp up (1/32 ... 1/2 of it): the GPU
            // starts after a small parse instead of a full batch's; a read's result does not depend
            // on its batch
            const uint32_t cap = !opt->max_reads && index < kRamp ? std::max<uint32_t>(1, maxReads >> (kRamp - index)) : maxReads;
            while (s->n < cap) {
                const bool more1 = c1.next(m1, eb);
                const bool more2 = paired && c2.next(m2, eb);
                if (eb.failed) {
                    end = true;
                    break;
                }
                if (!more1 || (paired && !more2)) {
                    if (more1 || more2) eb.set(MTB_ERR_IO, kUnequal);
                    end = true;
                    break;
                }
                // the mates' blocks may be cut at different reads: take the stretch both still hold
                const RecordBlock& x = *c1.b;
                const uint32_t lim = paired ? std::min(x.n, c1.at + (c2.b->n - c2.at)) : x.n;
                uint32_t k = c1.at;
                while (k < lim && s->n + (k - c1.at) < cap) {
                    uint64_t len = x.off[k + 1] - x.off[k];
                    if (paired) len += c2.b->off[c2.at + (k - c1.at) + 1] - c2.b->off[c2.at + (k - c1.at)];
                    if (s->bases + len > maxBases && s->n + (k - c1.at) > 0) break;
                    s->bases += len;
                    k++;
                }
                const uint32_t got = k - c1.at;
                if (got == 0) break;  // the bases budget is full
                take1.push_back({c1.b, {c1.at, k}});
                b1 += x.off[k] - x.off[c1.at];
                if (paired) {
                    take2.push_back({c2.b, {c2.at, c2.at + got}});
                    b2 += c2.b->off[c2.at + got] - c2.b->off[c2.at];
                    c2.at += got;
                }
                s->n += got;
                c1.at = k;
                if (s->bases >= maxBases) break;
            }
            if (eb.failed || s->n == 0) {
                freeQ[d]->push(s);
                break;
            }
            const auto f0 = Clock::now();
            // the blocks' stretches are copied into the pinned batch by a few threads at once
            struct Piece {
                const RecordBlock* b;
                uint32_t lo, hi, r;  // r: the batch index of read lo
                uint64_t seqAt, nameAt;
                int mate;
            };
            std::vector<Piece> pieces;
            uint64_t nameBytes = 0;
            for (int mate = 0; mate < (paired ? 2 : 1); mate++) {
                uint64_t at = 0;
                uint32_t r = 0;
                for (auto& tk : mate ? take2 : take1) {
                    const RecordBlock& b = *tk.first;
                    const uint32_t lo = tk.second.first, hi = tk.second.second;
                    pieces.push_back({&b, lo, hi, r, at, nameBytes, mate});
                    at += b.off[hi] - b.off[lo];
                    r += hi - lo;
                    if (!mate) nameBytes += b.noff[hi] - b.noff[lo];
                }
            }
            if (s->off1.ensure((size_t)s->n + 1) != hipSuccess ||
                (paired && s->off2.ensure((size_t)s->n + 1) != hipSuccess)) {
                eb.set(MTB_ERR_OOM, "cannot allocate pinned host batch buffers");
                freeQ[d]->push(s);
                break;
            }
            s->names.resize(nameBytes);
            s->noff.resize((size_t)s->n + 1);
            s->off1.p[0] = 0;
            if (paired) s->off2.p[0] = 0;
            // the slot's device buffers live on its context's device (a new thread starts on device 0);
            // growing them frees the smaller ones, and hipFree waits for the whole device: not while
            // another context's batch runs there (growMu)
            const int dev = mtb_ctx_device(ctxs[d]);
            const size_t on = sizeof(uint64_t) * ((size_t)s->n + 1);
            bool ok = true;
            {
                std::unique_lock<std::mutex> gl(*growMu.at(dev), std::defer_lock);
                if (s->dseq1.cap < b1 + 1 || s->doff1.cap < on || (paired && (s->dseq2.cap < b2 + 1 || s->doff2.cap < on)))
                    gl.lock();
                ok = hipSetDevice(dev) == hipSuccess && s->dseq1.ensure(b1 + 1) == hipSuccess &&
                     s->doff1.ensure(on) == hipSuccess &&
                     (!paired || (s->dseq2.ensure(b2 + 1) == hipSuccess && s->doff2.ensure(on) == hipSuccess));
            }
            // offsets and names by piece; the bases by staging chunk: each copy thread fills one of
            // its pinned chunks from the pieces overlapping the chunk's range of the batch and
            // uploads it while filling the other
            auto pool = std::static_pointer_cast<SlotPool>(mtb::ctx_pipeline_cache(ctxs[d]));
            const uint64_t nCh1 = (b1 + kStageChunk - 1) / kStageChunk, nCh2 = paired ? (b2 + kStageChunk - 1) / kStageChunk : 0;
            size_t firstOf2 = 0;  // pieces are in mate order, by seqAt within a mate
            while (firstOf2 < pieces.size() && pieces[firstOf2].mate == 0) firstOf2++;
            std::atomic<size_t> nextPiece{0};
            std::atomic<uint64_t> nextChunk{0};
            std::atomic<bool> stageOk{true};
            auto copy = [&](size_t t) {
                for (size_t i; (i = nextPiece.fetch_add(1)) < pieces.size();) {
                    const Piece& pc = pieces[i];
                    const RecordBlock& b = *pc.b;
                    uint64_t* off = pc.mate ? s->off2.p : s->off1.p;
                    const uint64_t base = b.off[pc.lo];
                    for (uint32_t k = pc.lo; k < pc.hi; k++) off[pc.r + 1 + (k - pc.lo)] = pc.seqAt + (b.off[k + 1] - base);
                    if (!pc.mate) {
                        const uint64_t nb = b.noff[pc.lo];
                        memcpy(&s->names[pc.nameAt], b.names.data() + nb, b.noff[pc.hi] - nb);
                        for (uint32_t k = pc.lo; k < pc.hi; k++)
                            s->noff[pc.r + 1 + (k - pc.lo)] = pc.nameAt + (b.noff[k + 1] - nb);
                    }
                }
                Stager& g = *pool->stagers[t];
                for (uint64_t c; stageOk && (c = nextChunk.fetch_add(1)) < nCh1 + nCh2;) {
                    const int mate = c >= nCh1;
                    const uint64_t lo = (mate ? c - nCh1 : c) * kStageChunk;
                    const uint64_t hi = std::min<uint64_t>(lo + kStageChunk, mate ? b2 : b1);
                    if (g.used[g.k] && hipEventSynchronize(g.done[g.k]) != hipSuccess) stageOk = false;
                    char* dst = g.buf[g.k];
                    // the mate's pieces overlapping [lo, hi): the first one by binary search on seqAt
                    size_t a = mate ? firstOf2 : 0, e = mate ? pieces.size() : firstOf2;
                    size_t i0 = std::upper_bound(pieces.begin() + a, pieces.begin() + e, lo,
                                                 [](uint64_t x, const Piece& p) { return x < p.seqAt; }) -
                                pieces.begin();
                    for (size_t i = i0 > a ? i0 - 1 : a; i < e && pieces[i].seqAt < hi; i++) {
                        const Piece& pc = pieces[i];
                        const RecordBlock& b = *pc.b;
                        const uint64_t pLo = pc.seqAt, pHi = pc.seqAt + (b.off[pc.hi] - b.off[pc.lo]);
                        const uint64_t x0 = std::max(lo, pLo), x1 = std::min(hi, pHi);
                        if (x0 < x1) memcpy(dst + (x0 - lo), b.seq.data() + b.off[pc.lo] + (x0 - pLo), x1 - x0);
                    }
                    char* dseq = (char*)(mate ? s->dseq2.p : s->dseq1.p);
                    if (hipMemcpyAsync(dseq + lo, dst, hi - lo, hipMemcpyHostToDevice, g.st) != hipSuccess ||
                        hipEventRecord(g.done[g.k], g.st) != hipSuccess)
                        stageOk = false;
                    g.used[g.k] = true;
                    g.k ^= 1;
                }
            };
            const size_t nCopy = std::max<size_t>(1, std::min<size_t>(std::max<size_t>(pieces.size(), nCh1 + nCh2),
                                                                      kCopyThreads));
            for (size_t t = 0; ok && t < nCopy; t++) {
                if (!pool->stagers[t]) pool->stagers[t].reset(new Stager());
                ok = pool->stagers[t]->init(dev);
            }
            if (ok) {
                std::vector<std::thread> cp;
                for (size_t t = 1; t < nCopy; t++)
                    cp.emplace_back([&, t] {
                        mtb::background_thread();
                        copy(t);
                    });
                copy(0);
                for (auto& t : cp) t.join();
                ok = stageOk;
            }
            take1.clear();
            take2.clear();
            // the offsets behind the bases (the copy stream waits for every stager's last chunks)
            if (ok) {
                ok = hipSetDevice(dev) == hipSuccess;
                for (size_t t = 0; ok && t < nCopy; t++)
                    for (int k = 0; k < 2; k++)
                        if (pool->stagers[t]->used[k] && hipStreamWaitEvent(up[d], pool->stagers[t]->done[k], 0) != hipSuccess)
                            ok = false;
                ok = ok && hipMemcpyAsync(s->doff1.p, s->off1.p, on, hipMemcpyHostToDevice, up[d]) == hipSuccess &&
                     (!paired || hipMemcpyAsync(s->doff2.p, s->off2.p, on, hipMemcpyHostToDevice, up[d]) == hipSuccess) &&
                     hipEventRecord(s->uploaded, up[d]) == hipSuccess;
            }
            if (ok && partitioned) {  // the same batch on every further part's device: copied from the first
                bool same = s->peers.size() == (size_t)nCtx - 1;
                for (int p = 1; same && p < nCtx; p++) same = s->peers[p - 1]->device == mtb_ctx_device(ctxs[p]);
                if (!same) {
                    s->peers.clear();
                    for (int p = 1; p < nCtx; p++) {
                        auto pi = std::make_unique<PeerIn>();
                        pi->device = mtb_ctx_device(ctxs[p]);
                        hipSetDevice(pi->device);
                        hipEventCreateWithFlags(&pi->uploaded, hipEventDisableTiming);
                        s->peers.push_back(std::move(pi));
                    }
                }
                for (int p = 1; p < nCtx && ok; p++) {  // device to device (xGMI between GPUs, or host-staged)
                    PeerIn& pi = *s->peers[p - 1];
                    std::unique_lock<std::mutex> pl(*growMu.at(pi.device), std::defer_lock);
                    if (pi.dseq1.cap < b1 + 1 || pi.doff1.cap < on || (paired && (pi.dseq2.cap < b2 + 1 || pi.doff2.cap < on)))
                        pl.lock();
                    if (!links.direct[p * nCtx + 0]) ok = hipEventSynchronize(s->uploaded) == hipSuccess;  // staged: source ready
                    ok = ok && hipSetDevice(pi.device) == hipSuccess && pi.dseq1.ensure(b1 + 1) == hipSuccess &&
                         pi.doff1.ensure(on) == hipSuccess && hipStreamWaitEvent(up[p], s->uploaded, 0) == hipSuccess &&
                         links.copy(p, pi.dseq1.p, 0, s->dseq1.p, b1, up[p]) && links.copy(p, pi.doff1.p, 0, s->doff1.p, on, up[p]);
                    if (ok && paired)
                        ok = hipSetDevice(pi.device) == hipSuccess && pi.dseq2.ensure(b2 + 1) == hipSuccess &&
                             pi.doff2.ensure(on) == hipSuccess && links.copy(p, pi.dseq2.p, 0, s->dseq2.p, b2, up[p]) &&
                             links.copy(p, pi.doff2.p, 0, s->doff2.p, on, up[p]);
                    ok = ok && hipSetDevice(pi.device) == hipSuccess && hipEventRecord(pi.uploaded, up[p]) == hipSuccess;
                }
            }
            if (!ok) {
                eb.set(MTB_ERR_HIP, "batch upload failed");
                freeQ[d]->push(s);
                break;
            }
            fillS += secs(f0, Clock::now());
            if (index == 0) firstBatchS = secs(t0, Clock::now());
            s->index = index++;
            s->tReady = secs(t0, Clock::now());
            s->firstRead = firstRead;
            firstRead += s->n;
            if (!readyQ[d]->push(s)) break;
        }
        for (auto& q : readyQ) q->close();
    });

    // --em outputs requested: the mappings of every batch (Reporter::writeMappings)
    const bool em = opt->em_tsv || opt->em_report_tsv || opt->em_reclassify_report_tsv;
    // GPU workers, one per context: every batch they take goes on to the writer
    std::vector<double> waitS(nCtx, 0.0);
    // per context: the most reads a batch piece may hold after the workspace ran out (0: no limit)
    std::vector<uint32_t> pieceCap(nCtx, 0);
    std::atomic<uint64_t> splitBatches{0};
    if (const char* e = getenv("MTB_PIECE_READS")) pieceCap.assign(nCtx, (uint32_t)strtoul(e, nullptr, 10));  // tests
    // range-partitioned run: worker 0 takes each batch and hands it to the other parts' workers
    std::vector<std::unique_ptr<BoundedQueue<Slot*>>> partQ;
    std::unique_ptr<PartBatch> pb;
    if (partitioned) {
        for (int p = 0; p < nCtx; p++) partQ.emplace_back(new BoundedQueue<Slot*>(kSlots));
        pb.reset(new PartBatch(nCtx));
    }
    auto partition_worker = [&](int p) {
        mtb_ctx* c = ctxs[p];
        const int dev = mtb_ctx_device(c);
        PartBatch& B = *pb;
        const int P = nCtx;
        OwnerStage os;
        if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&os.st, hipStreamNonBlocking) != hipSuccess)
            eb.set(MTB_ERR_HIP, "cannot create the owner's copy stream");
        // after each step: p == 0 reads every worker's status; a context out of HBM halves the piece
        auto decide = [&](bool merge, uint32_t lo, uint32_t k, Slot* s) {
            bool retry = false;
            for (int q = 0; q < P; q++) {
                if (B.rc[q] == MTB_RETRY || B.rc[q] == MTB_ERR_OOM) retry = true;
                else if (B.rc[q] != MTB_OK && B.fail == MTB_OK) {
                    B.fail = B.rc[q];
                    B.failMsg = B.err[q];
                }
            }
            if (B.fail != MTB_OK) return;
            if (retry) {
                if (k < 2) {
                    B.fail = MTB_ERR_OOM;
                    B.failMsg = "out of HBM for a one-read piece of a range-partitioned batch";
                    return;
                }
                B.pieces.pop_front();
                B.pieces.push_front({lo + k / 2, lo + k});
                B.pieces.push_front({lo, lo + k / 2});
                if (!B.cap || k / 2 < B.cap) {
                    B.cap = k / 2;
                    fprintf(stderr, "[mtb] partitioned batch %llu: out of HBM; pieces of <= %u reads\n",
                            (unsigned long long)s->index, B.cap);
                }
                B.split = true;
                return;
            }
            if (!merge) return;
            for (int q = 0; q < P; q++) {  // the owners' lists in read order, offsets rebased
                const uint32_t a = (uint32_t)((uint64_t)k * q / P), b = (uint32_t)((uint64_t)k * (q + 1) / P);
                const uint32_t base = (uint32_t)B.all.size();
                for (uint32_t i = lo + a; i < lo + b; i++) s->res.p[i].taxcnt_offset += base;
                B.all.insert(B.all.end(), B.tc[q].begin(), B.tc[q].end());
            }
            B.pieces.pop_front();
        };
        Slot* s = nullptr;
        while (true) {
            if (p == 0) {
                const auto w0 = Clock::now();
                const bool got = readyQ[0]->pop(s);
                waitS[0] += secs(w0, Clock::now());
                for (int q = 1; q < P; q++)
                    if (got) partQ[q]->push(s);
                    else partQ[q]->close();
                if (!got) break;
            } else if (!partQ[p]->pop(s)) {
                break;
            }
            const auto g0 = Clock::now();
            const bool paired2 = paired;
            const char* q1 = p == 0 ? (const char*)s->dseq1.p : (const char*)s->peers[p - 1]->dseq1.p;
            const uint64_t* o1 = p == 0 ? (const uint64_t*)s->doff1.p : (const uint64_t*)s->peers[p - 1]->doff1.p;
            const char* q2 = !paired2 ? nullptr : p == 0 ? (const char*)s->dseq2.p : (const char*)s->peers[p - 1]->dseq2.p;
            const uint64_t* o2 = !paired2 ? nullptr : p == 0 ? (const uint64_t*)s->doff2.p
                                                             : (const uint64_t*)s->peers[p - 1]->doff2.p;
            hipSetDevice(dev);
            const bool upOk = hipEventSynchronize(p == 0 ? s->uploaded : s->peers[p - 1]->uploaded) == hipSuccess;
            B.rc[p] = upOk ? MTB_OK : MTB_ERR_HIP;
            B.err[p] = upOk ? "" : "batch upload failed";
            if (p == 0) {
                s->rc = MTB_OK;
                s->gpuS = 0;
                s->em.clear();
                s->tGpu0 = secs(t0, g0);
                B.pieces.clear();
                B.all.clear();
                B.split = false;
                B.fail = eb.failed ? MTB_ERR_INTERNAL : MTB_OK;  // skipped: an earlier failure ends the run
                if (s->res.ensure(std::max<uint32_t>(s->n, 1)) != hipSuccess) B.fail = MTB_ERR_OOM;
                const uint32_t step = B.cap && s->n > B.cap ? B.cap : std::max<uint32_t>(s->n, 1);
                for (uint32_t lo = 0; lo < s->n; lo += step) B.pieces.push_back({lo, std::min<uint32_t>(s->n, lo + step)});
                if (B.pieces.size() > 1) B.split = true;
            }
            B.bar.wait();
            if (p == 0) decide(false, 0, 0, s);  // an upload failure
            B.bar.wait();
            while (B.fail == MTB_OK && !B.pieces.empty()) {
                const uint32_t lo = B.pieces.front().first, k = B.pieces.front().second - lo;
                // 1. every part matches the whole piece
                int rc = mtb_classify_batch(c, q1, o1 + lo, q2, o2 ? o2 + lo : nullptr, k,
                                            MTB_INPUT_DEVICE | MTB_MATCH_ONLY, nullptr);
                if (rc == MTB_OK) rc = mtb::ctx_match_view(c, B.mOff[p], &B.m[p], &B.cnt[p], &B.ql[p]);
                B.rc[p] = rc;
                if (rc != MTB_OK) B.err[p] = mtb_last_error();
                B.bar.wait();
                const size_t nPieces = B.pieces.size();
                B.bar.wait();  // (every worker has read the piece count before p == 0 may change it)
                if (p == 0) decide(false, lo, k, s);
                B.bar.wait();
                if (B.fail != MTB_OK || B.pieces.size() != nPieces) continue;  // failed, or halved: again
                // 2. the owner's reads' segments from every part, its reads' query lengths
                const uint32_t a = (uint32_t)((uint64_t)k * p / P), b = (uint32_t)((uint64_t)k * (p + 1) / P),
                               no = b - a;
                uint64_t tot = 0;
                for (int q = 0; q < P; q++) tot += B.mOff[q][b] - B.mOff[q][a];
                rc = MTB_OK;
                if (os.m.ensure(sizeof(mtb_match) * std::max<uint64_t>(tot, 1)) != hipSuccess ||
                    os.cnt.ensure(sizeof(uint32_t) * ((size_t)P * no + 1)) != hipSuccess ||
                    os.ql.ensure(sizeof(uint32_t) * (no + 1)) != hipSuccess) {
                    (void)hipGetLastError();
                    rc = MTB_ERR_OOM;
                }
                uint64_t at = 0;
                for (int q = 0; q < P && rc == MTB_OK && no; q++) {
                    const uint64_t nm = B.mOff[q][b] - B.mOff[q][a];
                    if (!links.copy(p, (mtb_match*)os.m.p + at, q, B.m[q] + B.mOff[q][a], sizeof(mtb_match) * nm, os.st) ||
                        !links.copy(p, (uint32_t*)os.cnt.p + (size_t)q * no, q, B.cnt[q] + a, sizeof(uint32_t) * no, os.st))
                        rc = MTB_ERR_HIP;
                    at += nm;
                }
                if (rc == MTB_OK && no &&
                    (!links.copy(p, os.ql.p, p, B.ql[p] + a, sizeof(uint32_t) * no, os.st) ||
                     hipSetDevice(dev) != hipSuccess || hipStreamSynchronize(os.st) != hipSuccess))
                    rc = MTB_ERR_HIP;
                B.rc[p] = rc;
                if (rc != MTB_OK) B.err[p] = "range-partitioned match hand-over failed";
                B.bar.wait();  // every part's segments are copied: the contexts' workspaces may be reused
                if (p == 0) decide(false, lo, k, s);
                B.bar.wait();
                if (B.fail != MTB_OK || B.pieces.size() != nPieces) continue;
                // 3. the owner scores its reads (K5 + K6 over the chunks of every part)
                B.tc[p].clear();
                rc = MTB_OK;
                if (no) {
                    rc = mtb_assign_chunks(c, (const mtb_match*)os.m.p, tot, (const uint32_t*)os.cnt.p, (uint32_t)P,
                                           (const uint32_t*)os.ql.p, no, MTB_INPUT_DEVICE, s->res.p + lo + a);
                    uint64_t nt = 0;
                    if (rc == MTB_OK) {
                        mtb_get_taxcnt(c, nullptr, 0, &nt);
                        B.tc[p].resize(nt);
                        rc = mtb_get_taxcnt(c, B.tc[p].data(), nt, &nt);
                    }
                }
                B.rc[p] = rc;
                if (rc != MTB_OK) B.err[p] = mtb_last_error();
                B.bar.wait();
                if (p == 0) decide(true, lo, k, s);
                B.bar.wait();
            }
            // every worker has read the loop's exit condition (B.fail, B.pieces) before worker 0
            // finishes this batch and refills B with the next one's pieces
            B.bar.wait();
            if (p == 0) {
                if (B.fail == MTB_OK && s->tc.ensure(std::max<size_t>(B.all.size(), 1)) != hipSuccess) B.fail = MTB_ERR_OOM;
                if (B.fail == MTB_OK) std::copy(B.all.begin(), B.all.end(), s->tc.p);
                if (B.split) splitBatches++;
                s->gpuS = secs(g0, Clock::now());
                s->tGpu1 = s->tGpu0 + s->gpuS;
                s->rc = B.fail;
                if (B.fail != MTB_OK) {
                    s->err = B.failMsg;
                    if (!eb.failed) eb.set(B.fail, B.failMsg);
                }
                writeQ.push(s);
            }
        }
        if (os.st) hipStreamDestroy(os.st);
    };
    // MTB_GPU_SERIAL=1: the contexts sharing a device take turns for whole batches (their uploads,
    // syncs and result copies still overlap the other's kernels) instead of running kernels
    // concurrently, which slows each batch's memory-bound kernels
    const bool gpuSerial = getenv("MTB_GPU_SERIAL") && atoi(getenv("MTB_GPU_SERIAL")) != 0;
    std::vector<std::thread> workers;
    for (int d = 0; d < nCtx; d++)
        workers.emplace_back([&, d] {
            if (partitioned) {
                partition_worker(d);
                return;
            }
            mtb_ctx* c = ctxs[d];
            if (hipSetDevice(mtb_ctx_device(c)) != hipSuccess) eb.set(MTB_ERR_HIP, "cannot select the device");
            Slot* s = nullptr;
            while (true) {
                const auto w0 = Clock::now();
                if (!readyQ[d]->pop(s)) break;
                waitS[d] += secs(w0, Clock::now());
                s->rc = MTB_OK;
                s->gpuS = 0;
                s->em.clear();
                if (eb.failed) {
                    s->rc = MTB_ERR_INTERNAL;  // skipped: an earlier failure ends the run
                    writeQ.push(s);
                    continue;
                }
                const auto g0 = Clock::now();
                s->tGpu0 = secs(t0, g0);
                int rc = hipEventSynchronize(s->uploaded) == hipSuccess ? MTB_OK : MTB_ERR_HIP;
                if (s->res.ensure(std::max<uint32_t>(s->n, 1)) != hipSuccess) rc = MTB_ERR_OOM;
                // the ramp and every context's first full-size batch run alone on their device: they
                // grow the contexts' workspaces, and each growth step's hipFree waits for the whole
                // device — with two contexts on one GPU, for the other's batch; later batches reuse
                // the workspace and overlap
                std::unique_lock<std::mutex> gl(*growMu.at(mtb_ctx_device(c)), std::defer_lock);
                if (s->index < kRamp + (uint64_t)nCtx || gpuSerial) gl.lock();
                if (rc == MTB_OK && em && s->firstRead + s->n > 0xFFFFFFFFull) {
                    rc = MTB_ERR_ARG;
                    mtb::set_error("--em: more than 2^32 reads (MappingRes query IDs are 32-bit)");
                }
                // a ramp batch grows the workspace to a full batch's size at once (not in five steps,
                // each a device-wide hipFree)
                const double full = std::min<double>((double)maxBases, (double)maxReads * s->bases / std::max<uint32_t>(s->n, 1));
                mtb::ctx_set_grow(c, s->index < kRamp && !opt->max_reads && s->bases ? full / (double)s->bases : 1.0);
                if (rc == MTB_OK) rc = classify_slot(c, s, paired, em, pieceCap[d], splitBatches);
                mtb::ctx_set_grow(c, 1.0);
                if (gl.owns_lock()) gl.unlock();
                s->gpuS = secs(g0, Clock::now());
                s->tGpu1 = s->tGpu0 + s->gpuS;
                if (trace) {
                    float ms[5] = {0, 0, 0, 0, 0};
                    mtb_last_stage_ms(c, ms, 5);
                    s->devMs = ms[4];
                    s->ws = mtb::ctx_workspace_bytes(c);
                }
                s->rc = rc;
                if (rc != MTB_OK) {
                    s->err = mtb_last_error();  // the error string is per thread
                    eb.set(rc, s->err);
                }
                writeQ.push(s);
            }
        });

    // writer: the batches in input order -> TSV lines + per-taxon read counts (+ --em mappings).
    // The lines of a batch are formatted into one of two part sets while a flusher thread writes
    // the other set's lines of the batch before (Reporter.cpp:38-83 writes as it classifies).
    std::map<int32_t, uint64_t> taxCounts;
    std::vector<uint64_t> denseCounts;
    std::vector<mtb_em_map> emMaps;
    uint64_t reads = 0, bases = 0, batches = 0;
    double writeS = 0, gpuS = 0;
    FILE* tsv = fopen(opt->out_tsv, "wb");
    if (!tsv) {
        eb.set(MTB_ERR_IO, std::string("cannot write ") + opt->out_tsv);
    } else if (fputs(mtb::classification_header((opt->write_flags & MTB_WRITE_LINEAGE) != 0), tsv) < 0) {
        eb.set(MTB_ERR_IO, std::string("cannot write ") + opt->out_tsv);
    }
    std::vector<std::string> partSets[2];
    BoundedQueue<std::vector<std::string>*> toFlush(2), freeParts(2);
    freeParts.push(&partSets[0]);
    freeParts.push(&partSets[1]);
    std::thread flusher([&] {
        std::vector<std::string>* ps = nullptr;
        while (toFlush.pop(ps)) {
            if (tsv && !eb.failed)
                for (auto& x : *ps)
                    if (fwrite(x.data(), 1, x.size(), tsv) != x.size()) {
                        eb.set(MTB_ERR_IO, std::string("cannot write ") + opt->out_tsv);
                        break;
                    }
            freeParts.push(ps);
        }
    });
    const char* ft = getenv("MTB_FORMAT_THREADS");
    const unsigned formatThreads = ft && atoi(ft) > 0 ? (unsigned)atoi(ft) : kFormatThreads;
    std::thread writer([&] {
        uint64_t next = 0;
        std::map<uint64_t, Slot*> held;  // classified batches waiting for an earlier one
        Slot* s = nullptr;
        while (writeQ.pop(s)) {
            held[s->index] = s;
            while (!held.empty() && held.begin()->first == next) {
                s = held.begin()->second;
                held.erase(held.begin());
                next++;
                const auto w0 = Clock::now();
                if (!eb.failed && s->rc == MTB_OK) {
                    mtb_read_batch b{};
                    b.n_reads = s->n;
                    b.names = s->names.data();
                    b.name_off = s->noff.data();
                    std::vector<std::string>* ps = nullptr;
                    if (freeParts.pop(ps)) {
                        mtb::format_classifications(ctx0, b, s->res.p, s->tc.p, opt->write_flags, *ps, formatThreads);
                        toFlush.push(ps);
                    }
                    for (uint32_t i = 0; i < s->n; i++) {  // ++taxCounts[classification] (Classifier.cpp:201-203)
                        const int32_t t = s->res.p[i].is_classified ? s->res.p[i].classification : 0;
                        if (t >= 0 && t < (1 << 26)) {  // internal taxIDs are dense: a flat table
                            if ((size_t)t >= denseCounts.size()) denseCounts.resize((size_t)t * 2 + 1024, 0);
                            denseCounts[t]++;
                        } else {
                            taxCounts[t]++;
                        }
                    }
                    emMaps.insert(emMaps.end(), s->em.begin(), s->em.end());
                    reads += s->n;
                    bases += s->bases;
                    batches++;
                    gpuS += s->gpuS;
                }
                writeS += secs(w0, Clock::now());
                if (trace)
                    fprintf(trace, "%llu %d %u ready %.4f gpu %.4f %.4f write %.4f %.4f dev_ms %.1f ws_gb %.1f\n",
                            (unsigned long long)s->index, s->ctx, s->n, s->tReady, s->tGpu0, s->tGpu1, secs(t0, w0),
                            secs(t0, Clock::now()), s->devMs, s->ws * 1e-9);
                freeQ[s->ctx]->push(s);
            }
        }
        for (auto& kv : held) freeQ[kv.second->ctx]->push(kv.second);  // a failed run: batches never written
        toFlush.close();
    });

    assembler.join();
    for (auto& w : workers) w.join();
    writeQ.close();
    writer.join();
    flusher.join();
    if (tsv && fclose(tsv) != 0) eb.set(MTB_ERR_IO, std::string("write failed: ") + opt->out_tsv);
    if (trace) {
        fprintf(trace, "end %.4f\n", secs(t0, Clock::now()));
        fclose(trace);
    }
    for (auto& q : freeQ) q->close();
    m1.out.close();
    m2.out.close();
    m1.t.join();
    if (paired) m2.t.join();
    for (int d = 0; d < nCtx; d++) {
        hipSetDevice(mtb_ctx_device(ctxs[d]));
        hipStreamSynchronize(up[d]);
        hipStreamDestroy(up[d]);
    }
    for (Slot* s : slotMem) {  // back to the context's pool: the batch data is not kept
        s->em.clear();
        s->names.clear();
    }
    hipSetDevice(mtb_ctx_device(ctx0));
    if (eb.code != MTB_OK) {
        set_error(eb.msg);
        return eb.code;
    }
    for (size_t t = 0; t < denseCounts.size(); t++)
        if (denseCounts[t]) taxCounts[(int32_t)t] += denseCounts[t];
    if (opt->report_tsv) {
        std::vector<int32_t> ids;
        std::vector<uint32_t> cnt;
        for (auto& kv : taxCounts) {
            ids.push_back(kv.first);
            cnt.push_back((uint32_t)kv.second);
        }
        const int rc = mtb_write_report(ctx0, opt->report_tsv, reads, ids.data(), cnt.data(), ids.size());
        if (rc != MTB_OK) return rc;
    }
    if (em) {  // Classifier.cpp:152-161: EM, the reassigned reads and both EM reports
        std::vector<mtb_em_read> er(std::max<uint64_t>(reads, 1));
        const size_t cap = emMaps.size() + 1;
        std::vector<int32_t> spIds(cap);
        std::vector<double> spP(cap);
        std::vector<uint32_t> spC(cap);
        uint64_t nSp = 0;
        mtb_em_stats est{};
        int rc = mtb_em(ctx0, emMaps.data(), emMaps.size(), reads, er.data(), spIds.data(), spP.data(), spC.data(), cap,
                        &nSp, &est);
        if (rc != MTB_OK) return rc;
        if (opt->em_tsv) {
            rc = mtb_write_em_results(ctx0, opt->em_tsv, opt->out_tsv, er.data(), reads, opt->write_flags);
            if (rc != MTB_OK) return rc;
        }
        if (opt->em_report_tsv) {  // emTaxCounts: the top species, taxID 0 = the reads they leave unexplained
            std::vector<int32_t> ids(spIds.begin(), spIds.begin() + nSp);
            std::vector<uint32_t> cnt(spC.begin(), spC.begin() + nSp);
            uint64_t explained = 0;
            for (uint32_t c : cnt) explained += c;
            ids.push_back(0);
            cnt.push_back((uint32_t)(reads - explained));
            rc = mtb_write_report(ctx0, opt->em_report_tsv, reads, ids.data(), cnt.data(), ids.size());
            if (rc != MTB_OK) return rc;
        }
        if (opt->em_reclassify_report_tsv) {  // reclassifyTaxCounts: the reassigned reads per taxID
            std::map<int32_t, uint64_t> rc2;
            for (uint64_t i = 0; i < reads; i++)
                if (er[i].mapped == 1) rc2[er[i].tax_id]++;
            std::vector<int32_t> ids;
            std::vector<uint32_t> cnt;
            for (auto& kv : rc2) {
                ids.push_back(kv.first);
                cnt.push_back((uint32_t)kv.second);
            }
            rc = mtb_write_report(ctx0, opt->em_reclassify_report_tsv, reads, ids.data(), cnt.data(), ids.size());
            if (rc != MTB_OK) return rc;
        }
    }
    if (stats) {
        double w = 0;
        for (double x : waitS) w += x;
        stats->reads = reads;
        stats->bases = bases;
        stats->batches = batches;
        stats->wall_s = secs(t0, Clock::now());
        stats->gpu_s = gpuS;
        stats->input_wait_s = w;
        stats->write_s = writeS;
        stats->source_s = m1.sourceS + m2.sourceS;
        stats->scan_s = m1.scanS + m2.scanS;
        stats->parse_s = (double)(m1.parseNs + m2.parseNs) * 1e-9;
        stats->fill_s = fillS;
        stats->first_batch_s = firstBatchS;
        stats->split_batches = splitBatches;
    }
    return MTB_OK;
}
