// C-ABI of the MI355X classify path (include/mtb_gpu.h): context, DB residency in HBM and the
// per-batch pipeline K0 read metadata -> K1 extract -> K2 radix sort -> K4 match (count, scan,
// emit) -> K5/K6 per-read sort + assignment -> taxcnt compaction.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <memory>
#include <charconv>
#include <mutex>
#include <unordered_map>

#include "mtb_host.h"
#include "mtb_launch.h"
#include <cstdlib>

using namespace mtb;

// A failed HIP call ends the entry point: MTB_ERR_OOM when the device ran out of memory (a batch
// entry point turns that into MTB_RETRY: the caller splits the batch), MTB_ERR_HIP otherwise.
#define HIP_TRY(x)                                                                                   \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #x);                 \
            return e_ == hipErrorOutOfMemory ? MTB_ERR_OOM : MTB_ERR_HIP;                            \
        }                                                                                            \
    } while (0)

namespace {

// A context's batch workspace: the bytes its grow-only buffers hold, and an optional cap on them
// (MTB_WORKSPACE_CAP: a growth step past it fails as out of memory, so tests force the split that
// a full device causes).
struct WsBudget {
    size_t cap = 0;  // 0: the device's memory is the only limit
    size_t used = 0;
    double grow = 1.0;  // a growth step allocates need x grow when that fits (mtb::ctx_set_grow)
};

struct DevBuf {  // grow-only device allocation
    void* p = nullptr;
    size_t bytes = 0;
    WsBudget* budget = nullptr;  // the owning context's (batch buffers only)
    hipError_t ensure(size_t need) {
        if (need <= bytes) return hipSuccess;
        static const bool trace = getenv("MTB_ALLOC_TRACE") != nullptr;  // experiments: slow growth steps
        const auto t0 = std::chrono::steady_clock::now();
        const size_t old = bytes;
        if (p) hipFree(p);
        const auto t1 = std::chrono::steady_clock::now();
        p = nullptr;
        if (budget) budget->used -= bytes;
        bytes = 0;
        size_t b = need + need / 8 + 256;
        hipError_t e = hipErrorOutOfMemory;
        if (budget && budget->grow > 1.125) {  // a small batch of a ramp: straight to the full batch's size
            const size_t big = (size_t)((double)need * budget->grow) + 256;
            if (!budget->cap || budget->used + big <= budget->cap) {
                e = hipMalloc(&p, big);
                if (e == hipSuccess) b = big;
                else (void)hipGetLastError();
            }
        }
        if (e != hipSuccess) {
            if (budget && budget->cap && budget->used + b > budget->cap) return hipErrorOutOfMemory;
            e = hipMalloc(&p, b);
        }
        if (e == hipSuccess) bytes = b;
        if (e == hipSuccess && budget) budget->used += b;
        if (trace) {
            const auto t2 = std::chrono::steady_clock::now();
            const double f = std::chrono::duration<double>(t1 - t0).count(), m = std::chrono::duration<double>(t2 - t1).count();
            if (f + m > 0.02) fprintf(stderr, "[alloc] %.3f GB -> %.3f GB: free %.3f s, malloc %.3f s\n", old * 1e-9, b * 1e-9, f, m);
        }
        return e;
    }
    void release() {
        if (!p) return;
        hipFree(p);
        p = nullptr;
        if (budget) budget->used -= bytes;
        bytes = 0;
    }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }  // scratch DevBufs of an entry point are freed on every return path
    template <typename T>
    T* as() const { return (T*)p; }
};

// The DB-derived device arrays a context reads but never writes (records unless the caller owns
// them, AA directory, probe lines, run index, species map, taxonomy): freed with the last context
// holding them — a context and its clones (mtb_clone).
struct DbArrays {
    int device = 0;
    std::vector<void*> own;
    ~DbArrays() {
        hipSetDevice(device);
        for (void* p : own)
            if (p) hipFree(p);
    }
};

}  // namespace

struct mtb_ctx {
    int device = 0;
    mtb_params par{};
    hipStream_t stream = nullptr;
    bool ownStream = false;
    HostTables tables{};
    // DB residency
    uint64_t D = 0;
    DbRec* db = nullptr;      // D + kDbPad records: value (rank form) + taxID & mask
    bool borrowedDb = false;  // db belongs to the caller (mtb_open_resident)
    std::shared_ptr<DbArrays> dbArrays;  // owner of the DB-derived arrays below, shared with clones
    uint64_t* dirMem = nullptr;
    ProbeLine* lines = nullptr;  // probe lines: AA 8-mer membership + DB run heads (5.4 GB)
    uint64_t* lineP = nullptr;   // run index: present ranks before each line (0.7 GB) ...
    uint16_t* runOff = nullptr;  // ... and each present rank's run start in its line (2 B per present rank)
    ProbeExt* lineExt = nullptr;  // run-length lines (64 B per probe line; MTB_LINE_EXT=1, A/B)
    uint64_t* link = nullptr;     // link lines: K1F's window pairs (14.4 GB; MTB_LINK_LINES=0: none)
    AADir dir{};
    uint64_t rankLo = 0, rankHi = ~0ull;  // AA-rank range of the held DB part (K1F drops the rest)
    int joinMode = 0;            // MTB_JOIN: 0 default (sort-merge), 1 sort, 2 probe, 3 sweep
    // K4S DB-sweep join: DB tiles (built at the first sweep batch) and the nominal tile size
    uint64_t* tileRec = nullptr;
    uint32_t* tilePre = nullptr;
    uint64_t nTiles = 0;
    uint32_t sweepNom = 2048;    // MTB_SWEEP_NOM
    uint32_t sweepLdsCap = ~0u;  // MTB_SWEEP_LDS (tests): tiles over this many records search HBM
    bool sweepSmall = false;     // MTB_SWEEP_SMALL=1 (A/B): 24-KB LDS tiles (2048 records), nominal 1024
    bool filterThreadMajor = false;  // MTB_FILTER_PACK=thread (A/B): K1F's output in round 3's thread-major order
    int sweepPersist = 1;        // MTB_SWEEP_PERSIST: 1 persistent (default: profiles/r04/join_ab.json), 2 warp-specialised, 0 a block per tile
    uint32_t matchWinCap = ~0u;  // MTB_MATCH_WINDOW (tests force the HBM-search path with 0)
    bool directJoin = true;      // MTB_DIRECT=0: the sort-merge join stages its matches (+ transpose)
    bool directRetry = false;    // MTB_DIRECT=2: every direct join is treated as overflowed (tests)
    int pruneAfter = 2;          // MTB_PRUNE_AFTER (A/B): launch_segsort's register-sort mode (2 rank keys, 0 full keys, 1 sort then prune, 4 as 2 with the bitonic large sort)
    int bigGroups = 1;           // MTB_BIG_GROUPS=0: no k_match_paths_wave (every group on a thread)
    bool fuseFilter = true;      // MTB_FUSE_FILTER=0: K1 writes every window's key, K1F reads them back
    bool radixDigits = true;     // MTB_RADIX_DIGITS=0: K2's histograms read the keys, not 1-B digit side arrays
    bool radixAtomicFirst = false;  // MTB_RADIX_ATOMIC_FIRST=1 (A/B): K2's first pass ranks by LDS atomics
    // MTB_K1F_BINS: the fused K1F writes straight into K2's first-pass buckets (1: batches of >= 2^22
    // present-window slots, 2: every batch, 0: off, the default — measured even);
    // MTB_K1F_BINS_RC forces the bucket size (tests)
    int binnedSort = 0;
    uint64_t binRcForce = 0;
    bool binDigits = true;  // MTB_K1F_BINS_DIG=0: the binned K1F writes no second-pass digits (K2 reads the keys)
    // MTB_UNIFORM_UNITS: uniform K1 units (every read 6 per mate, k_read_units) when every frame of the
    // batch is one chunk, so K4 rebuilds a matched query's info from its slot and a 4-B read length
    // instead of a 16-B unit record (round 6)
    bool uniformUnits = true;
    uint32_t upr = 0;  // the last batch's units per read when uniform, else 0
    uint64_t binHost[kSortBins] = {};  // the last binned K1F's bucket counts
    bool noFilter = false;       // MTB_FILTER=0: no K1F; every non-blank window is sorted and joined
                                 // (with the sweep join the context then holds no probe lines either)
    uint32_t spillShift = 0;     // MTB_DIRECT=3: read stretches taken as a quarter (queries spill; tests)
    bool sparse = false;         // the batch's matches are still in the direct join's layout (mDirect, slotOff * chunkC)
    uint32_t maxW = 0;           // the batch's most windows in one frame of one read
    int sortLoFine = kQuerySortLoFine;  // MTB_SORT_LO_FINE (experiments)
    bool forceGeneric = false;   // MTB_FORCE_GENERIC=1: fast paths off, fallbacks only (tests)
    bool segsortGlobal = false;  // MTB_SEGSORT_GLOBAL=1: every K5 segment through global scratch (tests)
    uint32_t mergeSeg = 0;       // MTB_MERGE_SEG=<n>: K5 merge path above n matches (tests; default 8192)
    int waveTaxon = -1;          // MTB_WAVE_TAXON=0/1/2: K6 chooseBestTaxon thread / wave / 16-lane group per read (default auto)
    int emulateAll = 0;          // MTB_EMULATE_SORT=1: k_combine_wave emulates std::sort for every run (tests)
    bool pruneCompact = true;    // MTB_PRUNE_COMPACT=0: big K5 segments are not thinned before their sort (tests)
    bool noAlias = false;        // MTB_K6_ALIAS=0: K6 scratch in buffers of its own (A/B, tests)
    uint64_t aliasBytes = 0;     // K6 scratch bytes of the last batch carved out of dead buffers
    int32_t* spOf = nullptr;
    int32_t maxTax = 0;
    int32_t *tNodeOf = nullptr, *tNodeTax = nullptr, *tParent = nullptr, *tDepth = nullptr, *tSpParent = nullptr;
    uint8_t* tFlags = nullptr;
    uint32_t cladePerMatch = 2;
    std::vector<int32_t> hNodeOf;  // host copies for mtb_taxon_rank / the TSV writer
    std::vector<std::string> hRank;
    HostTaxonomy hTax;             // the report (mtb_write_report): names, parents, nodes.dmp order
    mutable std::vector<std::string> lineage;  // per node, built on first use (mtb_taxon_lineage)
    mutable std::once_flag lineageOnce;
    std::shared_ptr<void> pipelineCache;  // mtb_pipeline.cpp's slots, kept between runs
    mutable mtb::TaxText taxText;  // per taxID: original ID digits + rank, built on first use
    mutable std::once_flag taxTextOnce;
    // batch workspace. ws comes before every DevBuf: members are destroyed in reverse order, and a
    // DevBuf still holding memory at mtb_close gives its bytes back to ws in its destructor
    WsBudget ws;                            // the batch buffers' bytes (+ MTB_WORKSPACE_CAP)
    DevBuf seq1, off1, seq2, off2, meta, reserve, slotOff, qlen, scanTmp;
    DevBuf keysA, valsA, keysB, valsB, radixCounts, radixOffs;
    DevBuf readCnt, mOff, matches, matchesSorted, segScratch, maxSeg, errFlag;
    DevBuf ordKA, ordVA, ordKB, ordVB, matchWin, unitRead, unitInfo, mStage, mRank, mTotal, mDirect, ovFlag, waveList, waveCount, devStats;
    DevBuf qFrom, probeStats;
    DevBuf longList, longCnt;  // the direct join's long-run queries (k_match_long)
    DevBuf qStart;             // K4S: the sorted queries' sort-prefix bucket starts
    uint32_t longCap = 0;
    DevBuf chunkIn, chunkCnt, chunkSrcOff;  // mtb_assign_chunks staging
    DevBuf liveCnt, liveOff;                // K5 pruning: live matches per read, their offsets
    DevBuf segLen;                          // K5: survivors of the thinned big segments (k_thin_big)
    DevBuf sizeLists;                       // K5: reads of each size class above 128 matches (k_size_lists)
    DevBuf digA, digB;                      // K2 digit side arrays (1 B per kept query k-mer, ping-pong)
    DevBuf binCnt, binTab;                  // binned K1F: bucket counts (kSortBins u64), K2's tile table
    DevBuf maskOut1, maskOut2, maskProb, maskScale;  // K0M tantan masking: masked mates + scratch
    DevBuf readLens;                        // K0: the mates' lengths, 16 bits each (uniform units' K4)
    DevBuf readCnt64;                       // uniform units' K4: per-read count | mate lengths << 32
    uint64_t liveM = 0;                     // matches K6 read in the last batch
    // mtb_open_phases: seconds of the DB files' read, upload + K3 decode into records, AA directory,
    // probe lines, run index, taxonomy + species map, and the whole open
    double openS[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // [7]: the records' allocation (inside [1])
    static constexpr int kNumStats = 20;
    uint64_t stats[kNumStats] = {};  // mtb_last_stats
    uint32_t chunkC = 1;  // K1 windows per unit of the last batch
    uint64_t stageRegion = 0;  // slots per staging region of mStage (grows to the largest seen)
    uint64_t spillCap = 0;     // direct join: spilled matches mStage holds (grows to the largest seen)
    // --em: the last batch's mappings (kEmTop {species, score^2} per read, their counts), the
    // std::sort scratch (8 B per species run), DB k-mers per species (length factors)
    DevBuf emMap, emCnt, emScratch, emPacked, emCnt32, emOff;
    bool emValid = false;
    bool emPackedValid = false;                // emHost holds the last batch's packed mappings
    std::vector<mtb_em_map> emHost;
    std::vector<uint32_t> spKmers;
    std::string dbDir;
    DevBuf local, paths, comb, conn, spScore, spKeep,
        gFlag, sFlag, pathCnt, gScan, sScan, gStart, sStart, clade, tcPool, tcLen, tcOff, tcOut, results;
    // last batch
    uint32_t nReads = 0;
    uint64_t Q = 0, M = 0, nTaxcnt = 0;
    uint64_t Qall = 0;  // non-blank query k-mers (KmerMatcher.cpp:143-152), before the AA filter
    double presentShare = 0.5;  // the fused filter's output capacity, a share of the slots (grows)
    const uint64_t* qKeys = nullptr;   // the last batch's query k-mers (sorted on the sort-merge path)
    const uint32_t* qSlots = nullptr;
    bool keepStages = false;
    bool probed = false;  // the last batch took the probe join
    bool matchOnly = false;  // the last batch stopped after the join (MTB_MATCH_ONLY)
    float stageMs[5] = {0, 0, 0, 0, 0};
    hipEvent_t ev[6]{};
    // tight event pairs around the main kernels: extract, k-mer sort, match count, match emit,
    // per-read match sort, assign
    static constexpr int kNumKern = 7;
    float kernMs[kNumKern] = {0, 0, 0, 0, 0, 0, 0};
    hipEvent_t kev[2 * kNumKern]{};
};

static std::vector<DevBuf*> batch_bufs(mtb_ctx* c);

// The batch buffers account their bytes to the context's budget; MTB_WORKSPACE_CAP=<bytes>[K|M|G]
// caps it (tests: a batch past the cap returns MTB_RETRY, as one past the device's memory does).
static void bind_workspace(mtb_ctx* c, size_t cap) {
    c->ws.cap = cap;
    if (const char* e = getenv("MTB_WORKSPACE_CAP")) {
        char* end = nullptr;
        double v = strtod(e, &end);
        const char u = end ? *end : 0;
        v *= u == 'G' || u == 'g' ? 1e9 : u == 'M' || u == 'm' ? 1e6 : u == 'K' || u == 'k' ? 1e3 : 1.0;
        c->ws.cap = v > 0 ? (size_t)v : 0;
    }
    for (DevBuf* b : batch_bufs(c)) b->budget = &c->ws;
}

static void free_db(mtb_ctx* c) {
    if (c->dbArrays) {  // the last holder frees them
        c->dbArrays.reset();
        c->db = nullptr;
        c->dirMem = nullptr;
        c->lines = nullptr;
        c->lineP = nullptr;
        c->runOff = nullptr;
        c->lineExt = nullptr;
        c->link = nullptr;
        return;
    }
    if (c->borrowedDb) c->db = nullptr;  // caller-owned (mtb_open_resident)
    void* ptrs[] = {c->db, c->dirMem, c->lines, c->lineP, c->runOff, c->lineExt, c->link, c->spOf, c->tNodeOf, c->tNodeTax, c->tParent, c->tDepth, c->tSpParent, c->tFlags};
    for (void* p : ptrs)
        if (p) hipFree(p);
    c->db = nullptr;
    c->dirMem = nullptr;
    c->lines = nullptr;
    c->lineP = nullptr;
    c->runOff = nullptr;
    c->lineExt = nullptr;
    c->link = nullptr;
}

template <typename T>
static hipError_t upload(T** dst, const std::vector<T>& v, hipStream_t s) {
    hipError_t e = hipMalloc((void**)dst, std::max<size_t>(1, v.size()) * sizeof(T));
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
    return e;
}

static int validate_params(const mtb_params* p) {
    if (p->reduced_aa) { set_error("reduced-AA DBs (ReducedKmerMatcher) are out of scope"); return MTB_ERR_UNSUPPORTED; }
    if (p->em && p->db_parts > 1) { set_error("--em needs the whole DB in one context"); return MTB_ERR_UNSUPPORTED; }
    if (p->mask_mode && !(p->mask_prob > 0.0f && p->mask_prob <= 1.0f)) { set_error("mask_prob must be in (0, 1]"); return MTB_ERR_ARG; }
    if (p->kmer_format != 1 && p->kmer_format != 2) { set_error("kmer_format must be 1 or 2"); return MTB_ERR_UNSUPPORTED; }
    if (p->syncmer && p->kmer_format != 2) { set_error("syncmer requires kmer_format 2"); return MTB_ERR_UNSUPPORTED; }
    if (p->syncmer && (p->smer_len < 1 || p->smer_len > 8)) { set_error("smer_len must be in [1, 8]"); return MTB_ERR_ARG; }
    if (p->seq_mode < 1 || p->seq_mode > 3) { set_error("seq_mode must be 1, 2 or 3"); return MTB_ERR_ARG; }
    return MTB_OK;
}

static double since(std::chrono::steady_clock::time_point& t) {
    const auto now = std::chrono::steady_clock::now();
    const double d = std::chrono::duration<double>(now - t).count();
    t = now;
    return d;
}

// K3 at open: diffIdx decoded chunk by chunk straight into the 12-B records (values in rank form
// next to info & mask), so HBM holds the records plus one chunk's temporaries (~34 B per chunk word)
// instead of the whole decode's (2 + 4 + 8 + 8 B per word and 4 + 8 B per k-mer: > 400 GB at the
// GTDB scale's 12G k-mers). Each chunk's words come from the file (parallel preads into pinned
// buffers) or the caller's host arrays, uploaded while the threads fill the next buffers; its whole
// k-mers decode (the cut one goes to the next chunk), continuing the previous chunk's last value.
// validateDatabase.cpp:78-131's checks ride along: the terminators counted over every chunk must
// equal info's entries (checked before a chunk writes past them) and the last word must end a k-mer.
// openS[0] gets the reads and uploads, openS[1] the decode (set by the caller from its clock).
static int decode_db_chunked(mtb_ctx* c, HostDb& db, uint32_t mask, hipStream_t s) {
    const uint64_t nDiff = db.nDiff, D = c->D;
    uint64_t W = 1ull << 30;  // words per chunk (2 GB of diffIdx)
    if (const char* e = getenv("MTB_DECODE_CHUNK_WORDS")) W = std::max<uint64_t>(8, strtoull(e, nullptr, 10));
    W = std::max<uint64_t>(std::min(W, nDiff), 1);
    DevBuf dDiff, dFlag, dIdx, dTmp, dVal, dInfo;  // chunk temporaries, freed on every return
    HIP_TRY(dDiff.ensure(W * sizeof(uint16_t)));
    HIP_TRY(dFlag.ensure(W * sizeof(uint32_t)));
    HIP_TRY(dIdx.ensure((W + 2) * sizeof(uint64_t)));
    HIP_TRY(dTmp.ensure(scan_tmp_elems(W) * sizeof(uint64_t)));
    HIP_TRY(dVal.ensure(W * sizeof(uint64_t)));
    HIP_TRY(dInfo.ensure(W * sizeof(uint32_t)));
    auto a0 = std::chrono::steady_clock::now();
    HIP_TRY(hipMalloc(&c->db, (D + kDbPad) * sizeof(DbRec)));
    c->openS[7] = since(a0);  // the records' allocation (waits for any memory the runtime still releases)
    const bool fromFile = !db.diffFile.empty();
    double upS = 0;
    auto l0 = std::chrono::steady_clock::now();
    StageLanes lanes(c->device);  // pinned staging reused by every chunk's uploads
    upS += since(l0);
    uint64_t w0 = 0, k0 = 0, carry = 0, seen = 0;  // seen: terminators so far (k0 stops at D)
    HIP_TRY(hipStreamSynchronize(s));
    while (w0 < nDiff) {
        const uint64_t n = std::min(W, nDiff - w0);
        auto u0 = std::chrono::steady_clock::now();
        const bool got = fromFile ? read_to_device(db.diffFile, dDiff.p, n * sizeof(uint16_t), w0 * sizeof(uint16_t), &lanes)
                                  : upload_to_device(db.diffP + w0, dDiff.p, n * sizeof(uint16_t), &lanes);
        if (!got) return MTB_ERR_IO;
        upS += since(u0);
        uint64_t lastTerm = 0, lastValue = 0;
        const uint64_t terms = decode_diff_chunk(dDiff.as<uint16_t>(), n, carry, dVal.as<uint64_t>(),
                                                 dFlag.as<uint32_t>(), dIdx.as<uint64_t>(), dTmp.p, &lastTerm,
                                                 &lastValue, s);
        HIP_TRY(hipGetLastError());
        const bool lastChunk = w0 + n == nDiff;
        if (terms == 0) {  // no terminator in a whole chunk: a k-mer of > W words, or the tail ends mid k-mer
            set_error("diffIdx ends mid k-mer");
            return MTB_ERR_DB;
        }
        if (lastChunk && lastTerm != n - 1) {
            set_error("diffIdx ends mid k-mer");
            return MTB_ERR_DB;
        }
        seen += terms;
        if (seen <= D) {  // the records of these k-mers: info & mask next to the rank-form values
            u0 = std::chrono::steady_clock::now();
            const bool gotInfo = fromFile ? read_to_device(db.infoFile, dInfo.p, terms * sizeof(uint32_t),
                                                           k0 * sizeof(uint32_t), &lanes)
                                          : upload_to_device(db.infoP + k0, dInfo.p, terms * sizeof(uint32_t), &lanes);
            if (!gotInfo) return MTB_ERR_IO;
            upS += since(u0);
            launch_mask_info(dInfo.as<uint32_t>(), terms, mask, s);
            if (c->par.kmer_format == 2) launch_to_rank_form(dVal.as<uint64_t>(), terms, s);
            launch_pack_db(dVal.as<uint64_t>(), dInfo.as<uint32_t>(), terms, c->db + k0, s);
            HIP_TRY(hipStreamSynchronize(s));
            k0 += terms;
        }
        carry = lastValue;
        w0 += lastTerm + 1;
    }
    if (seen != D) {  // counted to the end, written only up to D
        set_error("diffIdx k-mer count " + std::to_string(seen) + " != info entries " + std::to_string(D));
        return MTB_ERR_DB;
    }
    c->openS[0] += upS;
    return MTB_OK;
}

// Everything of an opening after the argument checks, into a fresh context (the caller closes it
// on failure, so no error path leaks the context, its stream or device arrays).
static int open_into(mtb_ctx* c, HostDb& db, const mtb_params* par, int device, const mtb_db_resident* res,
                     double readS, std::chrono::steady_clock::time_point t0) {
    auto tp = t0;
    c->device = device;
    c->par = *par;
    c->tables = make_tables();
    c->openS[0] = readS;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->ownStream = true;
    for (auto& e : c->ev) HIP_TRY(hipEventCreate(&e));
    for (auto& e : c->kev) HIP_TRY(hipEventCreate(&e));
    hipStream_t s = c->stream;
    const uint32_t mask = ~((uint32_t)(par->skip_redundancy == 0) << 31);
    const DbRec padRec[kDbPad] = {{~0u, ~0u, 0}, {~0u, ~0u, 0}, {~0u, ~0u, 0}, {~0u, ~0u, 0},
                                  {~0u, ~0u, 0}, {~0u, ~0u, 0}, {~0u, ~0u, 0}, {~0u, ~0u, 0}};
    if (res) {  // caller-owned records, used in place (capacity n_kmers + kDbPad)
        c->D = res->n_kmers;
        c->db = reinterpret_cast<DbRec*>(res->records);
        c->borrowedDb = true;
        launch_rec_mask_info(c->db, c->D, mask, s);
        if (par->kmer_format == 2 && !res->rank_form) launch_rec_rank_form(c->db, c->D, s);
    } else {
        c->D = db.nInfo;
        // diffIdx -> values (K3), info & mask (KmerMatcher.cpp:204-205, :381), then one record per k-mer
        const int drc = decode_db_chunked(c, db, mask, s);
        if (drc != MTB_OK) return drc;
    }
    // + kDbPad records of value ~0 / taxID 0: the probe's 8-wide reads from any DB index need no bound
    HIP_TRY(hipMemcpyAsync(c->db + c->D, padRec, sizeof(padRec), hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (par->db_parts > 1) {  // the part's AA-rank range: its first k-mer up to its guard k-mer's run
        DbRec ends[2];
        HIP_TRY(hipMemcpyAsync(&ends[0], c->db, sizeof(DbRec), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&ends[1], c->db + c->D - 1, sizeof(DbRec), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        c->rankLo = ((uint64_t)ends[0].hi << 32 | ends[0].lo) >> 24;
        c->rankHi = par->db_part == par->db_parts - 1 ? ~0ull : ((uint64_t)ends[1].hi << 32 | ends[1].lo) >> 24;
    }
    c->openS[1] = since(tp) - (c->openS[0] - readS);  // the decode's uploads are in openS[0]
    set_ab_rank_free(getenv("MTB_AB_RANK_FREE") ? atoi(getenv("MTB_AB_RANK_FREE")) : 0);  // A/B only: invalid results
    set_match_prefetch(getenv("MTB_MATCH_PREFETCH") ? atoi(getenv("MTB_MATCH_PREFETCH")) : 0);
    set_pair_read(getenv("MTB_PAIR_READ") ? atoi(getenv("MTB_PAIR_READ")) : 0);
    set_match_xcd(getenv("MTB_MATCH_XCD") ? atoi(getenv("MTB_MATCH_XCD")) : 0);  // (device-wide: set at each open)
    // run sharing measured no gain (the repeated lookups already hit the L2: profiles/r05/ab_share*.json): off
    set_share_runs(getenv("MTB_SHARE_RUNS") ? atoi(getenv("MTB_SHARE_RUNS")) : 0);
    if (const char* e = getenv("MTB_AB_SWEEP_COUNT")) set_ab_sweep_count(atoi(e));  // A/B only: invalid results
    if (const char* e = getenv("MTB_MATCH_WINDOW")) c->matchWinCap = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("MTB_FORCE_GENERIC")) c->forceGeneric = atoi(e) != 0;
    if (const char* e = getenv("MTB_SORT_LO_FINE")) {  // experiments: the unstaged join's sort prefix
        const int v = atoi(e);
        if (v >= 24 && v <= 52 && (kQuerySortHi - v) % 8 == 0) c->sortLoFine = v;  // 44 / 52: coarser (A/B)
    }
    if (const char* e = getenv("MTB_DIRECT")) {  // 0: staged join; 2: direct, then rerun staged (tests the fallback)
        c->directJoin = atoi(e) != 0;
        c->directRetry = atoi(e) == 2;
        c->spillShift = atoi(e) == 3 ? 2 : 0;
    }
    if (const char* e = getenv("MTB_SEGSORT_GLOBAL")) c->segsortGlobal = atoi(e) != 0;
    if (const char* e = getenv("MTB_MERGE_SEG")) c->mergeSeg = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("MTB_WAVE_TAXON")) c->waveTaxon = atoi(e) == 2 ? 2 : atoi(e) ? 1 : 0;
    if (const char* e = getenv("MTB_PRUNE_COMPACT")) c->pruneCompact = atoi(e) != 0;
    if (const char* e = getenv("MTB_BIG_GROUPS")) c->bigGroups = atoi(e) != 0;
    if (const char* e = getenv("MTB_FUSE_FILTER")) c->fuseFilter = atoi(e) != 0;
    if (const char* e = getenv("MTB_PRESENT_SHARE")) c->presentShare = std::max(1e-6, atof(e));  // tests: filter reruns
    if (const char* e = getenv("MTB_PRUNE_AFTER")) c->pruneAfter = atoi(e) == 1 ? 1 : atoi(e) == 0 ? 0 : atoi(e) == 4 ? 4 : 2;
    if (const char* e = getenv("MTB_EMULATE_SORT")) c->emulateAll = atoi(e) != 0;
    if (const char* e = getenv("MTB_K6_ALIAS")) c->noAlias = atoi(e) == 0;
    if (c->forceGeneric) c->matchWinCap = 0;
    c->dir = make_aa_dir(c->D, par->kmer_format);
    HIP_TRY(hipMalloc(&c->dirMem, (c->dir.R + 1) * sizeof(uint64_t)));
    c->dir.dir = c->dirMem;
    build_aa_dir(c->db, c->D, c->dir, c->dirMem, s);
    HIP_TRY(hipStreamSynchronize(s));
    c->openS[2] = since(tp);
    if (const char* e = getenv("MTB_JOIN"))
        c->joinMode = !strcmp(e, "sort") ? 1 : !strcmp(e, "probe") ? 2 : !strcmp(e, "sweep") ? 3 : 0;
    if (const char* e = getenv("MTB_SWEEP_NOM")) c->sweepNom = std::max(64u, std::min(4096u, (uint32_t)atoi(e)));
    if (const char* e = getenv("MTB_SWEEP_LDS")) c->sweepLdsCap = (uint32_t)strtoul(e, nullptr, 10);
    if (const char* e = getenv("MTB_SWEEP_PERSIST")) c->sweepPersist = std::max(0, std::min(2, atoi(e)));
    if (const char* e = getenv("MTB_SWEEP_SMALL")) c->sweepSmall = atoi(e) != 0;
    if (const char* e = getenv("MTB_FILTER_PACK")) c->filterThreadMajor = std::string(e) == "thread";
    // the warp-specialised sweep stages 24-KB tiles: nominal 1024 records (tiles ~ one bucket)
    if ((c->sweepSmall || c->sweepPersist == 2) && !getenv("MTB_SWEEP_NOM")) c->sweepNom = 1024;
    if (const char* e = getenv("MTB_FILTER")) c->noFilter = atoi(e) == 0;
    if (const char* e = getenv("MTB_RADIX_DIGITS")) c->radixDigits = atoi(e) != 0;
    if (const char* e = getenv("MTB_RADIX_ATOMIC_FIRST")) c->radixAtomicFirst = atoi(e) != 0;
    if (const char* e = getenv("MTB_K1F_BINS")) c->binnedSort = atoi(e);
    if (const char* e = getenv("MTB_K1F_BINS_RC")) c->binRcForce = strtoull(e, nullptr, 10);
    if (const char* e = getenv("MTB_K1F_BINS_DIG")) c->binDigits = atoi(e) != 0;
    if (const char* e = getenv("MTB_UNIFORM_UNITS")) c->uniformUnits = atoi(e) != 0;
    if (!c->forceGeneric && !(c->joinMode == 3 && c->noFilter)) {
        HIP_TRY(hipMalloc(&c->lines, kProbeLines * sizeof(ProbeLine)));
        HIP_TRY(hipMemsetAsync(c->lines, 0, kProbeLines * sizeof(ProbeLine), s));
        build_probe_lines(c->db, c->D, c->dir, c->lines, s);
        // link lines for the fused K1F (the sort-merge join's; MTB_LINK_LINES=0, A/B: probe lines only).
        // A device without the 14.4 GB left for them runs without (same results, one probe per window)
        const char* ll = getenv("MTB_LINK_LINES");
        if ((!ll || atoi(ll) != 0) && c->joinMode != 2 && c->joinMode != 3) {
            if (hipMalloc(&c->link, kLinkSlots * sizeof(uint64_t)) == hipSuccess) {
                build_link_lines(c->lines, c->link, s);
            } else {
                (void)hipGetLastError();  // the failed allocation's error is not the open's
                c->link = nullptr;
            }
        }
        HIP_TRY(hipStreamSynchronize(s));
        c->openS[3] = since(tp);
        const char* ri = getenv("MTB_RUN_INDEX");  // 0: no run index (the unstaged join gallops)
        if ((!ri || atoi(ri) != 0) && c->joinMode != 3) {  // the sweep join reads no run index
            uint32_t* pop = nullptr;
            void* tmp = nullptr;
            uint64_t P = 0;
            HIP_TRY(hipMalloc(&c->lineP, (kProbeLines + 1) * sizeof(uint64_t)));
            HIP_TRY(hipMalloc(&pop, kProbeLines * sizeof(uint32_t)));
            HIP_TRY(hipMalloc(&tmp, scan_tmp_elems(kProbeLines) * sizeof(uint64_t)));
            build_line_prefix(c->lines, c->lineP, pop, tmp, s);
            HIP_TRY(hipMemcpyAsync(&P, c->lineP + kProbeLines, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            hipFree(pop);
            hipFree(tmp);
            HIP_TRY(hipMalloc(&c->runOff, (P + 1) * sizeof(uint16_t)));
            HIP_TRY(hipMemsetAsync(c->runOff + P, 0, sizeof(uint16_t), s));  // the end entry is never a run's
            build_run_offsets(c->db, c->D, c->lines, c->lineP, c->runOff, s);
            // MTB_LINE_EXT=1 (A/B, off: the join went 55.9 -> 57.2-60.2 ms, profiles/r05/ab_lineext.json):
            // run-length lines, so K4 finds most runs without the run-index read
            const char* le = getenv("MTB_LINE_EXT");
            if (le && atoi(le) != 0) {
                HIP_TRY(hipMalloc(&c->lineExt, kProbeLines * sizeof(ProbeExt)));
                build_line_ext(c->lines, c->lineP, c->runOff, c->lineExt, s);
            }
        }
    }
    HIP_TRY(hipGetLastError());  // a failed launch (e.g. a bad grid) must not pass silently
    HIP_TRY(hipStreamSynchronize(s));
    c->openS[4] = since(tp);
    // taxonomy + taxId2speciesId
    const HostTaxonomy& T = db.tax;
    c->maxTax = T.maxTax;
    c->hNodeOf = T.nodeOf;
    c->hRank = T.rank;
    c->hTax = T;
    HIP_TRY(upload(&c->spOf, db.speciesOf, s));
    HIP_TRY(upload(&c->tNodeOf, T.nodeOf, s));
    HIP_TRY(upload(&c->tNodeTax, T.nodeTax, s));
    HIP_TRY(upload(&c->tParent, T.parent, s));
    HIP_TRY(upload(&c->tDepth, T.depth, s));
    HIP_TRY(upload(&c->tSpParent, T.spParent, s));
    HIP_TRY(upload(&c->tFlags, T.flags, s));
    // clade scratch per match: 1 + deepest chain from a node up to its species
    int maxSub = 0;
    for (size_t i = 0; i < T.nodeTax.size(); i++) {
        int32_t sp = T.taxIdAtRank(T.nodeTax[i], "species");
        if (!T.exists(sp)) continue;
        int spNode = T.nodeOf[sp];
        if (T.lcaNode((int)i, spNode) != spNode) continue;
        maxSub = std::max(maxSub, T.depth[i] - T.depth[spNode]);
    }
    c->cladePerMatch = (uint32_t)(maxSub + 1);
    HIP_TRY(hipStreamSynchronize(s));
    c->dbArrays = std::make_shared<DbArrays>();
    c->dbArrays->device = device;
    c->dbArrays->own = {c->borrowedDb ? nullptr : c->db, c->dirMem, c->lines, c->lineP, c->runOff, c->lineExt, c->link, c->spOf,
                        c->tNodeOf, c->tNodeTax, c->tParent, c->tDepth, c->tSpParent, c->tFlags};
    bind_workspace(c, 0);
    c->openS[5] = since(tp);
    c->openS[6] = readS + std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return MTB_OK;
}


static int open_common(HostDb& db, const mtb_params* par, int device, mtb_ctx** out,
                       const mtb_db_resident* res = nullptr, double readS = 0) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc = validate_params(par);
    if (rc != MTB_OK) return rc;
    if (res) {
        // a resident part of a range-partitioned DB (db_parts > 1): the caller passes the part's own
        // records, its last one the next part's first k-mer (as slice_db_part keeps it), or none
        // after the last part
        if (!res->records || res->n_kmers < 2) { set_error("resident DB needs >= 2 k-mers"); return MTB_ERR_DB; }
    } else {
        if (!check_db(db)) return MTB_ERR_DB;
        if (db.nInfo < 2) { set_error("DB has fewer than 2 k-mers"); return MTB_ERR_DB; }
        if (par->db_parts > 1 && !slice_db_part(db, par->db_part, par->db_parts)) return MTB_ERR_DB;
    }
    mtb_ctx* c = new mtb_ctx();
    rc = open_into(c, db, par, device, res, readS, t0);
    if (rc != MTB_OK) {
        const std::string msg = mtb_last_error();  // mtb_close must not mask the opening's error
        mtb_close(c);
        set_error(msg);
        return rc;
    }
    *out = c;
    return MTB_OK;
}

extern "C" {

int mtb_open(const char* db_dir, const mtb_params* par, int device, mtb_ctx** out) {
    if (!db_dir || !par || !out) { set_error("null argument"); return MTB_ERR_ARG; }
    HostDb db;
    const auto t0 = std::chrono::steady_clock::now();
    // a whole-DB context reads diffIdx / info straight into HBM; a partition is cut on the host
    if (!load_db_files(db_dir, db, par->db_parts <= 1)) return MTB_ERR_IO;
    const double readS = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const int rc = open_common(db, par, device, out, nullptr, readS);
    if (rc == MTB_OK) (*out)->dbDir = db_dir;  // --em: sp2uniqKmerCnt lives next to the DB files
    return rc;
}

int mtb_open_host(const mtb_db_host* h, const mtb_params* par, int device, mtb_ctx** out) {
    if (!h || !par || !out) { set_error("null argument"); return MTB_ERR_ARG; }
    HostDb db;
    if (par->db_parts > 1) {  // the part is cut from host copies
        db.diffIdx.assign(h->diff_idx, h->diff_idx + h->n_diff_idx);
        db.info.assign(h->info, h->info + h->n_info);
        db.use_vectors();
    } else {  // the caller's arrays, uploaded in place
        db.diffP = h->diff_idx;
        db.nDiff = h->n_diff_idx;
        db.infoP = h->info;
        db.nInfo = h->n_info;
    }
    if (h->split) db.split.assign(h->split, h->split + 3 * h->n_split);
    db.taxIdList.assign(h->taxid_list, h->taxid_list + h->n_taxid_list);
    std::vector<std::string> ranks(h->n_nodes), names(h->n_nodes);
    for (uint64_t i = 0; i < h->n_nodes; i++) {
        ranks[i] = h->rank_pool + h->rank_off[i];
        if (h->name_pool) names[i] = h->name_pool + h->name_off[i];
    }
    if (!build_taxonomy(h->node_taxid, h->node_parent, h->n_nodes, ranks, names, h->merged_old, h->merged_new,
                        h->n_merged, db.tax) ||
        !build_species_map(db))
        return MTB_ERR_DB;
    return open_common(db, par, device, out);
}

int mtb_open_resident(const mtb_db_resident* r, const mtb_db_host* h, const mtb_params* par, int device,
                      mtb_ctx** out) {
    if (!r || !h || !par || !out) { set_error("null argument"); return MTB_ERR_ARG; }
    HostDb db;
    db.taxIdList.assign(h->taxid_list, h->taxid_list + h->n_taxid_list);
    std::vector<std::string> ranks(h->n_nodes), names(h->n_nodes);
    for (uint64_t i = 0; i < h->n_nodes; i++) {
        ranks[i] = h->rank_pool + h->rank_off[i];
        if (h->name_pool) names[i] = h->name_pool + h->name_off[i];
    }
    if (!build_taxonomy(h->node_taxid, h->node_parent, h->n_nodes, ranks, names, h->merged_old, h->merged_new,
                        h->n_merged, db.tax) ||
        !build_species_map(db))
        return MTB_ERR_DB;
    return open_common(db, par, device, out, r);
}

int mtb_clone(const mtb_ctx* src, mtb_ctx** out) {
    if (!src || !out) { set_error("null argument"); return MTB_ERR_ARG; }
    mtb_ctx* c = new mtb_ctx();
    c->device = src->device;
    c->par = src->par;
    c->tables = src->tables;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->ownStream = true;
    for (auto& e : c->ev) HIP_TRY(hipEventCreate(&e));
    for (auto& e : c->kev) HIP_TRY(hipEventCreate(&e));
    // the DB, its directory, probe lines and run index, the species map and the taxonomy: shared
    c->dbArrays = src->dbArrays;
    c->D = src->D;
    c->db = src->db;
    c->borrowedDb = src->borrowedDb;
    c->dirMem = src->dirMem;
    c->lines = src->lines;
    c->lineP = src->lineP;
    c->runOff = src->runOff;
    c->lineExt = src->lineExt;
    c->link = src->link;
    c->dir = src->dir;
    c->rankLo = src->rankLo;
    c->rankHi = src->rankHi;
    c->spOf = src->spOf;
    c->maxTax = src->maxTax;
    c->tNodeOf = src->tNodeOf;
    c->tNodeTax = src->tNodeTax;
    c->tParent = src->tParent;
    c->tDepth = src->tDepth;
    c->tSpParent = src->tSpParent;
    c->tFlags = src->tFlags;
    c->cladePerMatch = src->cladePerMatch;
    c->hNodeOf = src->hNodeOf;
    c->hRank = src->hRank;
    c->hTax = src->hTax;
    c->dbDir = src->dbDir;
    c->spKmers = src->spKmers;
    // the opening's knobs
    c->joinMode = src->joinMode;
    c->sweepNom = src->sweepNom;
    c->sweepLdsCap = src->sweepLdsCap;
    c->sweepSmall = src->sweepSmall;
    c->filterThreadMajor = src->filterThreadMajor;
    c->sweepPersist = src->sweepPersist;
    c->matchWinCap = src->matchWinCap;
    c->directJoin = src->directJoin;
    c->directRetry = src->directRetry;
    c->pruneAfter = src->pruneAfter;
    c->bigGroups = src->bigGroups;
    c->fuseFilter = src->fuseFilter;
    c->presentShare = src->presentShare;
    c->spillShift = src->spillShift;
    c->sortLoFine = src->sortLoFine;
    c->forceGeneric = src->forceGeneric;
    c->segsortGlobal = src->segsortGlobal;
    c->mergeSeg = src->mergeSeg;
    c->waveTaxon = src->waveTaxon;
    c->emulateAll = src->emulateAll;
    c->pruneCompact = src->pruneCompact;
    c->noAlias = src->noAlias;
    c->noFilter = src->noFilter;
    c->radixDigits = src->radixDigits;
    c->radixAtomicFirst = src->radixAtomicFirst;
    c->binnedSort = src->binnedSort;
    c->binRcForce = src->binRcForce;
    c->binDigits = src->binDigits;
    c->uniformUnits = src->uniformUnits;
    bind_workspace(c, src->ws.cap);
    *out = c;
    return MTB_OK;
}

// Every grow-only batch buffer of a context (freed by mtb_close; their sum is the context's
// workspace, mtb::ctx_workspace_bytes).
#define MTB_BATCH_BUFS(X) \
    X(seq1) X(off1) X(seq2) X(off2) X(meta) X(reserve) X(slotOff) X(qlen) X(scanTmp) X(keysA) X(valsA) X(keysB) \
    X(valsB) X(radixCounts) X(radixOffs) X(readCnt) X(mOff) X(matches) X(matchesSorted) X(segScratch) X(maxSeg) \
    X(errFlag) X(ordKA) X(ordVA) X(ordKB) X(ordVB) X(matchWin) X(unitRead) X(unitInfo) X(waveList) X(waveCount) \
    X(devStats) X(mStage) X(mRank) X(mDirect) X(ovFlag) X(mTotal) X(qFrom) X(probeStats) X(longList) X(longCnt) \
    X(qStart) X(chunkIn) X(chunkCnt) X(chunkSrcOff) X(liveCnt) X(liveOff) X(segLen) X(sizeLists) X(digA) \
    X(digB) X(binCnt) X(binTab) X(local) X(paths) X(comb) X(conn) X(spScore) X(spKeep) X(gFlag) X(sFlag) \
    X(pathCnt) X(gScan) X(sScan) X(gStart) X(sStart) X(clade) X(tcPool) X(tcLen) X(tcOff) X(tcOut) X(results) \
    X(emMap) X(emCnt) X(emScratch) X(emPacked) X(emCnt32) X(emOff) X(maskOut1) X(maskOut2) X(maskProb) \
    X(maskScale) X(readLens) X(readCnt64)
static std::vector<DevBuf*> batch_bufs(mtb_ctx* c) {
#define MTB_BUF_PTR(n) &c->n,
    return {MTB_BATCH_BUFS(MTB_BUF_PTR)};
#undef MTB_BUF_PTR
}

static const char* const* batch_buf_names() {
#define MTB_BUF_NAME(n) #n,
    static const char* const names[] = {MTB_BATCH_BUFS(MTB_BUF_NAME)};
#undef MTB_BUF_NAME
    return names;
}

void mtb_close(mtb_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    free_db(c);
    if (c->tileRec) hipFree(c->tileRec);
    if (c->tilePre) hipFree(c->tilePre);
    c->pipelineCache.reset();  // pinned slots and their device buffers (on c->device)
    hipSetDevice(c->device);
    for (DevBuf* b : batch_bufs(c)) b->release();
    for (auto& e : c->ev)
        if (e) hipEventDestroy(e);
    for (auto& e : c->kev)
        if (e) hipEventDestroy(e);
    if (c->ownStream && c->stream) hipStreamDestroy(c->stream);
    delete c;
}

int mtb_set_stream(mtb_ctx* c, void* stream) {
    if (!c) return MTB_ERR_ARG;
    if (c->ownStream && c->stream) hipStreamDestroy(c->stream);
    if (stream) {
        c->stream = (hipStream_t)stream;
        c->ownStream = false;
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->ownStream = true;
    }
    return MTB_OK;
}

uint64_t mtb_db_kmers(const mtb_ctx* c) { return c ? c->D : 0; }

uint64_t mtb_workspace_bytes(const mtb_ctx* c) { return c ? c->ws.used : 0; }

int mtb_open_phases(const mtb_ctx* c, double* sec, int n) {
    if (!c || !sec) return MTB_ERR_ARG;
    for (int i = 0; i < n && i < 8; i++) sec[i] = c->openS[i];
    return MTB_OK;
}

int mtb_set_workspace_cap(mtb_ctx* c, uint64_t bytes) {
    if (!c) return MTB_ERR_ARG;
    c->ws.cap = bytes;
    return MTB_OK;
}

int mtb_release_workspace(mtb_ctx* c) {
    if (!c) return MTB_ERR_ARG;
    mtb::ctx_release_workspace(c);
    // one allocation settles the runtime's deferred release of the freed buffers (measured: the
    // first allocation after giving back ~80 GB took 2.4 s)
    void* p = nullptr;
    if (hipMalloc(&p, 64u << 20) == hipSuccess) hipFree(p);
    return hipDeviceSynchronize() == hipSuccess ? MTB_OK : MTB_ERR_HIP;
}

int mtb_ctx_device(const mtb_ctx* c) { return c ? c->device : 0; }

}  // extern "C"

static AssignArgs assign_args(const mtb_params& p) {
    AssignArgs a;
    a.em = p.em ? 1 : 0;
    a.kmerFormat = p.kmer_format;
    if (p.syncmer) {  // Taxonomer.cpp:34-42
        a.dnaShift = (8 - p.smer_len) * 3;
        a.maxCodonShift = 8 - p.smer_len;
    } else {
        a.dnaShift = 3;
        a.maxCodonShift = 1;
    }
    a.denominator = (p.seq_mode == 1 || p.seq_mode == 2) ? 100 : 1000;  // Taxonomer.cpp:44-48
    a.minConsCnt = p.min_cons_cnt;
    a.minConsCntEuk = p.min_cons_cnt_euk;
    a.accessionLevel = p.accession_level;
    a.minScore = p.min_score;
    a.minSpScore = p.min_sp_score;
    a.tieRatio = p.tie_ratio;
    a.generic = 0;
    return a;
}

// K5 + K6 + taxcnt compaction on the matches already grouped by read in c->matches (mOff).
// keep: no dead-match pruning in K5, so matchesSorted holds every match in compareMatches order
// afterwards (mtb_get_matches); the caller decides, nothing is inherited from an earlier call.
static int assign_stage(mtb_ctx* c, uint32_t n, bool keep) {
    hipStream_t s = c->stream;
    HIP_TRY(c->errFlag.ensure(sizeof(int)));  // mtb_assign_* may run before any batch
    const uint64_t M = c->M;
    AssignArgs a = assign_args(c->par);
    a.generic = c->forceGeneric ? 1 : 0;
    a.waveTaxon = c->waveTaxon;
    a.bigGroups = c->bigGroups;
    a.emulateAll = c->emulateAll;
    if (a.dnaShift <= 0) { set_error("syncmer smer_len 8 gives a zero dnaShift"); return MTB_ERR_ARG; }
    HIP_TRY(c->readCnt.ensure(sizeof(uint32_t) * (n + 1)));
    const uint64_t Mc = std::max<uint64_t>(M, 1);
    HIP_TRY(c->results.ensure(sizeof(mtb_result) * std::max<uint32_t>(n, 1)));
    // K5: per-read segmented sort into compareMatches order
    HIP_TRY(c->matchesSorted.ensure(sizeof(mtb_match) * Mc));
    HIP_TRY(c->maxSeg.ensure(sizeof(uint32_t)));
    launch_max_seg(c->mOff.as<uint64_t>(), n, c->maxSeg.as<uint32_t>(), s);
    uint32_t maxSeg = 0;
    HIP_TRY(hipMemcpyAsync(&maxSeg, c->maxSeg.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // dead matches (species with no path-capable (species, frame) group) are dropped in K5 unless
    // the batch keeps its stages (mtb_get_matches returns every match) or runs the general paths
    const bool prune = !keep && !c->forceGeneric;
    if (maxSeg > kSegSortLds || c->forceGeneric || c->segsortGlobal || (c->mergeSeg && maxSeg > c->mergeSeg))
        HIP_TRY(c->segScratch.ensure(6 * sizeof(uint64_t) * Mc));
    const bool compact = prune && maxSeg > kSegSortRegs && !c->segsortGlobal && c->pruneCompact;
    if (compact) HIP_TRY(c->segLen.ensure(sizeof(uint32_t) * (n + 1)));  // big segments thinned before sorting
    if (maxSeg > 128) HIP_TRY(c->sizeLists.ensure(sizeof(uint32_t) * (4 * (size_t)n + 4)));
    c->keepStages = !prune;  // mtb_get_matches: matchesSorted is complete only without pruning
    HIP_TRY(c->liveCnt.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(c->liveOff.ensure(sizeof(uint64_t) * (n + 1)));
    HIP_TRY(c->scanTmp.ensure(sizeof(uint64_t) * scan_tmp_elems(n + 1)));
    HIP_TRY(hipEventRecord(c->kev[10], s));
    // K5 reads sparse segments up to kSegSortSparse, and thins bigger ones straight from their stretches
    if (c->sparse && (!prune || (maxSeg > kSegSortSparse && !compact) || c->segsortGlobal ||
                      (c->mergeSeg && maxSeg > c->mergeSeg))) {
        // the reads that overflowed their stretch were compacted with their spills by join_stage:
        // re-copying them would put stale stretch entries over the scattered spills
        launch_compact_segments(c->mDirect.as<SegMatch>(), c->slotOff.as<uint64_t>(), c->chunkC,
                                c->mOff.as<uint64_t>(), n, c->matches.as<mtb_match>(), c->spillShift, s,
                                c->stats[13] ? 2 : 0);
        c->sparse = false;
    }
    HIP_TRY(launch_segsort(c->matches.as<mtb_match>(), c->mOff.as<uint64_t>(), n, Mc, c->matchesSorted.as<mtb_match>(),
                           c->segScratch.as<uint64_t>(), maxSeg, c->forceGeneric || c->segsortGlobal,
                           prune ? c->liveCnt.as<uint32_t>() : nullptr, c->mergeSeg,
                           prune_min_matches(a.minConsCnt, a.minConsCntEuk, a.maxCodonShift), s,
                           c->sparse ? c->mDirect.as<SegMatch>() : nullptr, c->slotOff.as<uint64_t>(),
                           c->chunkC | c->spillShift << 16,
                           compact ? c->segLen.as<uint32_t>() : nullptr,
                           c->maxSeg.as<uint32_t>(), c->pruneAfter, maxSeg > 128 ? c->sizeLists.as<uint32_t>() : nullptr));
    c->sparse = false;
    const mtb_match* kIn = c->matchesSorted.as<mtb_match>();
    const uint64_t* kOff = c->mOff.as<uint64_t>();
    uint64_t kM = M;
    if (prune) {
        exclusive_scan_u32(c->liveCnt.as<uint32_t>(), n, c->liveOff.as<uint64_t>(), c->scanTmp.p, s);
        HIP_TRY(hipMemcpyAsync(&kM, c->liveOff.as<uint64_t>() + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        launch_pack_live(c->matchesSorted.as<mtb_match>(), c->mOff.as<uint64_t>(), c->liveOff.as<uint64_t>(), n,
                         c->matches.as<mtb_match>(), c->errFlag.as<int>(), s);  // K5's input buffer is free again
        HIP_TRY(hipStreamSynchronize(s));
        if (kM > M) { set_error("internal error: K5 kept more matches than it sorted"); return MTB_ERR_INTERNAL; }
        kIn = c->matches.as<mtb_match>();
        kOff = c->liveOff.as<uint64_t>();
    }
    c->liveM = kM;
    c->stats[11] = kM;
    // K6 scratch, per match K6 reads: sized by the live matches (less than half of all at GTDB scale).
    // It is carved out of the batch buffers K5 left dead — the direct join's slot-sized segments,
    // the query keys and slots, the unpruned sorted matches, K5's global scratch, the spill — and
    // only what does not fit there takes buffers of its own: at GTDB scale that is ~25 GB per
    // 2M-pair batch that the larger QuerySplits need.
    const uint64_t Kc = std::max<uint64_t>(kM, 1);
    const uint64_t Mn = std::max<uint64_t>(Kc, n);  // K6 work lists: groups (<= live matches) and the read order
    std::vector<std::pair<char*, size_t>> dead;      // (next free byte, bytes left) per dead buffer
    if (!c->noAlias) {
        std::vector<DevBuf*> d = {&c->mDirect, &c->segScratch, &c->mStage, &c->mRank, &c->matchWin, &c->chunkIn};
        if (prune) {  // else the sorted matches are the result and the query keys stay readable (mtb_get_*)
            for (DevBuf* b : {&c->matchesSorted, &c->keysA, &c->valsA, &c->keysB, &c->valsB}) d.push_back(b);
        } else {
            d.push_back(&c->matches);
        }
        for (DevBuf* b : d)
            if (b->p && b->bytes >= (1u << 20)) dead.push_back({b->as<char>(), b->bytes});
        std::sort(dead.begin(), dead.end(), [](auto& a, auto& b) { return a.second > b.second; });
    }
    struct Need {
        DevBuf* own;
        uint64_t bytes;
        void* p;
    };
    Need need[] = {{&c->local, path_bytes() * Kc, nullptr},
                   {&c->paths, path_bytes() * Kc, nullptr},
                   {&c->comb, path_bytes() * Kc, nullptr},
                   {&c->conn, Kc, nullptr},
                   {&c->spScore, sizeof(float) * Kc, nullptr},
                   {&c->spKeep, Kc, nullptr},
                   {&c->waveList, sizeof(uint64_t) * Kc, nullptr},
                   {&c->gFlag, sizeof(uint32_t) * (Kc + 1), nullptr},
                   {&c->pathCnt, sizeof(uint32_t) * (Kc + 1), nullptr},
                   {&c->sFlag, std::max<uint64_t>(sizeof(uint32_t) * (Kc + 1), run_index_tmp_bytes(Kc)), nullptr},
                   {&c->gScan, sizeof(uint64_t) * (Kc + 1), nullptr},
                   {&c->sScan, sizeof(uint64_t) * (Kc + 1), nullptr},
                   {&c->gStart, sizeof(uint64_t) * (Kc + 1), nullptr},
                   {&c->sStart, sizeof(uint64_t) * (Kc + 1), nullptr},
                   {&c->clade, clade_bytes() * Kc * c->cladePerMatch, nullptr},
                   {&c->tcPool, sizeof(mtb_taxcnt) * Kc, nullptr},
                   {&c->ordKA, sizeof(uint64_t) * (Mn + 1), nullptr},
                   {&c->ordVA, sizeof(uint64_t) * (Mn + 1), nullptr},
                   {&c->ordKB, sizeof(uint64_t) * (Mn + 1), nullptr},
                   {&c->ordVB, sizeof(uint64_t) * (Mn + 1), nullptr}};
    std::vector<Need*> order;
    for (Need& x : need) order.push_back(&x);
    std::stable_sort(order.begin(), order.end(), [](Need* a, Need* b) { return a->bytes > b->bytes; });
    c->aliasBytes = 0;
    for (Need* x : order) {  // first fit, largest first; 256-B aligned pieces
        const size_t b = (x->bytes + 255) & ~(size_t)255;
        for (auto& r : dead)
            if (r.second >= b) {
                x->p = r.first;
                r.first += b;
                r.second -= b;
                c->aliasBytes += b;
                break;
            }
        if (!x->p) {
            HIP_TRY(x->own->ensure(x->bytes));
            x->p = x->own->p;
        }
    }
    HIP_TRY(c->waveCount.ensure(sizeof(uint32_t)));
    HIP_TRY(hipEventRecord(c->kev[11], s));
    HIP_TRY(hipEventRecord(c->kev[12], s));
    HIP_TRY(c->radixCounts.ensure(sizeof(uint32_t) * radix_counts_elems(Mn + 1)));
    HIP_TRY(c->radixOffs.ensure(sizeof(uint64_t) * (radix_counts_elems(Mn + 1) + 1)));
    HIP_TRY(c->scanTmp.ensure(sizeof(uint64_t) * scan_tmp_elems(radix_counts_elems(Mn + 1) + n + Mn + 2)));
    TaxDevice t{c->tNodeOf, c->tNodeTax, c->tParent, c->tDepth, c->tFlags, c->tSpParent, c->maxTax};
    AssignScratch sc{need[0].p,
                     need[1].p,
                     need[2].p,
                     (uint8_t*)need[3].p,
                     (uint32_t*)need[7].p,
                     (uint32_t*)need[9].p,
                     (uint32_t*)need[8].p,
                     (uint64_t*)need[10].p,
                     (uint64_t*)need[11].p,
                     (uint64_t*)need[12].p,
                     (uint64_t*)need[13].p,
                     (float*)need[4].p,
                     (uint64_t*)need[6].p,
                     c->waveCount.as<uint32_t>(),
                     (uint8_t*)need[5].p,
                     c->scanTmp.p,
                     (uint64_t*)need[16].p,
                     (uint64_t*)need[17].p,
                     (uint64_t*)need[18].p,
                     (uint64_t*)need[19].p,
                     c->radixCounts.as<uint32_t>(),
                     c->radixOffs.as<uint64_t>(),
                     need[14].p,
                     c->cladePerMatch};
    mtb_taxcnt* tcPool = (mtb_taxcnt*)need[15].p;
    c->stats[3] = M;
    c->stats[4] = maxSeg;
    launch_assign(kIn, kOff, c->qlen.as<uint32_t>(), n, kM, a, t, sc, tcPool,
                  c->results.as<mtb_result>(), c->devStats.as<unsigned long long>(), c->stats + 5, s);
    HIP_TRY(hipEventRecord(c->kev[13], s));
    HIP_TRY(c->tcLen.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(c->tcOff.ensure(sizeof(uint64_t) * (n + 1)));
    launch_taxcnt_len(c->results.as<mtb_result>(), n, c->tcLen.as<uint32_t>(), s);
    exclusive_scan_u32(c->tcLen.as<uint32_t>(), n, c->tcOff.as<uint64_t>(), c->scanTmp.p, s);
    uint64_t NT = 0;
    HIP_TRY(hipMemcpyAsync(&NT, c->tcOff.as<uint64_t>() + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(c->tcOut.ensure(sizeof(mtb_taxcnt) * std::max<uint64_t>(NT, 1)));
    launch_compact_taxcnt(tcPool, kOff, c->results.as<mtb_result>(), c->tcOff.as<uint64_t>(), n,
                          c->tcOut.as<mtb_taxcnt>(), s);
    c->nTaxcnt = NT;
    c->emValid = false;
    c->emPackedValid = false;
    if (c->par.em) {  // the mappings of Reporter::writeMappings (kEmTop best species per classified read)
        const uint64_t nS = std::max<uint64_t>(c->stats[7], 1);
        HIP_TRY(c->emScratch.ensure(8 * nS));
        HIP_TRY(c->emMap.ensure(8 * (uint64_t)kEmTop * std::max<uint32_t>(n, 1)));
        HIP_TRY(c->emCnt.ensure(std::max<uint32_t>(n, 1)));
        launch_em_top(kIn, kOff, n, sc, c->results.as<mtb_result>(), c->emScratch.p, c->emMap.p,
                      c->emCnt.as<uint8_t>(), s);
        HIP_TRY(hipGetLastError());
        c->emValid = true;
    }
    return MTB_OK;
}

// K1 -> K1F filter -> K4 join (probe join, or radix sort + sort-merge join) -> transpose into
// per-read segments. Kernel timers: 0 extract, 1 filter, 2 sort, 3 join, 4 transpose.
static int join_stage(mtb_ctx* c, const uint8_t* dSeq1, const uint64_t* dOff1, const uint8_t* dSeq2,
                      const uint64_t* dOff2, uint32_t n, uint64_t U, uint32_t C, uint64_t R, uint64_t Rc) {
    hipStream_t s = c->stream;
    const bool probe = c->probed;
    const bool filt = c->lines && (!c->noFilter || probe);  // K1F: only the windows whose AA 8-mer the DB holds go on
    const bool fused = filt && !probe && c->fuseFilter;
    // The fused K1 + K1F writes only the present windows (Q, about half the slots at GTDB scale):
    // its output is sized by the largest present share seen (+1/8) instead of every slot, and the
    // sort's other side by Q once it is known; a batch past that share reruns the filter into a
    // larger buffer. The unfused paths write a key per slot.
    if (!fused) {
        HIP_TRY(c->keysA.ensure(8 * Rc));
        HIP_TRY(c->valsA.ensure(4 * Rc));
        HIP_TRY(c->keysB.ensure(8 * Rc));
        HIP_TRY(c->valsB.ensure(4 * Rc));
    }
    HIP_TRY(c->radixCounts.ensure(sizeof(uint32_t) * radix_counts_elems(Rc)));
    HIP_TRY(c->radixOffs.ensure(sizeof(uint64_t) * (radix_counts_elems(Rc) + 1)));
    HIP_TRY(c->scanTmp.ensure(sizeof(uint64_t) * scan_tmp_elems(radix_counts_elems(Rc) + n + 1)));
    HIP_TRY(c->mTotal.ensure(sizeof(unsigned long long) * kStageRegions));
    HIP_TRY(c->probeStats.ensure(sizeof(unsigned long long) * kProbeStatsLen));
    HIP_TRY(hipMemsetAsync(c->probeStats.p, 0, sizeof(unsigned long long) * kProbeStatsLen, s));
    // K1 extract: every window's key (the sentinel where no k-mer is emitted); fused with K1F for
    // the sort-merge join (the keys never reach HBM: timed as the filter)
    HIP_TRY(hipEventRecord(c->kev[0], s));
    if (!fused)
        launch_extract(dSeq1, dOff1, dSeq2, dOff2, c->meta.as<ReadMeta>(), c->slotOff.as<uint64_t>(),
                       c->unitRead.as<uint32_t>(), U, C, c->tables, c->par.kmer_format, c->par.syncmer,
                       c->par.smer_len, c->keysA.as<uint64_t>(), c->unitInfo.as<uint64_t>(), s, c->upr);
    HIP_TRY(hipEventRecord(c->kev[1], s));
    // K1F: the windows whose AA 8-mer the DB holds (MTB_FORCE_GENERIC: no filter, the sort's first
    // pass drops the sentinels)
    uint64_t Q = R;
    const uint64_t* qk = c->keysA.as<uint64_t>();
    const uint32_t* qi = nullptr;
    const uint64_t* qf = nullptr;
    HIP_TRY(hipEventRecord(c->kev[2], s));
    // K2's digit side arrays: the fused K1F writes each kept key's first-pass digit (bits kQuerySortLo..)
    const bool digits = fused && c->radixDigits && c->sortLoFine == kQuerySortLo;
    uint64_t binRc = 0;  // > 0: the batch's K1F wrote K2's first-pass buckets of binRc slots
    if (fused) {
        uint64_t cap = std::min<uint64_t>(R, (uint64_t)((double)R * c->presentShare) + 4096);
        // binned K1F: 2048 buckets (first digit x XCD) of rc slots, 1/16 over the expected present
        // share plus 256 (the digits are near-uniform: the bits are the middle of a base-21 rank); a
        // bucket past rc sends the batch through the packed K1F once more (counted as a rerun)
        bool binned = digits && c->binnedSort && (c->binnedSort == 2 || cap >= (1ull << 22));
        for (int pass = 0; pass < 2 && binned; pass++) {
            uint64_t rc = c->binRcForce ? c->binRcForce : (cap + cap / 16) / kSortBins + 256;
            rc = (rc + 63) / 64 * 64;  // tile starts 16-B aligned for the digit loads
            const uint64_t slots = rc * kSortBins;
            HIP_TRY(c->keysB.ensure(8 * slots));
            HIP_TRY(c->valsB.ensure(4 * slots));
            HIP_TRY(c->digA.ensure(slots));
            HIP_TRY(c->binCnt.ensure(sizeof(unsigned long long) * kSortBins));
            Q = launch_extract_filter(dSeq1, dOff1, dSeq2, dOff2, c->meta.as<ReadMeta>(), c->slotOff.as<uint64_t>(),
                                      c->unitRead.as<uint32_t>(), U, C, c->tables, c->par.kmer_format, c->par.syncmer,
                                      c->par.smer_len, c->unitInfo.as<uint64_t>(), c->lines, c->keysB.as<uint64_t>(),
                                      c->valsB.as<uint32_t>(), c->mTotal.as<unsigned long long>(), c->rankLo,
                                      c->rankHi, &c->Qall, slots, false, s,
                                      c->binDigits ? c->digA.as<uint8_t>() : nullptr,
                                      c->binCnt.as<unsigned long long>(), rc, c->binHost, c->upr);
            HIP_TRY(hipGetLastError());
            if (R) c->presentShare = std::max(c->presentShare, std::min(1.0, 1.125 * (double)Q / (double)R));
            bool over = false;
            for (int r = 0; r < kSortBins; r++) over |= c->binHost[r] > rc;
            if (!over) {
                binRc = rc;
                break;
            }
            c->stats[15]++;  // a bucket overflowed: rerun packed, sized by the count just taken
            cap = std::min<uint64_t>(R, Q + Q / 8);
            binned = false;
        }
        for (int pass = 0; pass < 2 && !binRc; pass++) {
            HIP_TRY(c->keysB.ensure(8 * cap));
            HIP_TRY(c->valsB.ensure(4 * cap));
            if (digits) HIP_TRY(c->digA.ensure(cap));
            cap = std::min<uint64_t>(c->keysB.bytes / 8, c->valsB.bytes / 4);  // all the buffers hold
            if (digits) cap = std::min<uint64_t>(cap, c->digA.bytes);
            Q = launch_extract_filter(dSeq1, dOff1, dSeq2, dOff2, c->meta.as<ReadMeta>(), c->slotOff.as<uint64_t>(),
                                      c->unitRead.as<uint32_t>(), U, C, c->tables, c->par.kmer_format, c->par.syncmer,
                                      c->par.smer_len, c->unitInfo.as<uint64_t>(), c->lines, c->keysB.as<uint64_t>(),
                                      c->valsB.as<uint32_t>(), c->mTotal.as<unsigned long long>(), c->rankLo,
                                      c->rankHi, &c->Qall, cap, c->filterThreadMajor, s,
                                      digits ? c->digA.as<uint8_t>() : nullptr, nullptr, 0, nullptr, c->upr, c->link);
            HIP_TRY(hipGetLastError());
            if (Q == ~0ull) {  // launch_extract_filter's flag: a block's bases past K1F's LDS stage
                set_error("internal error: K1F sequence stage overflow");
                return MTB_ERR_INTERNAL;
            }
            if (R) c->presentShare = std::max(c->presentShare, std::min(1.0, 1.125 * (double)Q / (double)R));
            if (Q <= cap) break;
            cap = std::min<uint64_t>(R, Q + Q / 8);  // Q <= R: the second pass fits
            c->stats[15]++;                          // filter reruns (a batch past the present share)
        }
        HIP_TRY(c->keysA.ensure(8 * std::max<uint64_t>(Q, 1)));
        HIP_TRY(c->valsA.ensure(4 * std::max<uint64_t>(Q, 1)));
        if (digits) HIP_TRY(c->digB.ensure(std::max<uint64_t>(Q, 16)));
        qk = c->keysB.as<uint64_t>();
        qi = c->valsB.as<uint32_t>();
    } else if (filt) {
        if (probe) HIP_TRY(c->qFrom.ensure(8 * Rc + 8 * kDbPad));
        Q = launch_filter(c->keysA.as<uint64_t>(), R, c->lines, c->keysB.as<uint64_t>(), c->valsB.as<uint32_t>(),
                          probe ? c->qFrom.as<uint64_t>() : nullptr, c->mTotal.as<unsigned long long>(), c->rankLo,
                          c->rankHi, &c->Qall, s);
        qk = c->keysB.as<uint64_t>();
        qi = c->valsB.as<uint32_t>();
        qf = c->qFrom.as<uint64_t>();
    }
    HIP_TRY(hipEventRecord(c->kev[3], s));
    HIP_TRY(hipEventRecord(c->ev[1], s));
    // K2 (sort-merge join only): radix sort on the top 24 bits of the 36-bit AA rank. The join does
    // not need a total order (K5 puts each read's matches in compareMatches order); a sort prefix
    // of ~6 amino acids is all the locality its DB windows need: three passes instead of five.
    HIP_TRY(hipEventRecord(c->kev[4], s));
    const bool sweepJoin = c->joinMode == 3 && !probe && c->directJoin && !c->forceGeneric;
    const int sortLo = !sweepJoin && unstaged_join(c->lines != nullptr, c->D, Q, std::min<uint32_t>(c->matchWinCap, 3072))
                           ? c->sortLoFine : kQuerySortLo;
    if (!probe) {
        bool inB = false;
        if (binRc) {  // the first pass was K1F's: the tile table over its buckets, then the rest
            HIP_TRY(c->binTab.ensure(sizeof(uint64_t) * std::max<uint64_t>(radix_binned_tiles(c->binHost, binRc), 1)));
            const uint64_t rcn = radix_counts_elems(Q) + 256ull * kSortBins;
            HIP_TRY(c->radixCounts.ensure(sizeof(uint32_t) * rcn));
            HIP_TRY(c->radixOffs.ensure(sizeof(uint64_t) * (rcn + 1)));
            HIP_TRY(c->scanTmp.ensure(sizeof(uint64_t) * scan_tmp_elems(rcn + n + 1)));
            Q = radix_sort_binned(c->keysB.as<uint64_t>(), c->valsB.as<uint32_t>(), c->keysA.as<uint64_t>(),
                                  c->valsA.as<uint32_t>(), c->binHost, c->binCnt.as<unsigned long long>(), binRc,
                                  kQuerySortLo, kQuerySortHi, c->radixCounts.as<uint32_t>(),
                                  c->radixOffs.as<uint64_t>(), c->scanTmp.p, c->binTab.as<uint64_t>(), &inB, s,
                                  c->binDigits ? c->digA.as<uint8_t>() : nullptr, c->digB.as<uint8_t>());
            qk = inB ? c->keysA.as<uint64_t>() : c->keysB.as<uint64_t>();
            qi = inB ? c->valsA.as<uint32_t>() : c->valsB.as<uint32_t>();
        } else if (filt) {
            const bool dg = digits && sortLo == kQuerySortLo;
            Q = radix_sort_pairs(c->keysB.as<uint64_t>(), c->valsB.as<uint32_t>(), c->keysA.as<uint64_t>(),
                                 c->valsA.as<uint32_t>(), Q, sortLo, kQuerySortHi, false, false,
                                 c->radixCounts.as<uint32_t>(), c->radixOffs.as<uint64_t>(), c->scanTmp.p, &inB, s,
                                 dg ? c->digA.as<uint8_t>() : nullptr, dg ? c->digB.as<uint8_t>() : nullptr,
                                 c->radixAtomicFirst);
            qk = inB ? c->keysA.as<uint64_t>() : c->keysB.as<uint64_t>();
            qi = inB ? c->valsA.as<uint32_t>() : c->valsB.as<uint32_t>();
        } else {
            Q = radix_sort_pairs(c->keysA.as<uint64_t>(), c->valsA.as<uint32_t>(), c->keysB.as<uint64_t>(),
                                 c->valsB.as<uint32_t>(), R, kQuerySortLo, kQuerySortHi, true, true,
                                 c->radixCounts.as<uint32_t>(), c->radixOffs.as<uint64_t>(), c->scanTmp.p, &inB, s,
                                 nullptr, nullptr, c->radixAtomicFirst);
            qk = inB ? c->keysB.as<uint64_t>() : c->keysA.as<uint64_t>();
            qi = inB ? c->valsB.as<uint32_t>() : c->valsA.as<uint32_t>();
            c->Qall = Q;  // no membership filter: every non-blank window was sorted
        }
    }
    HIP_TRY(hipEventRecord(c->kev[5], s));
    HIP_TRY(hipEventRecord(c->ev[2], s));
    c->Q = Q;
    c->stats[1] = Q;
    const char* dupEnv = getenv("MTB_DUP_STATS");  // read per batch (a diagnostic the bench turns on for one batch)
    if (dupEnv && atoi(dupEnv) != 0 && !probe) {  // after the sort, before the join: what K4's blocks could share
        unsigned long long dup[2] = {0, 0};
        HIP_TRY(c->devStats.ensure(sizeof(unsigned long long) * 4));
        HIP_TRY(hipMemsetAsync(c->devStats.as<unsigned long long>() + 2, 0, 2 * sizeof(unsigned long long), s));
        launch_dup_stats(qk, Q, c->devStats.as<unsigned long long>() + 2, s);
        HIP_TRY(hipMemcpyAsync(dup, c->devStats.as<unsigned long long>() + 2, sizeof(dup), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        c->stats[17] = dup[0];
        c->stats[18] = dup[1];
    }
    c->qKeys = qk;
    c->qSlots = qi;
    // K4 join: per-read counts and ranks, matches staged in the join's order, then moved into
    // per-read segments by the transpose (KmerMatcher::matchKmers)
    HIP_TRY(c->readCnt.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(c->matchWin.ensure(sizeof(uint64_t) * std::max<uint64_t>(match_window_elems(Q), 1)));
    c->stageRegion = std::max<uint64_t>(c->stageRegion, std::max<uint64_t>(Q / kStageRegions, 64));
    // direct join (sort-merge join): each read's matches go straight into its K1 slot stretch
    // (a read has at most one query k-mer per slot, and in practice fewer matches than slots), no
    // staging buffer and no transpose; a read with more matches than slots sends the batch through
    // the staged join
    // (16-B segment matches hold 24-bit taxIDs: a taxonomy with larger IDs runs staged; and 29-bit
    // positions: reads of < 2^29 bases)
    bool direct = !probe && c->directJoin && (uint64_t)c->maxTax <= kSegMaxTax && c->maxW < (1u << 26);
    if (direct && c->mDirect.ensure(sizeof(SegMatch) * Rc) != hipSuccess) {
        (void)hipGetLastError();  // no room for a slot-sized match buffer (e.g. a long-read batch): staged join
        direct = false;
    }
    if (direct) {  // + the spill buffer (queries past their read's stretch), in mStage / mRank
        HIP_TRY(c->ovFlag.ensure(sizeof(int)));
        c->spillCap = std::max<uint64_t>(c->spillCap, std::max<uint64_t>(Q / 64, 1u << 12));
        if (c->mStage.ensure(sizeof(mtb_match) * c->spillCap) != hipSuccess ||
            c->mRank.ensure(sizeof(uint32_t) * c->spillCap) != hipSuccess) {
            (void)hipGetLastError();
            direct = false;
        }
    }
    if (!direct) {
        HIP_TRY(c->mStage.ensure(sizeof(mtb_match) * c->stageRegion * kStageRegions));
        HIP_TRY(c->mRank.ensure(sizeof(uint32_t) * c->stageRegion * kStageRegions));
    }
    HIP_TRY(hipEventRecord(c->kev[6], s));
    // the windows only serve the staged join
    if (!probe && !(sweepJoin && direct) && !unstaged_join(c->lines != nullptr, c->D, Q, std::min<uint32_t>(c->matchWinCap, 3072)))
        launch_match_windows(qk, Q, c->db, c->D, c->dir, c->par.kmer_format, c->matchWin.as<uint64_t>(), s);
    uint64_t M = 0, nSpill = 0;
    std::vector<unsigned long long> regTot(kStageRegions);
    const bool sweep = sweepJoin && direct;
    if (sweep) {  // K4S: the DB's tiles (once per context) and this batch's query bucket starts
        if (!c->tileRec) {
            const uint64_t nT = sweep_tiles(c->D, c->sweepNom);
            DevBuf tmp, rec, pre;  // freed on every return; the tiles are kept only once built
            HIP_TRY(tmp.ensure(sizeof(uint64_t) * kSweepStartsTmp));
            HIP_TRY(rec.ensure(sizeof(uint64_t) * (nT + 1)));
            HIP_TRY(pre.ensure(sizeof(uint32_t) * (nT + 1)));
            build_sweep_tiles(c->db, c->D, c->sweepNom, tmp.as<uint64_t>(), rec.as<uint64_t>(), pre.as<uint32_t>(), s);
            HIP_TRY(hipStreamSynchronize(s));
            c->tileRec = rec.as<uint64_t>();
            c->tilePre = pre.as<uint32_t>();
            rec.p = pre.p = nullptr;  // owned by the context now (mtb_close frees them)
            c->nTiles = nT;
        }
        HIP_TRY(c->qStart.ensure(sizeof(uint32_t) * (kSweepStartsTmp + c->nTiles + 1)));
        build_query_starts(qk, Q, c->qStart.as<uint32_t>(), c->tilePre, c->nTiles,
                           c->qStart.as<uint32_t>() + kSweepStartsTmp, s);
    }
    if (direct) {  // the long-run list: grown to the largest seen
        c->longCap = std::max<uint32_t>(c->longCap, (uint32_t)std::min<uint64_t>(std::max<uint64_t>(Q / 256, 1u << 12), 1u << 30));
        HIP_TRY(c->longList.ensure(sizeof(LongRun) * c->longCap));
        HIP_TRY(c->longCnt.ensure(sizeof(uint32_t)));
    }
    bool spillGrown = false;  // the spill buffer grows once per batch (then the staged join)
    // uniform units on the sort-merge join: its rank atomics go to 64-bit counters that also hand back
    // the read's lengths (k_match), copied to readCnt after the join
    unsigned long long* cnt64 = nullptr;
    if (c->upr && !probe && !(sweep && direct)) {
        HIP_TRY(c->readCnt64.ensure(sizeof(unsigned long long) * (n + 1)));
        cnt64 = c->readCnt64.as<unsigned long long>();
    }
    for (int attempt = 0; attempt < 5; attempt++) {
        HIP_TRY(hipMemsetAsync(c->readCnt.p, 0, sizeof(uint32_t) * (n + 1), s));
        if (cnt64) launch_cnt64_init(c->readLens.as<uint32_t>(), n, cnt64, s);
        HIP_TRY(hipMemsetAsync(c->mTotal.p, 0, sizeof(unsigned long long) * kStageRegions, s));
        int overflow = 0;
        uint32_t longN = 0;
        if (direct) HIP_TRY(hipMemsetAsync(c->ovFlag.p, 0, sizeof(int), s));
        if (direct) HIP_TRY(hipMemsetAsync(c->longCnt.p, 0, sizeof(uint32_t), s));
        if (probe)
            launch_probe(qk, qi, qf, Q, c->unitInfo.as<uint64_t>(), C, c->db, c->D, c->spOf,
                         (uint32_t)c->maxTax, c->par.kmer_format, c->readCnt.as<uint32_t>(),
                         c->mTotal.as<unsigned long long>(), c->mStage.as<mtb_match>(), c->mRank.as<uint32_t>(),
                         c->stageRegion, c->errFlag.as<int>(), c->probeStats.as<unsigned long long>(), s);
        else if (sweep && direct)
            launch_sweep(c->tileRec, c->qStart.as<uint32_t>() + kSweepStartsTmp, c->nTiles, qk, qi,
                         c->unitInfo.as<uint64_t>(), C, c->db, c->D, c->spOf, (uint32_t)c->maxTax, c->par.kmer_format,
                         c->readCnt.as<uint32_t>(), c->mTotal.as<unsigned long long>(), c->mStage.as<mtb_match>(),
                         c->mRank.as<uint32_t>(), c->spillCap, c->errFlag.as<int>(),
                         c->probeStats.as<unsigned long long>(), c->mDirect.as<SegMatch>(), c->ovFlag.as<int>(),
                         c->spillShift, c->longList.as<LongRun>(), c->longCap, c->longCnt.as<uint32_t>(),
                         c->sweepLdsCap, c->sweepSmall, c->sweepPersist, s);
        else
            launch_match(qk, qi, c->unitInfo.as<uint64_t>(), C, Q, c->db, c->D, c->dir, c->spOf,
                         (uint32_t)c->maxTax, c->par.kmer_format, c->readCnt.as<uint32_t>(),
                         c->mTotal.as<unsigned long long>(), c->mStage.as<mtb_match>(), c->mRank.as<uint32_t>(),
                         direct ? c->spillCap : c->stageRegion, c->errFlag.as<int>(), c->matchWinCap,
                         c->matchWin.as<uint64_t>(),
                         c->lines, c->lineP, c->runOff, sortLo, c->probeStats.as<unsigned long long>(),
                         direct ? c->mDirect.as<SegMatch>() : nullptr, c->slotOff.as<uint64_t>(),
                         c->ovFlag.as<int>(), c->spillShift, direct ? c->longList.as<LongRun>() : nullptr,
                         c->longCap, c->longCnt.as<uint32_t>(), s, c->lineExt, cnt64 ? c->upr : 0u, cnt64);
        HIP_TRY(hipMemcpyAsync(regTot.data(), c->mTotal.p, sizeof(unsigned long long) * kStageRegions,
                               hipMemcpyDeviceToHost, s));
        if (direct) HIP_TRY(hipMemcpyAsync(&overflow, c->ovFlag.p, sizeof(int), hipMemcpyDeviceToHost, s));
        if (direct) HIP_TRY(hipMemcpyAsync(&longN, c->longCnt.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (direct && longN > c->longCap) {  // the list outgrew its buffer: once more, larger
            c->longCap = longN + longN / 8;
            HIP_TRY(c->longList.ensure(sizeof(LongRun) * c->longCap));
            HIP_TRY(hipMemsetAsync(c->probeStats.p, 0, sizeof(unsigned long long) * kProbeStatsLen, s));
            continue;
        }
        c->stats[14] = direct ? longN : 0;
        if (direct && longN) {  // the long runs, a wave each; then the spill count and flag again
            launch_match_long(c->longList.as<LongRun>(), longN, qk, qi, c->unitInfo.as<uint64_t>(), C, c->db, c->D, c->spOf,
                              (uint32_t)c->maxTax, c->par.kmer_format, c->readCnt.as<uint32_t>(),
                              c->mTotal.as<unsigned long long>(), c->mStage.as<mtb_match>(), c->mRank.as<uint32_t>(),
                              c->spillCap, c->errFlag.as<int>(), c->mDirect.as<SegMatch>(),
                              c->slotOff.as<uint64_t>(), c->ovFlag.as<int>(), c->spillShift,
                              c->probeStats.as<unsigned long long>(), s, cnt64);
            HIP_TRY(hipMemcpyAsync(regTot.data(), c->mTotal.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(&overflow, c->ovFlag.p, sizeof(int), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
        }
        if (direct) {
            nSpill = regTot[0];
            if (!overflow && !c->directRetry) break;
            if (overflow && !spillGrown && !c->directRetry) {  // the spill outgrew its buffer: once more, larger
                spillGrown = true;
                const uint64_t want = nSpill + nSpill / 8;
                if (c->mStage.ensure(sizeof(mtb_match) * want) == hipSuccess &&
                    c->mRank.ensure(sizeof(uint32_t) * want) == hipSuccess) {
                    c->spillCap = want;
                    HIP_TRY(hipMemsetAsync(c->probeStats.p, 0, sizeof(unsigned long long) * kProbeStatsLen, s));
                    continue;
                }
                (void)hipGetLastError();
            }
            nSpill = 0;
            direct = false;  // rerun staged
            // the sweep built no windows (it needs none); the staged join does, unless it runs unstaged
            if (sweep && !unstaged_join(c->lines != nullptr, c->D, Q, std::min<uint32_t>(c->matchWinCap, 3072)))
                launch_match_windows(qk, Q, c->db, c->D, c->dir, c->par.kmer_format, c->matchWin.as<uint64_t>(), s);
            HIP_TRY(c->mStage.ensure(sizeof(mtb_match) * c->stageRegion * kStageRegions));
            HIP_TRY(c->mRank.ensure(sizeof(uint32_t) * c->stageRegion * kStageRegions));
            HIP_TRY(hipMemsetAsync(c->probeStats.p, 0, sizeof(unsigned long long) * kProbeStatsLen, s));
            continue;
        }
        M = 0;
        uint64_t most = 0;
        for (unsigned long long t : regTot) {
            M += t;
            most = std::max<uint64_t>(most, t);
        }
        if (most <= c->stageRegion || M >= kMaxBatchMatches) break;
        c->stageRegion = most + most / 8;  // grow once to the largest region (+12%) and rerun
        HIP_TRY(c->mStage.ensure(sizeof(mtb_match) * c->stageRegion * kStageRegions));
        HIP_TRY(c->mRank.ensure(sizeof(uint32_t) * c->stageRegion * kStageRegions));
        HIP_TRY(hipMemsetAsync(c->probeStats.p, 0, sizeof(unsigned long long) * kProbeStatsLen, s));
    }
    if (cnt64) launch_cnt64_counts(cnt64, n, c->readCnt.as<uint32_t>(), s);
    HIP_TRY(hipEventRecord(c->kev[7], s));
    exclusive_scan_u32(c->readCnt.as<uint32_t>(), n, c->mOff.as<uint64_t>(), c->scanTmp.p, s);
    if (direct) {  // M = the per-read counts' total (the direct join claims no staging stretches)
        HIP_TRY(hipMemcpyAsync(&M, c->mOff.as<uint64_t>() + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    if (M >= kMaxBatchMatches) {
        set_error("batch produced >= 2^32 matches: split it into smaller batches");
        return MTB_ERR_ARG;
    }
    c->M = M;
    HIP_TRY(c->matches.ensure(sizeof(mtb_match) * std::max<uint64_t>(M, 1)));
    HIP_TRY(hipEventRecord(c->kev[8], s));
    // a batch that goes on to K5 with pruning reads the direct join's segments in place (the
    // register and mid sorts, segments of <= kSegSortSparse matches); otherwise they are compacted here
    c->stats[13] = nSpill;
    c->sparse = direct && !c->keepStages && !c->forceGeneric && !c->matchOnly;
    if (c->sparse && nSpill) {  // only the reads that overflowed their stretch: compacted + their spills
        launch_compact_segments(c->mDirect.as<SegMatch>(), c->slotOff.as<uint64_t>(), C, c->mOff.as<uint64_t>(), n,
                                c->matches.as<mtb_match>(), c->spillShift, s, 1);
        launch_spill_scatter(c->mStage.as<mtb_match>(), c->mRank.as<uint32_t>(), c->mTotal.as<unsigned long long>(),
                             nSpill, c->mOff.as<uint64_t>(), n, c->matches.as<mtb_match>(), c->errFlag.as<int>(), s);
    } else if (direct && !c->sparse) {
        launch_compact_segments(c->mDirect.as<SegMatch>(), c->slotOff.as<uint64_t>(), C, c->mOff.as<uint64_t>(), n,
                                c->matches.as<mtb_match>(), c->spillShift, s);
        launch_spill_scatter(c->mStage.as<mtb_match>(), c->mRank.as<uint32_t>(), c->mTotal.as<unsigned long long>(),
                             nSpill, c->mOff.as<uint64_t>(), n, c->matches.as<mtb_match>(), c->errFlag.as<int>(), s);
    } else if (!direct)
        launch_match_transpose(c->mStage.as<mtb_match>(), c->mRank.as<uint32_t>(), c->stageRegion,
                               c->mTotal.as<unsigned long long>(), c->mOff.as<uint64_t>(), n,
                               c->matches.as<mtb_match>(), c->errFlag.as<int>(), s);
    HIP_TRY(hipEventRecord(c->kev[9], s));
    HIP_TRY(hipEventRecord(c->ev[3], s));
    return MTB_OK;
}

// A batch's device-side error flag (mtb_launch.h kErr*) as the entry point's status and message.
static int batch_error(int err) {
    switch (err) {
        case kErrTaxid:
            set_error("a selected reference k-mer has taxID 0 or no species in taxID_list (KmerMatcher.cpp:432-441)");
            return MTB_ERR_DB;
        case kErrProbeStash:
            set_error("a DB AA run holds >= 2^24 k-mers (probe join stash limit): use MTB_JOIN=sort");
            return MTB_ERR_DB;
        case kErrStagedRead:
            set_error("internal error: a staged or spilled match names a read outside the batch or past its segment");
            return MTB_ERR_INTERNAL;
        case kErrProbeCount:
            set_error("internal error: emitted matches disagree with the probe counts");
            return MTB_ERR_INTERNAL;
        case kErrRunOutsideDb:
            set_error("internal error: K4 found an AA run starting past the DB's end (run index or probe lines "
                      "inconsistent with the DB records)");
            return MTB_ERR_INTERNAL;
        case kErrLiveCount:
            set_error("internal error: K5 kept more live matches than a read's segment holds");
            return MTB_ERR_INTERNAL;
        default:
            set_error("internal error: device error flag " + std::to_string(err));
            return MTB_ERR_INTERNAL;
    }
}

// After an mtb_assign_* call: a device-side consistency check is reported.
static int check_err_flag(mtb_ctx* c) {
    int err = 0;
    HIP_TRY(hipMemcpy(&err, c->errFlag.p, sizeof(int), hipMemcpyDeviceToHost));
    return err ? batch_error(err) : MTB_OK;
}

// SeqIterator::maskLowComplexityRegions on the device for the batch's mates: masked copies in
// maskOut1/2 (the extraction reads those), tantan's scratch sized by the longer mate array.
static int mask_mates(mtb_ctx* c, const uint8_t* seq1, const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2,
                      uint32_t n, const uint8_t** out1, const uint8_t** out2) {
    hipStream_t s = c->stream;
    uint64_t nb[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&nb[0], off1 + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    if (seq2) HIP_TRY(hipMemcpyAsync(&nb[1], off2 + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t most = std::max(nb[0], nb[1]);
    HIP_TRY(c->maskProb.ensure(sizeof(float) * (most + 1)));
    HIP_TRY(c->maskScale.ensure(sizeof(double) * tantan_scale_elems(most, n)));
    const TantanTables tt = make_tantan_tables(c->par.mask_prob);
    HIP_TRY(c->maskOut1.ensure(nb[0] + 1));
    launch_tantan_mask(seq1, off1, n, tt, c->maskProb.as<float>(), c->maskScale.as<double>(), c->maskOut1.as<uint8_t>(), s);
    *out1 = c->maskOut1.as<uint8_t>();
    if (seq2) {
        HIP_TRY(c->maskOut2.ensure(nb[1] + 1));
        launch_tantan_mask(seq2, off2, n, tt, c->maskProb.as<float>(), c->maskScale.as<double>(),
                           c->maskOut2.as<uint8_t>(), s);
        *out2 = c->maskOut2.as<uint8_t>();
    }
    HIP_TRY(hipGetLastError());
    return MTB_OK;
}

extern "C" {

int mtb_memcpy(void* dst, const void* src, uint64_t bytes) {
    if (bytes && (!dst || !src)) { set_error("null argument"); return MTB_ERR_ARG; }
    if (bytes) HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
    return MTB_OK;
}

int mtb_line_ext_check(mtb_ctx* c, uint64_t* out) {
    if (!c || !out) return MTB_ERR_ARG;
    out[0] = out[1] = out[2] = 0;
    if (!c->lineExt || !c->runOff) { set_error("no run-length lines (MTB_LINE_EXT=0, or no run index)"); return MTB_ERR_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    DevBuf cnt;
    HIP_TRY(cnt.ensure(3 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(cnt.p, 0, 3 * sizeof(unsigned long long), c->stream));
    launch_line_ext_check(c->lines, c->lineP, c->runOff, c->lineExt, cnt.as<unsigned long long>(), c->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, cnt.p, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (out[2]) {
        set_error("internal error: " + std::to_string(out[2]) + " runs from the run-length lines disagree with the run index");
        return MTB_ERR_INTERNAL;
    }
    return MTB_OK;
}

int mtb_link_check(mtb_ctx* c, uint64_t* out) {
    if (!c || !out) return MTB_ERR_ARG;
    out[0] = out[1] = out[2] = 0;
    if (!c->link || !c->lines) { set_error("no link lines (MTB_LINK_LINES=0, the probe or sweep join, or no memory for them)"); return MTB_ERR_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    DevBuf cnt;
    HIP_TRY(cnt.ensure(3 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(cnt.p, 0, 3 * sizeof(unsigned long long), c->stream));
    launch_link_check(c->lines, c->link, cnt.as<unsigned long long>(), c->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, cnt.p, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (out[2]) {
        set_error("internal error: " + std::to_string(out[2]) + " link-line bits disagree with the probe lines");
        return MTB_ERR_INTERNAL;
    }
    return MTB_OK;
}

int mtb_hamming(int device, const uint64_t* query, const uint64_t* target, uint64_t n, uint8_t* sum, uint16_t* fwd,
                uint16_t* rev) {
    if (n && (!query || !target || !sum || !fwd || !rev)) { set_error("null argument"); return MTB_ERR_ARG; }
    if (!n) return MTB_OK;
    HIP_TRY(hipSetDevice(device));
    DevBuf a, b, s8, f16, r16, bad;
    HIP_TRY(a.ensure(8 * n));
    HIP_TRY(b.ensure(8 * n));
    HIP_TRY(s8.ensure(n));
    HIP_TRY(f16.ensure(2 * n));
    HIP_TRY(r16.ensure(2 * n));
    HIP_TRY(bad.ensure(8));
    HIP_TRY(hipMemcpy(a.p, query, 8 * n, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(b.p, target, 8 * n, hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(bad.p, 0, 8));
    launch_hamming_check(a.as<uint64_t>(), b.as<uint64_t>(), n, s8.as<uint8_t>(), f16.as<uint16_t>(),
                         r16.as<uint16_t>(), bad.as<unsigned long long>(), nullptr);
    HIP_TRY(hipGetLastError());
    unsigned long long nBad = 0;
    HIP_TRY(hipMemcpy(&nBad, bad.p, 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(sum, s8.p, n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fwd, f16.p, 2 * n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(rev, r16.p, 2 * n, hipMemcpyDeviceToHost));
    if (nBad) {
        set_error("internal error: K4's row-cached Hamming forms disagree with the plain forms on " +
                  std::to_string(nBad) + " pairs");
        return MTB_ERR_INTERNAL;
    }
    return MTB_OK;
}

int mtb_mask_reads(mtb_ctx* c, const char* seq, const uint64_t* off, uint32_t n, char* out) {
    if (!c || (n && (!seq || !off || !out))) { set_error("null argument"); return MTB_ERR_ARG; }
    if (!n) return MTB_OK;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint64_t nb = off[n];
    HIP_TRY(c->seq1.ensure(nb + 1));
    HIP_TRY(c->off1.ensure(sizeof(uint64_t) * (n + 1)));
    HIP_TRY(hipMemcpyAsync(c->seq1.p, seq, nb, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->off1.p, off, sizeof(uint64_t) * (n + 1), hipMemcpyHostToDevice, s));
    const uint8_t *m1 = nullptr, *m2 = nullptr;
    int rc = mask_mates(c, c->seq1.as<uint8_t>(), c->off1.as<uint64_t>(), nullptr, nullptr, n, &m1, &m2);
    if (rc != MTB_OK) return rc;
    HIP_TRY(hipMemcpyAsync(out, m1, nb, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return MTB_OK;
}

static int classify_batch(mtb_ctx* c, const char* seq, const uint64_t* off, const char* seq2, const uint64_t* off2,
                          uint32_t n, uint32_t flags, mtb_result* results) {
    if (!c || !off || !seq) { set_error("null argument"); return MTB_ERR_ARG; }
    const bool paired = c->par.seq_mode == 2;
    if (paired && (!seq2 || !off2)) { set_error("seq_mode 2 needs both mates"); return MTB_ERR_ARG; }
    if (n >= (1u << 29)) { set_error("batch exceeds the 29-bit seqID field (Kmer.h:14)"); return MTB_ERR_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    c->nReads = n;
    c->keepStages = (flags & MTB_KEEP_STAGES) != 0;
    const uint64_t *dOff1, *dOff2 = nullptr;
    const uint8_t *dSeq1, *dSeq2 = nullptr;
    HIP_TRY(hipEventRecord(c->ev[0], s));
    if (flags & MTB_INPUT_DEVICE) {
        dSeq1 = (const uint8_t*)seq;
        dOff1 = off;
        dSeq2 = (const uint8_t*)seq2;
        dOff2 = off2;
    } else {
        uint64_t b1 = off[n], b2 = paired ? off2[n] : 0;
        HIP_TRY(c->seq1.ensure(b1 + 1));
        HIP_TRY(c->off1.ensure(sizeof(uint64_t) * (n + 1)));
        HIP_TRY(hipMemcpyAsync(c->seq1.p, seq, b1, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(c->off1.p, off, sizeof(uint64_t) * (n + 1), hipMemcpyHostToDevice, s));
        dSeq1 = c->seq1.as<uint8_t>();
        dOff1 = c->off1.as<uint64_t>();
        if (paired) {
            HIP_TRY(c->seq2.ensure(b2 + 1));
            HIP_TRY(c->off2.ensure(sizeof(uint64_t) * (n + 1)));
            HIP_TRY(hipMemcpyAsync(c->seq2.p, seq2, b2, hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(c->off2.p, off2, sizeof(uint64_t) * (n + 1), hipMemcpyHostToDevice, s));
            dSeq2 = c->seq2.as<uint8_t>();
            dOff2 = c->off2.as<uint64_t>();
        }
    }
    if (c->par.mask_mode) {  // K0M: tantan masking of every mate (KmerExtractor.cpp:328-335)
        int rc = mask_mates(c, dSeq1, dOff1, dSeq2, dOff2, n, &dSeq1, &dSeq2);
        if (rc != MTB_OK) return rc;
    }
    for (uint64_t& x : c->stats) x = 0;
    HIP_TRY(c->devStats.ensure(sizeof(unsigned long long) * 4));
    HIP_TRY(hipMemsetAsync(c->devStats.p, 0, sizeof(unsigned long long) * 4, s));
    // K0: read metadata (KmerExtractor.cpp:442-494) and K1 work units
    HIP_TRY(c->meta.ensure(sizeof(ReadMeta) * (n + 1)));
    HIP_TRY(c->reserve.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(c->slotOff.ensure(sizeof(uint64_t) * (n + 1)));
    HIP_TRY(c->qlen.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(c->maxSeg.ensure(sizeof(uint32_t)));
    HIP_TRY(c->scanTmp.ensure(sizeof(uint64_t) * scan_tmp_elems(n + 1)));
    HIP_TRY(c->readLens.ensure(sizeof(uint32_t) * (n + 1)));
    launch_read_meta(dOff1, dOff2, n, paired, c->meta.as<ReadMeta>(), c->qlen.as<uint32_t>(), c->maxSeg.as<uint32_t>(),
                     c->readLens.as<uint32_t>(), s);
    uint32_t maxW = 0;
    HIP_TRY(hipMemcpyAsync(&maxW, c->maxSeg.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // chunk = the longest frame when it is short (no padding for uniform short reads), else 64
    const uint32_t C = std::min<uint32_t>(std::max<uint32_t>(maxW, 1), 64);
    c->maxW = maxW;
    // uniform units: every frame one chunk (maxW <= 64), 6 units per mate for every read
    c->upr = c->uniformUnits && maxW <= 64 ? (paired ? 12u : 6u) : 0u;
    c->stats[19] = c->upr;
    launch_read_units(c->meta.as<ReadMeta>(), n, C, c->upr, c->reserve.as<uint32_t>(), s);
    exclusive_scan_u32(c->reserve.as<uint32_t>(), n, c->slotOff.as<uint64_t>(), c->scanTmp.p, s);
    uint64_t U = 0;
    HIP_TRY(hipMemcpyAsync(&U, c->slotOff.as<uint64_t>() + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(c->unitRead.ensure(sizeof(uint32_t) * std::max<uint64_t>(U, 1)));
    launch_unit_read(c->slotOff.as<uint64_t>(), n, c->unitRead.as<uint32_t>(), s);
    const uint64_t R = extract_slots(U, C);
    const uint64_t Rc = std::max<uint64_t>(R, 1);
    if (R >= 0xFFFFFFFFull) { set_error("batch has >= 2^32 k-mer slots: split it"); return MTB_ERR_ARG; }
    c->chunkC = C;
    c->stats[0] = R;
    c->stats[15] = 0;
    HIP_TRY(c->unitInfo.ensure(16 * std::max<uint64_t>(U, 1)));  // 16-B unit records (mtb_device.h)
    HIP_TRY(c->errFlag.ensure(sizeof(int)));
    HIP_TRY(hipMemsetAsync(c->errFlag.p, 0, sizeof(int), s));
    HIP_TRY(c->mOff.ensure(sizeof(uint64_t) * (n + 1)));
    c->probed = !c->forceGeneric && c->joinMode == 2;  // the sort-merge join is the default (faster here)
    c->stats[10] = c->probed ? 0 : 1;
    c->matchOnly = (flags & MTB_MATCH_ONLY) != 0;
    int jrc = join_stage(c, dSeq1, dOff1, dSeq2, dOff2, n, U, C, R, Rc);
    if (jrc != MTB_OK) return jrc;
    if (c->matchOnly) {  // range-partitioned DB: the read owner sorts and scores (mtb_assign_chunks)
        for (int k = 10; k < 14; k++) HIP_TRY(hipEventRecord(c->kev[k], s));
        c->nTaxcnt = 0;
    } else {  // K5 + K6
        int rc = assign_stage(c, n, c->keepStages);
        if (rc != MTB_OK) return rc;
    }
    HIP_TRY(hipEventRecord(c->ev[4], s));
    HIP_TRY(hipGetLastError());
    int err = 0;
    unsigned long long dstat[4] = {0, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(&err, c->errFlag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(dstat, c->devStats.p, sizeof(dstat), hipMemcpyDeviceToHost, s));
    if (results && !c->matchOnly)
        HIP_TRY(hipMemcpyAsync(results, c->results.p, sizeof(mtb_result) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->stats[9] = dstat[1];
    {
        std::vector<unsigned long long> ps(kProbeStatsLen);
        HIP_TRY(hipMemcpy(ps.data(), c->probeStats.p, sizeof(unsigned long long) * ps.size(), hipMemcpyDeviceToHost));
        c->stats[2] = 0;
        for (uint32_t i = 0; i < kStatStripes; i++) c->stats[2] += ps[i];  // queries with >= 1 match
        c->stats[12] = ps[kStatStripes];  // run-index fallbacks (gallop searches) of the probe join
        c->stats[16] = 0;
        for (uint32_t i = 0; i < kStatStripes; i++) c->stats[16] += ps[kStatStripes + 1 + i];  // K4S: DB records read
    }
    for (int k = 0; k < 4; k++) HIP_TRY(hipEventElapsedTime(&c->stageMs[k], c->ev[k], c->ev[k + 1]));
    HIP_TRY(hipEventElapsedTime(&c->stageMs[4], c->ev[0], c->ev[4]));
    for (int k = 0; k < mtb_ctx::kNumKern; k++)
        HIP_TRY(hipEventElapsedTime(&c->kernMs[k], c->kev[2 * k], c->kev[2 * k + 1]));
    if (const char* e = getenv("MTB_WS_REPORT"); e && atoi(e)) {  // diagnostics: the batch buffers >= 256 MB
        const std::vector<DevBuf*> bufs = batch_bufs(c);
        const char* const* names = batch_buf_names();
        std::vector<std::pair<uint64_t, const char*>> big;
        for (size_t i = 0; i < bufs.size(); i++)
            if (bufs[i]->bytes >= (256ull << 20)) big.push_back({bufs[i]->bytes, names[i]});
        std::sort(big.begin(), big.end(), [](auto& a, auto& b) { return a.first > b.first; });
        fprintf(stderr, "[mtb ws] %u reads, Q %llu, M %llu, live %llu: workspace %.2f GB (K6 scratch aliased %.2f GB):",
                n, (unsigned long long)c->Q, (unsigned long long)c->M, (unsigned long long)c->liveM,
                ctx_workspace_bytes(c) / 1e9, c->aliasBytes / 1e9);
        for (auto& b : big) fprintf(stderr, " %s %.2f", b.second, b.first / 1e9);
        fprintf(stderr, "\n");
    }
    return err ? batch_error(err) : MTB_OK;
}

// The reference's match-buffer exhaustion is a retry (KmerMatcher.cpp:474-476 returns false,
// Classifier.cpp:127-130 enlarges matchPerKmer and searches that split again). Here the batch
// workspace grows with the batch's matches, so running out of HBM (or of MTB_WORKSPACE_CAP) is
// MTB_RETRY: the context stays usable (the failed buffer is gone, the others are reused, every
// stage is rerun by the next call) and the caller classifies the batch in smaller pieces
// (mtb_start_classify halves it down to one read).
int mtb_classify_batch(mtb_ctx* c, const char* seq, const uint64_t* off, const char* seq2, const uint64_t* off2,
                       uint32_t n, uint32_t flags, mtb_result* results) {
    const int rc = classify_batch(c, seq, off, seq2, off2, n, flags, results);
    if (rc != MTB_ERR_OOM) return rc;
    (void)hipGetLastError();
    // the buffers the failed attempt grew would otherwise stay at its size: the pieces start clean
    const double held = c->ws.used * 1e-9;
    mtb::ctx_release_workspace(c);
    char msg[200];
    snprintf(msg, sizeof msg, "out of HBM for the workspace of a %u-read batch (%.2f GB held%s): classify it in smaller "
             "pieces", n, held, c->ws.cap ? ", capped" : "");
    set_error(msg);
    return MTB_RETRY;
}

int mtb_get_taxcnt(mtb_ctx* c, mtb_taxcnt* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return MTB_ERR_ARG;
    *n_out = c->nTaxcnt;
    if (cap < c->nTaxcnt) return MTB_RETRY;
    if (c->nTaxcnt) HIP_TRY(hipMemcpy(out, c->tcOut.p, sizeof(mtb_taxcnt) * c->nTaxcnt, hipMemcpyDeviceToHost));
    return MTB_OK;
}

int mtb_device_results(mtb_ctx* c, void** results, void** taxcnt, uint64_t* n_taxcnt) {
    if (!c) return MTB_ERR_ARG;
    if (results) *results = c->results.p;
    if (taxcnt) *taxcnt = c->tcOut.p;
    if (n_taxcnt) *n_taxcnt = c->nTaxcnt;
    return MTB_OK;
}

int mtb_last_counts(const mtb_ctx* c, uint64_t* q, uint64_t* m) {
    if (!c) return MTB_ERR_ARG;
    if (q) *q = c->Qall;
    if (m) *m = c->M;
    return MTB_OK;
}

// Kraken-style report. Clade counts: each taxID's reads added to itself and every ancestor below
// the root's self-loop (getCladeCounts); children of a taxon in nodes.dmp order (getParentToChildren),
// sorted by clade count, descending, with std::sort as SORT_SERIAL does (ties in libstdc++'s order);
// a taxon is written only with a nonzero clade count, depth-first, two spaces of indent per level.
namespace {
struct CladeCounts {
    uint32_t taxCount = 0, cladeCount = 0;
};
struct ReportWriter {
    const HostTaxonomy& T;
    const std::unordered_map<int32_t, CladeCounts>& cc;
    const std::vector<std::vector<int32_t>>& children;  // by node
    unsigned long total;
    std::string out;
    uint32_t cladeOf(int32_t t) const {
        auto it = cc.find(t);
        return it == cc.end() ? 0 : it->second.cladeCount;
    }
    void line(uint32_t clade, uint32_t taxc, const std::string& rank, int32_t t, int depth, const std::string& name) {
        char buf[96];
        // 100 * cladeCount is unsigned int arithmetic in the reference (Reporter.cpp:233)
        snprintf(buf, sizeof buf, "%.4f\t%i\t%i\t", 100u * clade / double(total), (int)clade, (int)taxc);
        out += buf;
        out += rank;
        snprintf(buf, sizeof buf, "\t%i\t", t);
        out += buf;
        out.append(2 * depth, ' ');
        out += name;
        out += '\n';
    }
    void walk(int32_t t, int depth) {  // Reporter::writeReport, Reporter.cpp:217-244
        auto it = cc.find(t);
        const uint32_t clade = it == cc.end() ? 0 : it->second.cladeCount;
        if (t == 0) {
            if (clade > 0) {
                char buf[96];
                snprintf(buf, sizeof buf, "%.4f\t%i\t%i\tno rank\t0\tunclassified\n", 100u * clade / double(total),
                         (int)clade, (int)it->second.taxCount);
                out += buf;
            }
            walk(1, 0);
            return;
        }
        if (clade == 0) return;
        const int node = T.nodeOf[t];
        line(clade, it->second.taxCount, T.rank[node], T.original(t), depth, T.name[node]);  // getOriginalTaxID
        std::vector<int32_t> ch = children[node];
        std::sort(ch.begin(), ch.end(), [&](int32_t a, int32_t b) { return cladeOf(a) > cladeOf(b); });
        for (int32_t x : ch) {
            if (!cc.count(x)) break;
            walk(x, depth + 1);
        }
    }
};
}  // namespace

int mtb_write_report(const mtb_ctx* c, const char* path, uint64_t total_reads, const int32_t* tax_ids,
                     const uint32_t* counts, uint64_t n) {
    if (!c || !path || (n && (!tax_ids || !counts))) { set_error("null argument"); return MTB_ERR_ARG; }
    const HostTaxonomy& T = c->hTax;
    if (!T.exists(1)) { set_error("context has no taxonomy"); return MTB_ERR_ARG; }
    std::unordered_map<int32_t, CladeCounts> cc;
    for (uint64_t i = 0; i < n; i++) {
        const int32_t t = tax_ids[i];
        cc[t].taxCount = counts[i];
        cc[t].cladeCount += counts[i];
        if (!T.exists(t)) continue;
        int node = T.nodeOf[t];
        while (T.parent[node] != node) {  // the root is its own parent
            node = T.parent[node];
            cc[T.nodeTax[node]].cladeCount += counts[i];
        }
    }
    std::vector<std::vector<int32_t>> children(T.nodeTax.size());
    for (size_t i = 0; i < T.nodeTax.size(); i++)
        if ((int)i != T.parent[i]) children[T.parent[i]].push_back(T.nodeTax[i]);
    ReportWriter w{T, cc, children, (unsigned long)(int)total_reads, {}};  // numOfQuery is an int
    w.out = "#clade_proportion\tclade_count\ttaxon_count\trank\ttaxID\tname\n";
    w.walk(0, 0);
    FILE* f = fopen(path, "wb");
    if (!f) { set_error(std::string("cannot write ") + path); return MTB_ERR_IO; }
    fwrite(w.out.data(), 1, w.out.size(), f);
    if (fclose(f) != 0) { set_error(std::string("write failed: ") + path); return MTB_ERR_IO; }
    return MTB_OK;
}

const char* mtb_taxon_rank(const mtb_ctx* c, int32_t t) {
    if (!c || t < 0 || (size_t)t >= c->hNodeOf.size() || c->hNodeOf[t] < 0) return "-";
    return c->hRank[c->hNodeOf[t]].c_str();
}

int32_t mtb_original_taxid(const mtb_ctx* c, int32_t t) { return c ? c->hTax.original(t) : t; }

// TaxonomyWrapper::taxLineage2(node, infoAsName = true) (TaxonomyWrapper.cpp:431-454): the node and
// its ancestors below the root, root-most first, each as findShortRank2(rank) + "_" + name (short
// ranks of TaxonomyWrapper.h:8-24, "-" otherwise), joined by ';'. Built once per context.
const char* mtb_taxon_lineage(const mtb_ctx* c, int32_t t) {
    if (!c || !c->hTax.exists(t)) return "-";
    const HostTaxonomy& T = c->hTax;
    std::call_once(c->lineageOnce, [c, &T] {
        static const std::unordered_map<std::string, std::string> shortRank = {
            {"subspecies", "ss"}, {"species", "s"}, {"subgenus", "sg"}, {"genus", "g"}, {"subfamily", "sf"},
            {"family", "f"}, {"suborder", "so"}, {"order", "o"}, {"subclass", "sc"}, {"class", "c"},
            {"subphylum", "sp"}, {"phylum", "p"}, {"subkingdom", "sk"}, {"kingdom", "k"},
            {"superkingdom", "d"}, {"domain", "d"}, {"realm", "r"}};
        c->lineage.resize(T.nodeTax.size());
        std::vector<int> chain;
        for (size_t i = 0; i < T.nodeTax.size(); i++) {
            chain.clear();
            int node = (int)i;
            do {
                chain.push_back(node);
                node = T.parent[node];
            } while (T.parent[node] != node && chain.size() <= T.nodeTax.size());
            std::string& out = c->lineage[i];
            for (size_t k = chain.size(); k-- > 0;) {
                auto it = shortRank.find(T.rank[chain[k]]);
                out += it == shortRank.end() ? "-" : it->second;
                out += '_';
                out += T.name[chain[k]];
                if (k > 0) out += ';';
            }
        }
    });
    return c->lineage[T.nodeOf[t]].c_str();
}

}  // extern "C"

namespace mtb {
const TaxText& tax_text(const mtb_ctx* c) {
    std::call_once(c->taxTextOnce, [c] {
        TaxText& x = c->taxText;
        const HostTaxonomy& T = c->hTax;
        x.n = T.maxTax >= 0 && T.maxTax < (1 << 26) ? (uint32_t)T.maxTax + 1 : 0;  // else: formatted per line
        x.idOff.resize(x.n + 1);
        x.rankOff.resize(x.n + 1);
        char tmp[16];
        for (uint32_t t = 0; t < x.n; t++) {
            x.idOff[t] = (uint32_t)x.buf.size();
            const auto r = std::to_chars(tmp, tmp + sizeof tmp, T.original((int32_t)t));
            x.buf.append(tmp, r.ptr);
        }
        x.idOff[x.n] = (uint32_t)x.buf.size();
        for (uint32_t t = 0; t < x.n; t++) {
            x.rankOff[t] = (uint32_t)x.buf.size();
            x.buf += mtb_taxon_rank(c, (int32_t)t);
        }
        x.rankOff[x.n] = (uint32_t)x.buf.size();
    });
    return c->taxText;
}

void ctx_release_workspace(mtb_ctx* c) {
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (DevBuf* b : batch_bufs(c)) b->release();
    // the last batch's results went with the buffers: the getters (mtb_get_taxcnt / _matches /
    // _query_kmers / _em_mappings) see an empty batch instead of freed device pointers
    c->nReads = 0;
    c->M = c->Q = c->Qall = c->nTaxcnt = c->liveM = 0;
    c->qKeys = nullptr;
    c->qSlots = nullptr;
    c->sparse = false;
    c->keepStages = false;
    c->emValid = c->emPackedValid = false;
    c->emHost.clear();
    for (auto& v : c->stats) v = 0;  // mtb_last_stats / _stage_ms / _kernel_ms: the empty batch too
    for (auto& v : c->stageMs) v = 0.f;
    for (auto& v : c->kernMs) v = 0.f;
}

std::shared_ptr<void>& ctx_pipeline_cache(mtb_ctx* c) { return c->pipelineCache; }

const mtb_params& ctx_params(const mtb_ctx* c) { return c->par; }

void ctx_set_grow(mtb_ctx* c, double scale) { c->ws.grow = scale < 1.0 ? 1.0 : scale > 32.0 ? 32.0 : scale; }

int ctx_match_view(mtb_ctx* c, std::vector<uint64_t>& mOff, const mtb_match** m, const uint32_t** counts,
                   const uint32_t** qlen) {
    if (!c->matchOnly) { set_error("batch was not run with MTB_MATCH_ONLY"); return MTB_ERR_ARG; }
    mOff.resize((size_t)c->nReads + 1);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpy(mOff.data(), c->mOff.p, sizeof(uint64_t) * mOff.size(), hipMemcpyDeviceToHost));
    *m = c->matches.as<mtb_match>();
    *counts = c->readCnt.as<uint32_t>();
    *qlen = c->qlen.as<uint32_t>();
    return MTB_OK;
}

uint64_t ctx_workspace_bytes(const mtb_ctx* c) {
    uint64_t b = 0;
    for (DevBuf* x : batch_bufs(const_cast<mtb_ctx*>(c))) b += x->bytes;
    return b;
}
}  // namespace mtb

extern "C" {

int mtb_last_stats(const mtb_ctx* c, uint64_t* out, int n) {
    if (!c || !out) return MTB_ERR_ARG;
    for (int i = 0; i < n && i < mtb_ctx::kNumStats; i++) out[i] = c->stats[i];
    return MTB_OK;
}

int mtb_last_stage_ms(const mtb_ctx* c, float* ms, int n) {
    if (!c || !ms) return MTB_ERR_ARG;
    for (int i = 0; i < n && i < 5; i++) ms[i] = c->stageMs[i];
    return MTB_OK;
}

int mtb_last_kernel_ms(const mtb_ctx* c, float* ms, int n) {
    if (!c || !ms) return MTB_ERR_ARG;
    for (int i = 0; i < n && i < mtb_ctx::kNumKern; i++) ms[i] = c->kernMs[i];
    return MTB_OK;
}

int mtb_copy_results(mtb_ctx* c, void* dst, int dst_on_device) {
    if (!c || !dst) return MTB_ERR_ARG;
    HIP_TRY(hipMemcpyAsync(dst, c->results.p, sizeof(mtb_result) * c->nReads,
                           dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MTB_OK;
}

int mtb_get_em_mappings(mtb_ctx* c, uint32_t query_offset, mtb_em_map* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) { set_error("null argument"); return MTB_ERR_ARG; }
    if (!c->par.em) { set_error("the context was opened without em"); return MTB_ERR_ARG; }
    *n_out = 0;
    const uint32_t n = c->nReads;
    if (!c->emValid || n == 0) return MTB_OK;
    if (!c->emPackedValid) {  // packed on the device once per batch, then served from the host copy
        HIP_TRY(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        HIP_TRY(c->emCnt32.ensure(sizeof(uint32_t) * (n + 1)));
        HIP_TRY(c->emOff.ensure(sizeof(uint64_t) * (n + 1)));
        HIP_TRY(c->scanTmp.ensure(sizeof(uint64_t) * scan_tmp_elems(n + 1)));
        HIP_TRY(c->emPacked.ensure(sizeof(mtb_em_map) * (uint64_t)kEmTop * n));
        launch_em_pack(c->emMap.p, c->emCnt.as<uint8_t>(), n, c->emCnt32.as<uint32_t>(), c->emOff.as<uint64_t>(),
                       c->scanTmp.p, c->emPacked.as<mtb_em_map>(), s);
        uint64_t tot = 0;
        HIP_TRY(hipMemcpyAsync(&tot, c->emOff.as<uint64_t>() + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        c->emHost.resize(tot);
        if (tot) HIP_TRY(hipMemcpy(c->emHost.data(), c->emPacked.p, sizeof(mtb_em_map) * tot, hipMemcpyDeviceToHost));
        c->emPackedValid = true;
    }
    const uint64_t tot = c->emHost.size();
    *n_out = tot;
    if (tot > cap || (tot && !out)) return MTB_RETRY;
    for (uint64_t w = 0; w < tot; w++) {
        out[w] = c->emHost[w];
        out[w].query_id += query_offset;
    }
    return MTB_OK;
}

// DB k-mers per species: dbDir/sp2uniqKmerCnt ("taxID count" lines) when present, else counted on
// the device and written there (Classifier::countUniqueKmerPerSpecies, Classifier.cpp:388-431).
static int species_kmers(mtb_ctx* c) {
    if (!c->spKmers.empty()) return MTB_OK;
    c->spKmers.assign((size_t)c->maxTax + 1, 0);
    const std::string path = c->dbDir.empty() ? std::string() : c->dbDir + "/sp2uniqKmerCnt";
    if (!path.empty()) {
        if (FILE* f = fopen(path.c_str(), "r")) {
            long long t = 0;
            unsigned long long k = 0;
            while (fscanf(f, "%lld %llu", &t, &k) == 2)
                if (t >= 0 && t < (long long)c->spKmers.size()) c->spKmers[(size_t)t] = (uint32_t)k;
            fclose(f);
            return MTB_OK;
        }
    }
    DevBuf cnt;
    HIP_TRY(cnt.ensure(sizeof(uint32_t) * c->spKmers.size()));
    HIP_TRY(hipMemsetAsync(cnt.p, 0, sizeof(uint32_t) * c->spKmers.size(), c->stream));
    launch_species_kmers(c->db, c->D, c->spOf, (uint32_t)c->maxTax, cnt.as<uint32_t>(), c->stream);
    HIP_TRY(hipMemcpyAsync(c->spKmers.data(), cnt.p, sizeof(uint32_t) * c->spKmers.size(), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!path.empty()) {
        if (FILE* f = fopen(path.c_str(), "w")) {
            for (size_t i = 0; i < c->spKmers.size(); i++)
                if (c->spKmers[i] > 0) fprintf(f, "%zu %u\n", i, c->spKmers[i]);
            fclose(f);
        }
    }
    return MTB_OK;
}

int mtb_em(mtb_ctx* c, const mtb_em_map* maps, uint64_t n_maps, uint64_t total_reads, mtb_em_read* reads_out,
           int32_t* sp_ids, double* sp_probs, uint32_t* sp_counts, uint64_t cap, uint64_t* n_sp, mtb_em_stats* st) {
    if (!c || (!maps && n_maps) || !reads_out || !n_sp) { set_error("null argument"); return MTB_ERR_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    // queries (Classifier.cpp:224-233): runs of one query_id, ascending
    std::vector<uint64_t> qOff;
    std::vector<uint32_t> qId;
    for (uint64_t j = 0; j < n_maps; j++) {
        if (maps[j].query_id >= total_reads) { set_error("a mapping names a read past total_reads"); return MTB_ERR_ARG; }
        if (j == 0 || maps[j].query_id != maps[j - 1].query_id) {
            if (j && maps[j].query_id < maps[j - 1].query_id) { set_error("mappings must be in query order"); return MTB_ERR_ARG; }
            qOff.push_back(j);
            qId.push_back(maps[j].query_id);
        } else if (j - qOff.back() >= (uint64_t)kEmTop) {
            set_error("more than 10 mappings for one query");
            return MTB_ERR_ARG;
        }
    }
    const uint64_t nQ = qId.size();
    qOff.push_back(n_maps);
    // dense species (ascending taxID); the top species: each query's first mapping (getTopSpecies)
    std::vector<int32_t> spTax(n_maps);
    for (uint64_t j = 0; j < n_maps; j++) spTax[j] = maps[j].species_id;
    std::sort(spTax.begin(), spTax.end());
    spTax.erase(std::unique(spTax.begin(), spTax.end()), spTax.end());
    const uint32_t S = (uint32_t)spTax.size();
    std::vector<uint32_t> spIdx(n_maps);
    std::vector<float> score(n_maps);
    std::vector<uint64_t> spCnt(S + 1, 0);
    for (uint64_t j = 0; j < n_maps; j++) {
        spIdx[j] = (uint32_t)(std::lower_bound(spTax.begin(), spTax.end(), maps[j].species_id) - spTax.begin());
        score[j] = maps[j].score;
        spCnt[spIdx[j] + 1]++;
    }
    std::vector<uint8_t> isTop(S, 0);
    for (uint64_t q = 0; q < nQ; q++) isTop[spIdx[qOff[q]]] = 1;
    uint32_t nTop = 0;
    for (uint32_t i = 0; i < S; i++) nTop += isTop[i];
    // species order: each mapping's position (query order inside a species), slices of <= kSlice
    constexpr uint64_t kSlice = 4096;
    for (uint32_t i = 0; i < S; i++) spCnt[i + 1] += spCnt[i];
    std::vector<uint64_t> pos(n_maps), cur(spCnt.begin(), spCnt.end() - 1);
    for (uint64_t j = 0; j < n_maps; j++) pos[j] = cur[spIdx[j]]++;
    std::vector<uint64_t> sliceOff, spSlice(S + 1, 0);
    for (uint32_t i = 0; i < S; i++) {
        spSlice[i] = sliceOff.size();
        for (uint64_t a = spCnt[i]; a < spCnt[i + 1]; a += kSlice) sliceOff.push_back(a);
    }
    spSlice[S] = sliceOff.size();
    const uint64_t nSl = sliceOff.size();
    sliceOff.push_back(n_maps);
    // length factors 1 / log(k-mers) (0 for a species without DB k-mers), initial abundances
    int rc = species_kmers(c);
    if (rc != MTB_OK) return rc;
    std::vector<double> lf(S), p(S, 0.0);
    for (uint32_t i = 0; i < S; i++) {
        const int32_t t = spTax[i];
        const uint32_t k = t >= 0 && t < (int32_t)c->spKmers.size() ? c->spKmers[(size_t)t] : 0;
        lf[i] = k > 0 ? 1.0 / log((double)k) : 0.0;
        if (isTop[i]) p[i] = 1.0 / (double)nTop;
    }
    // device arrays
    DevBuf dScore, dSpIdx, dQOff, dPos, dLf, dP, dPNew, dW, dQc, dSliceOff, dPart, dSpSlice, dTop, dAbsd, dDelta,
        dSpTax, dQId, dOut;
    auto up = [&](DevBuf& b, const void* h, size_t bytes) -> hipError_t {
        hipError_t e = b.ensure(std::max<size_t>(bytes, 8));
        if (e == hipSuccess && bytes) e = hipMemcpyAsync(b.p, h, bytes, hipMemcpyHostToDevice, s);
        return e;
    };
    HIP_TRY(up(dScore, score.data(), 4 * n_maps));
    HIP_TRY(up(dSpIdx, spIdx.data(), 4 * n_maps));
    HIP_TRY(up(dQOff, qOff.data(), 8 * qOff.size()));
    HIP_TRY(up(dPos, pos.data(), 8 * n_maps));
    HIP_TRY(up(dLf, lf.data(), 8 * S));
    HIP_TRY(up(dP, p.data(), 8 * S));
    HIP_TRY(dPNew.ensure(8 * std::max<uint32_t>(S, 1)));
    HIP_TRY(dW.ensure(8 * std::max<uint64_t>(n_maps, 1)));
    HIP_TRY(dQc.ensure(8));
    HIP_TRY(up(dSliceOff, sliceOff.data(), 8 * sliceOff.size()));
    HIP_TRY(dPart.ensure(8 * std::max<uint64_t>(nSl, 1)));
    HIP_TRY(up(dSpSlice, spSlice.data(), 8 * spSlice.size()));
    HIP_TRY(up(dTop, isTop.data(), S));
    HIP_TRY(dAbsd.ensure(8 * std::max<uint32_t>(S, 1)));
    HIP_TRY(dDelta.ensure(8));
    // Classifier.cpp:247-309: at most 1000 iterations, until delta < 1e-6
    uint32_t iters = 0;
    double delta = 0.0;
    unsigned long long qc = 0;
    double *pa = dP.as<double>(), *pb = dPNew.as<double>();
    for (uint32_t it = 0; it < 1000; it++) {
        launch_em_iteration(dScore.as<float>(), dSpIdx.as<uint32_t>(), dQOff.as<uint64_t>(), nQ, dPos.as<uint64_t>(),
                            pa, dLf.as<double>(), dW.as<double>(), dQc.as<unsigned long long>(),
                            dSliceOff.as<uint64_t>(), nSl, dPart.as<double>(), dSpSlice.as<uint64_t>(), S,
                            dTop.as<uint8_t>(), pb, dAbsd.as<double>(), it > 10 ? 1 : 0, dDelta.as<double>(), s);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(&delta, dDelta.p, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(&qc, dQc.p, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        std::swap(pa, pb);  // taxProbs.swap(Fnew)
        iters++;
        if (delta < 1e-6) break;
    }
    HIP_TRY(hipMemcpy(p.data(), pa, 8 * S, hipMemcpyDeviceToHost));
    // per-read reassignment (Classifier::reclassify)
    std::vector<int32_t> spTaxD(spTax.begin(), spTax.end());
    HIP_TRY(up(dSpTax, spTaxD.data(), 4 * S));
    HIP_TRY(up(dQId, qId.data(), 4 * nQ));
    HIP_TRY(dOut.ensure(sizeof(mtb_em_read) * std::max<uint64_t>(total_reads, 1)));
    HIP_TRY(hipMemsetAsync(dOut.p, 0, sizeof(mtb_em_read) * total_reads, s));
    TaxDevice t{c->tNodeOf, c->tNodeTax, c->tParent, c->tDepth, c->tFlags, c->tSpParent, c->maxTax};
    launch_em_reclassify(dScore.as<float>(), dSpIdx.as<uint32_t>(), dSpTax.as<int32_t>(), dQOff.as<uint64_t>(),
                         dQId.as<uint32_t>(), nQ, pa, dLf.as<double>(), t, dOut.as<mtb_em_read>(), s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(reads_out, dOut.p, sizeof(mtb_em_read) * total_reads, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // emTaxCounts (Classifier.cpp:312-318): the top species' (unsigned)(p * queryCount)
    *n_sp = nTop;
    if (st) {
        st->query_count = qc;
        st->iterations = iters;
        st->n_species = nTop;
        st->delta = delta;
    }
    if (nTop > cap) return MTB_RETRY;
    uint64_t w = 0;
    for (uint32_t i = 0; i < S; i++) {
        if (!isTop[i]) continue;
        if (sp_ids) sp_ids[w] = spTax[i];
        if (sp_probs) sp_probs[w] = p[i];
        if (sp_counts) sp_counts[w] = (unsigned int)(p[i] * (double)qc);
        w++;
    }
    return MTB_OK;
}

int mtb_copy_taxcnt(mtb_ctx* c, void* dst, int dst_on_device, uint64_t* n_out) {
    if (!c || (!dst && c->nTaxcnt)) return MTB_ERR_ARG;
    if (n_out) *n_out = c->nTaxcnt;
    if (c->nTaxcnt)
        HIP_TRY(hipMemcpyAsync(dst, c->tcOut.p, sizeof(mtb_taxcnt) * c->nTaxcnt,
                               dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MTB_OK;
}

int mtb_get_query_kmers(mtb_ctx* c, mtb_kmer* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return MTB_ERR_ARG;
    *n_out = c->Q;
    if (!c->keepStages) { set_error("batch was not run with MTB_KEEP_STAGES"); return MTB_ERR_ARG; }
    if (c->probed) { set_error("the probe join keeps no sorted query k-mers (MTB_JOIN=probe)"); return MTB_ERR_ARG; }
    if (!c->qSlots) { set_error("no query k-mers kept"); return MTB_ERR_ARG; }
    if (cap < c->Q) return MTB_RETRY;
    // the unit records' buffer is sized need + need / 8 + 256 bytes (DevBuf::ensure): not a multiple of 8
    std::vector<uint64_t> k(c->Q), ui((c->unitInfo.bytes + 7) / 8);
    std::vector<uint32_t> v(c->Q);
    const void* kp = c->qKeys;
    const void* vp = c->qSlots;
    if (c->Q) {
        HIP_TRY(hipMemcpy(k.data(), kp, 8 * c->Q, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(v.data(), vp, 4 * c->Q, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(ui.data(), c->unitInfo.p, c->unitInfo.bytes, hipMemcpyDeviceToHost));
    }
    const bool packed = c->par.kmer_format == 2;  // back from the resident rank form
    for (uint64_t i = 0; i < c->Q; i++)
        out[i] = mtb_kmer{packed ? host_from_rank_form(k[i]) : k[i], slot_info(v[i], c->chunkC, ui.data(),
                                                                               c->par.kmer_format)};
    return MTB_OK;
}

int mtb_copy_matches(mtb_ctx* c, mtb_match* matches, uint32_t* read_counts, uint32_t* query_len, int dst_on_device) {
    if (!c) return MTB_ERR_ARG;
    if (!c->matchOnly) { set_error("batch was not run with MTB_MATCH_ONLY"); return MTB_ERR_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    const hipMemcpyKind k = dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (matches && c->M) HIP_TRY(hipMemcpyAsync(matches, c->matches.p, sizeof(mtb_match) * c->M, k, c->stream));
    if (read_counts && c->nReads)
        HIP_TRY(hipMemcpyAsync(read_counts, c->readCnt.p, sizeof(uint32_t) * c->nReads, k, c->stream));
    if (query_len && c->nReads)
        HIP_TRY(hipMemcpyAsync(query_len, c->qlen.p, sizeof(uint32_t) * c->nReads, k, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MTB_OK;
}

int mtb_assign_chunks(mtb_ctx* c, const mtb_match* m, uint64_t nm, const uint32_t* cnt, uint32_t nChunks,
                      const uint32_t* qlen, uint32_t n, uint32_t flags, mtb_result* results) {
    if (!c || (!m && nm) || (!cnt && n && nChunks) || !qlen) { set_error("null argument"); return MTB_ERR_ARG; }
    if (nm >= kMaxBatchMatches) { set_error("more than 2^32 - 1 matches in one call"); return MTB_ERR_ARG; }
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const bool dev = (flags & MTB_INPUT_DEVICE) != 0;
    const hipMemcpyKind k = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const uint64_t nc = (uint64_t)nChunks * n;
    for (uint64_t& x : c->stats) x = 0;
    HIP_TRY(c->devStats.ensure(sizeof(unsigned long long) * 4));
    HIP_TRY(hipMemsetAsync(c->devStats.p, 0, sizeof(unsigned long long) * 4, s));
    HIP_TRY(hipEventRecord(c->ev[0], s));
    for (int e = 1; e < 4; e++) HIP_TRY(hipEventRecord(c->ev[e], s));
    const mtb_match* dm = m;
    const uint32_t* dc = cnt;
    if (!dev) {
        HIP_TRY(c->chunkIn.ensure(sizeof(mtb_match) * std::max<uint64_t>(nm, 1)));
        HIP_TRY(c->chunkCnt.ensure(sizeof(uint32_t) * std::max<uint64_t>(nc, 1)));
        if (nm) HIP_TRY(hipMemcpyAsync(c->chunkIn.p, m, sizeof(mtb_match) * nm, k, s));
        if (nc) HIP_TRY(hipMemcpyAsync(c->chunkCnt.p, cnt, sizeof(uint32_t) * nc, k, s));
        dm = c->chunkIn.as<mtb_match>();
        dc = c->chunkCnt.as<uint32_t>();
    }
    c->sparse = false;
    HIP_TRY(c->matches.ensure(sizeof(mtb_match) * std::max<uint64_t>(nm, 1)));
    HIP_TRY(c->readCnt.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(c->mOff.ensure(sizeof(uint64_t) * (n + 1)));
    HIP_TRY(c->qlen.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(c->chunkSrcOff.ensure(sizeof(uint64_t) * (nc + 1)));
    HIP_TRY(c->scanTmp.ensure(sizeof(uint64_t) * scan_tmp_elems(nc + n + 1)));
    if (n) HIP_TRY(hipMemcpyAsync(c->qlen.p, qlen, sizeof(uint32_t) * n, k, s));
    launch_regroup_chunks(dm, dc, nChunks, n, c->readCnt.as<uint32_t>(), c->chunkSrcOff.as<uint64_t>(),
                          c->mOff.as<uint64_t>(), c->scanTmp.p, c->matches.as<mtb_match>(), s);
    uint64_t total = 0;  // the chunks' counts must add up to the matches handed over
    if (n) HIP_TRY(hipMemcpyAsync(&total, c->mOff.as<uint64_t>() + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (total != nm) { set_error("chunk counts do not add up to n_matches"); return MTB_ERR_ARG; }
    c->M = nm;
    c->Q = 0;
    c->Qall = 0;
    c->qKeys = nullptr;
    c->qSlots = nullptr;
    c->nReads = n;
    c->matchOnly = false;
    HIP_TRY(c->errFlag.ensure(sizeof(int)));
    HIP_TRY(hipMemsetAsync(c->errFlag.p, 0, sizeof(int), s));
    int rc = assign_stage(c, n, (flags & MTB_KEEP_STAGES) != 0);
    if (rc != MTB_OK) return rc;
    HIP_TRY(hipEventRecord(c->ev[4], s));
    if (results) HIP_TRY(hipMemcpyAsync(results, c->results.p, sizeof(mtb_result) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    for (int e = 0; e < 4; e++) HIP_TRY(hipEventElapsedTime(&c->stageMs[e], c->ev[e], c->ev[e + 1]));
    HIP_TRY(hipEventElapsedTime(&c->stageMs[4], c->ev[0], c->ev[4]));
    return check_err_flag(c);
}

int mtb_get_matches(mtb_ctx* c, mtb_match* out, uint64_t cap, uint64_t* n_out) {
    if (!c || !n_out) return MTB_ERR_ARG;
    *n_out = c->M;
    if (!c->keepStages) { set_error("the last K5 pruned dead matches: run the batch with MTB_KEEP_STAGES"); return MTB_ERR_ARG; }
    if (cap < c->M) return MTB_RETRY;
    if (c->M) HIP_TRY(hipMemcpy(out, c->matchesSorted.p, sizeof(mtb_match) * c->M, hipMemcpyDeviceToHost));
    return MTB_OK;
}

int mtb_assign_matches(mtb_ctx* c, const mtb_match* m, uint64_t nm, const uint32_t* qlen, uint32_t n,
                       mtb_result* results) {
    if (!c || (!m && nm) || !qlen) return MTB_ERR_ARG;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    for (uint64_t& x : c->stats) x = 0;
    HIP_TRY(c->devStats.ensure(sizeof(unsigned long long) * 4));
    HIP_TRY(hipMemsetAsync(c->devStats.p, 0, sizeof(unsigned long long) * 4, s));
    // group by read (counting sort by seqID) on the host, then K5 + K6 on the device
    std::vector<uint64_t> off(n + 1, 0);
    for (uint64_t i = 0; i < nm; i++) {
        uint32_t sq = info_seq(m[i].qinfo);
        if (sq == 0 || sq > n) { set_error("match seqID out of range"); return MTB_ERR_ARG; }
        off[sq]++;
    }
    for (uint32_t i = 0; i < n; i++) off[i + 1] += off[i];
    std::vector<mtb_match> grouped(std::max<uint64_t>(nm, 1));
    std::vector<uint64_t> cur(off.begin(), off.end() - 1);
    for (uint64_t i = 0; i < nm; i++) grouped[cur[info_seq(m[i].qinfo) - 1]++] = m[i];
    if (nm >= kMaxBatchMatches) { set_error("more than 2^32 - 1 matches in one call"); return MTB_ERR_ARG; }
    c->M = nm;
    c->Q = 0;
    c->Qall = 0;
    c->qKeys = nullptr;
    c->qSlots = nullptr;
    c->nReads = n;
    c->sparse = false;
    HIP_TRY(c->matches.ensure(sizeof(mtb_match) * std::max<uint64_t>(nm, 1)));
    HIP_TRY(c->mOff.ensure(sizeof(uint64_t) * (n + 1)));
    HIP_TRY(c->qlen.ensure(sizeof(uint32_t) * (n + 1)));
    HIP_TRY(hipMemcpyAsync(c->matches.p, grouped.data(), sizeof(mtb_match) * nm, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->mOff.p, off.data(), sizeof(uint64_t) * (n + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->qlen.p, qlen, sizeof(uint32_t) * n, hipMemcpyHostToDevice, s));
    HIP_TRY(c->errFlag.ensure(sizeof(int)));
    HIP_TRY(hipMemsetAsync(c->errFlag.p, 0, sizeof(int), s));
    int rc = assign_stage(c, n, true);  // staged entry point: every match stays readable
    if (rc != MTB_OK) return rc;
    if (results) HIP_TRY(hipMemcpyAsync(results, c->results.p, sizeof(mtb_result) * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return check_err_flag(c);
}

}  // extern "C"

extern "C" int mtb_pin_eval(int device, int fn, const int64_t* param, const uint64_t* a, const uint64_t* b,
                            uint64_t n, int64_t* out, uint64_t* n_out) {
    if (!n_out || (n && (!a || !out || (fn != MTB_PIN_DECODE_DIFF_IDX && !param)))) {
        set_error("null argument");
        return MTB_ERR_ARG;
    }
    *n_out = 0;
    if (fn < MTB_PIN_SCORE_INCREMENT || fn > MTB_PIN_DECODE_DIFF_IDX) { set_error("unknown pin function"); return MTB_ERR_ARG; }
    if (fn == MTB_PIN_TAXONOMER_SHAPE) {  // the host-side parameters the assign kernels get (assign_args)
        for (uint64_t i = 0; i < n; i++) {
            mtb_params par;
            mtb_default_params(&par);
            par.syncmer = (int)(a[i] >> 16);
            par.smer_len = (int)(a[i] & 0xFF);
            par.seq_mode = (int)b[i];
            const AssignArgs g = assign_args(par);
            const int64_t v[6] = {g.dnaShift, g.maxCodonShift, g.denominator, kBitsPerCodon, kTotalDnaBits,
                                  (int64_t)((1u << (kTotalDnaBits - kBitsPerCodon)) - 1u)};
            for (int k = 0; k < 6; k++) out[6 * i + k] = v[k];
        }
        *n_out = n;
        return MTB_OK;
    }
    if (!n) return MTB_OK;
    HIP_TRY(hipSetDevice(device));
    if (fn == MTB_PIN_DECODE_DIFF_IDX) {  // K3 as mtb_open runs it: one chunk from the stream's start
        std::vector<uint16_t> w(n);
        for (uint64_t i = 0; i < n; i++) w[i] = (uint16_t)a[i];
        DevBuf diff, flag, idx, tmp, val;
        HIP_TRY(diff.ensure(2 * n));
        HIP_TRY(flag.ensure(4 * n));
        HIP_TRY(idx.ensure(8 * (n + 2)));
        HIP_TRY(tmp.ensure(scan_tmp_elems(n) * sizeof(uint64_t)));
        HIP_TRY(val.ensure(8 * n));
        HIP_TRY(hipMemcpy(diff.p, w.data(), 2 * n, hipMemcpyHostToDevice));
        uint64_t lastTerm = 0, lastValue = 0;
        const uint64_t terms = decode_diff_chunk(diff.as<uint16_t>(), n, 0, val.as<uint64_t>(), flag.as<uint32_t>(),
                                                 idx.as<uint64_t>(), tmp.p, &lastTerm, &lastValue, nullptr);
        HIP_TRY(hipGetLastError());
        if (terms && lastTerm != n - 1) { set_error("diffIdx ends mid k-mer"); return MTB_ERR_DB; }
        HIP_TRY(hipMemcpy(out, val.p, 8 * terms, hipMemcpyDeviceToHost));
        *n_out = terms;
        return MTB_OK;
    }
    DevBuf dp, da, db, dout;
    HIP_TRY(dp.ensure(8 * n));
    HIP_TRY(da.ensure(8 * n));
    HIP_TRY(db.ensure(8 * n));
    HIP_TRY(dout.ensure(8 * n));
    HIP_TRY(hipMemcpy(dp.p, param, 8 * n, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(da.p, a, 8 * n, hipMemcpyHostToDevice));
    if (b) HIP_TRY(hipMemcpy(db.p, b, 8 * n, hipMemcpyHostToDevice));
    else HIP_TRY(hipMemset(db.p, 0, 8 * n));
    launch_pin_eval(fn, dp.as<int64_t>(), da.as<uint64_t>(), db.as<uint64_t>(), n, dout.as<int64_t>(), nullptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(out, dout.p, 8 * n, hipMemcpyDeviceToHost));
    *n_out = n;
    return MTB_OK;
}

// K2 alone (staged entry): the (key, 32-bit value) pairs sorted on key bits [bit_lo, bit_hi) by the
// LSD radix sort the query sort runs (radix_sort_pairs: every pass stable, with the knobs it reads —
// MTB_RADIX_ORRANK, MTB_RADIX_TILE, MTB_RADIX_FULLTILE, MTB_RADIX_XCD), 8-bit digits. Host arrays.
extern "C" int mtb_sort_pairs(int device, const uint64_t* keys, const uint32_t* vals, uint64_t n, int bit_lo,
                              int bit_hi, uint64_t* keys_out, uint32_t* vals_out) {
    if (n && (!keys || !vals || !keys_out || !vals_out)) { set_error("null argument"); return MTB_ERR_ARG; }
    if (bit_lo < 0 || bit_hi > 64 || bit_lo >= bit_hi || n >= (1ull << 32)) { set_error("bad sort range"); return MTB_ERR_ARG; }
    if (!n) return MTB_OK;
    HIP_TRY(hipSetDevice(device));
    DevBuf ka, va, kb, vb, cnt, offs, tmp;
    const uint64_t rc = radix_counts_elems(n);
    HIP_TRY(ka.ensure(8 * n));
    HIP_TRY(va.ensure(4 * n));
    HIP_TRY(kb.ensure(8 * n));
    HIP_TRY(vb.ensure(4 * n));
    HIP_TRY(cnt.ensure(4 * rc));
    HIP_TRY(offs.ensure(8 * (rc + 1)));
    HIP_TRY(tmp.ensure(8 * scan_tmp_elems(rc)));
    HIP_TRY(hipMemcpy(ka.p, keys, 8 * n, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(va.p, vals, 4 * n, hipMemcpyHostToDevice));
    bool inB = false;
    radix_sort_pairs(ka.as<uint64_t>(), va.as<uint32_t>(), kb.as<uint64_t>(), vb.as<uint32_t>(), n, bit_lo, bit_hi,
                     false, false, cnt.as<uint32_t>(), offs.as<uint64_t>(), tmp.p, &inB, nullptr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(keys_out, inB ? kb.p : ka.p, 8 * n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(vals_out, inB ? vb.p : va.p, 4 * n, hipMemcpyDeviceToHost));
    return MTB_OK;
}
