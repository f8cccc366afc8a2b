// Internal interface between the C-ABI orchestration (mtb_api.hip) and the kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "mtb_device.h"

namespace mtb {

// The batch's device-side error flag (errFlag, last writer wins); mtb_api.hip turns each into
// its own message, so a failure names the check that caught it.
constexpr int kErrTaxid = 1;         // a selected DB k-mer with taxID 0 or no species (KmerMatcher.cpp:432-441)
constexpr int kErrStagedRead = 2;    // a staged or spilled match names a read outside the batch / past its segment
constexpr int kErrProbeStash = 3;    // a DB AA run of >= 2^24 k-mers (probe join)
constexpr int kErrProbeCount = 4;    // the probe join emitted other counts than it reserved
constexpr int kErrRunOutsideDb = 5;  // K4: an AA run starting past the DB's end (run index / probe line inconsistent)
constexpr int kErrLiveCount = 6;     // K5: a read's live-match count above its segment

struct ReadMeta {  // per read: raw lengths, covered lengths, windows per frame of each mate
    int32_t len1, len2, ql1, ql2, w1, w2;
};

struct HostTables {  // restated genetic code (mtb_host.cpp)
    uint8_t base[256];
    int8_t aa[64];
    int8_t num[64];
};

struct TaxDevice {
    const int32_t* nodeOf;
    const int32_t* nodeTax;
    const int32_t* parent;
    const int32_t* depth;
    const uint8_t* flags;
    const int32_t* spParent;
    int32_t maxTax;
};

struct AssignArgs {
    int kmerFormat, dnaShift, maxCodonShift, denominator, minConsCnt, minConsCntEuk, accessionLevel;
    float minScore, minSpScore, tieRatio;
    int generic;  // MTB_FORCE_GENERIC: general code paths only (parity tests of the fallbacks)
    int waveTaxon = -1;  // MTB_WAVE_TAXON: -1 auto, 0 thread, 1 wave, 2 16-lane group per read (K6 chooseBestTaxon)
    int emulateAll = 0;  // MTB_EMULATE_SORT=1: every k_combine_wave run takes the std::sort emulation (tests)
    int em = 0;          // --em: classified reads keep their best species; mappings for the EM
    int bigGroups = 1;   // MTB_BIG_GROUPS=0: every (species, frame) group on a thread (A/B, tests)
};

struct AssignScratch {  // per match unless noted
    void* local;           // Path
    void* paths;           // Path
    void* comb;            // Path
    uint8_t* conn;
    uint32_t *gFlag, *sFlag, *pathCnt;
    uint64_t *gScan, *sScan, *gStart, *sStart;  // M + 1 entries
    float* spScore;        // per species run
    uint64_t* waveList;    // per species run: runs queued for k_combine_wave
    uint32_t* waveCount;   // 1
    uint8_t* spKeep;       // per species run
    void* scanTmp;         // scan_tmp_elems(radix_counts_elems(M + 1) + M + 2) u64
    uint64_t *ordKA, *ordVA, *ordKB, *ordVB;  // M + 1 each: group work list (radix_sort_pairs)
    uint32_t* radixCounts;                    // radix_counts_elems(M + 1)
    uint64_t* radixOffs;                      // radix_counts_elems(M + 1) + 1
    void* clade;           // cladePerMatch per match
    uint32_t cladePerMatch;
};

// scans (out has n+1 entries; tmp needs scan_tmp_elems(n) u64)
uint64_t scan_tmp_elems(uint64_t n);
// Grid of a grid-stride launch over n items: one launch holds < 2^32 work-items in x, and DB-wide
// arrays (12G k-mers at GTDB scale, ~30G diffIdx words) are larger.
inline unsigned stride_grid(uint64_t n, unsigned block = 256) {
    const uint64_t b = (n + block - 1) / block;
    return (unsigned)(b < 1 ? 1 : (b > (1ull << 22) ? (1ull << 22) : b));
}
#define MTB_GRID_STRIDE(i, n) \
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (uint64_t)gridDim.x * blockDim.x)
void exclusive_scan_u32(const uint32_t* in, uint64_t n, uint64_t* out, void* tmp, hipStream_t s);
void exclusive_scan_u64(const uint64_t* in, uint64_t n, uint64_t* out, void* tmp, hipStream_t s);
// K6 run index of nM sorted matches: flags nM bytes, tileSum run_index_tmp_bytes(nM); writes
// gScan/sScan (nM + 1) and gStart/sStart (count + 1)
uint64_t run_index_tmp_bytes(uint64_t nM);
void launch_run_index(const mtb_match* M, uint64_t nM, uint8_t* flags, unsigned long long* tileSum, uint64_t* gScan,
                      uint64_t* sScan, uint64_t* gStart, uint64_t* sStart, hipStream_t s);

void launch_read_meta(const uint64_t* off1, const uint64_t* off2, uint32_t n, int paired, ReadMeta* meta,
                      uint32_t* qlen, uint32_t* maxW, uint32_t* readLens, hipStream_t s);
// upr > 0: uniform units (every read upr units, one per (mate, frame); k_read_units)
void launch_read_units(const ReadMeta* meta, uint32_t n, uint32_t C, uint32_t upr, uint32_t* units, hipStream_t s);
void launch_unit_read(const uint64_t* uOff, uint32_t n, uint32_t* unitRead, hipStream_t s);
uint64_t extract_slots(uint64_t nUnits, uint32_t C);
// K1 over nUnits chunks of <= C windows; writes extract_slots(nUnits, C) slots
void launch_extract(const uint8_t* seq1, const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2,
                    const ReadMeta* meta, const uint64_t* uOff, const uint32_t* unitRead, uint64_t nUnits,
                    uint32_t C, const HostTables& t, int kmerFormat, int syncmer, int smerLen, uint64_t* keys,
                    uint64_t* unitInfo, hipStream_t s, uint32_t upr = 0);  // keys per slot, info per unit (slot_info)

uint64_t radix_counts_elems(uint64_t n);
// V = uint64_t or uint32_t; genVals: the values are the input positions (valsA not read).
// digA / digB (nullable, n bytes each; not with filter): digit side arrays — digA holds every key's
// first-pass digit (bits [bitLo, bitLo + 8)), each scatter writes the next pass's digits, and the
// histograms read 1 B per key instead of the 8-B key.
template <typename V>
uint64_t radix_sort_pairs(uint64_t* keysA, V* valsA, uint64_t* keysB, V* valsB, uint64_t n, int bitLo, int bitHi,
                          bool filter, bool genVals, uint32_t* counts, uint64_t* offs, void* scanTmp, bool* inB,
                          hipStream_t s, uint8_t* digA = nullptr, uint8_t* digB = nullptr, bool unstableFirst = false);
// unstableFirst: the first pass may permute keys of one digit (its input order carries nothing: the
// query sort); it then ranks by LDS atomics instead of the stable 8-ballot ranking
// K2 after a binned K1F (binRc > 0 above): the pairs already sit in the first pass's buckets —
// kSortBins regions of rc slots, region d * 8 + XCD for first digit d (bits [bitLo, bitLo + 8)), the
// region counts in binDev (device) and binHost (host copy) — with each key's second-pass digit in
// digR. Sorts the remaining passes through a tile table over the regions (tileTab: at least
// radix_binned_tiles(binHost, rc) entries); counts / offs sized radix_counts_elems(Q) + 256 * kSortBins.
// Returns Q; *inT: the result is in (keysT, valsT), else in (keysR, valsR) from slot 0.
constexpr int kSortBins = 2048;
uint64_t radix_binned_tiles(const uint64_t* binHost, uint64_t rc);
template <typename V>
uint64_t radix_sort_binned(uint64_t* keysR, V* valsR, uint64_t* keysT, V* valsT, const uint64_t* binHost,
                           const unsigned long long* binDev, uint64_t rc, int bitLo, int bitHi, uint32_t* counts,
                           uint64_t* offs, void* scanTmp, uint64_t* tileTab, bool* inT, hipStream_t s, uint8_t* digR,
                           uint8_t* digT);
// format-2 DB values -> resident rank form (mtb_kernels.hip, to_rank_form); host inverse for getters
void launch_to_rank_form(uint64_t* v, uint64_t n, hipStream_t s);
uint64_t host_from_rank_form(uint64_t v);
// AA 8-mers: base-21 ranks 0 .. 21^8 - 1
constexpr uint64_t kAARankEnd = 37822859361ull;
// query k-mers are ordered by these bits of their rank-form key (AA rank << 24 | DNA part)
constexpr int kQuerySortLo = 36, kQuerySortHi = 60;
constexpr int kQuerySortLoFine = 36;  // unstaged K4 sort prefix: 3 passes (4 passes, 28, measured 1.5 ms slower with the run index)

// K3 over one chunk of diffIdx words starting at a k-mer's first word: returns the whole k-mers it
// holds, their values (continuing from carry, the previous chunk's last value) in values, the chunk
// index of its last terminator word in *lastTerm and the last value in *lastValue (idxTmp n + 2 u64,
// flagTmp n u32, scanTmp scan_tmp_elems(n) u64)
uint64_t decode_diff_chunk(const uint16_t* diff, uint64_t n, uint64_t carry, uint64_t* values, uint32_t* flagTmp,
                           uint64_t* idxTmp, void* scanTmp, uint64_t* lastTerm, uint64_t* lastValue, hipStream_t s);
void launch_mask_info(uint32_t* info, uint64_t n, uint32_t mask, hipStream_t s);

// A resident DB k-mer: its value in rank form (low / high 32 bits) and its taxID (info & mask) in
// one 12-B record, so the join reads a candidate's value and taxID from one cache line.
struct DbRec {
    uint32_t lo, hi, tax;
};
static_assert(sizeof(DbRec) == 12, "12-B DB records");
// values + taxIDs -> records (out may not alias the inputs)
void launch_pack_db(const uint64_t* v, const uint32_t* tax, uint64_t n, DbRec* out, hipStream_t s);
// in place on records: format-2 values to rank form; taxIDs & mask
void launch_rec_rank_form(DbRec* db, uint64_t n, hipStream_t s);
void launch_rec_mask_info(DbRec* db, uint64_t n, uint32_t mask, hipStream_t s);

// AA-prefix directory over the decoded DB: dir[b] = first DB index whose value is >= the
// smallest value of bucket b (first L AAs ranked in base 21), dir[R] = D.
struct AADir {
    const uint64_t* dir;
    uint64_t R;    // 21^L buckets
    uint64_t div;  // 21^(8-L) (format 1 bucket = AA part / div)
    int L;
    int fmt;
};
AADir make_aa_dir(uint64_t D, int kmerFormat);
void build_aa_dir(const DbRec* db, uint64_t D, const AADir& d, uint64_t* dir, hipStream_t s);

// DB probe lines: the AA membership bitmap of the DB (bit r set iff some DB k-mer has AA rank r)
// cut into 64-B lines of kLineRanks ranks, each headed by the DB index of the first k-mer whose
// rank is >= the line's first rank. One random 64-B read answers "does the DB hold this AA
// 8-mer" and, when it does, names a DB index a few runs before the 8-mer's run.
constexpr uint32_t kLineRanks = 448;
struct alignas(64) ProbeLine {
    uint64_t base;
    uint32_t bits[kLineRanks / 32];
};
static_assert(sizeof(ProbeLine) == 64, "one probe line per 64-B segment");
constexpr uint32_t kStatStripes = 256;
// join statistics: [0, 256) matched-query stripes, [256] gallop fallbacks, [257, 513) K4S DB-record stripes
constexpr uint32_t kProbeStatsLen = 2 * kStatStripes + 1;
constexpr uint64_t kDbPad = 8;  // ~0 values after the resident DB
constexpr uint64_t kProbeLines = (kAARankEnd + kLineRanks - 1) / kLineRanks + 1;  // + an end line (base D)
void build_probe_lines(const DbRec* db, uint64_t D, const AADir& dir, ProbeLine* lines,
                       hipStream_t s);  // lines zeroed by the caller

// Run index (mtb_kernels.hip, k_run_offsets): lineP (kProbeLines + 1 u64: present ranks before
// each line, the total at [kProbeLines]; popTmp kProbeLines u32, scanTmp scan_tmp_elems(kProbeLines)),
// then runOff (lineP[kProbeLines] + 1 u16: each present rank's run start minus its line's base; lines
// of more than kRunIdxMax k-mers are not indexed)
constexpr uint64_t kRunIdxMax = 0xFFFF;
void build_line_prefix(const ProbeLine* lines, uint64_t* lineP, uint32_t* popTmp, void* scanTmp, hipStream_t s);
void build_run_offsets(const DbRec* db, uint64_t D, const ProbeLine* lines, const uint64_t* lineP,
                       uint16_t* runOff, hipStream_t s);
// Run-length lines (round 5): per probe line 64 B of 2-bit codes, one per present rank of the line
// (its first kExtRanks), code = min(run length - 1, 3), 3 an escape (a run of >= 4, or a line the run
// index does not cover: all codes 3). The unstaged K4 stages them beside the probe lines and finds a
// query's run as base + before + the codes' sum over the ranks before it, code + 1 long — no random
// run-index read — unless an escape lies at or before its rank (then runOff as before).
constexpr uint32_t kExtRanks = 256;
struct alignas(64) ProbeExt {
    uint32_t w[kExtRanks / 16];
};
static_assert(sizeof(ProbeExt) == 64, "one run-length line per probe line");
void build_line_ext(const ProbeLine* lines, const uint64_t* lineP, const uint16_t* runOff, ProbeExt* ext,
                    hipStream_t s);
// out (3 device words, zeroed): present ranks within reach, resolved by the codes, mismatches vs runOff
void launch_line_ext_check(const ProbeLine* lines, const uint64_t* lineP, const uint16_t* runOff, const ProbeExt* ext,
                           unsigned long long* out, hipStream_t s);

// Link lines (round 6): per AA 7-mer S (kLinkSlots = 21^7 of them) one u64 — bit y (0..20) set iff the
// DB holds the 8-mer of rank 21 S + y (S then y), bit 32 + x iff it holds rank x 21^7 + S (x then S) —
// built from the probe lines (same membership). Consecutive windows of a frame share 7 AAs, so the
// fused K1F tests both with one random 8-B read of their shared 7-mer's word (14.4 GB) instead of two
// probe-line reads; a window without a partner reads its own word (as S then y).
constexpr uint64_t kLinkSlots = 1801088541ull;  // 21^7
static_assert(kLinkSlots * 21 == kAARankEnd, "21^8 AA ranks");
void build_link_lines(const ProbeLine* lines, uint64_t* link, hipStream_t s);
// out (3 device words, zeroed): AA ranks checked, present ranks, link bits that disagree with the probe lines
void launch_link_check(const ProbeLine* lines, const uint64_t* link, unsigned long long* out, hipStream_t s);

// K1F: the present windows of keys[0..R) (AA 8-mer in the DB) packed, in no particular order, into
// qkey/qslot (and, when qfrom is given, their DB lower bounds); returns their count and sets
// *emitted to the non-blank windows (the reference's query k-mer count). counter: 2 device words.
// keys whose AA rank lies outside [rankLo, rankHi) (a DB part's range) are dropped without a probe
// K1 + K1F in one pass (sort-merge join): the present windows' keys and slots straight from the
// reads (returns Q; *emitted = non-blank windows); unitInfo as launch_extract's. Only the first
// `cap` present windows are written: Q > cap means the output must grow and the pass rerun.
// threadMajor (A/B): round 3's output order (each thread's present windows together).
uint64_t launch_extract_filter(const uint8_t* seq1, const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2,
                               const ReadMeta* meta, const uint64_t* uOff, const uint32_t* unitRead, uint64_t nUnits,
                               uint32_t C, const HostTables& t, int kmerFormat, int syncmer, int smerLen,
                               uint64_t* unitInfo, const ProbeLine* lines, uint64_t* qkey, uint32_t* qslot,
                               unsigned long long* counter, uint64_t rankLo, uint64_t rankHi, uint64_t* emitted,
                               uint64_t cap, bool threadMajor, hipStream_t s,
                               uint8_t* qdig = nullptr, unsigned long long* binCnt = nullptr, uint64_t binRc = 0,
                               uint64_t* binHost = nullptr, uint32_t upr = 0, const uint64_t* link = nullptr);
uint64_t launch_filter(const uint64_t* keys, uint64_t R, const ProbeLine* lines, uint64_t* qkey, uint32_t* qslot,
                       uint64_t* qfrom, unsigned long long* counter, uint64_t rankLo, uint64_t rankHi,
                       uint64_t* emitted, hipStream_t s);
// K4P probe join over the filtered queries: same outputs as launch_match (per-read counts and
// ranks, staged matches); stats: kStatStripes counters of queries with >= 1 match.
void launch_probe(const uint64_t* qkey, const uint32_t* qslot, const uint64_t* qfrom, uint64_t Q,
                  const uint64_t* unitInfo, uint32_t C, const DbRec* db, uint64_t D,
                  const int32_t* spOf, uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total,
                  mtb_match* buf, uint32_t* bufRank, uint64_t region, int* err, unsigned long long* stats,
                  hipStream_t s);

// A match inside a read's segment of the direct join, 16 B: the read is implicit (the segment's),
// positions are < 2^29 (the sort key's width, K5) and taxIDs < 2^24 (kSegMaxTax; a taxonomy with
// larger IDs runs the staged join): pos | frame << 29, target | hamming << 24, species |
// rightEndHamming low byte << 24, dna (24 bits) | rightEndHamming high byte << 24. K5 and the
// compaction expand it to mtb_match (seg_expand).
constexpr uint32_t kSegMaxTax = (1u << 24) - 1;
struct SegMatch {
    uint32_t posFrame, targetHam, speciesReh, dnaReh;
};
static_assert(sizeof(SegMatch) == 16, "16-B segment matches");
__host__ __device__ inline SegMatch seg_pack(const mtb_match& m) {
    return SegMatch{(uint32_t)m.qinfo | (uint32_t)(m.qinfo >> 61) << 29, m.target_id | (uint32_t)m.hamming << 24,
                    m.species_id | (uint32_t)(m.right_end_hamming & 0xFFu) << 24,
                    (m.dna_encoding & 0xFFFFFFu) | (uint32_t)(m.right_end_hamming >> 8) << 24};
}
// the match of the segment whose qinfo carries seqBits (info_seq << 32)
__host__ __device__ inline mtb_match seg_expand(const SegMatch& s, uint64_t seqBits) {
    mtb_match m;
    m.qinfo = (uint64_t)(s.posFrame >> 29) << 61 | seqBits | (s.posFrame & 0x1FFFFFFFu);
    m.target_id = s.targetHam & 0xFFFFFFu;
    m.species_id = s.speciesReh & 0xFFFFFFu;
    m.dna_encoding = s.dnaReh & 0xFFFFFFu;
    m.right_end_hamming = (uint16_t)((s.speciesReh >> 24) | (s.dnaReh >> 24) << 8);
    m.hamming = (uint8_t)(s.targetHam >> 24);
    m.pad = 0;
    return m;
}

// K4 join: per-read counts into readCnt; matches staged in buf = kStageRegions regions of
// `region` slots, total[k] = matches claimed in region k (all written iff every total[k] <= region).
// winCap: max DB values staged in LDS per block.
constexpr uint32_t kStageRegions = 256;
// qslot: each query's K1 slot (its info is slot_info(slot, C, unitInfo))
// A direct-join query whose AA run is longer than kLongRun (mtb_kernels.hip) is deferred to the
// long-run list and scanned by a wave of its own (launch_match_long).
void set_ab_rank_free(int on);  // A/B only: k_match without the per-read rank atomic (invalid results)
void set_match_xcd(int on);     // MTB_MATCH_XCD (A/B): the unstaged join's blocks in one contiguous eighth per XCD
void set_share_runs(int on);    // MTB_SHARE_RUNS=1 (A/B, off by default): same-AA queries of a block share one run lookup
void set_match_prefetch(int m);
void set_pair_read(int on);  // MTB_PAIR_READ=1 (A/B): K4 reads a run's second record for one-record runs too
void set_ab_sweep_count(int on);  // A/B only: k_sweep_ws searches and selects but emits nothing (invalid results)

struct LongRun {
    uint64_t q;       // index into the sorted query arrays
    uint64_t lo, hi;  // its DB run
};
void launch_match_long(const LongRun* list, uint32_t n, const uint64_t* qkey, const uint32_t* qslot,
                       const uint64_t* unitInfo, uint32_t C, const DbRec* db, uint64_t D, const int32_t* spOf,
                       uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total, mtb_match* buf,
                       uint32_t* bufRank, uint64_t region, int* err, SegMatch* direct, const uint64_t* dirOff,
                       int* overflow, uint32_t capShift, unsigned long long* stats, hipStream_t s, unsigned long long* cnt64 = nullptr);
// K4S DB-sweep join (MTB_JOIN=sweep; direct output only): tiles of ~nom DB records ending at
// sort-prefix bucket bounds, built once per context (pstartTmp: kSweepStartsTmp u64 scratch; tileRec
// sweep_tiles + 1 u64, tilePre sweep_tiles + 1 u32); per batch the sorted queries' bucket starts
// (qStart: kSweepStartsTmp u32: the starts and their suffix-minimum scratch), then one block per tile.
uint64_t sweep_tiles(uint64_t D, uint32_t nom);
constexpr uint64_t kSweepStarts = (1ull << 24) + 1;
constexpr uint64_t kSweepStartsTmp = kSweepStarts + (kSweepStarts + 1023) / 1024;
void build_sweep_tiles(const DbRec* db, uint64_t D, uint32_t nom, uint64_t* pstartTmp, uint64_t* tileRec,
                       uint32_t* tilePre, hipStream_t s);
void build_query_starts(const uint64_t* qkey, uint64_t Q, uint32_t* qStart, const uint32_t* tilePre, uint64_t nTiles,
                        uint32_t* tileQ, hipStream_t s);  // + tileQ (nTiles + 1): each tile's first query
void launch_sweep(const uint64_t* tileRec, const uint32_t* tileQ, uint64_t nTiles, const uint64_t* qkey,
                  const uint32_t* qslot, const uint64_t* unitInfo, uint32_t C, const DbRec* db, uint64_t D,
                  const int32_t* spOf, uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total,
                  mtb_match* buf, uint32_t* bufRank, uint64_t region, int* err, unsigned long long* stats,
                  SegMatch* direct, int* overflow, uint32_t capShift, LongRun* longList, uint32_t longCap,
                  uint32_t* longCnt, uint32_t ldsCap, bool small, int persist, hipStream_t s);
// ldsCap: tests (HBM tiles); small: 24-KB tiles; persist: resident blocks per CU slot (0: a block per tile)
void launch_match(const uint64_t* qkey, const uint32_t* qslot, const uint64_t* unitInfo, uint32_t C, uint64_t Q,
                  const DbRec* db, uint64_t D, const AADir& dir, const int32_t* spOf,
                  uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total, mtb_match* buf,
                  uint32_t* bufRank, uint64_t region, int* err, uint32_t winCap, const uint64_t* win,
                  const ProbeLine* lines, const uint64_t* lineP, const uint16_t* runOff, int sortLo,
                  unsigned long long* stats, SegMatch* direct, const uint64_t* dirOff, int* overflow,
                  uint32_t capShift, LongRun* longList, uint32_t longCap, uint32_t* longCnt, hipStream_t s,
                  const ProbeExt* lineExt = nullptr, uint32_t upr = 0, unsigned long long* cnt64 = nullptr);
// uniform units (upr): k_match and k_match_long reserve ranks on 64-bit per-read counters whose high
// word holds the mate lengths (launch_cnt64_init from the K0 lengths, launch_cnt64_counts back to readCnt)
void launch_cnt64_init(const uint32_t* readLens, uint32_t n, unsigned long long* cnt64, hipStream_t s);
void launch_cnt64_counts(const unsigned long long* cnt64, uint32_t n, uint32_t* readCnt, hipStream_t s);
// direct (nullable): no staging; each read's matches go straight to direct + dirOff[r] * C (its K1
// slot stretch, dirOff = the per-read unit offsets) at its reserved ranks. A query whose ranks pass
// its read's stretch spills its matches and their ranks to buf / bufRank (total[0] of them; at most
// `region`, else *overflow is set and the caller reruns with a larger spill buffer or staged).
// capShift (tests): stretches are taken as their size >> capShift, so that queries spill.
void launch_compact_segments(const SegMatch* in, const uint64_t* dirOff, uint32_t C, const uint64_t* readOff,
                             uint32_t nReads, mtb_match* out, uint32_t capShift, hipStream_t s, int mode = 0);
// (mode 0: every read; 1: only the reads whose matches passed their stretch; 2: all but those)
// the spilled matches to readOff[r] + rank (after launch_compact_segments)
void launch_spill_scatter(const mtb_match* spill, const uint32_t* spillRank, const unsigned long long* total,
                          uint64_t nSpill, const uint64_t* readOff, uint32_t nReads, mtb_match* out, int* err,
                          hipStream_t s);
// K4 runs without LDS DB windows (probe-line lower bounds, no window staging): a DB much larger
// than the query stream; its queries are then sorted finer (kQuerySortLoFine: one more pass buys
// DRAM-page locality for the random DB reads, measured 28.8 -> 26.5 ms per 1M pairs at GTDB scale)
bool unstaged_join(bool lines, uint64_t D, uint64_t Q, uint32_t winCap);  // stats[0] += queries with >= 1 match
// staged matches -> per-read segments at readOff (cursor: zeroed per-read counters)
void launch_match_transpose(const mtb_match* buf, const uint32_t* bufRank, uint64_t region,
                            const unsigned long long* total, const uint64_t* readOff, uint32_t nReads, mtb_match* out,
                            int* err, hipStream_t s);
uint64_t match_window_elems(uint64_t Q);
// MTB_DUP_STATS (diagnostic): out[0] += queries repeating an earlier query's AA rank in their 256-query K4
// block, out[1] += queries repeating its whole key (u64 x 2, accumulated)
void launch_dup_stats(const uint64_t* qkey, uint64_t Q, unsigned long long* out, hipStream_t s);
// mtb_hamming's kernel (bad: u64 count of pairs where the row-cached and plain forms disagree)
void launch_hamming_check(const uint64_t* a, const uint64_t* b, uint64_t n, uint8_t* sum, uint16_t* fwd, uint16_t* rev,
                          unsigned long long* bad, hipStream_t s);
// mtb_pin_eval: the dependency-free helpers (score_fields, ham_fields, consecutive, max_covered_length,
// query_kmer_number: mtb_device.h) on case vectors, fn = MTB_PIN_* (include/mtb_gpu.h), one thread per case
void launch_pin_eval(int fn, const int64_t* param, const uint64_t* a, const uint64_t* b, uint64_t n, int64_t* out,
                     hipStream_t s);
void launch_match_windows(const uint64_t* qkey, uint64_t Q, const DbRec* db, uint64_t D, const AADir& dir,
                          int kmerFormat, uint64_t* win, hipStream_t s);

uint64_t path_bytes();
uint64_t clade_bytes();
// K5; maxSeg: the most matches of one read (picks the kernels to launch); global: every segment
// through the global-scratch network (gScratch 6*M words; parity tests of the general path).
// liveCnt (nullable): drop dead matches (species without a frame run of two, which K6 never
// reads) from segments of <= 512 matches, write each segment front-packed and its live count
// mergeSeg: segments over this many matches (default, 0: 8192, the LDS capacity) sort as LDS chunks of
// that size merged pairwise (tests lower it to exercise the merge path)
// seg (nullable, only with maxSeg <= 512 and !global): read segment r from seg + inOff[r] * inC (the
// direct join's layout, 16-B SegMatch) rather than in + mOff[r]
// Returns the first HIP error of its allocations, copies and launches (hipErrorInvalidValue for a
// sparse input outside the register sorts' range).
// pruneMin: a species is live when one of its (species, frame) groups holds >= pruneMin matches
// (prune_min_matches); >= 2 always.
// segLen / maxTmp (n u32 / 1 u32 device scratch, nullable): with pruning, segments over one LDS
// sort (8192 matches, or mergeSeg) are thinned in place in `in` before they are sorted (k_thin_big);
// `in` is overwritten then.
// pruneAfter (A/B): segments of 129-512 matches are pruned (LDS hash counts), then their live
// matches sorted (0, the default), or sorted whole, then pruned on the sorted order (1).
// lists (4 n + 4 u32 device scratch, nullable): the reads of each size class above 128 matches, so
// the bigger sorts launch a block per read of their class (null: over the whole batch).
hipError_t launch_segsort(const mtb_match* in, const uint64_t* mOff, uint32_t nReads, uint64_t M, mtb_match* out,
                          uint64_t* gScratch, uint32_t maxSeg, bool global, uint32_t* liveCnt, uint32_t mergeSeg,
                          uint32_t pruneMin, hipStream_t s, const SegMatch* seg = nullptr,
                          const uint64_t* inOff = nullptr, uint32_t inC = 0 /* C | capShift << 16 */,
                          uint32_t* segLen = nullptr,
                          uint32_t* maxTmp = nullptr, int pruneAfter = 0, uint32_t* lists = nullptr);
// The fewest matches a (species, frame) group needs for getMatchPaths to emit a path: a path of
// depth d chains >= 1 + ceil((d - 1) / maxCodonShift) matches (each link adds a shift of at most
// maxCodonShift codons, Taxonomer.cpp:487-648), paths are emitted at depth >= MIN_DEPTH
// (minConsCnt, or minConsCntEuk under Eukaryota: the smaller bounds both), and a group of one match
// is never searched (Taxonomer.cpp:334-344). A species with no path gets no score and is read by
// nothing downstream (Taxonomer.cpp:347-408), so its matches are dead.
inline uint32_t prune_min_matches(int minConsCnt, int minConsCntEuk, int maxCodonShift) {
    const int d = minConsCnt < minConsCntEuk ? minConsCnt : minConsCntEuk;
    const int sh = maxCodonShift > 0 ? maxCodonShift : 1;
    const int need = d <= 1 ? 1 : 1 + (d - 1 + sh - 1) / sh;
    return (uint32_t)(need < 2 ? 2 : need);
}
// the live prefix of each segment (mOff) to out at liveOff (exclusive scan of liveCnt)
void launch_pack_live(const mtb_match* in, const uint64_t* mOff, const uint64_t* liveOff, uint32_t nReads,
                      mtb_match* out, int* err, hipStream_t s);
void launch_max_u32(const uint32_t* x, uint32_t n, uint32_t* out, hipStream_t s);
void launch_max_seg(const uint64_t* off, uint32_t n, uint32_t* out, hipStream_t s);
constexpr uint32_t kSegSortLds = 8192;
constexpr uint32_t kSegSortRegs = 512;  // segments up to this many matches sort in registers (sparse input allowed)
constexpr uint32_t kSegSortSparse = 2048;  // K5 reads the direct join's sparse segments up to this many matches
// K6 indexes matches and groups with 32 bits
constexpr uint64_t kMaxBatchMatches = 0xFFFFFFFFull;  // segments up to this many matches sort in LDS
void launch_assign(const mtb_match* matches, const uint64_t* mOff, const uint32_t* qlen, uint32_t nReads, uint64_t nM, const AssignArgs& a, const TaxDevice& t, const AssignScratch& s,
                   mtb_taxcnt* tcPool, mtb_result* results, unsigned long long* devStats, uint64_t* hostStats,
                   hipStream_t st);  // devStats[1] += wave runs sent to the introsort emulation;
                                     // hostStats = {groups, groups >= 2 matches, species runs, wave runs}
// chunk-major per-(chunk, read) counts -> per-read totals, mOff (n + 1), segments in dst
void launch_regroup_chunks(const mtb_match* src, const uint32_t* cnt, uint32_t nChunks, uint32_t n, uint32_t* tot,
                           uint64_t* srcOff, uint64_t* mOff, void* scanTmp, mtb_match* dst, hipStream_t s);
void launch_taxcnt_len(const mtb_result* results, uint32_t nReads, uint32_t* len, hipStream_t s);
void launch_compact_taxcnt(const mtb_taxcnt* pool, const uint64_t* mOff, mtb_result* results, const uint64_t* tcOff,
                           uint32_t nReads, mtb_taxcnt* out, hipStream_t s);

// --em (mtb_assign.hip): per classified read its first kEmTop species by score (std::sort order)
// as (species, score^2) into maps[r * kEmTop ..] (8-B {species, float}), cnt[r] of them; scratch:
// 8 B per species run of the batch.
constexpr int kEmTop = 10;
void launch_em_top(const mtb_match* M, const uint64_t* mOff, uint32_t n, const AssignScratch& s,
                   const mtb_result* results, void* scratch, void* maps, uint8_t* cnt, hipStream_t st);
// those mappings packed in read order as mtb_em_map {batch read, species, score^2}: cnt32 / off
// (n u32 / n + 1 u64 scratch), out (sum of cnt entries; off[n] holds the total)
void launch_em_pack(const void* maps, const uint8_t* cnt, uint32_t n, uint32_t* cnt32, uint64_t* off, void* scanTmp,
                    mtb_em_map* out, hipStream_t s);
// DB k-mers per species taxID (cnt: maxTax + 1 u32, zeroed by the caller)
void launch_species_kmers(const DbRec* db, uint64_t D, const int32_t* spOf, uint32_t maxTax, uint32_t* cnt,
                          hipStream_t s);
// One EM iteration over nQ queries' mappings (qOff: their ranges; spIdx: dense species; pos: each
// mapping's position in species order; sliceOff: nSl slices of one species each; spSlice: each
// species' slices): p -> pNew, *delta = sum |pNew - p| over the top species.
void launch_em_iteration(const float* score, const uint32_t* spIdx, const uint64_t* qOff, uint64_t nQ,
                         const uint64_t* pos, const double* p, const double* lf, double* wS,
                         unsigned long long* qCount, const uint64_t* sliceOff, uint64_t nSl, double* part,
                         const uint64_t* spSlice, uint32_t S, const uint8_t* isTop, double* pNew, double* absd,
                         int afterTen, double* delta, hipStream_t s);
// reassignment of each query (qId: its read) from the final abundances
void launch_em_reclassify(const float* score, const uint32_t* spIdx, const int32_t* spTax, const uint64_t* qOff,
                          const uint32_t* qId, uint64_t nQ, const double* p, const double* lf, const TaxDevice& t,
                          mtb_em_read* out, hipStream_t s);

// ---- K0M: tantan low-complexity masking of the reads (mtb_mask.hip; --mask-residues 1) ----------
constexpr int kTantanOffsets = 50;  // tantan's maxCycleLength (SeqIterator.cpp:163)
struct TantanTables {
    double lr[25];               // likelihood ratios of letter codes (A C G T N) a, b: lr[5 a + b]
    double b2f[kTantanOffsets];  // background -> repeat offset i + 1
    double b2b, f2b, f2f;        // background stays, repeat ends, repeat continues
    double minMask;              // maskProb (minMaskProb) as the comparison uses it
};
TantanTables make_tantan_tables(float maskProb);  // mtb_host.cpp
uint64_t tantan_scale_elems(uint64_t bases, uint32_t n);
// masked copy of a batch's mate: out[b] = 'N' where tantan's repeat probability >= maskProb or the
// letter is not A/C/G/T/U, else seq[b]; prob: 4 B per base, scale: tantan_scale_elems doubles
void launch_tantan_mask(const uint8_t* seq, const uint64_t* off, uint32_t n, const TantanTables& tt, float* prob,
                        double* scale, uint8_t* out, hipStream_t s);

}  // namespace mtb
