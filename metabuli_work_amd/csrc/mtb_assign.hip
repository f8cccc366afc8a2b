// K5 + K6: per-read match sort and taxonomic assignment (Classifier::assignTaxonomy,
// Classifier.cpp:166-208; Taxonomer::chooseBestTaxon and helpers, Taxonomer.cpp:130-713).
//
// K5 sorts each read's match segment (k_segsort_*); K6 then runs one thread per read over the
// sorted segment, executing the reference's decision tree with per-read scratch carved from
// batch-wide arrays by the read's match offset. Float arithmetic
// follows the reference operation for operation (compiled with -ffp-contract=off).
#include <algorithm>
#include <vector>

#include "mtb_launch.h"
#include "mtb_stdsort.h"

namespace mtb {

struct Path {  // MatchPath (Taxonomer.h:35-59); start/end match as indices into the read segment
    int start, end;
    float score;
    int hd, depth;
    uint32_t sm, em;
};

// ------------------------------------------------------------------------------------------------
// K5 segmented sort of each read's matches into compareMatches order (KmerMatcher.cpp:1149-1166).
// Key = (species:32 | frame:3 | pos:29, hamming:8 | dna:24 | target:32), compared as 128 bits;
// the last field only makes the order total (a valid DB never ties before it).
// Small segments (<= 512): one wave64 per read, register-resident bitonic sort of keys + indices
// (up to 8 per lane, cross-lane shuffles), then a gather-permute of the 24-B records into the
// output segment (contiguous writes). Larger segments: one 1024-thread block per read, bitonic
// sort in LDS (<= 8192) or, beyond that, in a global key scratch.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void match_key(const mtb_match& m, uint64_t& hi, uint64_t& lo) {
    hi = ((uint64_t)m.species_id << 32) | ((uint64_t)info_frame(m.qinfo) << 29) | (info_pos(m.qinfo) & 0x1FFFFFFFu);
    lo = ((uint64_t)m.hamming << 56) | ((uint64_t)(m.dna_encoding & 0xFFFFFFu) << 32) | m.target_id;
}

__device__ __forceinline__ bool key_gt(uint64_t ah, uint64_t al, uint64_t bh, uint64_t bl) {
    return ah > bh || (ah == bh && al > bl);
}

constexpr int kSmallSeg = 512;  // segments up to this many matches sort in registers (one wave, <= 8 per lane)
static_assert(kSmallSeg == (int)kSegSortRegs, "one register-sort bound");
constexpr int kBlockSeg = 8192;
constexpr uint32_t kSegSkip = 0xFFFFFFFFu;  // segLen entry of a read another pass sorts

// The length of read r's segment: its mOff stretch, or segLen[r] when given (segments compacted in
// place by k_prune_compact); -1 = not this pass's read (kSegSkip).
__device__ __forceinline__ long seg_len(const uint64_t* __restrict__ mOff, const uint32_t* __restrict__ segLen,
                                        uint32_t r) {
    if (!segLen) return (long)(mOff[r + 1] - mOff[r]);
    const uint32_t v = segLen[r];
    return v == kSegSkip ? -1 : (long)v;
}

// Segments of up to 64E matches sort in registers: element e = 64*slot + lane. Exchanges at
// distance j < 64 swap with lane ^ j through DPP / permlane moves (xor_lane: no LDS crossbar),
// j >= 64 swap slots inside a lane;
// the network is unrolled at compile time so the slots stay in VGPRs. No LDS, no barriers.
// The (k, j) stages of a bitonic network over 64E elements, in order, as compile-time constants
// (f(k, j) per stage: the cross-lane moves need j as a template argument).
template <int K, int J, int E, typename F>
__device__ __forceinline__ void bitonic_stages(F& f) {
    f(std::integral_constant<int, K>{}, std::integral_constant<int, J>{});
    if constexpr (J > 1) bitonic_stages<K, J / 2, E>(f);
    else if constexpr (K < 64 * E) bitonic_stages<K * 2, K, E>(f);
}

template <int J>
__device__ __forceinline__ uint64_t xor_lane64c(uint64_t v, int lane) {
    return (uint64_t)xor_lane<J>((uint32_t)(v >> 32), lane) << 32 | xor_lane<J>((uint32_t)v, lane);
}

template <int E>
__device__ __forceinline__ void wave_bitonic_sort(uint64_t (&h)[E], uint64_t (&l)[E], uint32_t (&x)[E], int lane) {
    auto stage = [&](auto kc, auto jc) {
        constexpr int k = decltype(kc)::value, j = decltype(jc)::value;
        if constexpr (j >= 64) {
            constexpr int js = j >> 6;
#pragma unroll
            for (int sl = 0; sl < E; sl++) {
                if (sl & js) continue;
                const int s2 = sl | js;
                const bool up = ((64 * sl + lane) & k) == 0;
                if (key_gt(h[sl], l[sl], h[s2], l[s2]) == up) {
                    const uint64_t th = h[sl], tl = l[sl];
                    const uint32_t tx = x[sl];
                    h[sl] = h[s2]; l[sl] = l[s2]; x[sl] = x[s2];
                    h[s2] = th; l[s2] = tl; x[s2] = tx;
                }
            }
        } else {
            const bool lower = (lane & j) == 0;
#pragma unroll
            for (int sl = 0; sl < E; sl++) {
                const bool up = ((64 * sl + lane) & k) == 0;
                const uint64_t ph = xor_lane64c<j>(h[sl], lane), pl = xor_lane64c<j>(l[sl], lane);
                const uint32_t px = xor_lane<j>(x[sl], lane);
                // the lower lane of the pair keeps the smaller key when ascending
                const bool takeP = (key_gt(h[sl], l[sl], ph, pl) == (lower == up));
                if (takeP) { h[sl] = ph; l[sl] = pl; x[sl] = px; }
            }
        }
    };
    bitonic_stages<2, 1, E>(stage);
}

// Dead matches: a (species, frame) run of one match is never given to getMatchPaths
// (Taxonomer.cpp:334-344), so a species none of whose frame runs has two matches gets no path and
// no score; it can be neither the best species nor in bestSpeciesRange, the only matches
// filterRedundantMatches reads (Taxonomer.cpp:141-172,205-241). Its matches change nothing
// downstream and are dropped here (prune): the sorted segment is written front-packed with only
// the live matches, their count in liveCnt[r].
// K5 inputs: a segment of full matches, or of the direct join's 16-B SegMatch records of read r
// (expanded on load: qinfo from r, species from spOf).
struct MatchIn {
    const mtb_match* __restrict__ p;
    uint64_t base;
    __device__ __forceinline__ mtb_match full(uint32_t e) const { return p[base + e]; }
};
struct SegIn {
    const SegMatch* __restrict__ p;
    uint64_t base;
    uint64_t seqBits;
    __device__ __forceinline__ mtb_match full(uint32_t e) const { return seg_expand(p[base + e], seqBits); }
};

// The direct join's sparse input (seg: 16-B records in per-read slot stretches, read r's at
// seg + inOff[r] * C): inCS = C | capShift << 16. A read whose matches passed its stretch (some were
// spilled: n > the stretch) was compacted into the match array at mOff[r] with its spills, so K5 reads
// it from there; every other read is read in place.
__device__ __forceinline__ bool sparse_read(const SegMatch* seg, const uint64_t* __restrict__ inOff, uint32_t inCS,
                                            uint32_t r, long n) {
    if (!seg) return false;
    const uint64_t cap = ((inOff[r + 1] - inOff[r]) * (inCS & 0xFFFFu)) >> (inCS >> 16);
    return (uint64_t)n <= cap;
}
__device__ __forceinline__ SegIn sparse_in(const SegMatch* seg, const uint64_t* __restrict__ inOff, uint32_t inCS,
                                           uint32_t r) {
    return SegIn{seg, inOff[r] * (inCS & 0xFFFFu), (uint64_t)(r + 1) << 32};
}

// Open-addressing insert into a wave's LDS table of tn (power of two) slots, key 0 = empty; returns
// the key's slot.
template <typename K>
__device__ __forceinline__ uint32_t lds_insert(K* tab, uint32_t tn, K key) {
    uint32_t i = (uint32_t)(((uint64_t)key * 0x9E3779B97F4A7C15ull) >> 40) & (tn - 1);
    while (true) {
        const K prev = atomicCAS(&tab[i], (K)0, key);
        if (prev == 0 || prev == key) return i;
        i = (i + 1) & (tn - 1);
    }
}

// The pruned sort with the dead matches dropped BEFORE sorting: (species, frame) pairs are counted
// in an LDS hash table, a species with any pair counted twice is live (the run-of-two rule
// above), and only the live matches (43% at GTDB scale) are compacted through LDS and sorted, in
// the fewest register slots that hold them. The output is the live subset of the full sort's
// order (a total order), as segsort_regs writes it.
template <int E2>
__device__ __forceinline__ void sort_live(mtb_match* __restrict__ out, uint64_t seqBits,
                                          uint64_t base, int nLive, int lane, const uint64_t* cH,
                                          const uint64_t* cL, const uint32_t* cX) {
    uint64_t h[E2], l[E2];
    uint32_t x[E2];
#pragma unroll
    for (int sl = 0; sl < E2; sl++) {
        const int e = 64 * sl + lane;
        const bool v = e < nLive;
        h[sl] = v ? cH[e] : ~0ull;
        l[sl] = v ? cL[e] : ~0ull;
        x[sl] = v ? cX[e] : 0u;
    }
    wave_bitonic_sort<E2>(h, l, x, lane);
#pragma unroll
    for (int sl = 0; sl < E2; sl++) {
        const int e = 64 * sl + lane;
        if (e < nLive) {  // the record rebuilt from its key (+ rightEndHamming riding in x): no gather
            mtb_match m;
            m.qinfo = ((h[sl] >> 29) & 7ull) << 61 | seqBits | (uint32_t)(h[sl] & 0x1FFFFFFFu);
            m.target_id = (uint32_t)l[sl];
            m.species_id = (uint32_t)(h[sl] >> 32);
            m.dna_encoding = (uint32_t)(l[sl] >> 32) & 0xFFFFFFu;
            m.right_end_hamming = (uint16_t)(x[sl] >> 16);
            m.hamming = (uint8_t)(l[sl] >> 56);
            m.pad = 0;
            out[base + e] = m;
        }
    }
}

// prune_then_sort's LDS: the hash tables while the matches are counted, then (the live flags held
// in registers) the live keys gathered for the sort, in the same bytes: 20 B per match slot in all
// (12 KB for a 512-match wave), so that several waves share a CU and hide the shuffles' latency.
template <int E>
struct PruneLds {
    union {
        struct {
            uint32_t spKey[128 * E];    // species (> 0 for a valid DB) | live << 31
            uint32_t pairKey[128 * E];  // (species slot << 3 | frame) + 1
            uint32_t pairCnt[128 * E];
        } t;
        struct {
            uint64_t cH[64 * E], cL[64 * E];
            uint32_t cX[64 * E];
        } c;
    };
};
template <int E>
__device__ __forceinline__ PruneLds<E>& prune_lds() {
    __shared__ PruneLds<E> lds;
    return lds;
}
template <int E>
__device__ __forceinline__ uint8_t* run_live_lds() {
    __shared__ uint8_t runLive[64 * E];
    return runLive;
}

template <int E, typename In>
__device__ __forceinline__ void prune_then_sort(const In& in, mtb_match* __restrict__ out, uint64_t base, int n, int lane,
                                                uint32_t* __restrict__ liveCnt, uint32_t r, uint32_t pm) {
    constexpr uint32_t T = 128 * E;  // load <= 1/2
    constexpr uint32_t kLive = 0x80000000u;
    PruneLds<E>& L = prune_lds<E>();  // one LDS instance per E whatever the input type
    uint32_t *spKey = L.t.spKey, *pairKey = L.t.pairKey, *pairCnt = L.t.pairCnt;
    for (uint32_t i = lane; i < T; i += 64) {
        spKey[i] = 0;
        pairKey[i] = 0;
        pairCnt[i] = 0;
    }
    __syncthreads();
    uint64_t h[E], l[E];
    uint32_t ps[E], ss[E], rx[E];
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        h[sl] = l[sl] = 0;
        ps[sl] = ss[sl] = rx[sl] = 0;
        if (e < n) {
            const mtb_match m = in.full((uint32_t)e);
            match_key(m, h[sl], l[sl]);
            rx[sl] = (uint32_t)m.right_end_hamming << 16;
            ss[sl] = lds_insert<uint32_t>(spKey, T, (uint32_t)(h[sl] >> 32));
            ps[sl] = lds_insert<uint32_t>(pairKey, T, (ss[sl] << 3 | ((uint32_t)(h[sl] >> 29) & 7u)) + 1u);
            atomicAdd(&pairCnt[ps[sl]], 1u);
        }
    }
    __syncthreads();
#pragma unroll
    for (int sl = 0; sl < E; sl++)
        if (64 * sl + lane < n && pairCnt[ps[sl]] >= pm) spKey[ss[sl]] |= kLive;  // same value from every writer
    __syncthreads();
    bool live[E];
#pragma unroll
    for (int sl = 0; sl < E; sl++) live[sl] = 64 * sl + lane < n && (spKey[ss[sl]] & kLive);
    __syncthreads();  // the tables are dead: their bytes take the live keys
    uint64_t *cH = L.c.cH, *cL = L.c.cL;
    uint32_t* cX = L.c.cX;
    const uint64_t lt = (1ull << lane) - 1;
    int nLive = 0;
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const uint64_t m = __ballot(live[sl]);
        if (live[sl]) {
            const int p = nLive + (int)__popcll(m & lt);
            cH[p] = h[sl];
            cL[p] = l[sl];
            cX[p] = rx[sl] | (uint32_t)(64 * sl + lane);
        }
        nLive += (int)__popcll(m);
    }
    __syncthreads();
    // the segment's read (every match of a segment carries it); keys hold the rest of the record
    const uint64_t seqBits = nLive ? in.full(0).qinfo & (0x1FFFFFFFull << 32) : 0;
    if (nLive <= 64) sort_live<1>(out, seqBits, base, nLive, lane, cH, cL, cX);
    else if (E >= 2 && nLive <= 128) sort_live<(E >= 2 ? 2 : 1)>(out, seqBits, base, nLive, lane, cH, cL, cX);
    else if (E >= 4 && nLive <= 256) sort_live<(E >= 4 ? 4 : 1)>(out, seqBits, base, nLive, lane, cH, cL, cX);
    else sort_live<E>(out, seqBits, base, nLive, lane, cH, cL, cX);
    if (lane == 0) liveCnt[r] = (uint32_t)nLive;
}

// Bitonic sort of one key per element (no payload: the keys carry their record's index), the
// network of wave_bitonic_sort: element e = 64 * slot + lane.
template <int E, typename K>
__device__ __forceinline__ void wave_bitonic_keys(K (&k)[E], int lane) {
    auto stage = [&](auto kc, auto jc) {
        constexpr int kk = decltype(kc)::value, j = decltype(jc)::value;
        if constexpr (j >= 64) {
            constexpr int js = j >> 6;
#pragma unroll
            for (int sl = 0; sl < E; sl++) {
                if (sl & js) continue;
                const int s2 = sl | js;
                const bool up = ((64 * sl + lane) & kk) == 0;
                if ((k[sl] > k[s2]) == up) {
                    const K t = k[sl];
                    k[sl] = k[s2];
                    k[s2] = t;
                }
            }
        } else {
            const bool lower = (lane & j) == 0;
#pragma unroll
            for (int sl = 0; sl < E; sl++) {
                const bool up = ((64 * sl + lane) & kk) == 0;
                K pk;
                if constexpr (sizeof(K) == 8) pk = (K)xor_lane64c<j>((uint64_t)k[sl], lane);
                else pk = (K)xor_lane<j>((uint32_t)k[sl], lane);
                if ((k[sl] > pk) == (lower == up)) k[sl] = pk;
            }
        }
    };
    bitonic_stages<2, 1, E>(stage);
}

// n (<= 64 ES) keys of LDS array a sorted in place by one wave.
template <int ES, typename K>
__device__ __forceinline__ void lds_sort_keys(K* a, int n, int lane) {
    K k[ES];
#pragma unroll
    for (int sl = 0; sl < ES; sl++) {
        const int e = 64 * sl + lane;
        k[sl] = e < n ? a[e] : (K)~(K)0;
    }
    wave_bitonic_keys<ES, K>(k, lane);
#pragma unroll
    for (int sl = 0; sl < ES; sl++) {
        const int e = 64 * sl + lane;
        if (e < n) a[e] = k[sl];
    }
}

template <int E, typename K>
__device__ __forceinline__ void lds_sort_keys_n(K* a, int n, int lane) {
    if (n <= 64) lds_sort_keys<1, K>(a, n, lane);
    else if (E >= 2 && n <= 128) lds_sort_keys<(E >= 2 ? 2 : 1), K>(a, n, lane);
    else if (E >= 4 && n <= 256) lds_sort_keys<(E >= 4 ? 4 : 1), K>(a, n, lane);
    else lds_sort_keys<E, K>(a, n, lane);
}

// The pruned sort on compact keys (the default for 65-512 matches): prune as prune_then_sort does
// (LDS hash counts of (species, frame) pairs), then replace each live species by its rank among the
// read's live species (the distinct species sorted once, usually a few dozen), so that
// (rank:9 | frame:3 | pos:29 | record:9) is one 64-bit key in (species, frame, pos) order whose low
// bits name the LDS record: the network moves one 64-bit value per element instead of a 128-bit key
// and an index (fewer cross-lane shuffles, a third of the sort registers). Elements tied on
// (species, frame, pos) — one query k-mer matching several DB k-mers of the species — take their
// places inside the tie by (hamming, dna, target), the rest of compareMatches' order, counted from
// the LDS records (ties are short runs of neighbours). Same output as prune_then_sort.
template <int E>
struct RankLds {
    union {
        struct {
            uint32_t spKey[128 * E];    // species | live << 31
            uint32_t pairKey[128 * E];  // (species slot << 3 | frame) + 1; then the rank of a species slot
            uint32_t pairCnt[128 * E];  // pair counts; then the live species list
        } t;
        struct {
            uint64_t key[64 * E];  // the live matches' keys, sorted in place
            uint64_t lo[64 * E];   // record: hamming:8 | dna:24 | target:32
            uint32_t sp[64 * E];   // record: species
            uint32_t rx[64 * E];   // record: rightEndHamming << 16
        } c;
    };
};

template <int E>
__device__ __forceinline__ RankLds<E>& rank_lds() {  // one LDS instance per E whatever the input type
    __shared__ RankLds<E> lds;
    return lds;
}

template <int E, typename In>
__device__ __forceinline__ void prune_rank_sort(const In& in, mtb_match* __restrict__ out, uint64_t base, int n, int lane,
                                                uint32_t* __restrict__ liveCnt, uint32_t r, uint32_t pm) {
    constexpr uint32_t T = 128 * E;  // load <= 1/2
    constexpr uint32_t kLive = 0x80000000u;
    RankLds<E>& L = rank_lds<E>();
    uint32_t *spKey = L.t.spKey, *pairKey = L.t.pairKey, *pairCnt = L.t.pairCnt;
    for (uint32_t i = lane; i < T; i += 64) {
        spKey[i] = 0;
        pairKey[i] = 0;
        pairCnt[i] = 0;
    }
    __syncthreads();
    uint64_t h[E], l[E];
    uint32_t ps[E], ss[E], rx[E];
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        h[sl] = l[sl] = 0;
        ps[sl] = ss[sl] = rx[sl] = 0;
        if (e < n) {
            const mtb_match m = in.full((uint32_t)e);
            match_key(m, h[sl], l[sl]);
            rx[sl] = (uint32_t)m.right_end_hamming << 16;
            ss[sl] = lds_insert<uint32_t>(spKey, T, (uint32_t)(h[sl] >> 32));
            ps[sl] = lds_insert<uint32_t>(pairKey, T, (ss[sl] << 3 | ((uint32_t)(h[sl] >> 29) & 7u)) + 1u);
            atomicAdd(&pairCnt[ps[sl]], 1u);
        }
    }
    __syncthreads();
#pragma unroll
    for (int sl = 0; sl < E; sl++)
        if (64 * sl + lane < n && pairCnt[ps[sl]] >= pm) spKey[ss[sl]] |= kLive;  // same value from every writer
    __syncthreads();
    bool live[E];
#pragma unroll
    for (int sl = 0; sl < E; sl++) live[sl] = 64 * sl + lane < n && (spKey[ss[sl]] & kLive);
    // the live species, sorted: their ranks (pairKey and pairCnt are dead now)
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t* spList = pairCnt;
    int S = 0;
    for (uint32_t i0 = 0; i0 < T; i0 += 64) {
        const uint32_t v = spKey[i0 + lane];
        const bool lv = (v & kLive) != 0;
        const uint64_t m = __ballot(lv);
        if (lv) spList[S + (int)__popcll(m & lt)] = v & ~kLive;
        S += (int)__popcll(m);
    }
    __syncthreads();
    lds_sort_keys_n<E, uint32_t>(spList, S, lane);
    __syncthreads();
    for (int e = lane; e < S; e += 64) {  // rank of each live species, stored at its table slot
        const uint32_t v = spList[e];
        uint32_t i = (uint32_t)(((uint64_t)v * 0x9E3779B97F4A7C15ull) >> 40) & (T - 1);
        while ((spKey[i] & ~kLive) != v) i = (i + 1) & (T - 1);
        pairKey[i] = (uint32_t)e;
    }
    __syncthreads();
    uint64_t key[E];
    int nLive = 0;
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const uint64_t m = __ballot(live[sl]);
        const uint32_t p = (uint32_t)(nLive + (int)__popcll(m & lt));
        key[sl] = live[sl] ? ((uint64_t)pairKey[ss[sl]] << 41 | ((h[sl] >> 29) & 7ull) << 38 |
                              (h[sl] & 0x1FFFFFFFull) << 9 | p)
                           : 0;
        nLive += (int)__popcll(m);
    }
    __syncthreads();  // the tables are dead: their bytes take the live records and keys
#pragma unroll
    for (int sl = 0; sl < E; sl++)
        if (live[sl]) {
            const uint32_t p = (uint32_t)(key[sl] & 511u);
            L.c.key[p] = key[sl];
            L.c.lo[p] = l[sl];
            L.c.sp[p] = (uint32_t)(h[sl] >> 32);
            L.c.rx[p] = rx[sl];
        }
    __syncthreads();
    lds_sort_keys_n<E, uint64_t>(L.c.key, nLive, lane);
    __syncthreads();
    // the segment's read (every match of a segment carries it); the keys and records hold the rest
    const uint64_t seqBits = nLive ? in.full(0).qinfo & (0x1FFFFFFFull << 32) : 0;
    for (int e = lane; e < nLive; e += 64) {
        const uint64_t k = L.c.key[e];
        const uint32_t p = (uint32_t)(k & 511u);
        const uint64_t pre = k >> 9, lo = L.c.lo[p];
        int at = e;  // place inside a (species, frame, pos) tie: by (hamming, dna, target)
        for (int j = e - 1; j >= 0 && (L.c.key[j] >> 9) == pre; j--) at -= L.c.lo[L.c.key[j] & 511u] > lo;
        for (int j = e + 1; j < nLive && (L.c.key[j] >> 9) == pre; j++) at += L.c.lo[L.c.key[j] & 511u] < lo;
        mtb_match m;
        m.qinfo = ((k >> 38) & 7ull) << 61 | seqBits | (uint32_t)((k >> 9) & 0x1FFFFFFFu);
        m.target_id = (uint32_t)lo;
        m.species_id = L.c.sp[p];
        m.dna_encoding = (uint32_t)(lo >> 32) & 0xFFFFFFu;
        m.right_end_hamming = (uint16_t)(L.c.rx[p] >> 16);
        m.hamming = (uint8_t)(lo >> 56);
        m.pad = 0;
        out[base + at] = m;
    }
    if (lane == 0) liveCnt[r] = (uint32_t)nLive;
}

// Sort all, then prune on the sorted segment (kAfter, and E == 1): a (species, frame) group of >= pm
// matches starts at e when e + pm - 1 holds its pair; a species run with such a group is live. Its
// LDS is 64E bytes, so occupancy is bound by registers, not by prune_then_sort's hash tables.
template <int E, typename In>
__device__ __forceinline__ void sort_then_prune(const In& in, mtb_match* __restrict__ out, uint64_t base, int n,
                                                int lane, uint32_t* __restrict__ liveCnt, uint32_t r, uint32_t pm) {
    uint64_t h[E], l[E];
    uint32_t x[E];
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        h[sl] = ~0ull;
        l[sl] = ~0ull;
        x[sl] = 0;
        if (e < n) {
            const mtb_match m = in.full((uint32_t)e);
            match_key(m, h[sl], l[sl]);
            x[sl] = (uint32_t)m.right_end_hamming << 16;
        }
    }
    const uint64_t seqBits = in.full(0).qinfo & (0x1FFFFFFFull << 32);
    wave_bitonic_sort<E>(h, l, x, lane);
    uint8_t* runLive = run_live_lds<E>();
    const uint64_t lt = (1ull << lane) - 1;
    const int far = lane + (int)pm - 1;  // pm <= 64 (the caller checks)
    uint32_t rid[E];
    bool pair[E];
    uint32_t runs = 0;
    uint64_t prevLast = ~0ull;  // the previous slot's last (species, frame)
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        const uint64_t sf = h[sl] >> 29;  // species << 3 | frame
        const uint64_t a = __shfl(sf, far & 63, 64);
        const uint64_t b = __shfl(h[sl + 1 < E ? sl + 1 : sl] >> 29, far & 63, 64);
        uint64_t pv = __shfl_up(sf, 1, 64);
        if (lane == 0) pv = prevLast;
        prevLast = __shfl(sf, 63, 64);
        pair[sl] = e + (int)pm - 1 < n && (far < 64 ? a : b) == sf;
        const bool start = e < n && (e == 0 || (pv >> 3) != (sf >> 3));
        const uint64_t m = __ballot(start);
        rid[sl] = runs + (uint32_t)__popcll(m & lt) + (uint32_t)start - 1u;
        runs += (uint32_t)__popcll(m);
        runLive[64 * sl + lane] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int sl = 0; sl < E; sl++)
        if (pair[sl]) runLive[rid[sl]] = 1;
    __syncthreads();
    uint32_t kept = 0;
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        const bool live = e < n && runLive[rid[sl]];
        const uint64_t m = __ballot(live);
        if (live) {  // the record rebuilt from its key (+ rightEndHamming riding in x): no gather
            mtb_match o;
            o.qinfo = ((h[sl] >> 29) & 7ull) << 61 | seqBits | (uint32_t)(h[sl] & 0x1FFFFFFFu);
            o.target_id = (uint32_t)l[sl];
            o.species_id = (uint32_t)(h[sl] >> 32);
            o.dna_encoding = (uint32_t)(l[sl] >> 32) & 0xFFFFFFu;
            o.right_end_hamming = (uint16_t)(x[sl] >> 16);
            o.hamming = (uint8_t)(l[sl] >> 56);
            o.pad = 0;
            out[base + kept + (uint32_t)__popcll(m & lt)] = o;
        }
        kept += (uint32_t)__popcll(m);
    }
    if (lane == 0) liveCnt[r] = kept;
}

// kMode (E >= 2, with pruning): 2 = prune, then sort the live matches on compact rank keys
// (prune_rank_sort, the default); 0 = prune, then sort the live matches' full keys
// (prune_then_sort); 1 = sort all, then prune (sort_then_prune).
// kMode 3: no pruning (the full sort below), a kernel of its own so that its 128-bit network does not
// set the pruned kernels' register budget.
template <int E, typename In, int kMode = 2>
__device__ __forceinline__ void segsort_regs(const In& in, mtb_match* __restrict__ out, uint64_t base, int n, int lane,
                                             uint32_t* __restrict__ liveCnt, uint32_t r, uint32_t pm) {
    if constexpr (E >= 2 && kMode == 2) {
        if (liveCnt) {
            prune_rank_sort<E>(in, out, base, n, lane, liveCnt, r, pm);
            return;
        }
        // unpruned: the small kernel (E 2) falls through to the full sort; launch_sorts sends the
        // E 4 / 8 kernels' unpruned batches to kMode 3
        if constexpr (E > 2) return;
    } else if constexpr (E >= 2 && kMode == 1) {
        if (liveCnt && pm <= 64) {
            sort_then_prune<E>(in, out, base, n, lane, liveCnt, r, pm);
            return;
        }
    } else if constexpr (E >= 2 && kMode == 0) {
        if (liveCnt) {
            prune_then_sort<E>(in, out, base, n, lane, liveCnt, r, pm);
            return;
        }
        if constexpr (E > 2) return;
    }
    uint64_t h[E], l[E];
    uint32_t x[E];
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        h[sl] = ~0ull;
        l[sl] = ~0ull;
        x[sl] = (uint32_t)e;
        if (e < n) match_key(in.full((uint32_t)e), h[sl], l[sl]);
    }
    wave_bitonic_sort<E>(h, l, x, lane);
    if (!liveCnt) {
#pragma unroll
        for (int sl = 0; sl < E; sl++) {
            const int e = 64 * sl + lane;
            if (e < n) out[base + e] = in.full(x[sl]);
        }
        return;
    }
    if constexpr (E == 1) {  // E >= 2 prunes before sorting (prune_then_sort)
    uint8_t* runLive = run_live_lds<E>();
    const uint64_t lt = (1ull << lane) - 1;
    bool pair[E];
    uint32_t rid[E];
    uint32_t runs = 0;
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        const uint64_t sf = h[sl] >> 29;  // species << 3 | frame
        // sorted: a (species, frame) group of >= pm matches starts at e when e + pm - 1 has its pair
        const uint64_t far = __shfl(sf, min(lane + (int)pm - 1, 63), 64);
        uint64_t pv = __shfl_up(sf, 1, 64);  // every lane takes part in the shuffles
        if (lane == 0) pv = ~0ull;
        pair[sl] = e + (int)pm - 1 < n && far == sf;
        const bool start = e < n && (e == 0 || (pv >> 3) != (sf >> 3));
        const uint64_t m = __ballot(start);
        rid[sl] = runs + (uint32_t)__popcll(m & lt) + (uint32_t)start - 1u;  // starts at or before e, - 1
        runs += (uint32_t)__popcll(m);
        runLive[64 * sl + lane] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int sl = 0; sl < E; sl++)
        if (pair[sl]) runLive[rid[sl]] = 1;
    __syncthreads();
    uint32_t kept = 0;
#pragma unroll
    for (int sl = 0; sl < E; sl++) {
        const int e = 64 * sl + lane;
        const bool live = e < n && runLive[rid[sl]];
        const uint64_t m = __ballot(live);
        if (live) out[base + kept + (uint32_t)__popcll(m & lt)] = in.full(x[sl]);
        kept += (uint32_t)__popcll(m);
    }
    if (lane == 0) liveCnt[r] = kept;
    }
}

// inOff (nullable): the segments are read from in + inOff[r] * inC (the direct join's per-read slot
// stretches) instead of in + mOff[r]; the output is at out + mOff[r] either way.
template <typename In>
__device__ __forceinline__ void segsort_small_run(const In& in, mtb_match* __restrict__ out, uint64_t base, int n,
                                                  int lane, uint32_t* __restrict__ liveCnt, uint32_t r, uint32_t pm) {
    if (n <= 1 || (liveCnt && n < (int)pm)) {  // too few matches for one live (species, frame) group
        if (lane == 0 && n == 1 && !liveCnt) out[base] = in.full(0);
        if (lane == 0 && liveCnt) liveCnt[r] = 0;
        return;
    }
    if (n <= 64) segsort_regs<1>(in, out, base, n, lane, liveCnt, r, pm);
    else segsort_regs<2>(in, out, base, n, lane, liveCnt, r, pm);
}

__global__ void __launch_bounds__(64) k_segsort_small(const mtb_match* __restrict__ in, const uint64_t* __restrict__ mOff,
                                                      const SegMatch* __restrict__ seg,
                                                      const uint64_t* __restrict__ inOff, uint32_t inC,
                                                      uint32_t nReads, mtb_match* __restrict__ out,
                                                      uint32_t* __restrict__ liveCnt, uint32_t pm,
                                                      const uint32_t* __restrict__ segLen) {
    const uint32_t r = blockIdx.x;
    if (r >= nReads) return;
    const uint64_t base = mOff[r];
    const long nl = seg_len(mOff, segLen, r);
    if (nl < 0 || nl > 128) return;
    const int n = (int)nl;
    if (sparse_read(seg, inOff, inC, r, n)) segsort_small_run(sparse_in(seg, inOff, inC, r), out, base, n, threadIdx.x, liveCnt, r, pm);
    else segsort_small_run(MatchIn{in, base}, out, base, n, threadIdx.x, liveCnt, r, pm);
}

// 129..256 (E = 4) and 257..512 (E = 8) matches: the same register network with more slots per
// lane, in kernels of their own so the small kernel keeps its register budget (occupancy).
template <int E, int kMode>
__global__ void __launch_bounds__(64) k_segsort_regs(const mtb_match* __restrict__ in, const uint64_t* __restrict__ mOff,
                                                     const SegMatch* __restrict__ seg,
                                                     const uint64_t* __restrict__ inOff, uint32_t inC,
                                                     uint32_t nReads, mtb_match* __restrict__ out,
                                                     uint32_t* __restrict__ liveCnt, uint32_t pm,
                                                     const uint32_t* __restrict__ segLen,
                                                     const uint32_t* __restrict__ list) {
    const uint32_t r = list ? list[blockIdx.x] : blockIdx.x;  // list: the reads of this size class
    if (r >= nReads) return;
    const uint64_t base = mOff[r];
    const long nl = seg_len(mOff, segLen, r);
    if (nl <= 32 * E || nl > 64 * E) return;
    const int n = (int)nl;
    if (sparse_read(seg, inOff, inC, r, n))
        segsort_regs<E, SegIn, kMode>(sparse_in(seg, inOff, inC, r), out, base, n,
                                       (int)threadIdx.x, liveCnt, r, pm);
    else
        segsort_regs<E, MatchIn, kMode>(MatchIn{in, base}, out, base, n, (int)threadIdx.x, liveCnt, r, pm);
}

// One block per large segment (the block loops over the reads of its 256-read slice). Segments with
// p2 <= 4096 sort in LDS; larger ones in global scratch laid out as three arrays of 2*M words
// (keys hi, keys lo, indices), the read's slice at offset 2*base (p2 <= 2n).
// Bitonic sort of p2 (power of two) 128-bit keys with a permutation, one compare-exchange pair
// per thread and step: pair t covers i = t with a zero bit inserted at log2(j), and i + j.
template <int kThreads, typename Idx>
__device__ void block_bitonic(uint64_t* H, uint64_t* Lo, Idx* I, long p2) {
    for (long k = 2; k <= p2; k <<= 1)
        for (long j = k >> 1; j > 0; j >>= 1) {
            for (long t = threadIdx.x; t < (p2 >> 1); t += kThreads) {
                const long i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                const long ixj = i + j;
                const bool up = (i & k) == 0;
                const uint64_t ah = H[i], al = Lo[i], bh = H[ixj], bl = Lo[ixj];
                if (key_gt(ah, al, bh, bl) == up) {
                    H[i] = bh; Lo[i] = bl; H[ixj] = ah; Lo[ixj] = al;
                    const Idx x = I[i]; I[i] = I[ixj]; I[ixj] = x;
                }
            }
            __threadfence_block();
            __syncthreads();
        }
}

// Exclusive block scan for kThreads-thread blocks (wave shuffles + one LDS word per wave).
template <int kThreads>
__device__ uint32_t block_scan_u32(uint32_t x, uint32_t* total, uint32_t* sWave) {
    constexpr int kW = kThreads / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) sWave[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int i = 0; i < kW; i++) {
            const uint32_t t = sWave[i];
            sWave[i] = run;
            run += t;
        }
        sWave[kW] = run;
    }
    __syncthreads();
    const uint32_t r = sWave[w] + inc - x;
    *total = sWave[kW];
    __syncthreads();
    return r;
}

// Dead-match pruning for a segment sorted by a block (see segsort_regs): elements 0..n-1 in
// sorted order, hi keys in H (species << 32 | frame << 29 | pos), the permutation in I. Each thread
// takes a contiguous chunk: species-run ids by a block scan of run starts, a flag per run that has
// a (species, frame) pair, then the live elements written in order. rid: n words, runLive: n bytes
// of scratch. Returns the live count.
// kSp / kSpf: the right shifts of a key that leave its species / (species, frame) — 32 / 29 for the
// hi word of match_key, 40 / 37 for the compact keys of the large sort.
template <int kThreads, typename Idx, typename In, int kSp = 32, int kSpf = 29>
__device__ uint32_t prune_pack_block(const uint64_t* H, const Idx* I, uint32_t* rid, uint8_t* runLive, long n,
                                     const In& in, mtb_match* __restrict__ out, uint64_t base,
                                     uint32_t* sWave, uint32_t pm) {
    const long per = (n + kThreads - 1) / kThreads;
    const long b = (long)threadIdx.x * per, e = min(n, b + per);
    uint32_t starts = 0;
    for (long i = b; i < e; i++) starts += (i == 0 || (H[i] >> kSp) != (H[i - 1] >> kSp)) ? 1u : 0u;
    uint32_t nRuns;
    uint32_t run = block_scan_u32<kThreads>(starts, &nRuns, sWave);
    for (long i = b; i < e; i++) {
        if (i == 0 || (H[i] >> kSp) != (H[i - 1] >> kSp)) run++;
        rid[i] = run - 1;
    }
    for (long i = threadIdx.x; i < (long)nRuns; i += kThreads) runLive[i] = 0;
    __threadfence_block();  // the scratch may be global memory (segments over kBlockSeg)
    __syncthreads();
    for (long i = b; i < e; i++)
        if (i + (long)pm - 1 < n && (H[i] >> kSpf) == (H[i + pm - 1] >> kSpf)) runLive[rid[i]] = 1;  // a group of >= pm
    __threadfence_block();
    __syncthreads();
    uint32_t mine = 0;
    for (long i = b; i < e; i++) mine += runLive[rid[i]];
    uint32_t kept;
    uint32_t at = block_scan_u32<kThreads>(mine, &kept, sWave);
    for (long i = b; i < e; i++)
        if (runLive[rid[i]]) out[base + at++] = in.full((uint32_t)I[i]);
    return kept;
}

// Lossy pre-prune for the block sorts (segments over 512 matches): (species, frame) pairs counted
// in a hash indexed by the pair (collisions merge pairs), species flagged live in a hash indexed by
// the species when one of their pairs counts twice. A collision can only keep a dead match (the
// exact pruning after the sort still drops it), never drop a live one. The tables (T u32 each)
// live in the LDS the sort uses afterwards; each thread keeps its <= 8 elements' keys in registers,
// and the live ones are then written compacted into H / L / I. Returns the live count.
template <int kThreads, int kPer, typename Idx, typename In>
__device__ long preprune_load(const In& in, long n, uint32_t* cnt, uint32_t* flag,
                              uint32_t logT, uint64_t* H, uint64_t* L, Idx* I, uint32_t* sWave, uint32_t pm) {
    const uint32_t T = 1u << logT;
    for (uint32_t i = threadIdx.x; i < T; i += kThreads) {
        cnt[i] = 0;
        flag[i] = 0;
    }
    const long b = (long)threadIdx.x * kPer;
    uint64_t h[kPer], l[kPer];
    uint32_t hp[kPer], hs[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        h[k] = l[k] = 0;
        hp[k] = hs[k] = 0;
        if (b + k < n) {
            match_key(in.full((uint32_t)(b + k)), h[k], l[k]);
            hp[k] = (uint32_t)(((h[k] >> 29) * 0x9E3779B97F4A7C15ull) >> (64 - logT));
            hs[k] = (uint32_t)(((h[k] >> 32) * 0xC2B2AE3D27D4EB4Full) >> (64 - logT));
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (b + k < n) atomicAdd(&cnt[hp[k]], 1u);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (b + k < n && cnt[hp[k]] >= pm) flag[hs[k]] = 1;
    __syncthreads();
    uint32_t mask = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (b + k < n && flag[hs[k]]) mask |= 1u << k;
    uint32_t nLive;
    uint32_t at = block_scan_u32<kThreads>((uint32_t)__popc(mask), &nLive, sWave);  // syncs: the tables are free
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if ((mask >> k) & 1u) {
            H[at] = h[k];
            L[at] = l[k];
            I[at] = (Idx)(b + k);
            at++;
        }
    __syncthreads();
    return (long)nLive;
}

// Segments of 513..kBlockSeg matches sort in LDS with one 1024-thread block per read (long reads:
// ~2.5k matches at N50 10 kb); larger ones run the same network over a global key scratch.
constexpr int kLargeThreads = 1024;

// Segments of 513..2048 matches: the same LDS sort with a 2048-entry tile and 256 threads, so four
// blocks share a CU (the 8192-entry kernel holds 147 KB of LDS: one block per CU).
constexpr int kMidSeg = 2048;
constexpr int kMidThreads = 256;
static_assert(kMidSeg == (int)kSegSortSparse, "the sparse-input bound of launch_segsort");

struct MidLds {
    uint64_t sh[kMidSeg], sl[kMidSeg];
    uint16_t si[kMidSeg];
    uint32_t sWave[kMidThreads / 64 + 1];
};

template <typename In>
__device__ __forceinline__ void segsort_mid_run(const In& in, MidLds& L, mtb_match* __restrict__ out, uint64_t base,
                                                long n, uint32_t* __restrict__ liveCnt, uint32_t r, uint32_t pm) {
    uint64_t *sh = L.sh, *sl = L.sl;
    uint16_t* si = L.si;
    long m = n;  // elements sorted: the pre-pruned live ones (prune), or all
    if (liveCnt) {
        static_assert(kMidSeg / kMidThreads == 8 && 2 * kMidSeg == 4096, "pre-prune geometry");
        m = preprune_load<kMidThreads, 8, uint16_t>(in, n, reinterpret_cast<uint32_t*>(sh),
                                                    reinterpret_cast<uint32_t*>(sl), 12, sh, sl, si, L.sWave, pm);
        if (m == 0) {
            if (threadIdx.x == 0) liveCnt[r] = 0;
            return;
        }
    }
    long p2 = 2;
    while (p2 < m) p2 <<= 1;
    for (long i = threadIdx.x; i < p2; i += kMidThreads) {
        if (liveCnt && i < m) continue;  // loaded by the pre-prune
        uint64_t h = ~0ull, l = ~0ull;
        if (i < m) match_key(in.full((uint32_t)i), h, l);
        sh[i] = h; sl[i] = l; si[i] = (uint16_t)i;
    }
    __syncthreads();
    block_bitonic<kMidThreads, uint16_t>(sh, sl, si, p2);
    if (liveCnt) {
        n = m;
        uint32_t* rid = reinterpret_cast<uint32_t*>(sl);
        const uint32_t kept = prune_pack_block<kMidThreads, uint16_t>(sh, si, rid, reinterpret_cast<uint8_t*>(rid + n), n,
                                                                      in, out, base, L.sWave, pm);
        if (threadIdx.x == 0) liveCnt[r] = kept;
        return;
    }
    for (long i = threadIdx.x; i < n; i += kMidThreads) out[base + i] = in.full(si[i]);
}

template <int kThreads, int kSeg, typename In>
__device__ bool segsort_compact(const In& in, long n, uint64_t* K, uint64_t* Lo, uint16_t* orig, uint32_t* sWave,
                                mtb_match* __restrict__ out, uint64_t base, uint32_t* __restrict__ liveCnt, uint32_t r,
                                uint32_t pm, bool bitonic);

// seg (nullable): the direct join's sparse per-read stretches (seg + inOff[r] * inC), as
// k_segsort_small reads them, so that batches of <= kMidSeg matches per read need no compaction.
// compact (pruning only): 1 the compact-key sort (segsort_compact), 2 the same on the bitonic network.
__global__ void __launch_bounds__(kMidThreads) k_segsort_mid(const mtb_match* __restrict__ in,
                                                             const uint64_t* __restrict__ mOff, uint32_t nReads,
                                                             mtb_match* __restrict__ out, uint32_t* __restrict__ liveCnt,
                                                             long mergeSeg, uint32_t pm,
                                                             const uint32_t* __restrict__ segLen,
                                                             const SegMatch* __restrict__ seg,
                                                             const uint64_t* __restrict__ inOff, uint32_t inC,
                                                             int compact, const uint32_t* __restrict__ list) {
    __shared__ MidLds L;
    const uint32_t r = list ? list[blockIdx.x] : blockIdx.x;
    if (r >= nReads) return;
    const uint64_t base = mOff[r];
    const long n = seg_len(mOff, segLen, r);
    if (n <= kSmallSeg || n > kMidSeg || n > mergeSeg) return;  // larger: k_segsort_large / merge path
    if (sparse_read(seg, inOff, inC, r, n)) {
        const auto sin = sparse_in(seg, inOff, inC, r);
        if (liveCnt && compact &&
            segsort_compact<kMidThreads, kMidSeg>(sin, n, L.sh, L.sl, L.si, L.sWave, out, base, liveCnt, r, pm, compact == 2))
            return;
        segsort_mid_run(sin, L, out, base, n, liveCnt, r, pm);
    } else {
        if (liveCnt && compact &&
            segsort_compact<kMidThreads, kMidSeg>(MatchIn{in, base}, n, L.sh, L.sl, L.si, L.sWave, out, base, liveCnt, r,
                                                  pm, compact == 2))
            return;
        segsort_mid_run(MatchIn{in, base}, L, out, base, n, liveCnt, r, pm);
    }
}

// The LDS pruned sorts on compact keys (segments of 513..2048 matches on 256 threads, 2049..8192 on
// 1024: long reads), as the register sorts do (prune_rank_sort): species:24 | frame:3 | pos:24 | slot:13
// in one 64-bit key, the slot naming the element's record (its lo key and original index) in LDS, so
// the sort moves 8 B per element instead of a 128-bit key and an index. Elements tied on (species, frame, pos)
// are placed inside their tie by the lo key (hamming, dna, target), the rest of compareMatches'
// order. Segments with a species or a position of 2^24 or more take the full-key sort (returns false).
constexpr int kCSp = 40, kCSpf = 37, kCPos = 13;

template <int kThreads>
__device__ __forceinline__ void block_bitonic_u64(uint64_t* K, long p2) {
    for (long k = 2; k <= p2; k <<= 1)
        for (long j = k >> 1; j > 0; j >>= 1) {
            for (long t = threadIdx.x; t < (p2 >> 1); t += kThreads) {
                const long i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                const long ixj = i + j;
                const bool up = (i & k) == 0;
                const uint64_t a = K[i], b = K[ixj];
                if ((a > b) == up) {
                    K[i] = b;
                    K[ixj] = a;
                }
            }
            __syncthreads();
        }
}

// One wave's register bitonic sort of 64E keys (element e = 64 * slot + lane), as wave_bitonic_sort
// on a single 64-bit key.
template <int E>
__device__ __forceinline__ void wave_sort_u64(uint64_t (&k)[E], int lane) {
    auto stage = [&](auto kc, auto jc) {
        constexpr int kk = decltype(kc)::value, j = decltype(jc)::value;
        if constexpr (j >= 64) {
            constexpr int js = j >> 6;
#pragma unroll
            for (int sl = 0; sl < E; sl++) {
                if (sl & js) continue;
                const int s2 = sl | js;
                const bool up = ((64 * sl + lane) & kk) == 0;
                const uint64_t a = k[sl], b = k[s2];
                if ((a > b) == up) {
                    k[sl] = b;
                    k[s2] = a;
                }
            }
        } else {
            const bool lower = (lane & j) == 0;
#pragma unroll
            for (int sl = 0; sl < E; sl++) {
                const bool up = ((64 * sl + lane) & kk) == 0;
                const uint64_t p = xor_lane64c<j>(k[sl], lane);
                if ((k[sl] > p) == (lower == up)) k[sl] = p;
            }
        }
    };
    bitonic_stages<2, 1, E>(stage);
}

// Sorts K[0, p2) ascending (p2 a power of two <= kSeg; every thread of the kThreads-thread block).
// From max(kThreads, 512) keys on: runs of 512 sort in registers, a wave each (DPP / permlane moves,
// no barriers), then log2(p2 / 512) merge rounds in place — each thread finds the merge-path split of
// its p2 / kThreads outputs, merges them into registers and writes them back after a barrier —
// instead of the bitonic network's up to ~90 barrier-separated LDS stages. Keys are distinct but for
// the ~0 padding.
template <int kThreads, int kSeg>
__device__ void block_sort_u64(uint64_t* K, long p2) {
    constexpr int E = 8, kRun = 64 * E, kOut = kSeg / kThreads;
    static_assert(kSeg <= kRun * (kThreads / 64) && kOut <= 8, "a run per wave, <= 8 outputs per thread");
    if (p2 < kThreads || p2 < kRun) {
        block_bitonic_u64<kThreads>(K, p2);
        return;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if ((long)w * kRun < p2) {
        uint64_t k[E];
#pragma unroll
        for (int sl = 0; sl < E; sl++) k[sl] = K[w * kRun + 64 * sl + lane];
        wave_sort_u64<E>(k, lane);
#pragma unroll
        for (int sl = 0; sl < E; sl++) K[w * kRun + 64 * sl + lane] = k[sl];
    }
    __syncthreads();
    const int per = (int)(p2 / kThreads);  // outputs per thread: 1..kOut
    for (long run = kRun; run < p2; run <<= 1) {
        const long d0 = (long)threadIdx.x * per, ps = d0 & ~(2 * run - 1), d = d0 - ps;
        const uint64_t* A = K + ps;
        const uint64_t* B = A + run;
        long lo = max(0l, d - run), hi = min(d, run);
        while (lo < hi) {  // the first d outputs take i keys of A and d - i of B
            const long i = (lo + hi) >> 1;
            if (B[d - i - 1] > A[i]) lo = i + 1;
            else hi = i;
        }
        long i = lo, j = d - lo;
        uint64_t o[kOut];
#pragma unroll
        for (int t = 0; t < kOut; t++) {
            if (t >= per) break;
            const uint64_t a = i < run ? A[i] : ~0ull, b = j < run ? B[j] : ~0ull;
            const bool takeA = j >= run || (i < run && a <= b);
            o[t] = takeA ? a : b;
            i += takeA;
            j += !takeA;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < kOut; t++)
            if (t < per) K[d0 + t] = o[t];
        __syncthreads();
    }
}

template <int kThreads, int kSeg, typename In>
__device__ bool segsort_compact(const In& in, long n, uint64_t* K, uint64_t* Lo, uint16_t* orig, uint32_t* sWave,
                                mtb_match* __restrict__ out, uint64_t base, uint32_t* __restrict__ liveCnt, uint32_t r,
                                uint32_t pm, bool bitonic) {
    constexpr int kPer = kSeg / kThreads;  // 8
    static_assert(kPer == 8 && (kSeg == 2048 || kSeg == 8192) && kSeg <= (1 << kCPos), "compact geometry");
    constexpr uint32_t logT = kSeg == 8192 ? 14 : 12, T = 1u << logT;  // pair / species hashes in K and Lo (2 kSeg words)
    uint32_t* cnt = reinterpret_cast<uint32_t*>(K);
    uint32_t* flag = reinterpret_cast<uint32_t*>(Lo);
    const long b = (long)threadIdx.x * kPer;
    uint64_t h[kPer], l[kPer];
    uint32_t hp[kPer], hs[kPer];
    bool bad = false;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        h[k] = l[k] = 0;
        hp[k] = hs[k] = 0;
        if (b + k < n) {
            match_key(in.full((uint32_t)(b + k)), h[k], l[k]);
            bad |= (h[k] >> 32) >= (1ull << 24) || (h[k] & 0x1FFFFFFFull) >= (1ull << 24);
            hp[k] = (uint32_t)(((h[k] >> 29) * 0x9E3779B97F4A7C15ull) >> (64 - logT));
            hs[k] = (uint32_t)(((h[k] >> 32) * 0xC2B2AE3D27D4EB4Full) >> (64 - logT));
        }
    }
    if (__syncthreads_or(bad)) return false;
    for (uint32_t i = threadIdx.x; i < T; i += kThreads) {
        cnt[i] = 0;
        flag[i] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (b + k < n) atomicAdd(&cnt[hp[k]], 1u);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (b + k < n && cnt[hp[k]] >= pm) flag[hs[k]] = 1;
    __syncthreads();
    uint32_t mask = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (b + k < n && flag[hs[k]]) mask |= 1u << k;
    uint32_t m;
    uint32_t at = block_scan_u32<kThreads>((uint32_t)__popc(mask), &m, sWave);  // syncs: the tables are free
    if (m == 0) {
        if (threadIdx.x == 0) liveCnt[r] = 0;
        return true;
    }
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if ((mask >> k) & 1u) {
            K[at] = (h[k] >> 32) << kCSp | ((h[k] >> 29) & 7ull) << kCSpf | (h[k] & 0xFFFFFFull) << kCPos | at;
            Lo[at] = l[k];
            orig[at] = (uint16_t)(b + k);
            at++;
        }
    long p2 = 2;
    while (p2 < (long)m) p2 <<= 1;
    for (long i = (long)m + threadIdx.x; i < p2; i += kThreads) K[i] = ~0ull;
    __syncthreads();
    if (bitonic) block_bitonic_u64<kThreads>(K, p2);  // A/B: the plain LDS network
    else block_sort_u64<kThreads, kSeg>(K, p2);
    // places inside (species, frame, pos) ties, then the original index at each place
    uint16_t pos[kPer], idx[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        const long e = threadIdx.x + (long)j * kThreads;
        pos[j] = idx[j] = 0;
        if (e < (long)m) {
            const uint64_t k = K[e], pre = k >> kCPos, lo = Lo[k & (kSeg - 1)];
            long a = e;
            for (long q = e - 1; q >= 0 && (K[q] >> kCPos) == pre; q--) a -= Lo[K[q] & (kSeg - 1)] > lo;
            for (long q = e + 1; q < (long)m && (K[q] >> kCPos) == pre; q++) a += Lo[K[q] & (kSeg - 1)] < lo;
            pos[j] = (uint16_t)a;
            idx[j] = orig[k & (kSeg - 1)];
        }
    }
    __syncthreads();  // the lo keys are dead: their LDS takes the placed indices, run ids and flags
    uint16_t* placed = reinterpret_cast<uint16_t*>(Lo);
#pragma unroll
    for (int j = 0; j < kPer; j++)
        if (threadIdx.x + (long)j * kThreads < (long)m) placed[pos[j]] = idx[j];
    __syncthreads();
    uint32_t* rid = reinterpret_cast<uint32_t*>(placed + kSeg);
    const uint32_t kept = prune_pack_block<kThreads, uint16_t, In, kCSp, kCSpf>(
        K, placed, rid, reinterpret_cast<uint8_t*>(rid + kSeg), (long)m, in, out, base, sWave, pm);
    if (threadIdx.x == 0) liveCnt[r] = kept;
    return true;
}

__global__ void __launch_bounds__(kLargeThreads) k_segsort_large(const mtb_match* __restrict__ in,
                                                                 const uint64_t* __restrict__ mOff, uint32_t nReads,
                                                                 uint64_t M, mtb_match* __restrict__ out,
                                                                 uint64_t* __restrict__ gScratch, int global,
                                                                 uint32_t* __restrict__ liveCnt, long mergeSeg, uint32_t pm,
                                                                 const uint32_t* __restrict__ segLen, int compact,
                                                                 const uint32_t* __restrict__ list) {
    __shared__ uint64_t sh[kBlockSeg], sl[kBlockSeg];
    __shared__ uint16_t si[kBlockSeg];
    const uint32_t r = list ? list[blockIdx.x] : blockIdx.x;  // one block per read (of its size class)
    if (r >= nReads) return;
    const uint64_t base = mOff[r];
    long n = seg_len(mOff, segLen, r);
    if (n < 0) return;
    if (global && n == 0 && liveCnt && threadIdx.x == 0) liveCnt[r] = 0;  // k_segsort_small is not launched
    if (global ? n == 0 : n <= kMidSeg) return;  // global: every segment takes the scratch path (tests)
    __shared__ uint32_t sWave[kLargeThreads / 64 + 1];
    long p2 = 2;
    while (p2 < n) p2 <<= 1;
    if (!global && n > mergeSeg) return;  // chunked LDS sorts + merge path (launch_segsort)
    if (!global && liveCnt && compact &&
        segsort_compact<kLargeThreads, kBlockSeg>(MatchIn{in, base}, n, sh, sl, si, sWave, out, base, liveCnt, r, pm,
                                                  compact == 2))
        return;
    if (!global) {
        long m = n;  // elements sorted: the pre-pruned live ones (prune), or all
        if (liveCnt) {
            static_assert(kBlockSeg / kLargeThreads == 8 && 2 * kBlockSeg == 16384, "pre-prune geometry");
            m = preprune_load<kLargeThreads, 8, uint16_t>(MatchIn{in, base}, n, reinterpret_cast<uint32_t*>(sh),
                                                          reinterpret_cast<uint32_t*>(sl), 14, sh, sl, si, sWave, pm);
            if (m == 0) {
                if (threadIdx.x == 0) liveCnt[r] = 0;
                return;
            }
            p2 = 2;
            while (p2 < m) p2 <<= 1;
        }
        for (long i = threadIdx.x; i < p2; i += kLargeThreads) {
            if (liveCnt && i < m) continue;  // loaded by the pre-prune
            uint64_t h = ~0ull, l = ~0ull;
            if (i < m) match_key(in[base + i], h, l);
            sh[i] = h; sl[i] = l; si[i] = (uint16_t)i;
        }
        __syncthreads();
        block_bitonic<kLargeThreads, uint16_t>(sh, sl, si, p2);
        n = m;
        if (liveCnt) {  // the lo keys are no longer needed: their LDS holds the run ids and flags
            uint32_t* rid = reinterpret_cast<uint32_t*>(sl);
            const uint32_t kept = prune_pack_block<kLargeThreads, uint16_t>(sh, si, rid, reinterpret_cast<uint8_t*>(rid + n),
                                                                            n, MatchIn{in, base}, out, base, sWave, pm);
            if (threadIdx.x == 0) liveCnt[r] = kept;
            return;
        }
        for (long i = threadIdx.x; i < n; i += kLargeThreads) out[base + i] = in[base + si[i]];
        return;
    }
    uint64_t* H = gScratch + 2 * base;
    uint64_t* Lo = gScratch + 2 * M + 2 * base;
    uint32_t* I = (uint32_t*)(gScratch + 4 * M) + 2 * base;
    for (long i = threadIdx.x; i < p2; i += kLargeThreads) {
        uint64_t h = ~0ull, l = ~0ull;
        if (i < n) match_key(in[base + i], h, l);
        H[i] = h; Lo[i] = l; I[i] = (uint32_t)i;
    }
    __threadfence_block();
    __syncthreads();
    block_bitonic<kLargeThreads, uint32_t>(H, Lo, I, p2);
    if (liveCnt) {  // run ids and flags in the lo-key scratch (2 * p2 words, p2 >= n)
        uint32_t* rid = reinterpret_cast<uint32_t*>(Lo);
        const uint32_t kept =
            prune_pack_block<kLargeThreads, uint32_t>(H, I, rid, reinterpret_cast<uint8_t*>(rid + n), n, MatchIn{in, base},
                                                      out, base, sWave, pm);
        if (threadIdx.x == 0) liveCnt[r] = kept;
        return;
    }
    for (long i = threadIdx.x; i < n; i += kLargeThreads) out[base + i] = in[base + I[i]];
}

// Batch maxima: 8 elements per thread, a wave and a block reduction, then one atomic per 256-thread
// block (one atomicMax per wave on one address had serialised ~100k atomics: 0.59 ms per 3.33M-pair
// batch).
constexpr int kMaxPer = 8;
__device__ __forceinline__ void block_max_to(uint32_t v, uint32_t* __restrict__ out) {
    __shared__ uint32_t sM[4];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = max(v, (uint32_t)__shfl_xor(v, d, 64));
    if ((threadIdx.x & 63) == 0) sM[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t m = max(max(sM[0], sM[1]), max(sM[2], sM[3]));
        if (m) atomicMax(out, m);
    }
}
__device__ __forceinline__ uint64_t max_elem(uint32_t k) { return (uint64_t)blockIdx.x * (256 * kMaxPer) + k * 256 + threadIdx.x; }
__host__ __device__ constexpr uint32_t max_blocks(uint32_t n) { return (n + 256 * kMaxPer - 1) / (256 * kMaxPer); }

__global__ void __launch_bounds__(256) k_max_u32(const uint32_t* __restrict__ x, uint32_t n, uint32_t* __restrict__ out) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < kMaxPer; k++)
        if (max_elem(k) < n) v = max(v, x[max_elem(k)]);
    block_max_to(v, out);
}

// ---- segments over kBlockSeg matches (long reads): each kBlockSeg chunk sorts in LDS, then the
// sorted runs are merged pairwise (merge path: every thread finds its output diagonal's split by
// binary search and merges 8 elements), then pruning / the gather-permute. Keys + segment-local
// indices ping-pong between two scratch buffers indexed by the match's global position:
// buffer b: hi keys at b*3M, lo keys at b*3M + M, indices (u32) at b*3M + 2M words.
struct MergeBuf {
    uint64_t* h;
    uint64_t* l;
    uint32_t* x;
};
__device__ __forceinline__ MergeBuf merge_buf(uint64_t* scratch, uint64_t M, int b) {
    uint64_t* p = scratch + (uint64_t)b * 3 * M;
    return MergeBuf{p, p + M, reinterpret_cast<uint32_t*>(p + 2 * M)};
}

__global__ void __launch_bounds__(kLargeThreads) k_chunk_sort(const mtb_match* __restrict__ in,
                                                              const uint64_t* __restrict__ mOff,
                                                              const uint2* __restrict__ chunks, uint64_t M,
                                                              uint64_t* __restrict__ scratch, long chunk,
                                                              const uint32_t* __restrict__ segLen) {
    __shared__ uint64_t sh[kBlockSeg], sl[kBlockSeg];
    __shared__ uint16_t si[kBlockSeg];
    const uint2 ck = chunks[blockIdx.x];  // (read, chunk start)
    const uint64_t base = mOff[ck.x];
    const long n = seg_len(mOff, segLen, ck.x);
    const long cs = ck.y, len = min(chunk, n - cs);
    long p2 = 2;
    while (p2 < len) p2 <<= 1;
    for (long i = threadIdx.x; i < p2; i += kLargeThreads) {
        uint64_t h = ~0ull, l = ~0ull;
        if (i < len) match_key(in[base + cs + i], h, l);
        sh[i] = h; sl[i] = l; si[i] = (uint16_t)i;
    }
    __syncthreads();
    block_bitonic<kLargeThreads, uint16_t>(sh, sl, si, p2);
    const MergeBuf o = merge_buf(scratch, M, 0);
    for (long i = threadIdx.x; i < len; i += kLargeThreads) {
        o.h[base + cs + i] = sh[i];
        o.l[base + cs + i] = sl[i];
        o.x[base + cs + i] = (uint32_t)(cs + si[i]);
    }
}

constexpr int kMergePer = 8;                   // outputs per thread
constexpr int kMergeTile = 256 * kMergePer;    // outputs per block

// One tile of the merge of runs A = [ps, ps + w) and B = [ps + w, ps + 2w) (clipped to n) of a
// segment, from buffer src into dst. tiles: (read, pair start, tile start).
__global__ void __launch_bounds__(256) k_merge_tiles(const uint64_t* __restrict__ mOff, const uint4* __restrict__ tiles,
                                                     uint64_t M, uint64_t* __restrict__ scratch, int src, long w,
                                                     const uint32_t* __restrict__ segLen) {
    const uint4 t = tiles[blockIdx.x];
    const uint64_t base = mOff[t.x];
    const long n = seg_len(mOff, segLen, t.x);
    const long ps = t.y;
    const long na = min(w, n - ps), nb = max(0l, min(w, n - ps - w));
    const MergeBuf S = merge_buf(scratch, M, src), D = merge_buf(scratch, M, src ^ 1);
    const uint64_t a0 = base + ps, b0 = a0 + na;
    long d = (long)t.z + (long)threadIdx.x * kMergePer;
    if (d >= na + nb) return;
    // merge path: the first d outputs take i from A and d - i from B
    long lo = max(0l, d - nb), hi = min(d, na);
    while (lo < hi) {
        const long i = (lo + hi) >> 1;
        // A[i] goes before B[d - i - 1] ?  (ties cannot occur: the key is a total order)
        if (key_gt(S.h[b0 + d - i - 1], S.l[b0 + d - i - 1], S.h[a0 + i], S.l[a0 + i])) lo = i + 1;
        else hi = i;
    }
    long i = lo, j = d - lo;
    const long end = min(na + nb, d + kMergePer);
    for (; d < end; d++) {
        const bool takeA = j >= nb || (i < na && !key_gt(S.h[a0 + i], S.l[a0 + i], S.h[b0 + j], S.l[b0 + j]));
        const uint64_t from = takeA ? a0 + i : b0 + j;
        D.h[a0 + d] = S.h[from];
        D.l[a0 + d] = S.l[from];
        D.x[a0 + d] = S.x[from];
        if (takeA) i++; else j++;
    }
}

// The merged segment in buffer b: pruning (run ids and flags in the other buffer's lo keys) or the
// plain gather-permute.
__global__ void __launch_bounds__(kLargeThreads) k_merge_finish(const mtb_match* __restrict__ in,
                                                                const uint64_t* __restrict__ mOff,
                                                                const uint32_t* __restrict__ reads, uint64_t M,
                                                                uint64_t* __restrict__ scratch, int b,
                                                                mtb_match* __restrict__ out,
                                                                uint32_t* __restrict__ liveCnt, uint32_t pm,
                                                                const uint32_t* __restrict__ segLen) {
    __shared__ uint32_t sWave[kLargeThreads / 64 + 1];
    const uint32_t r = reads[blockIdx.x];
    const uint64_t base = mOff[r];
    const long n = seg_len(mOff, segLen, r);
    const MergeBuf S = merge_buf(scratch, M, b), T = merge_buf(scratch, M, b ^ 1);
    if (liveCnt) {
        uint32_t* rid = reinterpret_cast<uint32_t*>(T.l + base);
        const uint32_t kept = prune_pack_block<kLargeThreads, uint32_t>(S.h + base, S.x + base, rid,
                                                                        reinterpret_cast<uint8_t*>(rid + n), n,
                                                                        MatchIn{in, base}, out, base, sWave, pm);
        if (threadIdx.x == 0) liveCnt[r] = kept;
        return;
    }
    for (long i = threadIdx.x; i < n; i += kLargeThreads) out[base + i] = in[base + S.x[base + i]];
}

#define MTB_HIP_RET(x)                       \
    do {                                     \
        const hipError_t e_ = (x);           \
        if (e_ != hipSuccess) return e_;     \
    } while (0)

static hipError_t launch_merge_path(const mtb_match* in, const uint64_t* mOff, uint32_t nReads, uint64_t M,
                                    mtb_match* out, uint64_t* scratch, uint32_t* liveCnt, long chunk, uint32_t pm,
                                    const uint32_t* segLen, hipStream_t s) {
    std::vector<uint64_t> off(nReads + 1);
    std::vector<uint32_t> len;
    MTB_HIP_RET(hipMemcpyAsync(off.data(), mOff, sizeof(uint64_t) * (nReads + 1), hipMemcpyDeviceToHost, s));
    if (segLen) {
        len.resize(nReads);
        MTB_HIP_RET(hipMemcpyAsync(len.data(), segLen, sizeof(uint32_t) * nReads, hipMemcpyDeviceToHost, s));
    }
    MTB_HIP_RET(hipStreamSynchronize(s));
    auto nOf = [&](uint32_t r) -> long {
        if (!segLen) return (long)(off[r + 1] - off[r]);
        return len[r] == kSegSkip ? -1 : (long)len[r];
    };
    std::vector<uint32_t> big;
    std::vector<uint2> chunks;
    long maxN = 0;
    for (uint32_t r = 0; r < nReads; r++) {
        const long n = nOf(r);
        if (n <= chunk) continue;
        big.push_back(r);
        maxN = std::max(maxN, n);
        for (long c = 0; c < n; c += chunk) chunks.push_back(make_uint2(r, (uint32_t)c));
    }
    if (big.empty()) return hipSuccess;
    uint2* dChunks = nullptr;
    uint4* dTiles = nullptr;
    uint32_t* dBig = nullptr;
    // every allocation and copy is checked: a kernel must never launch over a null buffer
    hipError_t e = hipMallocAsync((void**)&dChunks, sizeof(uint2) * chunks.size(), s);
    if (e == hipSuccess) e = hipMallocAsync((void**)&dBig, sizeof(uint32_t) * big.size(), s);
    if (e == hipSuccess) e = hipMemcpyAsync(dChunks, chunks.data(), sizeof(uint2) * chunks.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(dBig, big.data(), sizeof(uint32_t) * big.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) {
        k_chunk_sort<<<(unsigned)chunks.size(), kLargeThreads, 0, s>>>(in, mOff, dChunks, M, scratch, chunk, segLen);
        e = hipGetLastError();
    }
    // every round's tiles planned at once and uploaded in one copy: the rounds then follow each other
    // in stream order with no host round trip between them
    int b = 0;
    std::vector<uint4> tiles;
    std::vector<size_t> roundAt;
    for (long w = chunk; w < maxN; w *= 2) {
        roundAt.push_back(tiles.size());
        for (uint32_t r : big) {
            const long n = nOf(r);
            for (long ps = 0; ps < n; ps += 2 * w) {
                const long len2 = std::min(2 * w, n - ps);
                for (long t = 0; t < len2; t += kMergeTile) tiles.push_back(make_uint4(r, (uint32_t)ps, (uint32_t)t, 0));
            }
        }
    }
    roundAt.push_back(tiles.size());
    if (e == hipSuccess && !tiles.empty()) {
        e = hipMallocAsync((void**)&dTiles, sizeof(uint4) * tiles.size(), s);
        if (e == hipSuccess) e = hipMemcpyAsync(dTiles, tiles.data(), sizeof(uint4) * tiles.size(), hipMemcpyHostToDevice, s);
    }
    long w = chunk;
    for (size_t rr = 0; e == hipSuccess && rr + 1 < roundAt.size(); rr++, w *= 2) {
        k_merge_tiles<<<(unsigned)(roundAt[rr + 1] - roundAt[rr]), 256, 0, s>>>(mOff, dTiles + roundAt[rr], M, scratch, b, w,
                                                                                segLen);
        e = hipGetLastError();
        b ^= 1;
    }
    if (e == hipSuccess) {
        k_merge_finish<<<(unsigned)big.size(), kLargeThreads, 0, s>>>(in, mOff, dBig, M, scratch, b, out, liveCnt, pm,
                                                                       segLen);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the host vectors the copies read stay alive until here
    if (dTiles) hipFreeAsync(dTiles, s);
    if (dChunks) hipFreeAsync(dChunks, s);
    if (dBig) hipFreeAsync(dBig, s);
    return e;
}

// Segments too big for one LDS sort (> chunk matches, long reads; ~75% of their matches are dead)
// are thinned before they are sorted: one block per read counts the read's (species, frame) pairs
// in an LDS hash indexed by the pair and flags species in a hash indexed by the species when a pair
// reaches pm (collisions merge counters, so a dead match may survive but a live one never drops:
// the sort kernels' exact pruning then runs on the survivors), and packs the survivors to the front
// of the read's segment in place, staged through the (not yet written) output segment.
// segLen[r] = survivors; reads at or below `chunk` get kSegSkip (sorted and pruned the usual way).
constexpr int kThinLog = 14;  // 2^14 counters + 2^14 flags: 128 KB of LDS

template <typename In>
__device__ void thin_run(const In& in, bool inPlace, mtb_match* __restrict__ io, mtb_match* __restrict__ stage,
                         uint64_t base, long n, uint32_t pm, uint32_t* __restrict__ segLen, uint32_t r, uint32_t* cnt,
                         uint32_t* flag, uint32_t& sCount);

// seg (nullable): the direct join's sparse stretches; a read that fits its stretch is read there
// (no compaction of the batch first) and its survivors are written straight to io.
__global__ void __launch_bounds__(kLargeThreads) k_thin_big(mtb_match* __restrict__ io, mtb_match* __restrict__ stage,
                                                            const uint64_t* __restrict__ mOff, uint32_t nReads,
                                                            long chunk, uint32_t pm, uint32_t* __restrict__ segLen,
                                                            const SegMatch* __restrict__ seg,
                                                            const uint64_t* __restrict__ inOff, uint32_t inC) {
    __shared__ uint32_t cnt[1 << kThinLog], flag[1 << kThinLog];
    __shared__ uint32_t sCount;
    const uint32_t r = blockIdx.x;
    if (r >= nReads) return;
    const uint64_t base = mOff[r];
    const long n = (long)(mOff[r + 1] - base);
    if (n <= chunk) {
        if (threadIdx.x == 0) segLen[r] = kSegSkip;
        return;
    }
    if (sparse_read(seg, inOff, inC, r, n))
        thin_run(sparse_in(seg, inOff, inC, r), false, io, stage, base, n, pm, segLen, r, cnt, flag, sCount);
    else
        thin_run(MatchIn{io, base}, true, io, stage, base, n, pm, segLen, r, cnt, flag, sCount);
}

template <typename In>
__device__ void thin_run(const In& in, bool inPlace, mtb_match* __restrict__ io, mtb_match* __restrict__ stage,
                         uint64_t base, long n, uint32_t pm, uint32_t* __restrict__ segLen, uint32_t r, uint32_t* cnt,
                         uint32_t* flag, uint32_t& sCount) {
    constexpr uint32_t T = 1u << kThinLog;
    for (uint32_t i = threadIdx.x; i < T; i += kLargeThreads) { cnt[i] = 0; flag[i] = 0; }
    if (threadIdx.x == 0) sCount = 0;
    __syncthreads();
    auto pairSlot = [](const mtb_match& m) {
        const uint64_t k = ((uint64_t)m.species_id << 3) | info_frame(m.qinfo);
        return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> (64 - kThinLog));
    };
    auto spSlot = [](const mtb_match& m) {
        return (uint32_t)(((uint64_t)m.species_id * 0xC2B2AE3D27D4EB4Full) >> (64 - kThinLog));
    };
    // the first kThinReg elements of each thread keep their two hash slots in registers, so the flag
    // pass and the survivors' test read no records again (a record is re-read only if it survives)
    constexpr int kThinReg = 16;
    static_assert(kThinLog <= 16, "two slots per register");
    uint32_t hs2[kThinReg];
#pragma unroll
    for (int t = 0; t < kThinReg; t++) {
        const long i = threadIdx.x + (long)t * kLargeThreads;
        hs2[t] = 0;
        if (i < n) {
            const mtb_match m = in.full((uint32_t)i);
            hs2[t] = pairSlot(m) | spSlot(m) << 16;
            atomicAdd(&cnt[hs2[t] & 0xFFFFu], 1u);
        }
    }
    for (long i = threadIdx.x + (long)kThinReg * kLargeThreads; i < n; i += kLargeThreads)
        atomicAdd(&cnt[pairSlot(in.full((uint32_t)i))], 1u);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kThinReg; t++)
        if (threadIdx.x + (long)t * kLargeThreads < n && cnt[hs2[t] & 0xFFFFu] >= pm) flag[hs2[t] >> 16] = 1;
    for (long i = threadIdx.x + (long)kThinReg * kLargeThreads; i < n; i += kLargeThreads) {
        const mtb_match m = in.full((uint32_t)i);
        if (cnt[pairSlot(m)] >= pm) flag[spSlot(m)] = 1;
    }
    __syncthreads();
    // survivors, one LDS atomic per wave: staged through the (not yet written) output segment when
    // they overwrite their own input, else straight to io
    mtb_match* dst = inPlace ? stage : io;
    const int lane = threadIdx.x & 63;
    for (long i0 = 0; i0 < n; i0 += kLargeThreads) {
        const long i = i0 + threadIdx.x;
        const int t = (int)(i0 / kLargeThreads);
        mtb_match m;
        bool keep = false;
        if (i < n) {
            uint32_t h = 0;
#pragma unroll
            for (int x = 0; x < kThinReg; x++)
                if (x == t) h = hs2[x];
            if (t < kThinReg) {
                keep = flag[h >> 16] != 0;
                if (keep) m = in.full((uint32_t)i);
            } else {
                m = in.full((uint32_t)i);
                keep = flag[spSlot(m)] != 0;
            }
        }
        const unsigned long long mk = __ballot(keep);
        uint32_t at = 0;
        if (lane == 0 && mk) at = atomicAdd(&sCount, (uint32_t)__popcll(mk));
        at = __shfl(at, 0, 64);
        if (keep) dst[base + at + (uint32_t)__popcll(mk & ((1ull << lane) - 1))] = m;
    }
    __threadfence_block();
    __syncthreads();
    const uint32_t surv = sCount;
    if (inPlace)
        for (long i = threadIdx.x; i < (long)surv; i += kLargeThreads) io[base + i] = stage[base + i];
    if (threadIdx.x == 0) segLen[r] = surv;
}

__global__ void __launch_bounds__(256) k_max_seg_len(const uint32_t* __restrict__ segLen, uint32_t n,
                                                     uint32_t* __restrict__ out) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < kMaxPer; k++)
        if (max_elem(k) < n && segLen[max_elem(k)] != kSegSkip) v = max(v, segLen[max_elem(k)]);
    block_max_to(v, out);
}

// The reads of each size class above the small kernel's bound — (128, 256], (256, 512],
// (512, 2048], (2048, ...) matches — as lists, so each register / LDS sort kernel launches one block
// per read of its class instead of one per read of the batch (a read of another class exited at once
// but held the kernel's LDS while it read its bounds: ~0.7 ms per kernel over a 3.33M-pair batch).
// A block takes 1024 reads; one global atomic per class and block.
constexpr int kSizeClasses = 4;
constexpr int kSizeListReads = 1024;

__global__ void __launch_bounds__(256) k_size_lists(const uint64_t* __restrict__ mOff, const uint32_t* __restrict__ segLen,
                                                    uint32_t nReads, uint32_t maxSeg, uint32_t* __restrict__ lists,
                                                    uint32_t* __restrict__ counts) {
    __shared__ uint32_t sCnt[kSizeClasses], sBase[kSizeClasses];
    if (threadIdx.x < kSizeClasses) sCnt[threadIdx.x] = 0;
    __syncthreads();
    constexpr int kPer = kSizeListReads / 256;
    int cls[kPer];
    uint32_t at[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t r = blockIdx.x * kSizeListReads + k * 256 + threadIdx.x;
        cls[k] = -1;
        at[k] = 0;
        if (r < nReads) {
            const long n = seg_len(mOff, segLen, r);  // segments over maxSeg are another pass's (thinned first)
            cls[k] = n > (long)maxSeg ? -1 : n > kMidSeg ? 3 : n > kSmallSeg ? 2 : n > 256 ? 1 : n > 128 ? 0 : -1;
        }
        if (cls[k] >= 0) at[k] = atomicAdd(&sCnt[cls[k]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kSizeClasses)
        sBase[threadIdx.x] = sCnt[threadIdx.x] ? atomicAdd(&counts[threadIdx.x], sCnt[threadIdx.x]) : 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (cls[k] >= 0)
            lists[(uint64_t)cls[k] * nReads + sBase[cls[k]] + at[k]] = blockIdx.x * kSizeListReads + k * 256 + threadIdx.x;
}

// Sort (and, with liveCnt and no segLen, prune) the segments of the given lengths.
static hipError_t launch_sorts(const mtb_match* in, const uint64_t* mOff, uint32_t nReads, uint64_t M, mtb_match* out,
                               uint64_t* gScratch, uint32_t maxSeg, uint32_t* liveCnt, long chunk, uint32_t pm,
                               const uint32_t* segLen, hipStream_t s, const SegMatch* seg, const uint64_t* inOff,
                               uint32_t inC, int mode, uint32_t* lists) {
    k_segsort_small<<<nReads, 64, 0, s>>>(in, mOff, seg, inOff, inC, nReads, out, liveCnt, pm, segLen);
    if (maxSeg <= 128) return hipGetLastError();
    // MTB_SIZE_LISTS=0 (A/B): every bigger sort kernel over the whole batch, as before round 4
    static const bool useLists = !(getenv("MTB_SIZE_LISTS") && atoi(getenv("MTB_SIZE_LISTS")) == 0);
    if (!useLists || !lists) {
#define MTB_REGS(E, M) k_segsort_regs<E, M><<<nReads, 64, 0, s>>>(in, mOff, seg, inOff, inC, nReads, out, liveCnt, pm, segLen, nullptr)
        if (!liveCnt) mode = 3;
        if (maxSeg > 128) {
            if (mode == 1) MTB_REGS(4, 1);
            else if (mode == 0) MTB_REGS(4, 0);
            else if (mode == 3) MTB_REGS(4, 3);
            else MTB_REGS(4, 2);
        }
        if (maxSeg > 256) {
            if (mode == 1) MTB_REGS(8, 1);
            else if (mode == 0) MTB_REGS(8, 0);
            else if (mode == 3) MTB_REGS(8, 3);
            else MTB_REGS(8, 2);
        }
#undef MTB_REGS
        if (maxSeg > kSmallSeg)
            k_segsort_mid<<<nReads, kMidThreads, 0, s>>>(in, mOff, nReads, out, liveCnt, chunk, pm, segLen, seg, inOff,
                                                         inC, mode == 2 ? 1 : mode == 4 ? 2 : 0, nullptr);
        if (maxSeg > kMidSeg)
            k_segsort_large<<<nReads, kLargeThreads, 0, s>>>(in, mOff, nReads, M, out, gScratch, 0, liveCnt, chunk, pm,
                                                             segLen, mode == 2 ? 1 : mode == 4 ? 2 : 0, nullptr);
        MTB_HIP_RET(hipGetLastError());
        if (maxSeg > chunk) return launch_merge_path(in, mOff, nReads, M, out, gScratch, liveCnt, chunk, pm, segLen, s);
        return hipSuccess;
    }
    // the bigger segments' reads by size class (one host round trip for the four counts)
    // lists: kSizeClasses * nReads + kSizeClasses words of the caller's workspace
    uint32_t* dCnt = lists + (size_t)kSizeClasses * nReads;
    uint32_t cnt[kSizeClasses] = {0, 0, 0, 0};
    hipError_t e = hipMemsetAsync(dCnt, 0, sizeof(cnt), s);
    if (e == hipSuccess) {
        k_size_lists<<<(nReads + kSizeListReads - 1) / kSizeListReads, 256, 0, s>>>(mOff, segLen, nReads, maxSeg, lists, dCnt);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(cnt, dCnt, sizeof(cnt), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    const uint32_t* list4 = lists;
    const uint32_t* list8 = lists + (size_t)nReads;
    const uint32_t* listMid = lists + 2 * (size_t)nReads;
    const uint32_t* listLarge = lists + 3 * (size_t)nReads;
    // mode (MTB_PRUNE_AFTER, A/B): segsort_regs' kMode of the E 4 and E 8 register sorts (4: as 2, with
    // the compact large sort on the plain bitonic network)
    // MTB_SEGSORT_PAD=<bytes> (A/B diagnostic): unused dynamic LDS per block, to cap the waves per SIMD
    static const size_t segPad = getenv("MTB_SEGSORT_PAD") ? (size_t)atoi(getenv("MTB_SEGSORT_PAD")) : 0;
#define MTB_REGS(E, M, N, L) \
    k_segsort_regs<E, M><<<N, 64, segPad, s>>>(in, mOff, seg, inOff, inC, nReads, out, liveCnt, pm, segLen, L)
    if (!liveCnt) mode = 3;  // no pruning: the full-key sort
    if (e == hipSuccess && cnt[0]) {
        if (mode == 1) MTB_REGS(4, 1, cnt[0], list4);
        else if (mode == 0) MTB_REGS(4, 0, cnt[0], list4);
        else if (mode == 3) MTB_REGS(4, 3, cnt[0], list4);
        else MTB_REGS(4, 2, cnt[0], list4);
    }
    if (e == hipSuccess && cnt[1]) {
        if (mode == 1) MTB_REGS(8, 1, cnt[1], list8);
        else if (mode == 0) MTB_REGS(8, 0, cnt[1], list8);
        else if (mode == 3) MTB_REGS(8, 3, cnt[1], list8);
        else MTB_REGS(8, 2, cnt[1], list8);
    }
#undef MTB_REGS
    if (e == hipSuccess && cnt[2])
        k_segsort_mid<<<cnt[2], kMidThreads, 0, s>>>(in, mOff, nReads, out, liveCnt, chunk, pm, segLen, seg, inOff, inC,
                                                     mode == 2 ? 1 : mode == 4 ? 2 : 0, listMid);
    if (e == hipSuccess && cnt[3])
        k_segsort_large<<<cnt[3], kLargeThreads, 0, s>>>(in, mOff, nReads, M, out, gScratch, 0, liveCnt, chunk, pm,
                                                         segLen, mode == 2 ? 1 : mode == 4 ? 2 : 0, listLarge);
    if (e == hipSuccess) e = hipGetLastError();
    MTB_HIP_RET(e);
    if (maxSeg > chunk) return launch_merge_path(in, mOff, nReads, M, out, gScratch, liveCnt, chunk, pm, segLen, s);
    return hipSuccess;
}

hipError_t launch_segsort(const mtb_match* in, const uint64_t* mOff, uint32_t nReads, uint64_t M, mtb_match* out,
                          uint64_t* gScratch, uint32_t maxSeg, bool global, uint32_t* liveCnt, uint32_t mergeSeg,
                          uint32_t pm, hipStream_t s, const SegMatch* seg, const uint64_t* inOff, uint32_t inC,
                          uint32_t* segLen, uint32_t* maxTmp, int after, uint32_t* lists) {
    pm = max(pm, 2u);
    if (nReads == 0) return hipSuccess;
    // sparse input: the register sorts and the mid sort (segments of <= kSegSortSparse), and the
    // thinning of the bigger ones (read in their stretches, survivors compacted)
    const bool thin = liveCnt && segLen;
    if (seg && (global || (maxSeg > kSegSortSparse && !thin))) return hipErrorInvalidValue;
    const long chunk = std::max<long>(kSmallSeg, std::min<long>(mergeSeg ? mergeSeg : kBlockSeg, kBlockSeg));
    if (global) {
        k_segsort_large<<<nReads, kLargeThreads, 0, s>>>(in, mOff, nReads, M, out, gScratch, 1, liveCnt, chunk, pm,
                                                         nullptr, 0, nullptr);
        return hipGetLastError();
    }
    // segments over thinAbove matches are thinned first when pruning (most of a long read's matches
    // are dead: sorting the survivors, mostly within one 2048-entry LDS tile, beats sorting all)
    const long thinAbove = std::min<long>(chunk, kMidSeg);
    if (!liveCnt || maxSeg <= (uint32_t)thinAbove || !segLen)
        return launch_sorts(in, mOff, nReads, M, out, gScratch, maxSeg, liveCnt, chunk, pm, nullptr, s, seg, inOff, inC, after,
                            lists);
    // the others are sorted and pruned as usual; the big ones are thinned in place first
    // (k_thin_big), then sorted and pruned on their survivors
    MTB_HIP_RET(launch_sorts(in, mOff, nReads, M, out, gScratch, (uint32_t)thinAbove, liveCnt, chunk, pm, nullptr, s,
                             seg, inOff, inC, after, lists));
    mtb_match* io = const_cast<mtb_match*>(in);  // K5's input buffer: the caller's, free to overwrite
    k_thin_big<<<nReads, kLargeThreads, 0, s>>>(io, out, mOff, nReads, thinAbove, pm, segLen, seg, inOff, inC);
    MTB_HIP_RET(hipMemsetAsync(maxTmp, 0, sizeof(uint32_t), s));
    k_max_seg_len<<<max_blocks(nReads), 256, 0, s>>>(segLen, nReads, maxTmp);
    uint32_t maxSurv = 0;
    MTB_HIP_RET(hipMemcpyAsync(&maxSurv, maxTmp, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    MTB_HIP_RET(hipStreamSynchronize(s));
    if (maxSurv == 0) return hipSuccess;
    return launch_sorts(in, mOff, nReads, M, out, gScratch, maxSurv, liveCnt, chunk, pm, segLen, s, nullptr, nullptr, 0, after,
                        lists);
}

// Live matches (front-packed in each sorted segment) into one dense array: a wave per read.
__global__ void __launch_bounds__(256) k_pack_live(const mtb_match* __restrict__ in, const uint64_t* __restrict__ mOff,
                                                   const uint64_t* __restrict__ liveOff, uint32_t nReads,
                                                   mtb_match* __restrict__ out, int* __restrict__ err) {
    const uint32_t r = blockIdx.x * 4 + threadIdx.x / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (r >= nReads) return;
    const uint64_t live = liveOff[r + 1] - liveOff[r];
    // a live count above the segment, or live offsets past the matches, would be a K5 bug: never
    // copy out of bounds
    if (live > mOff[r + 1] - mOff[r] || liveOff[r + 1] > mOff[nReads]) {
        if (lane == 0) atomicExch(err, kErrLiveCount);
        return;
    }
    const uint64_t* src = reinterpret_cast<const uint64_t*>(in + mOff[r]);
    uint64_t* dst = reinterpret_cast<uint64_t*>(out + liveOff[r]);
    for (uint64_t w = lane; w < live * 3; w += 64) dst[w] = src[w];
}

void launch_pack_live(const mtb_match* in, const uint64_t* mOff, const uint64_t* liveOff, uint32_t nReads,
                      mtb_match* out, int* err, hipStream_t s) {
    if (nReads) k_pack_live<<<(nReads + 3) / 4, 256, 0, s>>>(in, mOff, liveOff, nReads, out, err);
}

__global__ void __launch_bounds__(256) k_max_seg(const uint64_t* __restrict__ off, uint32_t n, uint32_t* __restrict__ out) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < kMaxPer; k++)
        if (max_elem(k) < n) v = max(v, (uint32_t)min<uint64_t>(off[max_elem(k) + 1] - off[max_elem(k)], 0xFFFFFFFFull));
    block_max_to(v, out);
}

void launch_max_seg(const uint64_t* off, uint32_t n, uint32_t* out, hipStream_t s) {
    hipMemsetAsync(out, 0, sizeof(uint32_t), s);
    if (n) k_max_seg<<<max_blocks(n), 256, 0, s>>>(off, n, out);
}

void launch_max_u32(const uint32_t* x, uint32_t n, uint32_t* out, hipStream_t s) {
    hipMemsetAsync(out, 0, sizeof(uint32_t), s);
    if (n) k_max_u32<<<max_blocks(n), 256, 0, s>>>(x, n, out);
}

struct TaxView {
    const int32_t* nodeOf;    // taxID -> node index, -1 if absent (D array)
    const int32_t* nodeTax;   // node -> taxID
    const int32_t* parent;    // node -> parent node
    const int32_t* depth;     // node -> depth below taxID 1
    const uint8_t* flags;     // bit0: IsAncestor(Eukaryota, taxID); bit1: rank "" or "accession"
    const int32_t* spParent;  // node -> parentTaxId of taxonNode(getTaxIdAtRank(taxID, "species"))
    int32_t maxTax;
    __device__ bool exists(int32_t t) const { return t >= 0 && t <= maxTax && nodeOf[t] >= 0; }
    // NcbiTaxonomy::lcaHelper on node indices: node 0 short-circuits, otherwise the tree LCA.
    __device__ int lca_node(int i, int j) const {
        if (i == 0 || j == 0) return 0;
        while (i != j) {
            int di = depth[i], dj = depth[j];
            if (di >= dj) i = parent[i];
            if (dj >= di) j = parent[j];
        }
        return i;
    }
    __device__ int32_t lca(int32_t a, int32_t b) const {  // NcbiTaxonomy::LCA(TaxID, TaxID)
        if (!exists(a)) return b;
        if (!exists(b)) return a;
        return nodeTax[lca_node(nodeOf[a], nodeOf[b])];
    }
};

struct AssignCfg {
    int kmerFormat, dnaShift, maxCodonShift, denominator, minConsCnt, minConsCntEuk, accessionLevel;
    float minScore, minSpScore, tieRatio;
    int generic;  // 1: skip the register fast path (tests)
    int emulateAll;  // 1: k_combine_wave takes the std::sort emulation for every run (tests)
    int em;          // --em: a classified read keeps its best species (Taxonomer.cpp:193-201)
};

struct Clade {
    int32_t tax, parentTax;
    uint32_t count;
    int32_t removed;
};


// ------------------------------------------------------------------------------------------------
// K6 as three kernels over the sorted match array. Work items are the runs the reference loops
// over (Taxonomer.cpp:316-408): (read, species, frame) groups for getMatchPaths, (read, species)
// runs for combineMatchPaths, reads for chooseBestTaxon onward. Neighbouring lanes take
// neighbouring runs, so a wave's loads and scratch writes fall in one contiguous stretch of the
// match array instead of 64 unrelated per-read segments.
// ------------------------------------------------------------------------------------------------

// Run boundaries (group and species-run starts, their exclusive counts): launch_run_index,
// mtb_kernels.hip.

// Work list for k_match_paths: the groups that can emit a path (>= prune_min_matches matches: a
// single match is never searched, and fewer matches cannot chain MIN_DEPTH codons) in batch order,
// so a wave's lanes still walk neighbouring groups (ordering them by size instead was slower: the
// lost locality costs more than the divergence it removes). The others get the sentinel key and
// zero paths; one stable radix pass on an all-zero digit compacts the rest.
__global__ void k_group_keys(const uint64_t* __restrict__ gStart, uint64_t nG, uint64_t* __restrict__ keys,
                             uint64_t* __restrict__ vals, uint32_t* __restrict__ pathCnt, uint32_t minGroup) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nG) return;
    const uint64_t n = gStart[g + 1] - gStart[g];
    if (n < minGroup) {  // too few matches to chain a path of MIN_DEPTH (prune_min_matches): no paths
        pathCnt[g] = 0;
        keys[g] = kSentinel;
    } else {
        keys[g] = g;
    }
    vals[g] = 0;
}


// getMatchPaths with the DP state in registers: only the current and the next position group are
// live, and both are almost always small (one DB k-mer per strain at a position). Returns false,
// having written nothing that counts, if a position group holds more than kRegPos matches; the
// caller then reruns the group through the general version.
constexpr int kRegPos = 4;
constexpr uint64_t kBigGroup = 256;  // groups of at least this many matches: k_match_paths_wave

// The fields getMatchPaths reads of match k: from the match array, or from a wave's LDS copy of
// its groups' span (k_match_paths: one coalesced load of the span instead of per-lane record loads).
struct GlobalRecs {
    const mtb_match* __restrict__ M;
    __device__ __forceinline__ uint32_t pos(uint64_t k) const { return info_pos(M[k].qinfo); }
    __device__ __forceinline__ uint32_t dna(uint64_t k) const { return M[k].dna_encoding; }
    __device__ __forceinline__ uint32_t reh(uint64_t k) const { return M[k].right_end_hamming; }
    __device__ __forceinline__ uint32_t ham(uint64_t k) const { return M[k].hamming; }
};
struct LdsRecs {
    const uint32_t* p;   // pos
    const uint32_t* dh;  // dna | hamming << 24
    const uint16_t* rh;  // rightEndHamming
    uint64_t base;       // match index of entry 0
    __device__ __forceinline__ uint32_t pos(uint64_t k) const { return p[k - base]; }
    __device__ __forceinline__ uint32_t dna(uint64_t k) const { return dh[k - base] & 0xFFFFFFu; }
    __device__ __forceinline__ uint32_t reh(uint64_t k) const { return rh[k - base]; }
    __device__ __forceinline__ uint32_t ham(uint64_t k) const { return dh[k - base] >> 24; }
};

template <typename R>
__device__ __forceinline__ bool match_paths_regs(const R& M, uint64_t start, uint64_t end,
                                                 const AssignCfg& cfg, int minDepth, bool fwd,
                                                 Path* __restrict__ P, uint64_t& nPout, bool emitLone = false) {
    Path cp[kRegPos], np[kRegPos];
    uint32_t cd[kRegPos], nd[kRegPos], nr[kRegPos];
    bool cc[kRegPos];
    int nc = 0, nn = 0;
    uint64_t nP = start;
    uint64_t k = start;
    uint32_t currPos = M.pos(k);
    // first position group
    while (k < end) {
        if (M.pos(k) != currPos) break;
        if (nc == kRegPos) return false;
        const uint32_t mreh = M.reh(k), mham = M.ham(k), mdna = M.dna(k);
#pragma unroll
        for (int x = 0; x < kRegPos; x++)
            if (x == nc) {
                cp[x].start = (int)currPos;
                cp[x].end = (int)currPos + 23;
                cp[x].score = score_fields(mreh, 8, false);
                cp[x].hd = (int)mham;
                cp[x].depth = 1;
                cp[x].sm = cp[x].em = (uint32_t)k;
                cd[x] = mdna;
                cc[x] = false;
            }
        nc++;
        k++;
    }
    const bool stepped = k < end;  // a next position group follows (emitLone: see match_paths_serial)
    while (k < end) {
        const uint32_t nextPos = M.pos(k);
        nn = 0;
        while (k < end) {
            if (M.pos(k) != nextPos) break;
            if (nn == kRegPos) return false;
            const uint32_t mreh = M.reh(k), mham = M.ham(k), mdna = M.dna(k);
#pragma unroll
            for (int x = 0; x < kRegPos; x++)
                if (x == nn) {
                    np[x].start = (int)nextPos;
                    np[x].end = (int)nextPos + 23;
                    np[x].score = score_fields(mreh, 8, false);
                    np[x].hd = (int)mham;
                    np[x].depth = 1;
                    np[x].sm = np[x].em = (uint32_t)k;
                    nd[x] = mdna;
                    nr[x] = mreh;
                }
            nn++;
            k++;
        }
        const int shift = (int)((nextPos - currPos) / 3);
        if (shift > 0 && shift <= cfg.maxCodonShift) {
            const uint32_t sh = kBitsPerCodon * (uint32_t)shift;
            const uint32_t lowMask = (1u << (kTotalDnaBits - sh)) - 1u;
#pragma unroll
            for (int x = 0; x < kRegPos; x++) {
                if (x >= nn) continue;
                const float inc = score_fields(nr[x], shift, false);  // calScoreIncrement
                const int hinc = ham_fields(nr[x], shift, false);     // calHammingDistIncrement
                bool found = false;
                float bestScore = 0.0f;
                Path bp{};
#pragma unroll
                for (int y = 0; y < kRegPos; y++) {
                    if (y >= nc) continue;
                    if (consecutive(cd[y], nd[x], sh, lowMask, fwd, cfg.kmerFormat)) {
                        cc[y] = true;
                        if (cp[y].score > bestScore) { found = true; bestScore = cp[y].score; bp = cp[y]; }
                    }
                }
                if (found) {
                    np[x].start = bp.start;
                    np[x].score = bp.score + inc;
                    np[x].hd = bp.hd + hinc;
                    np[x].depth = bp.depth + shift;
                    np[x].sm = bp.sm;
                }
            }
        }
#pragma unroll
        for (int y = 0; y < kRegPos; y++)
            if (y < nc && !cc[y] && cp[y].depth >= minDepth) P[nP++] = cp[y];
        if (k == end) {
#pragma unroll
            for (int x = 0; x < kRegPos; x++)
                if (x < nn && np[x].depth >= minDepth) P[nP++] = np[x];
        }
#pragma unroll
        for (int x = 0; x < kRegPos; x++) {
            cp[x] = np[x];
            cd[x] = nd[x];
            cc[x] = false;
        }
        nc = nn;
        currPos = nextPos;
    }
    if (!stepped && emitLone)
#pragma unroll
        for (int y = 0; y < kRegPos; y++)
            if (y < nc && cp[y].depth >= minDepth) P[nP++] = cp[y];
    nPout = nP;
    return true;
}

// getMatchPaths' loop (Taxonomer.cpp:487-648) over the matches [start, end) of one (species,
// frame) group, DP state in L / conn (indexed by match); paths to P from index start in emission
// order; returns the end of the emitted paths. emitLone: [start, end) is a stretch of a larger group
// that ends at a break (the next position is not within maxCodonShift codons): a stretch of a
// single position group emits its paths too, as the whole group's loop would when it moves past it.
template <typename R>
__device__ uint64_t match_paths_serial(const R& M, uint64_t start, uint64_t end,
                                       const AssignCfg& cfg, int minDepth, bool fwd, Path* __restrict__ L,
                                       Path* __restrict__ P, uint8_t* __restrict__ conn, bool emitLone) {
    for (uint64_t x = start; x < end; x++) conn[x] = 0;
    uint64_t nP = start;
    uint64_t k = start;
    uint64_t currPos = M.pos(start);
    bool stepped = false;  // a next position group was processed
    auto initPath = [&](uint64_t idx) {
        Path p;
        p.start = (int)M.pos(idx);
        p.end = p.start + 23;
        p.score = score_fields(M.reh(idx), 8, false);
        p.hd = (int)M.ham(idx);
        p.depth = 1;
        p.sm = p.em = (uint32_t)idx;
        L[idx] = p;
    };
    uint64_t curS = k;
    while (k < end && M.pos(k) == currPos) { initPath(k); ++k; }
    uint64_t curE = k;
    while (k < end) {
        const uint32_t nextPos = M.pos(k);
        const uint64_t nxS = k;
        while (k < end && M.pos(k) == nextPos) { initPath(k); ++k; }
        const uint64_t nxE = k;
        stepped = true;
        const int shift = (int)(((uint64_t)nextPos - currPos) / 3);
        if (shift > 0 && shift <= cfg.maxCodonShift) {
            const uint32_t sh = kBitsPerCodon * (uint32_t)shift;
            const uint32_t lowMask = (1u << (kTotalDnaBits - sh)) - 1u;
            for (uint64_t nx = nxS; nx < nxE; nx++) {
                const uint32_t nreh = M.reh(nx);
                const float inc = score_fields(nreh, shift, false);  // calScoreIncrement
                const int hinc = ham_fields(nreh, shift, false);     // calHammingDistIncrement
                int64_t best = -1;
                float bestScore = 0.0f;
                const uint32_t dn = M.dna(nx);
                for (uint64_t cu = curS; cu < curE; cu++) {
                    const uint32_t dc = M.dna(cu);
                    if (consecutive(dc, dn, sh, lowMask, fwd, cfg.kmerFormat)) {
                        conn[cu] = 1;
                        if (L[cu].score > bestScore) { best = (int64_t)cu; bestScore = L[cu].score; }
                    }
                }
                if (best >= 0) {
                    const Path bp = L[best];
                    Path& np = L[nx];
                    np.start = bp.start;
                    np.score = bp.score + inc;
                    np.hd = bp.hd + hinc;
                    np.depth = bp.depth + shift;
                    np.sm = bp.sm;
                }
            }
        }
        for (uint64_t cu = curS; cu < curE; cu++)
            if (!conn[cu] && L[cu].depth >= minDepth) P[nP++] = L[cu];
        if (k == end)
            for (uint64_t nx = nxS; nx < nxE; nx++)
                if (L[nx].depth >= minDepth) P[nP++] = L[nx];
        curS = nxS;
        curE = nxE;
        currPos = nextPos;
    }
    if (!stepped && emitLone)
        for (uint64_t cu = start; cu < end; cu++)
            if (L[cu].depth >= minDepth) P[nP++] = L[cu];
    return nP;
}

// getMatchPaths (Taxonomer.cpp:487-648) on one (read, species, frame) group [gs, ge). Paths go to
// P[gs + k] in emission order; L and conn are indexed by match.
template <typename R>
__device__ __forceinline__ void match_paths_group(const R& recs, const mtb_match* __restrict__ M, uint64_t g,
                                                  uint64_t start, uint64_t end, const AssignCfg& cfg,
                                                  const TaxView& tax, Path* __restrict__ L, Path* __restrict__ P,
                                                  uint8_t* __restrict__ conn, uint32_t* __restrict__ pathCnt) {
    const int32_t sp = (int32_t)M[start].species_id;
    const uint32_t curFrame = info_frame(M[start].qinfo);
    int minDepth = cfg.minConsCnt;
    if (tax.exists(sp) && (tax.flags[tax.nodeOf[sp]] & 1u)) minDepth = cfg.minConsCntEuk;
    const bool fwd = curFrame < 3;
    {
        uint64_t nPr = start;
        if (!cfg.generic && match_paths_regs(recs, start, end, cfg, minDepth, fwd, P, nPr)) {
            pathCnt[g] = (uint32_t)(nPr - start);
            return;
        }
    }
    const uint64_t nP = match_paths_serial(recs, start, end, cfg, minDepth, fwd, L, P, conn, false);
    pathCnt[g] = (uint32_t)(nP - start);
}

// A wave per 64 work items (groups in batch order, so their matches form one stretch of the array):
// the stretch's pos / dna / hamming / rightEndHamming are staged in LDS with coalesced loads (the
// groups' own loads would be 64 scattered lines per instruction), unless it is longer than
// kPathStage matches.
constexpr int kPathStage = 1024;

// kLds = false (MTB_PATHS_NOLDS=1, A/B): no stage at all — at GTDB scale a wave's span of groups
// rarely fits one (~2,200 matches) — so neither the 10-KB stage nor the register budget holds the
// kernel at 4 waves per SIMD (kW: the waves the registers are held to)
template <bool kLds, int kW>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kW))) k_match_paths(const mtb_match* __restrict__ M, const uint64_t* __restrict__ gStart,
                                                    const uint64_t* __restrict__ order, uint64_t nWork, AssignCfg cfg,
                                                    TaxView tax, Path* __restrict__ L, Path* __restrict__ P,
                                                    uint8_t* __restrict__ conn, uint32_t* __restrict__ pathCnt,
                                                    uint64_t* __restrict__ bigList, uint32_t* __restrict__ bigCount) {
    __shared__ uint32_t sPos[kLds ? kPathStage : 1], sDh[kLds ? kPathStage : 1];
    __shared__ uint16_t sReh[kLds ? kPathStage : 1];
    const uint64_t w0 = (uint64_t)blockIdx.x * 64;
    const uint64_t i = w0 + threadIdx.x;
    const uint64_t wLast = min(w0 + 63, nWork - 1);
    const uint64_t spanLo = kLds ? gStart[(uint32_t)order[w0]] : 0, spanHi = kLds ? gStart[(uint32_t)order[wLast] + 1] : 0;
    const bool staged = kLds && spanHi - spanLo <= (uint64_t)kPathStage;
    if (staged) {
        for (uint64_t k = spanLo + threadIdx.x; k < spanHi; k += 64) {
            const mtb_match m = M[k];
            sPos[k - spanLo] = info_pos(m.qinfo);
            sDh[k - spanLo] = (m.dna_encoding & 0xFFFFFFu) | ((uint32_t)m.hamming << 24);
            sReh[k - spanLo] = m.right_end_hamming;
        }
        __syncthreads();
    }
    if (i >= nWork) return;
    const uint64_t g = (uint32_t)order[i];
    const uint64_t start = gStart[g], end = gStart[g + 1];
    if (bigList && end - start >= kBigGroup) {  // k_match_paths_wave takes it
        bigList[atomicAdd(bigCount, 1u)] = g;
        return;
    }
    if (staged)
        match_paths_group(LdsRecs{sPos, sDh, sReh, spanLo}, M, g, start, end, cfg, tax, L, P, conn, pathCnt);
    else
        match_paths_group(GlobalRecs{M}, M, g, start, end, cfg, tax, L, P, conn, pathCnt);
}

// A group of >= kBigGroup matches (long reads) with a wave: each lane takes a stretch of ~n/64
// matches widened to whole break-delimited stretches (a break: the next position is not within
// maxCodonShift codons, so no path crosses it and the serial loop's state restarts there), runs the
// serial loop on it with its paths to P at the stretch's own offset, and the stretches' paths are
// then packed in lane order (= the serial emission order) through L.
__device__ __forceinline__ bool group_break(const mtb_match* __restrict__ M, uint64_t start, uint64_t i,
                                            int maxCodonShift) {
    if (i == start) return true;
    const uint32_t p = info_pos(M[i].qinfo), pp = info_pos(M[i - 1].qinfo);
    if (p == pp) return false;
    const int shift = (int)((p - pp) / 3);
    return !(shift > 0 && shift <= maxCodonShift);
}

__global__ void __launch_bounds__(64) k_match_paths_wave(const mtb_match* __restrict__ M,
                                                         const uint64_t* __restrict__ gStart,
                                                         const uint64_t* __restrict__ bigList, AssignCfg cfg,
                                                         TaxView tax, Path* __restrict__ L, Path* __restrict__ P,
                                                         uint8_t* __restrict__ conn, uint32_t* __restrict__ pathCnt) {
    const uint64_t g = bigList[blockIdx.x];
    const int lane = threadIdx.x;
    const uint64_t start = gStart[g], end = gStart[g + 1], n = end - start;
    const int32_t sp = (int32_t)M[start].species_id;
    int minDepth = cfg.minConsCnt;
    if (tax.exists(sp) && (tax.flags[tax.nodeOf[sp]] & 1u)) minDepth = cfg.minConsCntEuk;
    const bool fwd = info_frame(M[start].qinfo) < 3;
    const bool multi = info_pos(M[start].qinfo) != info_pos(M[end - 1].qinfo);
    // this lane's stretch: from the first break at or after its nominal start
    uint64_t a = start + n * (uint64_t)lane / 64;
    while (a < end && !group_break(M, start, a, cfg.maxCodonShift)) a++;
    uint64_t b = __shfl_down(a, 1, 64);
    if (lane == 63) b = end;
    if (b < a) b = a;
    uint64_t cnt = 0;
    if (a < b) {  // the register DP when no position of the stretch holds more than kRegPos matches
        uint64_t nPr = a;
        if (!cfg.generic && match_paths_regs(GlobalRecs{M}, a, b, cfg, minDepth, fwd, P, nPr, multi)) cnt = nPr - a;
        else cnt = match_paths_serial(GlobalRecs{M}, a, b, cfg, minDepth, fwd, L, P, conn, multi) - a;
    }
    // exclusive scan of the counts over the lanes
    uint64_t inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    const uint64_t off = inc - cnt, total = __shfl(inc, 63, 64);
    __syncthreads();  // every stretch's DP done: L is free
    for (uint64_t k = 0; k < cnt; k++) L[start + off + k] = P[a + k];
    __syncthreads();
    for (uint64_t k = lane; k < total; k += 64) P[start + k] = L[start + k];
    if (lane == 0) pathCnt[g] = (uint32_t)total;
}

// trimMatchPath (Taxonomer.cpp:475-485): p overlaps c by ol < 24 bases at one end
__device__ __forceinline__ void trim_path(const mtb_match* __restrict__ M, Path& p, const Path& c, int ol) {
    const int range = ol / 3;
    if (p.start < c.start) {
        const uint32_t reh = M[p.em].right_end_hamming;
        p.end = c.start - 1;
        p.hd = max(0, p.hd - ham_fields(reh, range, false));
        p.score = p.score - score_fields(reh, range, false) - (float)(ol % 3);
    } else {
        const uint32_t reh = M[p.sm].right_end_hamming;
        p.start = c.end + 1;
        p.hd = max(0, p.hd - ham_fields(reh, range, true));
        p.score = p.score - score_fields(reh, range, true) - (float)(ol % 3);
    }
}

// trim_path with the end matches' rightEndHamming already at hand (rehS: p.sm's, rehE: p.em's)
__device__ __forceinline__ void trim_path_reh(Path& p, const Path& c, int ol, uint32_t rehS, uint32_t rehE) {
    const int range = ol / 3;
    if (p.start < c.start) {
        p.end = c.start - 1;
        p.hd = max(0, p.hd - ham_fields(rehE, range, false));
        p.score = p.score - score_fields(rehE, range, false) - (float)(ol % 3);
    } else {
        p.start = c.end + 1;
        p.hd = max(0, p.hd - ham_fields(rehS, range, true));
        p.score = p.score - score_fields(rehS, range, true) - (float)(ol % 3);
    }
}

// combineMatchPaths (Taxonomer.cpp:410-468) on nP packed paths in global memory: the libstdc++
// introsort emulation, then the greedy overlap pass. Returns the summed score.
__device__ float combine_serial(const mtb_match* __restrict__ M, Path* Ps, long nP, Path* Cs) {
    stdsort::sort(Ps, Ps + nP, [](const Path& a, const Path& b) {
        if (a.score != b.score) return a.score > b.score;
        if (a.hd != b.hd) return a.hd < b.hd;
        return a.start > b.start;
    });
    long nC = 0;
    float score = 0.0f;
    for (long pi = 0; pi < nP; pi++) {
        if (nC == 0) {
            Cs[nC++] = Ps[pi];
            score += Ps[pi].score;
            continue;
        }
        bool overlapped = false;
        for (long j = 0; j < nC; j++) {
            Path& p = Ps[pi];
            const Path c = Cs[j];
            if ((p.end < c.start) || (c.end < p.start)) continue;
            const int ol = min(p.end, c.end) - max(p.start, c.start) + 1;
            if (ol == p.end - p.start + 1) { overlapped = true; break; }
            if (ol < 24) {
                trim_path(M, p, c, ol);
                continue;
            }
            overlapped = true;
            break;
        }
        if (!overlapped) {
            Cs[nC++] = Ps[pi];
            score += Ps[pi].score;
        }
    }
    return score;
}

__device__ __forceinline__ void species_score(float score, int readLength, const AssignCfg& cfg, float* spScore,
                                              uint8_t* spKeep, uint64_t s) {
    score = score / (float)readLength;
    score = (1.0f < score) ? 1.0f : score;  // std::min(score, 1.0f)
    spScore[s] = score;
    spKeep[s] = !(score < cfg.minScore);
}

// The species score (:380-395) for one (read, species) run [ss, se): its groups' paths are packed
// in frame order (the order the reference appends them) and combined. Runs of more than
// kWaveCombineMin paths (long reads) are queued for k_combine_wave instead.
constexpr int kWaveCombineMin = 24;
constexpr int kWaveCombineMax = 1024;

__global__ void __launch_bounds__(256) k_combine_paths(const mtb_match* __restrict__ M, const uint64_t* __restrict__ sStart,
                                                       uint64_t nS, const uint64_t* __restrict__ gScan,
                                                       const uint64_t* __restrict__ gStart,
                                                       const uint32_t* __restrict__ pathCnt,
                                                       const uint32_t* __restrict__ qlen, AssignCfg cfg,
                                                       Path* __restrict__ P, Path* __restrict__ C,
                                                       float* __restrict__ spScore, uint8_t* __restrict__ spKeep,
                                                       uint64_t* __restrict__ waveList, uint32_t* __restrict__ waveCount) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nS) return;
    const uint64_t ss = sStart[s], se = sStart[s + 1];
    uint64_t w = ss;
    for (uint64_t g = gScan[ss]; gStart[g] < se; g++) {
        const uint64_t src = gStart[g];
        const uint32_t cnt = pathCnt[g];
        if (src != w)
            for (uint32_t k = 0; k < cnt; k++) P[w + k] = P[src + k];
        w += cnt;
    }
    if (w == ss) { spKeep[s] = 0; return; }
    const long nP = (long)(w - ss);
    if (!cfg.generic && nP > kWaveCombineMin && nP <= kWaveCombineMax) {
        waveList[atomicAdd(waveCount, 1u)] = ((uint64_t)nP << 32) | s;
        return;
    }
    const int readLength = (int)qlen[info_seq(M[ss].qinfo) - 1];
    species_score(combine_serial(M, P + ss, nP, C + ss), readLength, cfg, spScore, spKeep, s);
}

// One wave per queued run (list entry = nP << 32 | run; its nP paths are packed at P[ss..]). The
// paths are sorted in LDS by (score desc, hd asc, start desc): any correct sort places distinct
// keys the same way, and tied paths only need std::sort's exact order (the introsort emulation,
// combine_serial on lane 0) when they differ in a field the greedy pass reads. The greedy pass finds the first combined path a candidate
// overlaps with one ballot per 64 entries, and searches on from there after a trim.
__global__ void __launch_bounds__(64) k_combine_wave(const mtb_match* __restrict__ M, const uint64_t* __restrict__ sStart,
                                                     const uint64_t* __restrict__ waveList,
                                                     const uint32_t* __restrict__ qlen, AssignCfg cfg,
                                                     Path* __restrict__ P, Path* __restrict__ C,
                                                     float* __restrict__ spScore, uint8_t* __restrict__ spKeep,
                                                     unsigned long long* __restrict__ stats,
                                                     const uint64_t* __restrict__ order) {
    __shared__ uint64_t kbuf[2 * kWaveCombineMax];  // sort keys (kh, kl), or the emulation's compact keys
    uint64_t* kh = kbuf;
    uint64_t* kl = kbuf + kWaveCombineMax;
    // rightEndHamming of each sorted path's start / end match: a trim reads one (trimMatchPath), and
    // a dependent global load per trim in the serial greedy pass would cost ~1 us each
    __shared__ uint16_t qrs[kWaveCombineMax], qre[kWaveCombineMax];
    const uint64_t e = waveList[order ? order[blockIdx.x] : blockIdx.x];  // largest runs first
    const uint64_t s = (uint32_t)e;
    const int nP = (int)(e >> 32);
    const uint64_t ss = sStart[s];
    const Path* Ps = P + ss;
    const int lane = threadIdx.x;
    const int readLength = (int)qlen[info_seq(M[ss].qinfo) - 1];
    int p2 = 2;
    while (p2 < nP) p2 <<= 1;
    for (int i = lane; i < p2; i += 64) {
        if (i < nP) {
            const Path p = Ps[i];
            kh[i] = ((uint64_t)(~__float_as_uint(p.score)) << 32) | (uint32_t)p.hd;
            kl[i] = ((uint64_t)(~(uint32_t)p.start) << 32) | (uint32_t)i;
        } else {
            kh[i] = ~0ull;
            kl[i] = ~0ull;
        }
    }
    __syncthreads();
    for (int k = 2; k <= p2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = lane; t < (p2 >> 1); t += 64) {
                const int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                const int ixj = i + j;
                const bool up = (i & k) == 0;
                const uint64_t ah = kh[i], al = kl[i], bh = kh[ixj], bl = kl[ixj];
                if (key_gt(ah, al, bh, bl) == up) {
                    kh[i] = bh; kl[i] = bl; kh[ixj] = ah; kl[ixj] = al;
                }
            }
            __syncthreads();
        }
    }
    // A tie on the comparator's key only matters if the tied paths can act differently in the
    // greedy pass, which reads start, end, score and, when trimming, the end matches' hamming
    // fields; tied paths equal in all of those are interchangeable in any order.
    bool tie = false;
    for (int i = lane; i + 1 < nP; i += 64) {
        if (kh[i] != kh[i + 1] || (kl[i] >> 32) != (kl[i + 1] >> 32)) continue;
        const Path a = Ps[(uint32_t)kl[i]], b = Ps[(uint32_t)kl[i + 1]];
        tie |= a.end != b.end || M[a.sm].right_end_hamming != M[b.sm].right_end_hamming ||
               M[a.em].right_end_hamming != M[b.em].right_end_hamming;
    }
    // The order of tied paths is whatever libstdc++'s introsort leaves: emulated (mtb_stdsort.h) on
    // lane 0 over compact keys in LDS, from the paths' original order, in place of the bitonic
    // result; the greedy pass below is the same either way.
    struct EmuKey {
        float score;
        int hd, start;
        uint32_t idx;
    };
    static_assert(sizeof(EmuKey) * kWaveCombineMax == sizeof(uint64_t) * 2 * kWaveCombineMax, "emulation keys fit");
    EmuKey* K = reinterpret_cast<EmuKey*>(kbuf);
    const bool emulate = __syncthreads_or(tie || cfg.emulateAll);
    if (emulate) {
        if (lane == 0) atomicAdd(&stats[1], 1ull);
        for (int i = lane; i < nP; i += 64) {
            const Path q = Ps[i];
            K[i] = EmuKey{q.score, q.hd, q.start, (uint32_t)i};
        }
        __syncthreads();
        if (lane == 0)
            stdsort::sort(K, K + nP, [](const EmuKey& a, const EmuKey& b) {
                if (a.score != b.score) return a.score > b.score;
                if (a.hd != b.hd) return a.hd < b.hd;
                return a.start > b.start;
            });
        __syncthreads();
    }
    // the paths themselves, in sorted order, into LDS (over the dead key arrays, plus the end
    // matches' rightEndHamming) so the sequential pass below reads no global memory
    constexpr int kPerLane = kWaveCombineMax / 64;
    uint32_t src[kPerLane];
#pragma unroll
    for (int t = 0; t < kPerLane; t++) {
        const int i = lane + 64 * t;
        src[t] = i < nP ? (emulate ? K[i].idx : (uint32_t)kl[i]) : 0u;
    }
    __syncthreads();
    int* qs = reinterpret_cast<int*>(kh);
    int* qe = qs + kWaveCombineMax;
    float* qsc = reinterpret_cast<float*>(kl);
    int* qhd = reinterpret_cast<int*>(kl) + kWaveCombineMax;
#pragma unroll
    for (int t = 0; t < kPerLane; t++) {
        const int i = lane + 64 * t;
        if (i < nP) {
            const Path q = Ps[src[t]];
            qs[i] = q.start; qe[i] = q.end; qsc[i] = q.score; qhd[i] = q.hd;
            qrs[i] = M[q.sm].right_end_hamming;
            qre[i] = M[q.em].right_end_hamming;
        }
    }
    __syncthreads();
    // Combined paths are pairwise disjoint (a kept path overlaps none of them), so the entries a
    // candidate touches are found with one pass over the lane-distributed interval registers
    // (entry j in slot j / 64 of lane j % 64) and then visited in insertion order, re-checked
    // against the candidate as trims shrink it.
    constexpr int kSlots = kWaveCombineMax / 64;
    int rs[kSlots], re[kSlots];
#pragma unroll
    for (int t = 0; t < kSlots; t++) { rs[t] = 0; re[t] = -1; }
    float score = 0.0f;
    int nC = 0;
    for (int pi = 0; pi < nP; pi++) {
        Path p;  // wave-uniform
        p.start = qs[pi]; p.end = qe[pi]; p.score = qsc[pi]; p.hd = qhd[pi]; p.sm = 0; p.em = 0;
        const uint32_t rehS = qrs[pi], rehE = qre[pi];
        p.depth = 0;
        bool keep = true;
#pragma unroll
        for (int t = 0; t < kSlots; t++) {
            if (!keep || 64 * t >= nC) break;
            unsigned long long m = __ballot(64 * t + lane < nC && !(p.end < rs[t] || re[t] < p.start));
            while (keep && m) {
                const int l = __ffsll((long long)m) - 1;
                m &= m - 1;
                Path c;
                c.start = __shfl(rs[t], l, 64);
                c.end = __shfl(re[t], l, 64);
                if ((p.end < c.start) || (c.end < p.start)) continue;  // cleared by an earlier trim
                const int ol = min(p.end, c.end) - max(p.start, c.start) + 1;
                if (ol == p.end - p.start + 1) { keep = false; break; }
                if (ol < 24) { trim_path_reh(p, c, ol, rehS, rehE); continue; }
                keep = false;
            }
        }
        if (keep) {
#pragma unroll
            for (int t = 0; t < kSlots; t++)
                if (t == (nC >> 6) && lane == (nC & 63)) { rs[t] = p.start; re[t] = p.end; }
            nC++;
            score += p.score;
        }
    }
    if (lane == 0) species_score(score, readLength, cfg, spScore, spKeep, s);
}

// filterRedundantMatches (Taxonomer.cpp:205-241) for the best species' matches B[0, nb), serially.
// Per quotient q = pos / dnaShift: the best (lowest hamming) match's taxon, ties folded with LCA —
// an order-free reduction. Within the best species the matches are sorted by frame, then position,
// so each frame's quotients ascend: a <= 6-way merge over the frame runs visits each quotient once,
// in order, with no per-read quotient table. taxCnt goes to tc (capacity >= nb) in std::map order
// (ascending taxID); returns its length.
__device__ long filter_redundant_serial(const mtb_match* __restrict__ M, uint64_t bestFirst, uint64_t bestSecond,
                                        const uint64_t* __restrict__ gScan, const uint64_t* __restrict__ gStart,
                                        uint32_t dnaShift, const TaxView& tax, mtb_taxcnt* __restrict__ tc) {
    uint32_t fc[6], fin[6], head[6];
    const mtb_match* B = M + bestFirst;
    int nf = 0;
    for (uint64_t g = gScan[bestFirst]; nf < 6 && gStart[g] < bestSecond; g++) {
        fc[nf] = (uint32_t)(gStart[g] - bestFirst);
        fin[nf] = (uint32_t)(gStart[g + 1] - bestFirst);
        nf++;
    }
#pragma unroll
    for (int f = 0; f < 6; f++) head[f] = (f < nf) ? info_pos(B[fc[f]].qinfo) / dnaShift : 0xFFFFFFFFu;
    // taxCnt: the first distinct taxa stay in registers, the rest (rare) in the read's pool slice
    constexpr int kRegTc = 4;
    int32_t rt[kRegTc];
    uint32_t rc[kRegTc];
    long nTc = 0;
    while (true) {
        uint32_t qmin = 0xFFFFFFFFu;
#pragma unroll
        for (int f = 0; f < 6; f++) qmin = min(qmin, head[f]);
        if (qmin == 0xFFFFFFFFu) break;
        uint32_t minH = 256;
        int32_t t = 0;
#pragma unroll
        for (int f = 0; f < 6; f++) {
            while (head[f] == qmin) {
                const mtb_match& x = B[fc[f]];
                const uint32_t h = x.hamming;
                if (h < minH) { minH = h; t = (int32_t)x.target_id; }
                else if (h == minH) t = tax.lca(t, (int32_t)x.target_id);
                fc[f]++;
                head[f] = fc[f] < fin[f] ? info_pos(B[fc[f]].qinfo) / dnaShift : 0xFFFFFFFFu;
            }
        }
        long e = -1;
#pragma unroll
        for (int k = 0; k < kRegTc; k++)
            if (k < nTc && rt[k] == t) e = k;
        if (e >= 0) {
#pragma unroll
            for (int k = 0; k < kRegTc; k++)
                if (k == e) rc[k]++;
            continue;
        }
        if (nTc < kRegTc) {
#pragma unroll
            for (int k = 0; k < kRegTc; k++)
                if (k == nTc) { rt[k] = t; rc[k] = 1; }
            nTc++;
            continue;
        }
        e = kRegTc;
        while (e < nTc && tc[e].tax_id != t) e++;
        if (e == nTc) { tc[nTc].tax_id = t; tc[nTc].count = 0; nTc++; }
        tc[e].count++;
    }
#pragma unroll
    for (int k = 0; k < kRegTc; k++)
        if (k < nTc) { tc[k].tax_id = rt[k]; tc[k].count = rc[k]; }
    for (long a = 1; a < nTc; a++) {  // std::map order
        mtb_taxcnt v = tc[a];
        long b = a;
        while (b > 0 && tc[b - 1].tax_id > v.tax_id) { tc[b] = tc[b - 1]; b--; }
        tc[b] = v;
    }
    return nTc;
}

// chooseBestTaxon after filterRedundantMatches (Taxonomer.cpp:175-201): the parent of the species
// below minSpScore, else lowerRankClassification / getSpeciesCladeCounts / BFS (:252-314) over the
// taxCnt list tc[0, nTc). cl: the read's clade scratch (clCap entries).
__device__ void classify_tail(mtb_result& res, const mtb_taxcnt* __restrict__ tc, long nTc, float spTotal,
                              int32_t bestTax, int readLength, const AssignCfg& cfg, const TaxView& tax,
                              Clade* __restrict__ cl, long clCap) {
    res.taxcnt_offset = (uint32_t)0;
    res.taxcnt_len = (uint32_t)nTc;
    res.is_classified = 1;
    res.score = spTotal;
    if (spTotal < cfg.minSpScore) {
        res.classification = tax.exists(bestTax) ? tax.spParent[tax.nodeOf[bestTax]] : 0;
        return;
    }
    if (cfg.em) {  // no lowerRankClassification under --em
        res.classification = bestTax;
        return;
    }
    const int32_t spT = bestTax;
    long nCl = 0;
    auto findOrAdd = [&](int32_t t) -> long {
        for (long z = 0; z < nCl; z++)
            if (cl[z].tax == t) return z;
        if (nCl >= clCap) return -1;
        cl[nCl].tax = t;
        cl[nCl].parentTax = 0;
        cl[nCl].count = 0;
        cl[nCl].removed = 0;
        return nCl++;
    };
    for (long e = 0; e < nTc; e++) {
        const uint32_t c = tc[e].count;
        int node = tax.nodeOf[tc[e].tax_id];
        int32_t t = tax.nodeTax[node];
        long z = findOrAdd(t);
        if (z < 0) break;
        cl[z].count += c;
        int guard = 0;
        while (t != spT && guard++ < 64) {
            const int pnode = tax.parent[node];
            const int32_t pt = tax.nodeTax[pnode];
            cl[z].parentTax = pt;  // t is a child of pt
            long pz = findOrAdd(pt);
            if (pz < 0) break;
            cl[pz].count += c;
            node = pnode;
            t = pt;
            z = pz;
        }
    }
    if (cfg.accessionLevel == 2) {
        for (long z = 0; z < nCl; z++)
            if (cl[z].tax != spT && (tax.flags[tax.nodeOf[cl[z].tax]] & 2u)) cl[z].removed = 1;
    }
    const uint32_t thr = (uint32_t)((readLength - 1) / cfg.denominator);
    int32_t cur = spT;
    for (int step = 0; step < 64; step++) {
        uint32_t maxCnt = thr;
        long nBest = 0, best = -1, nChild = 0;
        for (long z = 0; z < nCl; z++) {
            if (cl[z].tax == spT || cl[z].removed || cl[z].parentTax != cur) continue;
            nChild++;
            const uint32_t cc = cl[z].count;
            if (cc > maxCnt) { maxCnt = cc; best = z; nBest = 1; }
            else if (cc == maxCnt) { if (nBest == 0) best = z; nBest++; }
        }
        if (nChild == 0 || nBest != 1) break;
        cur = cl[best].tax;
    }
    res.classification = cur;
}

__device__ __forceinline__ mtb_result empty_result(int readLength) {
    mtb_result res;
    res.classification = 0;
    res.score = 0.0f;
    res.hamming_dist = 0;
    res.query_length = (uint32_t)readLength;
    res.taxcnt_offset = (uint32_t)0;
    res.taxcnt_len = 0;
    res.is_classified = 0;
    for (int k = 0; k < 7; k++) res.pad[k] = 0;
    return res;
}

// chooseBestTaxon (Taxonomer.cpp:130-202), filterRedundantMatches (:205-241), taxCnt and the
// lower-rank BFS (:252-314): one thread per read (short reads).
__global__ void __launch_bounds__(256) k_choose_taxon(const mtb_match* __restrict__ M, const uint64_t* __restrict__ mOff,
                                                      const uint32_t* __restrict__ qlen, uint32_t nReads,
                                                      const uint64_t* __restrict__ sScan,
                                                      const uint64_t* __restrict__ sStart,
                                                      const uint64_t* __restrict__ gScan,
                                                      const uint64_t* __restrict__ gStart,
                                                      const float* __restrict__ spScore,
                                                      const uint8_t* __restrict__ spKeep, AssignCfg cfg, TaxView tax,
                                                      Clade* __restrict__ cladeP,
                                                      uint32_t cladePerMatch, mtb_taxcnt* __restrict__ tcP,
                                                      mtb_result* __restrict__ results) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nReads) return;
    const uint64_t base = mOff[r];
    const long n = (long)(mOff[r + 1] - base);
    const int readLength = (int)qlen[r];
    mtb_result res = empty_result(readLength);
    if (n == 0) { results[r] = res; return; }

    // ---- getBestSpeciesMatches tail (Taxonomer.cpp:380-408) over the read's species runs ----
    const uint64_t s0 = sScan[base], s1 = sScan[base + n];
    long meaningful = 0;
    float bestSpScore = 0.0f;
    uint64_t bestFirst = 0, bestSecond = 0;
    for (uint64_t s = s0; s < s1; s++) {
        if (!spKeep[s]) continue;
        const float score = spScore[s];
        if (score > 0.f) meaningful++;
        if (score > bestSpScore) { bestSpScore = score; bestFirst = sStart[s]; bestSecond = sStart[s + 1]; }
    }

    // ---- chooseBestTaxon (Taxonomer.cpp:130-202) ----
    float spTotal = 0.0f;
    int32_t bestTax = 0;
    bool isLCA = false;
    if (meaningful > 0) {
        const float thr = bestSpScore * cfg.tieRatio;
        long cnt = 0;
        int lcaNode = -1;
        for (uint64_t s = s0; s < s1; s++) {
            if (!spKeep[s]) continue;
            if (spScore[s] >= thr) {
                cnt++;
                spTotal += spScore[s];
                const int32_t t = (int32_t)M[sStart[s]].species_id;
                if (cnt == 1) bestTax = t;
                if (tax.exists(t)) lcaNode = lcaNode < 0 ? tax.nodeOf[t] : tax.lca_node(lcaNode, tax.nodeOf[t]);
            }
        }
        if (cnt > 1) {
            isLCA = true;
            bestTax = lcaNode >= 0 ? tax.nodeTax[lcaNode] : 0;
            spTotal = spTotal / (float)cnt;
        }
    }
    if (spTotal == 0 || spTotal < cfg.minScore) {
        res.score = spTotal;
        results[r] = res;
        return;
    }
    if (isLCA) {
        res.is_classified = 1;
        res.classification = bestTax;
        res.score = spTotal;
        results[r] = res;
        return;
    }
    mtb_taxcnt* tc = tcP + base;  // capacity n (each quotient holds >= 1 match)
    const long nTc = filter_redundant_serial(M, bestFirst, bestSecond, gScan, gStart, (uint32_t)cfg.dnaShift, tax, tc);
    classify_tail(res, tc, nTc, spTotal, bestTax, readLength, cfg, tax, cladeP + base * cladePerMatch,
                  n * (long)cladePerMatch);
    results[r] = res;
}

// The same for reads with many matches (long reads): one wave per read. The species-run scan is
// spread over the lanes (sum / max reductions, the first maximum by ballot; the tie set summed in
// species order, as the reference's float additions run); filterRedundantMatches is a parallel
// reduction over a per-quotient table in LDS (atomicMin of the hamming, then LCA folds of the
// minimal matches' taxa by compare-and-swap: an order-free reduction, as the serial fold is), and
// taxCnt a small LDS hash of (taxon, count). Reads whose quotients or distinct taxa do not fit take
// the serial code on lane 0.
constexpr int kWavePerReadMatches = 256;  // live matches per read above which K6 goes wave per read
constexpr int kQuotLds = 4096;   // quotients per LDS window (a 12 kb read at dnaShift 3 in one pass)
constexpr int kTcHash = 256;     // distinct taxa of one read's taxCnt in LDS

__device__ __forceinline__ float wave_max_f(float x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x = fmaxf(x, __shfl_xor(x, d, 64));
    return x;
}
__device__ __forceinline__ long wave_sum_l(long x) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

__global__ void __launch_bounds__(64) k_choose_taxon_wave(const mtb_match* __restrict__ M, const uint64_t* __restrict__ mOff,
                                                          const uint32_t* __restrict__ qlen, uint32_t nReads,
                                                          const uint64_t* __restrict__ sScan,
                                                          const uint64_t* __restrict__ sStart,
                                                          const uint64_t* __restrict__ gScan,
                                                          const uint64_t* __restrict__ gStart,
                                                          const float* __restrict__ spScore,
                                                          const uint8_t* __restrict__ spKeep, AssignCfg cfg,
                                                          TaxView tax, Clade* __restrict__ cladeP,
                                                          uint32_t cladePerMatch, mtb_taxcnt* __restrict__ tcP,
                                                          mtb_result* __restrict__ results,
                                                          const uint64_t* __restrict__ order) {
    // per quotient: min hamming << 24 | the LCA of the taxIDs at that hamming (taxIDs < 2^24: the
    // caller checks), one word (32 KB: twice the waves per CU of separate tables)
    __shared__ uint32_t qw[kQuotLds];
    __shared__ int32_t hk[kTcHash];
    __shared__ uint32_t hc[kTcHash];
    __shared__ int sFlag;
    if (blockIdx.x >= nReads) return;
    const uint32_t r = order ? (uint32_t)order[blockIdx.x] : blockIdx.x;  // reads with most matches first
    const int lane = threadIdx.x;
    const uint64_t base = mOff[r];
    const long n = (long)(mOff[r + 1] - base);
    const int readLength = (int)qlen[r];
    mtb_result res = empty_result(readLength);
    if (n == 0) {
        if (lane == 0) results[r] = res;
        return;
    }
    const uint64_t s0 = sScan[base], s1 = sScan[base + n];
    long meaningful = 0;
    float bestSpScore = 0.0f;
    for (uint64_t s = s0 + lane; s < s1; s += 64) {
        if (!spKeep[s]) continue;
        const float score = spScore[s];
        meaningful += score > 0.f;
        bestSpScore = fmaxf(bestSpScore, score);
    }
    meaningful = wave_sum_l(meaningful);
    bestSpScore = wave_max_f(bestSpScore);  // every lane: the maximum (> 0 when meaningful)
    float spTotal = 0.0f;
    int32_t bestTax = 0;
    bool isLCA = false;
    uint64_t bestFirst = 0, bestSecond = 0;
    if (meaningful > 0) {
        // the first species run reaching the maximum (the serial scan keeps the first strict max)
        for (uint64_t c = s0; c < s1; c += 64) {
            const uint64_t s = c + lane;
            const bool hit = s < s1 && spKeep[s] && spScore[s] == bestSpScore;
            const unsigned long long m = __ballot(hit);
            if (m) {
                const uint64_t sb = c + (uint64_t)(__ffsll((long long)m) - 1);
                bestFirst = sStart[sb];
                bestSecond = sStart[sb + 1];
                break;
            }
        }
        // the tie set in species order: scores summed one by one (wave-uniform), LCA folded
        const float thr = bestSpScore * cfg.tieRatio;
        long cnt = 0;
        int lcaNode = -1;
        for (uint64_t c = s0; c < s1; c += 64) {
            const uint64_t s = c + lane;
            const bool in = s < s1 && spKeep[s] && spScore[s] >= thr;
            const float sc = in ? spScore[s] : 0.0f;
            const int32_t sp = in ? (int32_t)M[sStart[s]].species_id : 0;
            unsigned long long m = __ballot(in);
            while (m) {
                const int b = __ffsll((long long)m) - 1;
                m &= m - 1;
                const float v = __shfl(sc, b, 64);
                const int32_t t = __shfl(sp, b, 64);
                cnt++;
                spTotal += v;
                if (cnt == 1) bestTax = t;
                if (tax.exists(t)) lcaNode = lcaNode < 0 ? tax.nodeOf[t] : tax.lca_node(lcaNode, tax.nodeOf[t]);
            }
        }
        if (cnt > 1) {
            isLCA = true;
            bestTax = lcaNode >= 0 ? tax.nodeTax[lcaNode] : 0;
            spTotal = spTotal / (float)cnt;
        }
    }
    if (spTotal == 0 || spTotal < cfg.minScore || isLCA) {
        if (lane == 0) {
            res.score = spTotal;
            if (isLCA && !(spTotal == 0 || spTotal < cfg.minScore)) {
                res.is_classified = 1;
                res.classification = bestTax;
            }
            results[r] = res;
        }
        return;
    }
    // ---- filterRedundantMatches over the best species' matches ----
    mtb_taxcnt* tc = tcP + base;  // capacity n
    const uint32_t dnaShift = (uint32_t)cfg.dnaShift;
    const long maxQ = (readLength + 3) / (long)dnaShift;
    const long nb = (long)(bestSecond - bestFirst);
    const mtb_match* B = M + bestFirst;
    long nTc = -1;  // -1: take the serial path
    if (tax.maxTax < 0xFFFFFF) {  // taxID 0xFFFFFF is the packed word's "empty" mark
        for (int k = lane; k < kTcHash; k += 64) { hk[k] = 0; hc[k] = 0; }
        if (lane == 0) sFlag = 0;
        // quotients in windows of kQuotLds (a read of > 12 kb takes several passes over its matches)
        for (long q0 = 0; q0 <= maxQ; q0 += kQuotLds) {
            const long q1 = min(maxQ + 1, q0 + (long)kQuotLds);
            for (long q = q0 + lane; q < q1; q += 64) qw[q - q0] = 0xFFFFFFFFu;
            __syncthreads();
            for (long i = lane; i < nb; i += 64) {
                const uint32_t q = info_pos(B[i].qinfo) / dnaShift;
                if (q > (uint32_t)maxQ || B[i].hamming > 254u) { sFlag = 1; continue; }
                if ((long)q < q0 || (long)q >= q1) continue;
                atomicMin(&qw[q - q0], (uint32_t)B[i].hamming << 24 | 0xFFFFFFu);  // the minimum, taxon part empty
            }
            __syncthreads();
            if (sFlag) break;
            for (long i = lane; i < nb; i += 64) {
                const uint32_t q = info_pos(B[i].qinfo) / dnaShift;
                if ((long)q < q0 || (long)q >= q1) continue;
                const uint32_t h = (uint32_t)B[i].hamming << 24;
                uint32_t old = qw[q - q0];
                if ((old & 0xFF000000u) != h) continue;
                const int32_t t = (int32_t)B[i].target_id;
                while (true) {  // taxon part = LCA(taxon part, t), 0xFFFFFF = empty
                    const uint32_t cur = old & 0xFFFFFFu;
                    const uint32_t nv = h | (uint32_t)(cur == 0xFFFFFFu ? t : tax.lca((int32_t)cur, t));
                    if (nv == old) break;
                    const uint32_t prev = atomicCAS(&qw[q - q0], old, nv);
                    if (prev == old) break;
                    old = prev;
                }
            }
            __syncthreads();
            for (long q = q0 + lane; q < q1; q += 64) {
                const uint32_t wq = qw[q - q0];
                const int32_t t = wq == 0xFFFFFFFFu ? 0 : (int32_t)(wq & 0xFFFFFFu);
                if (t == 0) continue;
                uint32_t h = ((uint32_t)t * 2654435761u) & (kTcHash - 1);
                int probes = 0;
                while (true) {
                    const int32_t prev = atomicCAS(&hk[h], 0, t);
                    if (prev == 0 || prev == t) { atomicAdd(&hc[h], 1u); break; }
                    h = (h + 1) & (kTcHash - 1);
                    if (++probes == kTcHash) { sFlag = 1; break; }
                }
            }
            __syncthreads();  // qw is rewritten by the next window
            if (sFlag) break;
        }
        if (!sFlag) {  // entries out in slot order, then std::map order (ascending taxID) on lane 0
            long at = 0;
            for (int k0 = 0; k0 < kTcHash; k0 += 64) {
                const int k = k0 + lane;
                const bool v = hk[k] != 0;
                const unsigned long long m = __ballot(v);
                if (v) {
                    const long p = at + (long)__popcll(m & ((1ull << lane) - 1));
                    tc[p].tax_id = hk[k];
                    tc[p].count = hc[k];
                }
                at += (long)__popcll(m);
            }
            nTc = at;
        }
    }
    if (lane != 0) return;
    if (nTc < 0) {
        nTc = filter_redundant_serial(M, bestFirst, bestSecond, gScan, gStart, dnaShift, tax, tc);
    } else {
        for (long a = 1; a < nTc; a++) {
            mtb_taxcnt v = tc[a];
            long b = a;
            while (b > 0 && tc[b - 1].tax_id > v.tax_id) { tc[b] = tc[b - 1]; b--; }
            tc[b] = v;
        }
    }
    classify_tail(res, tc, nTc, spTotal, bestTax, readLength, cfg, tax, cladeP + base * cladePerMatch,
                  n * (long)cladePerMatch);
    results[r] = res;
}

// The same for short reads with kGroupLanes lanes per read (16 reads per 256-thread block): the
// species-run scan, the tie set and filterRedundantMatches' per-quotient reduction as in the wave
// kernel, on a 16-lane group with per-group LDS tables (kGroupQ quotients, kGroupHash taxa); the
// group's first lane runs the tail. A read whose quotients or taxa do not fit takes the serial
// filter on that lane. Block-wide barriers order the LDS phases (every thread reaches them).
constexpr int kGroupLanes = 16;
constexpr int kGroupQ = 128;    // quotients of a read (a 2 x 150 bp pair at dnaShift 3: 101)
constexpr int kGroupHash = 64;  // distinct taxa of one read's taxCnt

__device__ __forceinline__ float group_max_f(float x) {
#pragma unroll
    for (int d = kGroupLanes / 2; d > 0; d >>= 1) x = fmaxf(x, __shfl_xor(x, d, kGroupLanes));
    return x;
}
__device__ __forceinline__ long group_sum_l(long x) {
#pragma unroll
    for (int d = kGroupLanes / 2; d > 0; d >>= 1) x += __shfl_xor(x, d, kGroupLanes);
    return x;
}

__global__ void __launch_bounds__(256) k_choose_taxon_group(const mtb_match* __restrict__ M,
                                                            const uint64_t* __restrict__ mOff,
                                                            const uint32_t* __restrict__ qlen, uint32_t nReads,
                                                            const uint64_t* __restrict__ sScan,
                                                            const uint64_t* __restrict__ sStart,
                                                            const uint64_t* __restrict__ gScan,
                                                            const uint64_t* __restrict__ gStart,
                                                            const float* __restrict__ spScore,
                                                            const uint8_t* __restrict__ spKeep, AssignCfg cfg,
                                                            TaxView tax, Clade* __restrict__ cladeP,
                                                            uint32_t cladePerMatch, mtb_taxcnt* __restrict__ tcP,
                                                            mtb_result* __restrict__ results) {
    constexpr int kGroups = 256 / kGroupLanes;
    __shared__ uint32_t qw[kGroups][kGroupQ];  // min hamming << 24 | LCA of the taxa at it (as the wave kernel)
    __shared__ int32_t hk[kGroups][kGroupHash];
    __shared__ uint32_t hc[kGroups][kGroupHash];
    __shared__ int gFlag[kGroups];
    const int g = threadIdx.x / kGroupLanes, gl = threadIdx.x % kGroupLanes;
    const int gLane0 = (threadIdx.x & 63) & ~(kGroupLanes - 1);  // the group's first lane in its wave
    const uint32_t r = blockIdx.x * kGroups + g;
    const bool valid = r < nReads;
    const uint64_t base = valid ? mOff[r] : 0;
    const long n = valid ? (long)(mOff[r + 1] - base) : 0;
    const int readLength = valid ? (int)qlen[r] : 0;
    mtb_result res = empty_result(readLength);
    float spTotal = 0.0f;
    int32_t bestTax = 0;
    bool isLCA = false, filter = false;
    uint64_t bestFirst = 0, bestSecond = 0;
    if (n > 0) {
        const uint64_t s0 = sScan[base], s1 = sScan[base + n];
        long meaningful = 0;
        float bestSpScore = 0.0f;
        for (uint64_t s = s0 + gl; s < s1; s += kGroupLanes) {
            if (!spKeep[s]) continue;
            const float score = spScore[s];
            meaningful += score > 0.f;
            bestSpScore = fmaxf(bestSpScore, score);
        }
        meaningful = group_sum_l(meaningful);
        bestSpScore = group_max_f(bestSpScore);
        if (meaningful > 0) {
            for (uint64_t c = s0; c < s1; c += kGroupLanes) {  // the first species run at the maximum
                const uint64_t s = c + gl;
                const bool hit = s < s1 && spKeep[s] && spScore[s] == bestSpScore;
                const uint32_t m = (uint32_t)(__ballot(hit) >> gLane0) & 0xFFFFu;
                if (m) {
                    const uint64_t sb = c + (uint64_t)(__ffs((int)m) - 1);
                    bestFirst = sStart[sb];
                    bestSecond = sStart[sb + 1];
                    break;
                }
            }
            const float thr = bestSpScore * cfg.tieRatio;  // the tie set in species order
            long cnt = 0;
            int lcaNode = -1;
            for (uint64_t c = s0; c < s1; c += kGroupLanes) {
                const uint64_t s = c + gl;
                const bool in = s < s1 && spKeep[s] && spScore[s] >= thr;
                const float sc = in ? spScore[s] : 0.0f;
                const int32_t sp = in ? (int32_t)M[sStart[s]].species_id : 0;
                uint32_t m = (uint32_t)(__ballot(in) >> gLane0) & 0xFFFFu;
                while (m) {
                    const int b = __ffs((int)m) - 1;
                    m &= m - 1;
                    const float v = __shfl(sc, b, kGroupLanes);
                    const int32_t t = __shfl(sp, b, kGroupLanes);
                    cnt++;
                    spTotal += v;
                    if (cnt == 1) bestTax = t;
                    if (tax.exists(t)) lcaNode = lcaNode < 0 ? tax.nodeOf[t] : tax.lca_node(lcaNode, tax.nodeOf[t]);
                }
            }
            if (cnt > 1) {
                isLCA = true;
                bestTax = lcaNode >= 0 ? tax.nodeTax[lcaNode] : 0;
                spTotal = spTotal / (float)cnt;
            }
        }
        filter = !(spTotal == 0 || spTotal < cfg.minScore || isLCA);
    }
    // filterRedundantMatches over the best species' matches, in the group's LDS tables
    const uint32_t dnaShift = (uint32_t)cfg.dnaShift;
    const long maxQ = (readLength + 3) / (long)dnaShift;
    const long nb = (long)(bestSecond - bestFirst);
    const mtb_match* B = M + bestFirst;
    const bool lds = filter && maxQ < kGroupQ && tax.maxTax < 0xFFFFFF;
    if (lds) {
        for (long q = gl; q <= maxQ; q += kGroupLanes) qw[g][q] = 0xFFFFFFFFu;
        for (int k = gl; k < kGroupHash; k += kGroupLanes) {
            hk[g][k] = 0;
            hc[g][k] = 0;
        }
        if (gl == 0) gFlag[g] = 0;
    }
    __syncthreads();
    if (lds) {
        for (long i = gl; i < nb; i += kGroupLanes) {
            const uint32_t q = info_pos(B[i].qinfo) / dnaShift;
            if (q > (uint32_t)maxQ || B[i].hamming > 254u) {
                gFlag[g] = 1;
                continue;
            }
            atomicMin(&qw[g][q], (uint32_t)B[i].hamming << 24 | 0xFFFFFFu);
        }
    }
    __syncthreads();
    const bool ok = lds && !gFlag[g];
    if (ok) {
        for (long i = gl; i < nb; i += kGroupLanes) {
            const uint32_t q = info_pos(B[i].qinfo) / dnaShift;
            const uint32_t h = (uint32_t)B[i].hamming << 24;
            uint32_t old = qw[g][q];
            if ((old & 0xFF000000u) != h) continue;
            const int32_t t = (int32_t)B[i].target_id;
            while (true) {  // taxon part = LCA(taxon part, t), 0xFFFFFF = empty
                const uint32_t cur = old & 0xFFFFFFu;
                const uint32_t nv = h | (uint32_t)(cur == 0xFFFFFFu ? t : tax.lca((int32_t)cur, t));
                if (nv == old) break;
                const uint32_t prev = atomicCAS(&qw[g][q], old, nv);
                if (prev == old) break;
                old = prev;
            }
        }
    }
    __syncthreads();
    if (ok) {
        for (long q = gl; q <= maxQ; q += kGroupLanes) {
            const uint32_t wq = qw[g][q];
            const int32_t t = wq == 0xFFFFFFFFu ? 0 : (int32_t)(wq & 0xFFFFFFu);
            if (t == 0) continue;
            uint32_t h = ((uint32_t)t * 2654435761u) & (kGroupHash - 1);
            int probes = 0;
            while (true) {
                const int32_t prev = atomicCAS(&hk[g][h], 0, t);
                if (prev == 0 || prev == t) {
                    atomicAdd(&hc[g][h], 1u);
                    break;
                }
                h = (h + 1) & (kGroupHash - 1);
                if (++probes == kGroupHash) {
                    gFlag[g] = 1;
                    break;
                }
            }
        }
    }
    __syncthreads();
    mtb_taxcnt* tc = tcP + base;  // capacity n
    long nTc = -1;                // -1: the serial filter
    if (ok && !gFlag[g]) {        // entries out in slot order (std::map order on the first lane below)
        long at = 0;
        for (int k0 = 0; k0 < kGroupHash; k0 += kGroupLanes) {
            const int k = k0 + gl;
            const bool v = hk[g][k] != 0;
            const uint32_t m = (uint32_t)(__ballot(v) >> gLane0) & 0xFFFFu;
            if (v) {
                const long p = at + (long)__popc(m & ((1u << gl) - 1));
                tc[p].tax_id = hk[g][k];
                tc[p].count = hc[g][k];
            }
            at += (long)__popc(m);
        }
        nTc = at;
    }
    if (gl != 0 || !valid) return;
    if (!filter) {
        res.score = spTotal;
        if (isLCA && n > 0 && !(spTotal == 0 || spTotal < cfg.minScore)) {
            res.is_classified = 1;
            res.classification = bestTax;
        }
        results[r] = res;
        return;
    }
    if (nTc < 0) {
        nTc = filter_redundant_serial(M, bestFirst, bestSecond, gScan, gStart, dnaShift, tax, tc);
    } else {
        for (long a = 1; a < nTc; a++) {
            mtb_taxcnt v = tc[a];
            long b = a;
            while (b > 0 && tc[b - 1].tax_id > v.tax_id) {
                tc[b] = tc[b - 1];
                b--;
            }
            tc[b] = v;
        }
    }
    classify_tail(res, tc, nTc, spTotal, bestTax, readLength, cfg, tax, cladeP + base * cladePerMatch,
                  n * (long)cladePerMatch);
    results[r] = res;
}

// Longest-first orders for the wave kernels (a wave kernel's time is otherwise set by its longest
// waves, started last): keys = a size bound minus the size, a stable LSD radix sort of the indices.
__global__ void k_wave_size_keys(const uint64_t* __restrict__ waveList, uint32_t n, uint64_t* __restrict__ keys) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = (uint64_t)(kWaveCombineMax - (uint32_t)(waveList[i] >> 32));
}
__global__ void k_read_size_keys(const uint64_t* __restrict__ mOff, uint32_t n, uint64_t* __restrict__ keys) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = 0xFFFFFFull - min<uint64_t>(mOff[i + 1] - mOff[i], 0xFFFFFFull);
}

static const uint64_t* longest_first(uint32_t n, int bits, const AssignScratch& s, hipStream_t st) {
    bool inB = false;
    radix_sort_pairs(s.ordKA, s.ordVA, s.ordKB, s.ordVB, n, 0, bits, false, true, s.radixCounts, s.radixOffs,
                     s.scanTmp, &inB, st);
    return inB ? s.ordVB : s.ordVA;
}

void launch_assign(const mtb_match* matches, const uint64_t* mOff, const uint32_t* qlen, uint32_t nReads, uint64_t nM, const AssignArgs& a, const TaxDevice& t, const AssignScratch& s,
                   mtb_taxcnt* tcPool, mtb_result* results, unsigned long long* devStats, uint64_t* hostStats,
                   hipStream_t st) {
    for (int i = 0; i < 4; i++) hostStats[i] = 0;
    if (nReads == 0) return;
    AssignCfg cfg{a.kmerFormat, a.dnaShift, a.maxCodonShift, a.denominator, a.minConsCnt, a.minConsCntEuk,
                  a.accessionLevel, a.minScore, a.minSpScore, a.tieRatio, a.generic, a.emulateAll, a.em};
    TaxView tv{t.nodeOf, t.nodeTax, t.parent, t.depth, t.flags, t.spParent, t.maxTax};
    if (nM) {
        // gFlag holds the flag bytes, sFlag the packed tile sums (run_index_tmp_bytes)
        launch_run_index(matches, nM, reinterpret_cast<uint8_t*>(s.gFlag),
                         reinterpret_cast<unsigned long long*>(s.sFlag), s.gScan, s.sScan, s.gStart, s.sStart, st);
        // groups and runs never outnumber matches: size the grids by nM, threads past the count exit
        uint64_t cnt[2] = {0, 0};
        hipMemcpyAsync(&cnt[0], s.gScan + nM, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(&cnt[1], s.sScan + nM, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
        hostStats[0] = cnt[0];
        hostStats[2] = cnt[1];
        if (cnt[0]) {
            k_group_keys<<<(unsigned)((cnt[0] + 255) / 256), 256, 0, st>>>(
                s.gStart, cnt[0], s.ordKA, s.ordVA, s.pathCnt,
                prune_min_matches(a.minConsCnt, a.minConsCntEuk, a.maxCodonShift));
            bool inB = false;
            const uint64_t heavy = radix_sort_pairs(s.ordKA, s.ordVA, s.ordKB, s.ordVB, cnt[0], 32, 40, true, false,
                                                    s.radixCounts, s.radixOffs, s.scanTmp, &inB, st);
            hostStats[1] = heavy;
            if (heavy) {
                // groups of >= kBigGroup matches queue for a wave each (long reads' serial tail)
                const bool waves = !a.generic && a.bigGroups && nM >= kBigGroup;
                if (waves) hipMemsetAsync(s.waveCount, 0, sizeof(uint32_t), st);
                // MTB_PATHS_NOLDS=<waves> (A/B, read per batch): the unstaged form held to 5 or 6 waves
                const char* nl = getenv("MTB_PATHS_NOLDS");
                const int nlw = nl ? atoi(nl) : 0;
#define MTB_PATHS(L, W)                                                                                             \
    k_match_paths<L, W><<<(unsigned)((heavy + 63) / 64), 64, 0, st>>>(                                              \
        matches, s.gStart, inB ? s.ordKB : s.ordKA, heavy, cfg, tv, (Path*)s.local, (Path*)s.paths, s.conn,         \
        s.pathCnt, waves ? s.waveList : nullptr, s.waveCount)
                if (nlw == 6) MTB_PATHS(false, 6);
                else if (nlw == 5) MTB_PATHS(false, 5);
                else if (nlw == 4) MTB_PATHS(false, 4);
                else MTB_PATHS(true, 1);
#undef MTB_PATHS
                if (waves) {
                    uint32_t nBig = 0;
                    hipMemcpyAsync(&nBig, s.waveCount, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
                    hipStreamSynchronize(st);
                    if (nBig)
                        k_match_paths_wave<<<nBig, 64, 0, st>>>(matches, s.gStart, s.waveList, cfg, tv, (Path*)s.local,
                                                                (Path*)s.paths, s.conn, s.pathCnt);
                }
            }
        }
        if (cnt[1]) {
            hipMemsetAsync(s.waveCount, 0, sizeof(uint32_t), st);
            k_combine_paths<<<(unsigned)((cnt[1] + 255) / 256), 256, 0, st>>>(
                matches, s.sStart, cnt[1], s.gScan, s.gStart, s.pathCnt, qlen, cfg, (Path*)s.paths, (Path*)s.comb,
                s.spScore, s.spKeep, s.waveList, s.waveCount);
            uint32_t nWave = 0;
            hipMemcpyAsync(&nWave, s.waveCount, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
            hipStreamSynchronize(st);
            if (nWave) {
                k_wave_size_keys<<<(nWave + 255) / 256, 256, 0, st>>>(s.waveList, nWave, s.ordKA);
                const uint64_t* order = longest_first(nWave, 16, s, st);
                k_combine_wave<<<nWave, 64, 0, st>>>(matches, s.sStart, s.waveList, qlen, cfg, (Path*)s.paths,
                                                     (Path*)s.comb, s.spScore, s.spKeep, devStats, order);
            }
            hostStats[3] = nWave;
        }
    } else {
        hipMemsetAsync(s.sScan, 0, sizeof(uint64_t), st);
    }
    // a wave per read when reads carry many matches (long reads: a thread per read would leave most
    // SIMDs idle and serialise each read's best-species scan), else a 16-lane group per read (a
    // thread per read with MTB_WAVE_TAXON=0, or under MTB_FORCE_GENERIC)
    const bool wave = a.waveTaxon >= 0 ? a.waveTaxon == 1 : (!a.generic && nM > (uint64_t)kWavePerReadMatches * nReads);
    // short reads: a 16-lane group per read by default (config 3: 1.78 -> 1.09 ms, 10.4 -> 2.5 GB
    // fetched per batch against a thread per read; profiles/r03/ab_k6_group.json)
    const bool group = a.waveTaxon == 2 || (a.waveTaxon < 0 && !wave && !a.generic);
    if (group) {
        k_choose_taxon_group<<<(nReads + 15) / 16, 256, 0, st>>>(matches, mOff, qlen, nReads, s.sScan, s.sStart,
                                                                 s.gScan, s.gStart, s.spScore, s.spKeep, cfg, tv,
                                                                 (Clade*)s.clade, s.cladePerMatch, tcPool, results);
    } else if (wave) {
        k_read_size_keys<<<(nReads + 255) / 256, 256, 0, st>>>(mOff, nReads, s.ordKA);
        const uint64_t* order = longest_first(nReads, 24, s, st);
        k_choose_taxon_wave<<<nReads, 64, 0, st>>>(matches, mOff, qlen, nReads, s.sScan, s.sStart, s.gScan, s.gStart,
                                                   s.spScore, s.spKeep, cfg, tv, (Clade*)s.clade, s.cladePerMatch,
                                                   tcPool, results, order);
    } else {
        const unsigned ctT = nReads < 256u * 256u ? 64u : 256u;
        k_choose_taxon<<<(nReads + ctT - 1) / ctT, ctT, 0, st>>>(matches, mOff, qlen, nReads, s.sScan, s.sStart,
                                                             s.gScan, s.gStart, s.spScore, s.spKeep, cfg, tv,
                                                             (Clade*)s.clade, s.cladePerMatch, tcPool, results);
    }
}

uint64_t path_bytes() { return sizeof(Path); }
uint64_t clade_bytes() { return sizeof(Clade); }

// Compaction of the per-read taxcnt slices (capacity = match count) into one pooled array.
__global__ void k_compact_taxcnt(const mtb_taxcnt* __restrict__ pool, const uint64_t* __restrict__ mOff,
                                 mtb_result* __restrict__ results, const uint64_t* __restrict__ tcOff, uint32_t nReads,
                                 mtb_taxcnt* __restrict__ out) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nReads) return;
    uint32_t len = results[r].taxcnt_len;
    uint64_t dst = tcOff[r];
    results[r].taxcnt_offset = (uint32_t)dst;
    for (uint32_t k = 0; k < len; k++) out[dst + k] = pool[mOff[r] + k];
}

__global__ void k_taxcnt_len(const mtb_result* __restrict__ results, uint32_t nReads, uint32_t* __restrict__ len) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < nReads) len[r] = results[r].taxcnt_len;
}

void launch_taxcnt_len(const mtb_result* results, uint32_t nReads, uint32_t* len, hipStream_t s) {
    if (nReads) k_taxcnt_len<<<(nReads + 255) / 256, 256, 0, s>>>(results, nReads, len);
}
void launch_compact_taxcnt(const mtb_taxcnt* pool, const uint64_t* mOff, mtb_result* results, const uint64_t* tcOff,
                           uint32_t nReads, mtb_taxcnt* out, hipStream_t s) {
    if (nReads) k_compact_taxcnt<<<(nReads + 255) / 256, 256, 0, s>>>(pool, mOff, results, tcOff, nReads, out);
}

// ---- all-to-all receive layout -> per-read segments (range-partitioned DB) ---------
// The owner of reads [0, n) receives one chunk per DB part, each grouped by read. Per-read totals
// (then scanned into mOff) and, per (chunk, read) piece, a wave copies it to its read's segment at
// the running offset of the chunks before it. srcOff = exclusive scan of the chunk-major counts.
__global__ void k_chunk_totals(const uint32_t* __restrict__ cnt, uint32_t nChunks, uint32_t n,
                               uint32_t* __restrict__ tot) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    uint32_t t = 0;
    for (uint32_t c = 0; c < nChunks; c++) t += cnt[(uint64_t)c * n + r];
    tot[r] = t;
}

__global__ void __launch_bounds__(256) k_regroup_chunks(const uint64_t* __restrict__ src, const uint32_t* __restrict__ cnt,
                                                        const uint64_t* __restrict__ srcOff, uint32_t nChunks, uint32_t n,
                                                        const uint64_t* __restrict__ mOff, uint64_t* __restrict__ dst) {
    const uint32_t r = blockIdx.x * 4 + threadIdx.x / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (r >= n) return;
    uint64_t at = mOff[r] * 3;  // 24-B records as 3 words
    for (uint32_t c = 0; c < nChunks; c++) {
        const uint64_t k = (uint64_t)c * n + r;
        const uint64_t words = (uint64_t)cnt[k] * 3, from = srcOff[k] * 3;
        for (uint64_t w = lane; w < words; w += 64) dst[at + w] = src[from + w];
        at += words;
    }
}

void launch_regroup_chunks(const mtb_match* src, const uint32_t* cnt, uint32_t nChunks, uint32_t n, uint32_t* tot,
                           uint64_t* srcOff, uint64_t* mOff, void* scanTmp, mtb_match* dst, hipStream_t s) {
    if (!n) return;
    k_chunk_totals<<<(n + 255) / 256, 256, 0, s>>>(cnt, nChunks, n, tot);
    exclusive_scan_u32(tot, n, mOff, scanTmp, s);
    exclusive_scan_u32(cnt, (uint64_t)nChunks * n, srcOff, scanTmp, s);
    k_regroup_chunks<<<(n + 3) / 4, 256, 0, s>>>((const uint64_t*)src, cnt, srcOff, nChunks, n, mOff, (uint64_t*)dst);
}

// ------------------------------------------------------------------------------------------------
// --em (Classifier.cpp:209-386, Taxonomer.cpp:377-386, Reporter.h:80-92): per classified read its
// species scores sorted by std::sort (score descending; the comparator is not a total order, so the
// libstdc++ emulation decides ties), the first ten kept as (species, score^2) "mappings"; then the
// EM re-estimation of species abundances over all mappings and the per-read reassignment.
// ------------------------------------------------------------------------------------------------
struct EmPair {
    int32_t sp;
    float sc;
};

__global__ void k_em_top(const mtb_match* __restrict__ M, const uint64_t* __restrict__ mOff, uint32_t n,
                         const uint64_t* __restrict__ sScan, const uint64_t* __restrict__ sStart,
                         const float* __restrict__ spScore, const uint8_t* __restrict__ spKeep,
                         const mtb_result* __restrict__ results, EmPair* __restrict__ scratch,
                         EmPair* __restrict__ maps, uint8_t* __restrict__ cnt) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    cnt[r] = 0;
    if (!results[r].is_classified) return;
    const uint64_t base = mOff[r], end = mOff[r + 1];
    const uint64_t s0 = sScan[base], s1 = sScan[end];
    EmPair* v = scratch + s0;
    long k = 0;
    for (uint64_t s = s0; s < s1; s++)  // sp2score in species order (Taxonomer.cpp:330-369)
        if (spKeep[s]) v[k++] = EmPair{(int32_t)M[sStart[s]].species_id, spScore[s]};
    stdsort::sort(v, v + k, [](const EmPair& a, const EmPair& b) { return a.sc > b.sc; });
    const long m = k < kEmTop ? k : kEmTop;
    for (long i = 0; i < m; i++) maps[(uint64_t)r * kEmTop + i] = EmPair{v[i].sp, v[i].sc * v[i].sc};
    cnt[r] = (uint8_t)m;
}

void launch_em_top(const mtb_match* M, const uint64_t* mOff, uint32_t n, const AssignScratch& s,
                   const mtb_result* results, void* scratch, void* maps, uint8_t* cnt, hipStream_t st) {
    if (!n) return;
    k_em_top<<<(n + 255) / 256, 256, 0, st>>>(M, mOff, n, s.sScan, s.sStart, s.spScore, s.spKeep, results,
                                              (EmPair*)scratch, (EmPair*)maps, cnt);
}

// The batch's mappings packed in read order (off: exclusive scan of cnt) as {read, species, score}.
__global__ void k_em_pack(const EmPair* __restrict__ maps, const uint8_t* __restrict__ cnt,
                          const uint64_t* __restrict__ off, uint32_t n, mtb_em_map* __restrict__ out) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t o = off[r];
    for (uint32_t k = 0; k < cnt[r]; k++) {
        const EmPair e = maps[(uint64_t)r * kEmTop + k];
        out[o + k] = mtb_em_map{r, e.sp, e.sc};
    }
}

__global__ void k_u8_to_u32(const uint8_t* __restrict__ in, uint32_t n, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

void launch_em_pack(const void* maps, const uint8_t* cnt, uint32_t n, uint32_t* cnt32, uint64_t* off, void* scanTmp,
                    mtb_em_map* out, hipStream_t s) {
    if (!n) return;
    k_u8_to_u32<<<(n + 255) / 256, 256, 0, s>>>(cnt, n, cnt32);
    exclusive_scan_u32(cnt32, n, off, scanTmp, s);
    k_em_pack<<<(n + 255) / 256, 256, 0, s>>>((const EmPair*)maps, cnt, off, n, out);
}

// DB k-mers per species (Classifier::countUniqueKmerPerSpecies, Classifier.cpp:388-431: every info
// entry's species, taxID_list mapping; entries without a species are not counted).
__global__ void k_species_kmers(const DbRec* __restrict__ db, uint64_t D, const int32_t* __restrict__ spOf,
                                uint32_t maxTax, uint32_t* __restrict__ cnt) {
    MTB_GRID_STRIDE(i, D) {
        const uint32_t t = db[i].tax;
        const int32_t sp = t <= maxTax ? spOf[t] : 0;
        if (sp > 0) atomicAdd(&cnt[sp], 1u);
    }
}

void launch_species_kmers(const DbRec* db, uint64_t D, const int32_t* spOf, uint32_t maxTax, uint32_t* cnt,
                          hipStream_t s) {
    if (D) k_species_kmers<<<stride_grid(D), 256, 0, s>>>(db, D, spOf, maxTax, cnt);
}

// One EM iteration, E step per query (the reference's loop body, Classifier.cpp:268-280): the
// query's terms score * p * lengthFactor summed in mapping order; a query with a zero sum adds
// nothing, the others add term / sum to their species. Contributions go to their species-sorted
// position (pos) so that the per-species sums below read them contiguously, in query order.
__global__ void k_em_estep(const float* __restrict__ score, const uint32_t* __restrict__ spIdx,
                           const uint64_t* __restrict__ qOff, uint64_t nQ, const uint64_t* __restrict__ pos,
                           const double* __restrict__ p, const double* __restrict__ lf, double* __restrict__ wS,
                           unsigned long long* __restrict__ qCount) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool counted = false;
    if (q < nQ) {
        const uint64_t a = qOff[q], b = qOff[q + 1];
        double denom = 0.0;
        for (uint64_t j = a; j < b; j++) denom += (double)score[j] * p[spIdx[j]] * lf[spIdx[j]];
        counted = !(denom == 0.0);
        for (uint64_t j = a; j < b; j++)
            wS[pos[j]] = counted ? ((double)score[j] * p[spIdx[j]] * lf[spIdx[j]]) / denom : 0.0;
    }
    const int c = __syncthreads_count(counted);
    if (threadIdx.x == 0 && c) atomicAdd(qCount, (unsigned long long)c);
}

// Per-species sums of the contributions: slices of <= kEmSlice consecutive entries of one species
// summed in order, then each species' slices in order (a species of <= kEmSlice entries sums
// exactly as the sequential loop does). M step (Classifier.cpp:291-309): top species divided by
// the counted queries, |new - old| for the convergence delta, and after ten iterations abundances
// below 1e-5 dropped to zero.
__global__ void k_em_slices(const double* __restrict__ wS, const uint64_t* __restrict__ sliceOff, uint64_t nSl,
                            double* __restrict__ part) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nSl) return;
    double f = 0.0;
    for (uint64_t j = sliceOff[i]; j < sliceOff[i + 1]; j++) f += wS[j];
    part[i] = f;
}

__global__ void k_em_mstep(const double* __restrict__ part, const uint64_t* __restrict__ spSlice, uint32_t S,
                           const uint8_t* __restrict__ isTop, const unsigned long long* __restrict__ qCount,
                           const double* __restrict__ p, double* __restrict__ pNew, double* __restrict__ absd,
                           int afterTen) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    double f = 0.0;
    for (uint64_t k = spSlice[i]; k < spSlice[i + 1]; k++) f += part[k];
    if (isTop[i]) {
        f /= (double)*qCount;
        absd[i] = fabs(f - p[i]);
        if (afterTen && f < 1e-5) f = 0.0;
    } else {
        absd[i] = 0.0;
    }
    pNew[i] = f;
}

// delta = sum of absd in species order: 256 ordered chunk sums, then those in order (fixed order,
// run to run identical)
__global__ void __launch_bounds__(256) k_em_delta(const double* __restrict__ absd, uint32_t S, double* __restrict__ out) {
    __shared__ double part[256];
    const uint32_t per = (S + 255) / 256, a = threadIdx.x * per, b = min(S, a + per);
    double d = 0.0;
    for (uint32_t i = a; i < b; i++) d += absd[i];
    part[threadIdx.x] = d;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < 256; k++) t += part[k];
        *out = t;
    }
}

void launch_em_iteration(const float* score, const uint32_t* spIdx, const uint64_t* qOff, uint64_t nQ,
                         const uint64_t* pos, const double* p, const double* lf, double* wS,
                         unsigned long long* qCount, const uint64_t* sliceOff, uint64_t nSl, double* part,
                         const uint64_t* spSlice, uint32_t S, const uint8_t* isTop, double* pNew, double* absd,
                         int afterTen, double* delta, hipStream_t s) {
    (void)hipMemsetAsync(qCount, 0, sizeof(unsigned long long), s);
    if (nQ) k_em_estep<<<(unsigned)((nQ + 255) / 256), 256, 0, s>>>(score, spIdx, qOff, nQ, pos, p, lf, wS, qCount);
    if (nSl) k_em_slices<<<(unsigned)((nSl + 255) / 256), 256, 0, s>>>(wS, sliceOff, nSl, part);
    if (S) k_em_mstep<<<(S + 255) / 256, 256, 0, s>>>(part, spSlice, S, isTop, qCount, p, pNew, absd, afterTen);
    k_em_delta<<<1, 256, 0, s>>>(absd, S, delta);
}

// Classifier::reclassify (Classifier.cpp:326-386) per query: p * score * lengthFactor normalised by
// their sum, sorted descending (std::sort: emulated), the leading species until the sum reaches 0.5,
// their LCA. mapped: 1 reassigned (counted in the reclassify report), 2 a zero sum (taxID 0, not
// counted).
struct EmPairD {
    int32_t sp;
    double pr;
};

__global__ void k_em_reclassify(const float* __restrict__ score, const uint32_t* __restrict__ spIdx,
                                const int32_t* __restrict__ spTax, const uint64_t* __restrict__ qOff,
                                const uint32_t* __restrict__ qId, uint64_t nQ, const double* __restrict__ p,
                                const double* __restrict__ lf, TaxView tax, mtb_em_read* __restrict__ out) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nQ) return;
    const uint64_t a = qOff[q], b = qOff[q + 1];
    EmPairD v[kEmTop];
    double denom = 0.0;
    long k = 0;
    for (uint64_t j = a; j < b && k < kEmTop; j++, k++) {
        const double sc = p[spIdx[j]] * (double)score[j] * lf[spIdx[j]];
        denom += sc;
        v[k] = EmPairD{spTax[spIdx[j]], sc};
    }
    mtb_em_read r;
    r.tax_id = 0;
    r.score = 0.0;
    if (denom == 0.0) {
        r.mapped = 2;
        out[qId[q]] = r;
        return;
    }
    for (long i = 0; i < k; i++) v[i].pr /= denom;
    stdsort::sort(v, v + k, [](const EmPairD& x, const EmPairD& y) { return x.pr > y.pr; });
    double sum = 0.0;
    int lcaNode = -1;
    for (long i = 0; i < k && sum < 0.5; i++) {
        sum += v[i].pr;
        const int32_t t = v[i].sp;
        if (tax.exists(t)) lcaNode = lcaNode < 0 ? tax.nodeOf[t] : tax.lca_node(lcaNode, tax.nodeOf[t]);
    }
    r.tax_id = lcaNode >= 0 ? tax.nodeTax[lcaNode] : 0;
    r.score = sum;
    r.mapped = 1;
    out[qId[q]] = r;
}

void launch_em_reclassify(const float* score, const uint32_t* spIdx, const int32_t* spTax, const uint64_t* qOff,
                          const uint32_t* qId, uint64_t nQ, const double* p, const double* lf, const TaxDevice& t,
                          mtb_em_read* out, hipStream_t s) {
    TaxView tv{t.nodeOf, t.nodeTax, t.parent, t.depth, t.flags, t.spParent, t.maxTax};
    if (nQ) k_em_reclassify<<<(unsigned)((nQ + 255) / 256), 256, 0, s>>>(score, spIdx, spTax, qOff, qId, nQ, p, lf, tv, out);
}

// ------------------------------------------------------------------------------------------------
// mtb_pin_eval: the helpers getMatchPaths, the path trims and K0 compute with, evaluated one case per
// thread exactly as those kernels call them (tests: tests/golden/ref_functions.json, computed by the
// reference's own function bodies).
// ------------------------------------------------------------------------------------------------
__global__ void k_pin_eval(int fn, const int64_t* __restrict__ param, const uint64_t* __restrict__ a,
                           const uint64_t* __restrict__ b, uint64_t n, int64_t* __restrict__ out) {
    MTB_GRID_STRIDE(i, n) {
        const int p = (int)param[i];
        const uint32_t x = (uint32_t)a[i];
        const uint32_t sh = kBitsPerCodon * (uint32_t)(p ? p : 1);  // shift 0: the shift-less form, one codon
        const uint32_t lowMask = (1u << (kTotalDnaBits - sh)) - 1u;
        int64_t r = 0;
        switch (fn) {
            case MTB_PIN_SCORE_INCREMENT: r = __float_as_uint(score_fields(x, p, false)); break;
            case MTB_PIN_HAMMING_INCREMENT: r = ham_fields(x, p, false); break;
            case MTB_PIN_IS_CONSECUTIVE: r = consecutive(x, (uint32_t)b[i], sh, lowMask, true, 1); break;
            case MTB_PIN_IS_CONSECUTIVE2: r = consecutive(x, (uint32_t)b[i], sh, lowMask, true, 2); break;
            case MTB_PIN_MATCH_SCORE: r = __float_as_uint(score_fields(x, 8, false)); break;
            case MTB_PIN_RIGHT_PART_SCORE: r = __float_as_uint(score_fields(x, p, false)); break;
            case MTB_PIN_LEFT_PART_SCORE: r = __float_as_uint(score_fields(x, p, true)); break;
            case MTB_PIN_RIGHT_PART_HAMMING: r = ham_fields(x, p, false); break;
            case MTB_PIN_LEFT_PART_HAMMING: r = ham_fields(x, p, true); break;
            case MTB_PIN_MAX_COVERED_LENGTH: r = max_covered_length((int)a[i]); break;
            case MTB_PIN_QUERY_KMER_NUMBER: r = query_kmer_number((int)a[i], p); break;
            default: r = -1;
        }
        out[i] = r;
    }
}

void launch_pin_eval(int fn, const int64_t* param, const uint64_t* a, const uint64_t* b, uint64_t n, int64_t* out,
                     hipStream_t s) {
    if (n) k_pin_eval<<<stride_grid(n), 256, 0, s>>>(fn, param, a, b, n, out);
}

}  // namespace mtb
