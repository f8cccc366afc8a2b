// Device-side helpers of the MI355X classify path: record packing, codon tables, Hamming LUTs.
// Every table here restates the reference's (cited per item); the oracle's copy is pinned
// against the reference's GeneticCode.h (tests/golden/genetic_code.json).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtb_gpu.h"

namespace mtb {

constexpr uint64_t kSentinel = ~0ull;          // blank reserved slot (never a valid metamer)
constexpr uint64_t kAAMask = ~0xFFFFFFull;     // AMINO_ACID_PART (KmerMatcher.h:22)

__host__ __device__ inline uint64_t pack_info(uint32_t seq, uint32_t pos, uint32_t frame) {
    return (uint64_t)pos | ((uint64_t)(seq & 0x1FFFFFFFu) << 32) | ((uint64_t)(frame & 7u) << 61);
}
__host__ __device__ inline uint32_t info_pos(uint64_t x) { return (uint32_t)x; }
__host__ __device__ inline uint32_t info_seq(uint64_t x) { return (uint32_t)((x >> 32) & 0x1FFFFFFFu); }
__host__ __device__ inline uint32_t info_frame(uint64_t x) { return (uint32_t)(x >> 61); }

// K1 slot layout: work unit u owns window p of its chunk at slot (u / 64) * 64C + 64p + u % 64.
// A unit's info (pack_info of its first window) plus the frame's direction gives every window's
// info, so the sort carries 32-bit slots and K4 rebuilds the info of the queries that matched.
// Unit records are 16 B: {pack_info of the unit's first window, the unit's read's slot stretch:
// its first unit (low 40 bits) | its unit count << 40} — the join's segment bounds come with the
// info in one aligned load instead of a second random read of the read's unit offsets.
constexpr uint64_t kStretchLoMask = (1ull << 40) - 1;

__host__ __device__ inline uint64_t unit_info_at(uint64_t ui, uint32_t p, int kmerFormat) {
    const uint32_t frame = (uint32_t)(ui >> 61);
    const bool fromLeft = (kmerFormat == 2) ? frame < 3 : frame >= 3;
    const uint32_t pos = fromLeft ? (uint32_t)ui + 3u * p : (uint32_t)ui - 3u * p;
    return (ui & ~0xFFFFFFFFull) | pos;
}

__host__ __device__ inline uint32_t slot_unit(uint32_t slot, uint32_t C, uint32_t& p) {
    const uint32_t wave = slot / (64u * C), rem = slot - wave * 64u * C;
    p = rem >> 6;
    return wave * 64u + (rem & 63u);
}

__host__ __device__ inline uint64_t slot_info(uint32_t slot, uint32_t C, const uint64_t* unitInfo, int kmerFormat) {
    uint32_t p;
    const uint32_t u = slot_unit(slot, C, p);
    return unit_info_at(unitInfo[2 * (uint64_t)u], p, kmerFormat);
}

// getMaxCoveredLength / getQueryKmerNumber (LocalUtil.h:45-59)
__host__ __device__ inline int max_covered_length(int len) {
    int r = len % 3;
    return r == 2 ? len - 2 : (r == 1 ? len - 4 : len - 3);
}
__host__ __device__ inline int query_kmer_number(int len, int spaceNum = 0, int kLength = 8) {
    return (max_covered_length(len) / 3 - kLength - spaceNum + 1) * 6;
}

// The Taxonomer's codon geometry (Taxonomer.cpp:50-58): 3-bit codons, 24 DNA bits (reduced-AA's
// 4-bit codons are refused).
constexpr uint32_t kBitsPerCodon = 3;
constexpr uint32_t kTotalDnaBits = 24;

// Base byte -> 2-bit code {A:0, C:1, T:2, G:3} or 7 (N / anything else). This is
// nuc2int(atcg[c]) (GeneticCode.h:6, common.cpp:13-17) folded into one 256-entry table; the
// complement of a valid code is code ^ 2 (iRCT, common.cpp:19-23).
struct BaseTable {
    uint8_t code[256];
};

// Codon tables indexed by (b1 << 4 | b2 << 2 | b3) over valid 2-bit codes (GeneticCode.h:33-194):
// aa in [0,20] (20 = stop) and the 3-bit synonymous-codon code. Invalid codons are handled by
// the caller (any base code 7 => AA -1).
struct CodonTable {
    int8_t aa[64];
    int8_t num[64];
};

// hammingLookup (KmerMatcher.h:66-70) packed as 3 bits per entry, one 24-bit row per query codon.
__device__ __forceinline__ uint32_t hamming_lookup_row(uint32_t q) {
    // rows: {0,1,1,1,2,1,3,3} {1,0,1,1,2,2,3,2} {1,1,0,1,2,2,2,3} {1,1,1,0,1,2,3,3}
    //       {2,2,2,1,0,1,4,4} {1,2,2,2,1,0,4,4} {3,3,2,3,4,4,0,1} {3,2,3,3,4,4,1,0}
    constexpr uint32_t R0 = 0u | 1u << 3 | 1u << 6 | 1u << 9 | 2u << 12 | 1u << 15 | 3u << 18 | 3u << 21;
    constexpr uint32_t R1 = 1u | 0u << 3 | 1u << 6 | 1u << 9 | 2u << 12 | 2u << 15 | 3u << 18 | 2u << 21;
    constexpr uint32_t R2 = 1u | 1u << 3 | 0u << 6 | 1u << 9 | 2u << 12 | 2u << 15 | 2u << 18 | 3u << 21;
    constexpr uint32_t R3 = 1u | 1u << 3 | 1u << 6 | 0u << 9 | 1u << 12 | 2u << 15 | 3u << 18 | 3u << 21;
    constexpr uint32_t R4 = 2u | 2u << 3 | 2u << 6 | 1u << 9 | 0u << 12 | 1u << 15 | 4u << 18 | 4u << 21;
    constexpr uint32_t R5 = 1u | 2u << 3 | 2u << 6 | 2u << 9 | 1u << 12 | 0u << 15 | 4u << 18 | 4u << 21;
    constexpr uint32_t R6 = 3u | 3u << 3 | 2u << 6 | 3u << 9 | 4u << 12 | 4u << 15 | 0u << 18 | 1u << 21;
    constexpr uint32_t R7 = 3u | 2u << 3 | 3u << 6 | 3u << 9 | 4u << 12 | 4u << 15 | 1u << 18 | 0u << 21;
    return q == 0 ? R0 : q == 1 ? R1 : q == 2 ? R2 : q == 3 ? R3 : q == 4 ? R4 : q == 5 ? R5 : q == 6 ? R6 : R7;
}

__device__ __forceinline__ uint32_t hamming_lookup(uint32_t q, uint32_t t) {
    return (hamming_lookup_row(q) >> (3 * t)) & 7u;
}

// getHammingDistanceSum (KmerMatcher.h:348-360): sum over the 8 codons of the DNA part.
__device__ __forceinline__ uint32_t hamming_sum(uint64_t a, uint64_t b) {
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += hamming_lookup((uint32_t)(a >> (3 * i)) & 7u, (uint32_t)(b >> (3 * i)) & 7u);
    return s;
}

// The 8 lookup rows of a query k-mer's codons, selected once per query; a candidate's hamming
// sum is then one 3-bit field extract per codon (hamming_sum_rows == hamming_sum).
struct HamRows {
    uint32_t r[8];
};

__device__ __forceinline__ HamRows hamming_rows(uint64_t key) {
    HamRows h;
#pragma unroll
    for (int i = 0; i < 8; i++) h.r[i] = hamming_lookup_row((uint32_t)(key >> (3 * i)) & 7u);
    return h;
}

__device__ __forceinline__ uint32_t hamming_sum_rows(const HamRows& h, uint64_t tv) {
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += (h.r[i] >> (3 * ((uint32_t)(tv >> (3 * i)) & 7u))) & 7u;
    return s;
}

// One 2-bit field of HAMMING_LUT0..7 (KmerMatcher.h:72-158): a distance of 4 is stored as 0,
// except field 7 where query rows 4-5 against target columns 6-7 read 1.
__device__ __forceinline__ uint32_t hamming_field(uint32_t q, uint32_t t, int field) {
    uint32_t h = hamming_lookup(q, t);
    if (field == 7 && (q == 4u || q == 5u) && (t == 6u || t == 7u)) return 1u;
    return h == 4u ? 0u : h;
}

// hammings() from the query's rows: a distance of 4 occurs exactly at (q in 4-5, t in 6-7) and
// (q in 6-7, t in 4-5); field 7 stores the first kind as 1, everything else stores 4 as 0.
__device__ __forceinline__ uint32_t hammings_rows(const HamRows& hr, uint64_t a, uint64_t b, bool reverse) {
    uint32_t h = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t q = (uint32_t)(a >> (3 * i)) & 7u, t = (uint32_t)(b >> (3 * i)) & 7u;
        const uint32_t d = (hr.r[i] >> (3 * t)) & 7u;
        const int field = reverse ? 7 - i : i;
        const uint32_t v = d == 4u ? ((field == 7 && q < 6u) ? 1u : 0u) : d;
        h |= v << (2 * field);
    }
    return h;
}

// getHammings (forward) / getHammings_reverse (KmerMatcher.h:386-416)
__device__ __forceinline__ uint32_t hammings(uint64_t a, uint64_t b, bool reverse) {
    uint32_t h = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t q = (uint32_t)(a >> (3 * i)) & 7u, t = (uint32_t)(b >> (3 * i)) & 7u;
        int field = reverse ? 7 - i : i;
        h |= hamming_field(q, t, field) << (2 * field);
    }
    return h;
}

// Match::getScore and partial scores (Match.h:32-70): 3 for an exact codon, else 2 - 0.5h.
__host__ __device__ inline float codon_score(uint32_t h) { return h == 0 ? 3.0f : 2.0f - 0.5f * (float)h; }

// The score of the first / last `range` codon fields of a rightEndHamming word, summed in the
// reference's order: Match::getScore (range 8), getRightPartScore / getLeftPartScore (Match.h:32-70),
// and Taxonomer::calScoreIncrement (the first `shift` fields, Taxonomer.cpp:650-661).
__host__ __device__ inline float score_fields(uint32_t reh, int range, bool left) {
    float s = 0.0f;
    for (int c = 0; c < range; c++) {
        uint32_t h = left ? (reh >> (14 - 2 * c)) & 3u : (reh >> (2 * c)) & 3u;
        s += codon_score(h);
    }
    return s;
}
// getRightPartHammingDist / getLeftPartHammingDist (Match.h:72-86), calHammingDistIncrement (Taxonomer.cpp:663-669)
__host__ __device__ inline int ham_fields(uint32_t reh, int range, bool left) {
    int s = 0;
    for (int c = 0; c < range; c++) s += (int)(left ? (reh >> (14 - 2 * c)) & 3u : (reh >> (2 * c)) & 3u);
    return s;
}

// isConsecutive / isConsecutive2 (Taxonomer.cpp:677-699) of a current match's DNA encoding (dc) and the
// next's (dn), shifted by sh = 3 * shift bits (lowMask = 2^(24 - sh) - 1); fwd false: the two swapped,
// as getMatchPaths' reverse frames call them (Taxonomer.cpp:600-620). Format 2 -> isConsecutive2.
__host__ __device__ inline bool consecutive(uint32_t dc, uint32_t dn, uint32_t sh, uint32_t lowMask, bool fwd,
                                            int kmerFormat) {
    if (kmerFormat == 2) return fwd ? ((dc & lowMask) == (dn >> sh)) : ((dn & lowMask) == (dc >> sh));
    return fwd ? ((dc >> sh) == (dn & lowMask)) : ((dn >> sh) == (dc & lowMask));
}

// The value of lane ^ J (J = 1..32) without the LDS crossbar (__shfl_xor is a ds_bpermute): DPP
// quad_perm for 1 and 2, row_shl / row_shr for 4, row_ror:8 for 8 (a rotation by half a 16-lane row
// is the xor), and gfx950's v_permlane16_swap / v_permlane32_swap for 16 and 32 (a swap of v with
// itself leaves the other half's value in each lane's [1] (lower half) or [0] (upper half)).
template <int J>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v, int lane) {
    static_assert(J == 1 || J == 2 || J == 4 || J == 8 || J == 16 || J == 32, "a power of two below 64");
    if constexpr (J == 1) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    } else if constexpr (J == 4) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xF, 0xF, false);  // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
        return (lane & 4) ? dn : up;
    } else if constexpr (J == 8) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (J == 16) {
        const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? p[0] : p[1];
    } else {
        const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? p[0] : p[1];
    }
}

// The same for a run-time j (a constant after unrolling: the switch folds away) and 32/64-bit values.
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v, int j, int lane) {
    switch (j) {
        case 1: return xor_lane<1>(v, lane);
        case 2: return xor_lane<2>(v, lane);
        case 4: return xor_lane<4>(v, lane);
        case 8: return xor_lane<8>(v, lane);
        case 16: return xor_lane<16>(v, lane);
        default: return xor_lane<32>(v, lane);
    }
}
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v, int j, int lane) {
    return (uint64_t)xor_lane32((uint32_t)(v >> 32), j, lane) << 32 | xor_lane32((uint32_t)v, j, lane);
}

}  // namespace mtb
