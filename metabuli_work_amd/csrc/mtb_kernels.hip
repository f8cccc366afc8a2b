// HIP kernels of the classify hot path for CDNA4 (gfx950): K1 extract, K2 radix sort,
// K3 diffIdx decode, K4 merge-match. K5/K6 (per-read match sort + assignment) are in
// mtb_assign.hip. All integer/byte work, HBM-bound: no MFMA.
#include "mtb_launch.h"

#include <cstring>

namespace mtb {

// ------------------------------------------------------------------------------------------------
// Block-wide scan helpers (256 threads = 4 wave64)
// ------------------------------------------------------------------------------------------------
constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

__device__ __forceinline__ unsigned long long wave_inclusive_scan(unsigned long long x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// Exclusive scan over the block; returns the exclusive prefix of x, *total = block sum.
__device__ __forceinline__ unsigned long long block_exclusive_scan(unsigned long long x, unsigned long long* total) {
    __shared__ unsigned long long wsum[kWaves];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned long long inc = wave_inclusive_scan(x);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    unsigned long long off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kWaves; i++) {
        if (i < w) off += wsum[i];
        tot += wsum[i];
    }
    __syncthreads();
    *total = tot;
    return off + inc - x;
}

// ------------------------------------------------------------------------------------------------
// Device-wide exclusive scan: out[i] = sum(in[0..i)), out[n] = total. Three launches:
// per-tile sums, scan of tile sums (one block), per-tile scan + carry.
// ------------------------------------------------------------------------------------------------
constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;

template <typename T>
__global__ void k_scan_tiles(const T* __restrict__ in, uint64_t n, unsigned long long* __restrict__ tileSum) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        uint64_t i = base + (uint64_t)k * kBlock + threadIdx.x;
        if (i < n) s += (unsigned long long)in[i];
    }
    unsigned long long tot;
    block_exclusive_scan(s, &tot);
    if (threadIdx.x == 0) tileSum[blockIdx.x] = tot;
}

__global__ void k_scan_tile_sums(unsigned long long* __restrict__ tileSum, uint64_t nTiles) {
    unsigned long long carry = 0;
    for (uint64_t b = 0; b < nTiles; b += kBlock) {
        uint64_t i = b + threadIdx.x;
        unsigned long long x = i < nTiles ? tileSum[i] : 0ull;
        unsigned long long tot;
        unsigned long long ex = block_exclusive_scan(x, &tot);
        if (i < nTiles) tileSum[i] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) tileSum[nTiles] = carry;
}

template <typename T>
__global__ void k_scan_apply(const T* __restrict__ in, uint64_t n, const unsigned long long* __restrict__ tileSum,
                             uint64_t* __restrict__ out) {
    // Thread-contiguous items so each tile is scanned in element order.
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    unsigned long long v[kScanItems];
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        uint64_t i = base + k;
        v[k] = i < n ? (unsigned long long)in[i] : 0ull;
        s += v[k];
    }
    unsigned long long tot;
    unsigned long long run = block_exclusive_scan(s, &tot) + tileSum[blockIdx.x];
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        uint64_t i = base + k;
        if (i < n) out[i] = run;
        run += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kBlock - 1) out[n] = tileSum[gridDim.x];
}

template <typename T>
static void scan_impl(const T* in, uint64_t n, uint64_t* out, unsigned long long* tmp, hipStream_t s) {
    uint64_t tiles = (n + kScanTile - 1) / kScanTile;
    if (tiles == 0) {
        hipMemsetAsync(out, 0, sizeof(uint64_t), s);
        return;
    }
    k_scan_tiles<T><<<(unsigned)tiles, kBlock, 0, s>>>(in, n, tmp);
    k_scan_tile_sums<<<1, kBlock, 0, s>>>(tmp, tiles);
    k_scan_apply<T><<<(unsigned)tiles, kBlock, 0, s>>>(in, n, tmp, out);
}

uint64_t scan_tmp_elems(uint64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

// ------------------------------------------------------------------------------------------------
// K6 run index over the sorted live matches (the loops of Taxonomer.cpp:316-408): a (read, species,
// frame) group starts where the read, species or frame changes, a (read, species) run where the
// read or species changes. Two passes over 8192-match tiles instead of flags + two device scans +
// a start scatter: pass 1 reads the matches once, writes one flag byte per match (bit 0 group,
// bit 1 run) and the tile's two counts packed in one u64 (groups low, runs high: both < 2^32);
// the tile sums are scanned as packed u64; pass 2 reads the bytes (32 per thread, two 16-B loads),
// scans them, and writes gScan/sScan (exclusive counts, u64) through LDS so the stores stay
// coalesced, and each group's / run's first match index. gScan[nM], sScan[nM] = the totals, and
// gStart / sStart end with nM.
// ------------------------------------------------------------------------------------------------
constexpr int kRunItems = 32;
constexpr int kRunTile = kBlock * kRunItems;  // 8192 matches

__global__ void __launch_bounds__(256) k_run_tiles(const mtb_match* __restrict__ M, uint64_t nM,
                                                   uint8_t* __restrict__ flags, unsigned long long* __restrict__ tileSum) {
    const uint64_t base = (uint64_t)blockIdx.x * kRunTile;
    unsigned long long s = 0;
#pragma unroll 8
    for (int k = 0; k < kRunItems; k++) {
        const uint64_t i = base + (uint64_t)k * kBlock + threadIdx.x;
        if (i >= nM) break;
        uint32_t g = 1, sp = 1;
        if (i > 0) {
            const uint64_t qa = M[i - 1].qinfo, qb = M[i].qinfo;
            const bool newSp = info_seq(qa) != info_seq(qb) || M[i - 1].species_id != M[i].species_id;
            sp = newSp;
            g = newSp || info_frame(qa) != info_frame(qb);
        }
        flags[i] = (uint8_t)(g | sp << 1);
        s += (unsigned long long)g | (unsigned long long)sp << 32;
    }
    unsigned long long tot;
    block_exclusive_scan(s, &tot);
    if (threadIdx.x == 0) tileSum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(256) k_run_index(const uint8_t* __restrict__ flags, uint64_t nM,
                                                   const unsigned long long* __restrict__ tileSum,
                                                   uint64_t* __restrict__ gScan, uint64_t* __restrict__ sScan,
                                                   uint64_t* __restrict__ gStart, uint64_t* __restrict__ sStart) {
    __shared__ uint32_t sIdx[kRunTile];  // tile-relative exclusive count of one kind, per match
    __shared__ uint8_t sF[kRunTile];
    const uint64_t base = (uint64_t)blockIdx.x * kRunTile;
    const uint32_t nT = (uint32_t)min<uint64_t>(kRunTile, nM - base);
    const int tid = threadIdx.x;
    // bytes in: coalesced 16-B loads into LDS (the tile is 8192 bytes), then 32 contiguous per thread
    if (nT == kRunTile) {
        const uint4* src = reinterpret_cast<const uint4*>(flags + base);
        uint4* dst = reinterpret_cast<uint4*>(sF);
        for (int x = tid; x < kRunTile / 16; x += kBlock) dst[x] = src[x];
    } else {
        for (uint32_t x = tid; x < nT; x += kBlock) sF[x] = flags[base + x];
    }
    __syncthreads();
    uint32_t f[kRunItems];
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < kRunItems; k++) {
        const uint32_t x = (uint32_t)tid * kRunItems + k;
        f[k] = x < nT ? sF[x] : 0u;
        s += (unsigned long long)(f[k] & 1u) | (unsigned long long)(f[k] >> 1) << 32;
    }
    unsigned long long tot;
    const unsigned long long ex = block_exclusive_scan(s, &tot);
    const unsigned long long tb = tileSum[blockIdx.x];
    const uint64_t gBase = tb & 0xFFFFFFFFull, sBase = tb >> 32;
#pragma unroll
    for (int kind = 0; kind < 2; kind++) {
        uint32_t run = kind ? (uint32_t)(ex >> 32) : (uint32_t)ex;
#pragma unroll
        for (int k = 0; k < kRunItems; k++) {
            sIdx[tid * kRunItems + k] = run;
            run += (f[k] >> kind) & 1u;
        }
        __syncthreads();
        uint64_t* scan = kind ? sScan : gScan;
        uint64_t* start = kind ? sStart : gStart;
        const uint64_t b0 = kind ? sBase : gBase;
        for (uint32_t x = tid; x < nT; x += kBlock) {
            const uint64_t v = b0 + sIdx[x];
            scan[base + x] = v;
            if ((sF[x] >> kind) & 1u) start[v] = base + x;
        }
        __syncthreads();
    }
    if (blockIdx.x == gridDim.x - 1 && tid == 0) {
        const unsigned long long all = tileSum[gridDim.x];
        gScan[nM] = all & 0xFFFFFFFFull;
        sScan[nM] = all >> 32;
        gStart[all & 0xFFFFFFFFull] = nM;
        sStart[all >> 32] = nM;
    }
}

uint64_t run_index_tmp_bytes(uint64_t nM) { return 8 * ((nM + kRunTile - 1) / kRunTile + 2); }

void launch_run_index(const mtb_match* M, uint64_t nM, uint8_t* flags, unsigned long long* tileSum, uint64_t* gScan,
                      uint64_t* sScan, uint64_t* gStart, uint64_t* sStart, hipStream_t s) {
    if (nM == 0) return;
    const uint64_t tiles = (nM + kRunTile - 1) / kRunTile;
    k_run_tiles<<<(unsigned)tiles, kBlock, 0, s>>>(M, nM, flags, tileSum);
    k_scan_tile_sums<<<1, kBlock, 0, s>>>(tileSum, tiles);
    k_run_index<<<(unsigned)tiles, kBlock, 0, s>>>(flags, nM, tileSum, gScan, sScan, gStart, sStart);
}
void exclusive_scan_u32(const uint32_t* in, uint64_t n, uint64_t* out, void* tmp, hipStream_t s) {
    scan_impl<uint32_t>(in, n, out, (unsigned long long*)tmp, s);
}
void exclusive_scan_u64(const uint64_t* in, uint64_t n, uint64_t* out, void* tmp, hipStream_t s) {
    scan_impl<uint64_t>(in, n, out, (unsigned long long*)tmp, s);
}

// ------------------------------------------------------------------------------------------------
// K0 read metadata: loadChunkOfReads (KmerExtractor.cpp:442-494). Per read: covered lengths and
// windows per frame of each mate (0 when the read is dropped by the shared empty rule); the batch
// maximum sizes K1's chunks.
// ------------------------------------------------------------------------------------------------
__global__ void k_read_meta(const uint64_t* __restrict__ off1, const uint64_t* __restrict__ off2, uint32_t n,
                            int paired, ReadMeta* __restrict__ meta, uint32_t* __restrict__ qlen,
                            uint32_t* __restrict__ maxW, uint32_t* __restrict__ readLens) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int len1 = (int)(off1[i + 1] - off1[i]);
    int ql1 = max_covered_length(len1);
    int w1 = query_kmer_number(len1) / 6;  // windows per frame (KmerExtractor.cpp:462,481)
    int len2 = 0, ql2 = 0, w2 = 0;
    bool empty = w1 < 1;
    if (paired) {
        len2 = (int)(off2[i + 1] - off2[i]);
        ql2 = max_covered_length(len2);
        w2 = query_kmer_number(len2) / 6;
        if (w2 < 1) empty = true;
    }
    ReadMeta m;
    m.len1 = len1; m.len2 = len2; m.ql1 = ql1; m.ql2 = ql2;
    m.w1 = empty ? 0 : w1;
    m.w2 = (empty || !paired) ? 0 : w2;
    meta[i] = m;
    qlen[i] = (uint32_t)(ql1 + ql2);
    // the mates' lengths in 16 bits each (K4 rebuilds a uniform unit's info from them; read only when
    // every frame is one chunk, i.e. reads of a few hundred bases)
    readLens[i] = (uint32_t)min(len1, 0xFFFF) | (uint32_t)min(len2, 0xFFFF) << 16;
    const uint32_t w = (uint32_t)max(m.w1, m.w2);
    if (w) atomicMax(maxW, w);
}

// K1 work units per read: each (mate, frame) is cut into chunks of C windows. Uniform units (upr > 0:
// every frame of the batch fits one chunk): every read gets upr = 6 per mate units, a read whose mate
// is too short included (its units hold no window), so unit u is read u / upr's (mate, frame)
// u % upr and K4 needs no unit record (unit_windows, k_match).
__global__ void k_read_units(const ReadMeta* __restrict__ meta, uint32_t n, uint32_t C, uint32_t upr,
                             uint32_t* __restrict__ units) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ReadMeta m = meta[i];
    units[i] = upr ? upr : 6u * ((uint32_t)(m.w1 + C - 1) / C + (uint32_t)(m.w2 + C - 1) / C);
}

__global__ void k_unit_read(const uint64_t* __restrict__ uOff, uint32_t n, uint32_t* __restrict__ unitRead) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (uint64_t u = uOff[i]; u < uOff[i + 1]; u++) unitRead[u] = i;
}

void launch_read_meta(const uint64_t* off1, const uint64_t* off2, uint32_t n, int paired, ReadMeta* meta,
                      uint32_t* qlen, uint32_t* maxW, uint32_t* readLens, hipStream_t s) {
    hipMemsetAsync(maxW, 0, sizeof(uint32_t), s);
    if (n == 0) return;
    k_read_meta<<<(n + 255) / 256, 256, 0, s>>>(off1, off2, n, paired, meta, qlen, maxW, readLens);
}

void launch_read_units(const ReadMeta* meta, uint32_t n, uint32_t C, uint32_t upr, uint32_t* units, hipStream_t s) {
    if (n) k_read_units<<<(n + 255) / 256, 256, 0, s>>>(meta, n, C, upr, units);
}

void launch_unit_read(const uint64_t* uOff, uint32_t n, uint32_t* unitRead, hipStream_t s) {
    if (n) k_unit_read<<<(n + 255) / 256, 256, 0, s>>>(uOff, n, unitRead);
}

// ------------------------------------------------------------------------------------------------
// K1 extract (fillQueryKmerBuffer, KmerExtractor.cpp:355-386): one thread per work unit = a chunk
// of C consecutive windows of one (read, mate, frame). It loads the chunk's codons plus the 7
// before its first window's last codon (a window depends on its own 8 codons only) and writes
// window p of the chunk to slot (unit / 64) * 64C + 64p + unit % 64: the 64 lanes of a wave
// store 64 consecutive slots per window step, so every store is one coalesced line. Pre-sort
// slot order is free (K2 reorders everything) and slots past a chunk's windows get the sentinel.
// A window
// is emitted iff its 8 codons translate (the N-restart of MetamerScanner::next,
// KmerScanner.h:82-117) and, with syncmers, its earliest-minimum s-mer sits at either end
// (SyncmerScanner::next, SyncmerScanner.h:36-102). Blank windows get the sentinel key, which
// the first radix pass drops.
//
// Load order j of a frame's codons: format 2 reads left to right (forward) or from the right end
// on the complement (reverse); format 1 (OldMetamerScanner, KmerScanner.h:137-181) reads the
// forward frame from the right end and the reverse frame from the left end, both with the first
// loaded codon most significant.
// ------------------------------------------------------------------------------------------------
struct ExtractTables {
    uint8_t base[256];
    int8_t aa[64];
    int8_t num[64];
};

// One K1 work unit: a chunk of <= C consecutive windows of one (read, mate, frame).
struct UnitWindows {
    const uint8_t* seq;
    int s0, e0;          // covered span of the frame (first / last base)
    int pFirst, nWin;    // first window of the chunk, windows in the chunk (0: nothing to do)
    bool fromLeft, comp;
    uint64_t info0;      // pack_info of the chunk's first window (window p: pos0 +- 3p, slot_info)
    uint64_t stretch;    // the read's first unit | its unit count << 40 (mtb_device.h)
};

__device__ __forceinline__ UnitWindows unit_windows(uint64_t u, uint64_t nUnits, uint32_t C,
                                                    const uint8_t* __restrict__ seq1, const uint64_t* __restrict__ off1,
                                                    const uint8_t* __restrict__ seq2, const uint64_t* __restrict__ off2,
                                                    const ReadMeta* __restrict__ meta, const uint64_t* __restrict__ uOff,
                                                    const uint32_t* __restrict__ unitRead, int kmerFormat,
                                                    uint32_t upr) {
    UnitWindows w{};
    if (u >= nUnits) return w;
    const uint32_t r = upr ? (uint32_t)(u / upr) : unitRead[u];
    const ReadMeta m = meta[r];
    const uint64_t first = upr ? (uint64_t)r * upr : uOff[r];
    w.stretch = first | (upr ? (uint64_t)upr : uOff[r + 1] - first) << 40;
    uint32_t local = (uint32_t)(u - first);
    // uniform units: one chunk per (mate, frame), windows or not (k_read_units)
    const uint32_t c1 = upr ? 1u : (uint32_t)(m.w1 + C - 1) / C, c2 = upr ? 1u : (uint32_t)(m.w2 + C - 1) / C;
    uint32_t cpf = c1;
    int mate = 0;
    if (local >= 6 * c1) { local -= 6 * c1; mate = 1; cpf = c2; }
    const int frame = (int)(local / cpf);
    const int chunk = (int)(local % cpf);
    const int W = mate ? m.w2 : m.w1;
    w.pFirst = chunk * (int)C;
    w.nWin = min((int)C, W - w.pFirst);
    if (w.nWin <= 0) return w;
    w.seq = mate ? seq2 + off2[r] : seq1 + off1[r];
    const int len = mate ? m.len2 : m.len1;
    const int used = mate ? m.ql2 : m.ql1;
    const uint32_t posOffset = mate ? (uint32_t)m.ql1 + 3u : 0u;  // KmerExtractor.cpp:341-345
    const bool fwd = frame < 3;
    int begin;
    if (fwd) begin = frame;
    else { begin = (len % 3) - (frame % 3); if (begin < 0) begin += 3; }
    w.s0 = begin;
    w.e0 = begin + used - 1;
    // which end the load order starts from, and whether codons are complemented
    w.fromLeft = (kmerFormat == 2) ? fwd : !fwd;
    w.comp = !fwd;
    const uint32_t pos0 = w.fromLeft ? (uint32_t)(w.s0 + 3 * w.pFirst) : (uint32_t)(w.e0 - 3 * (w.pFirst + 8) + 1);
    w.info0 = pack_info(r + 1, pos0 + posOffset, (uint32_t)frame);
    return w;
}

// The unit's windows one at a time: the scanner state of MetamerScanner / OldMetamerScanner /
// SyncmerScanner over the unit's codons in load order (the chunk's first window needs the 7
// codons before its last one: loaded by the constructor). next(): the next window's emission and
// its resident rank-form key (AA rank << 24 | DNA part; kSentinel when not emitted).
struct WinScanner {
    const UnitWindows& w;
    const uint8_t* seq;  // the unit's mate: w.seq in HBM, or its copy in the block's LDS stage (K1F)
    const uint8_t* sBase;
    const int8_t *sAA, *sNum;
    int syncmer, nSm;
    uint64_t smMask;
    uint64_t aaAcc = 0, dnaAcc = 0, smAcc = 0;
    uint64_t sm0 = 0, sm1 = 0, sm2 = 0, sm3 = 0, sm4 = 0, sm5 = 0, sm6 = 0, sm7 = 0;
    int run = 0, j;
    // the last window's rank split for the link lines: its first seven AAs' rank, first and last AA
    uint32_t first7 = 0, firstAA = 0, lastAA = 0;

    __device__ __forceinline__ WinScanner(const UnitWindows& w_, const uint8_t* b, const int8_t* a, const int8_t* n,
                                          int sync, int smerLen, const uint8_t* seqAt)
        : w(w_), seq(seqAt), sBase(b), sAA(a), sNum(n), syncmer(sync), nSm(8 - smerLen + 1),
          smMask((smerLen >= 13) ? ~0ull : ((1ull << (5 * smerLen)) - 1)), j(w_.pFirst) {
        if (w.nWin > 0)
            for (int k = 0; k < 7; k++) codon();
    }
    __device__ __forceinline__ void codon() {
        // branch-free (selects only): the loads of a codon sit in one basic block, so the wait before them
        // is for them alone, not a conservative drain of every load in flight (the K1F probes)
        const int d = w.fromLeft ? 1 : -1;
        const int c0 = w.fromLeft ? w.s0 + 3 * j : w.e0 - 3 * j;  // first base of the triplet in load order
        const uint32_t x = sBase[seq[c0]], y = sBase[seq[c0 + d]], z = sBase[seq[c0 + 2 * d]];
        // load order x, y, z is the codon's for a forward read from the left or a reverse one from the
        // right; the other two cases read it backwards
        const bool back = w.fromLeft == w.comp;
        const uint32_t cm = w.comp ? 2u : 0u;  // complement of a valid code (iRCT)
        const uint32_t b1 = (back ? z : x) ^ cm, b2 = y ^ cm, b3 = (back ? x : z) ^ cm;
        const bool valid = ((x | y | z) < 4u);
        const int idx = (int)(((b1 << 4) | (b2 << 2) | b3) & 63u);
        const int aaT = sAA[idx], numT = sNum[idx];
        const int aa = valid ? aaT : -1, num = valid ? numT : 0;
        const bool ok = aa >= 0;
        run = ok ? run + 1 : 0;
        aaAcc = ok ? (aaAcc << 5) | (uint64_t)aa : aaAcc;
        dnaAcc = ok ? (dnaAcc << 3) | (uint64_t)num : dnaAcc;
        smAcc = ok ? ((smAcc << 5) | (uint64_t)aa) & smMask : smAcc;
        if (syncmer) {
            sm7 = sm6; sm6 = sm5; sm5 = sm4; sm4 = sm3; sm3 = sm2; sm2 = sm1; sm1 = sm0; sm0 = smAcc;
        }
        j++;
    }
    __device__ __forceinline__ uint64_t next() {
        codon();
        bool ok = run >= 8;
        if (ok && syncmer) {
            // s-mers of the window: positions p..p+nSm-1 end at codons j-nSm+1..j = sm[nSm-1]..sm0.
            // Earliest minimum: scan from the oldest (k = nSm-1) to the newest with strict <.
            const uint64_t sv[8] = {sm0, sm1, sm2, sm3, sm4, sm5, sm6, sm7};
            int bestK = -1;
            uint64_t best = ~0ull;
#pragma unroll
            for (int k = 7; k >= 0; k--) {
                if (k <= nSm - 1 && sv[k] < best) { best = sv[k]; bestK = k; }
            }
            ok = (bestK == nSm - 1) || (bestK == 0);
        }
        if (!ok) return kSentinel;
        // both formats' resident key: base-21 rank of the 8 AA codes (to_rank_form)
        uint64_t aaPart = 0;
#pragma unroll
        for (int k = 7; k >= 1; k--) aaPart = aaPart * 21 + ((aaAcc >> (5 * k)) & 31u);
        first7 = (uint32_t)aaPart;
        lastAA = (uint32_t)(aaAcc & 31u);
        firstAA = (uint32_t)((aaAcc >> 35) & 31u);
        aaPart = aaPart * 21 + lastAA;
        return (aaPart << 24) | (dnaAcc & 0xFFFFFFull);
    }
};

// The unit's windows in order: f(p, ok, key) for p = 0 .. nWin-1 (p relative to the chunk).
template <typename F>
__device__ __forceinline__ void unit_scan(const UnitWindows& w, const uint8_t* sBase, const int8_t* sAA,
                                          const int8_t* sNum, int syncmer, int smerLen, F&& f) {
    WinScanner sc(w, sBase, sAA, sNum, syncmer, smerLen, w.seq);
    for (int p = 0; p < w.nWin; p++) {
        const uint64_t key = sc.next();
        f(p, key != kSentinel, key);
    }
}

__device__ __forceinline__ void load_extract_tables(const ExtractTables& tabs, uint8_t* sBase, int8_t* sAA,
                                                    int8_t* sNum) {
    sBase[threadIdx.x] = tabs.base[threadIdx.x];
    if (threadIdx.x < 64) { sAA[threadIdx.x] = tabs.aa[threadIdx.x]; sNum[threadIdx.x] = tabs.num[threadIdx.x]; }
    __syncthreads();
}

// The AA-membership word and bit of a rank in the probe lines.
__device__ __forceinline__ const uint32_t* line_word(const ProbeLine* lines, uint64_t rank, uint32_t& bit) {
    const uint64_t L = rank / kLineRanks;
    const uint32_t o = (uint32_t)(rank - L * kLineRanks);
    bit = o & 31u;
    return &lines[L].bits[o >> 5];
}

// DB index of the first k-mer of AA rank x, or below it: the line's base plus the present ranks
// before x in the line (each holds >= 1 DB k-mer). One 64-B line read.
__device__ __forceinline__ uint64_t line_lower_bound_at(const ProbeLine* line, uint32_t o) {
    const uint4* lp = reinterpret_cast<const uint4*>(line);
    const uint4 q0 = lp[0], q1 = lp[1], q2 = lp[2], q3 = lp[3];
    const uint32_t w[14] = {q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    uint32_t before = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        const uint32_t wi = (uint32_t)i;
        const uint32_t m = wi < (o >> 5) ? ~0u : (wi == (o >> 5) ? ((1u << (o & 31u)) - 1u) : 0u);
        before += __popc(w[i] & m);
    }
    return (((uint64_t)q0.x | (uint64_t)q0.y << 32) & ((1ull << 40) - 1)) + before;
}

// One line read for the run index: the head word; the present ranks before rank o of the line,
// in the whole line, and whether o itself is present.
__device__ __forceinline__ uint64_t line_scan(const ProbeLine* line, uint32_t o, uint32_t& before, uint32_t& total,
                                              bool& present) {
    const uint4* lp = reinterpret_cast<const uint4*>(line);
    const uint4 q0 = lp[0], q1 = lp[1], q2 = lp[2], q3 = lp[3];
    const uint32_t w[14] = {q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    before = 0;
    total = 0;
    uint32_t at = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        const uint32_t wi = (uint32_t)i;
        const uint32_t m = wi < (o >> 5) ? ~0u : (wi == (o >> 5) ? ((1u << (o & 31u)) - 1u) : 0u);
        before += __popc(w[i] & m);
        total += __popc(w[i]);
        if (wi == (o >> 5)) at = w[i];
    }
    present = (at >> (o & 31u)) & 1u;
    return (uint64_t)q0.x | (uint64_t)q0.y << 32;
}

__device__ __forceinline__ uint64_t line_lower_bound(const ProbeLine* __restrict__ lines, uint64_t x) {
    const uint64_t L = x / kLineRanks;
    return line_lower_bound_at(lines + L, (uint32_t)(x - L * kLineRanks));
}

// First index >= lo with a[i] >= key (an answer exists below D + kDbPad: the pad is ~0).
// Read views of the resident DB records (value / taxID by index), so one search code serves LDS
// windows (plain arrays) and the records in HBM.
struct DbVal {
    const DbRec* __restrict__ r;
    __device__ __forceinline__ uint64_t operator[](uint64_t i) const { return (uint64_t)r[i].hi << 32 | r[i].lo; }
};
struct DbTax {
    const DbRec* __restrict__ r;
    __device__ __forceinline__ uint32_t operator[](uint64_t i) const { return r[i].tax; }
};
template <typename A>
__device__ __forceinline__ uint64_t gallop_lower(const A& a, uint64_t lo, uint64_t key);
template <typename A>
__device__ __forceinline__ uint64_t gallop_lower1(const A& a, uint64_t lo, uint64_t key);

__global__ void __launch_bounds__(256) k_extract(const uint8_t* __restrict__ seq1, const uint64_t* __restrict__ off1,
                                                 const uint8_t* __restrict__ seq2, const uint64_t* __restrict__ off2,
                                                 const ReadMeta* __restrict__ meta, const uint64_t* __restrict__ uOff,
                                                 const uint32_t* __restrict__ unitRead, uint64_t nUnits, uint32_t C,
                                                 ExtractTables tabs, int kmerFormat, int syncmer, int smerLen,
                                                 uint64_t* __restrict__ keys, uint64_t* __restrict__ unitInfo,
                                                 uint32_t upr) {
    __shared__ uint8_t sBase[256];
    __shared__ int8_t sAA[64], sNum[64];
    load_extract_tables(tabs, sBase, sAA, sNum);
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t slotBase = (u >> 6) * 64ull * C + (u & 63u);
    const UnitWindows w = unit_windows(u, nUnits, C, seq1, off1, seq2, off2, meta, uOff, unitRead, kmerFormat, upr);
    // slots of this unit past its windows (and of padding units) hold the sentinel
    for (int p = max(w.nWin, 0); p < (int)C; p++) keys[slotBase + 64ull * p] = kSentinel;
    if (w.nWin <= 0) return;
    reinterpret_cast<ulonglong2*>(unitInfo)[u] = make_ulonglong2(w.info0, w.stretch);
    unit_scan(w, sBase, sAA, sNum, syncmer, smerLen,
              [&](int p, bool ok, uint64_t key) { keys[slotBase + 64ull * p] = ok ? key : kSentinel; });
}

uint64_t extract_slots(uint64_t nUnits, uint32_t C) { return (nUnits + 63) / 64 * 64 * C; }

static ExtractTables extract_tables(const HostTables& t) {
    ExtractTables tabs;
    for (int i = 0; i < 256; i++) tabs.base[i] = t.base[i];
    for (int i = 0; i < 64; i++) { tabs.aa[i] = t.aa[i]; tabs.num[i] = t.num[i]; }
    return tabs;
}

void launch_extract(const uint8_t* seq1, const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2,
                    const ReadMeta* meta, const uint64_t* uOff, const uint32_t* unitRead, uint64_t nUnits,
                    uint32_t C, const HostTables& t, int kmerFormat, int syncmer, int smerLen, uint64_t* keys,
                    uint64_t* unitInfo, hipStream_t s, uint32_t upr) {
    if (nUnits == 0) return;
    const uint64_t threads = (nUnits + 63) / 64 * 64;  // whole waves: padding units write sentinels
    k_extract<<<(unsigned)((threads + 255) / 256), 256, 0, s>>>(seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits,
                                                                C, extract_tables(t), kmerFormat, syncmer, smerLen,
                                                                keys, unitInfo, upr);
}

// ------------------------------------------------------------------------------------------------
// K2 LSD radix sort of (key, val) pairs on 8-bit digits of the key. Per pass: tile histograms
// (digit-major so one device scan yields stable global offsets), scan, stable scatter through an
// LDS-staged tile so each digit run leaves the block as one contiguous write. Each wave ranks its
// own 2048-key slice against a wave-private histogram (from per-digit lane masks, or match-any
// ballots), so the tile needs two block barriers per pass rather than several per 256 keys. The first pass (FILTER) drops
// sentinel keys: the compaction of blank reserved slots costs nothing extra.
// ------------------------------------------------------------------------------------------------
constexpr int kRadixItems = 32;
constexpr int kRadixTile = kBlock * kRadixItems;  // 8192 keys

// one 32-bit bit-field extract from the word holding the digit (shift is wave-uniform), not a 64-bit shift
__device__ __forceinline__ uint32_t radix_digit(uint64_t k, int shift) {
    if (shift >= 32) return __builtin_amdgcn_ubfe((uint32_t)(k >> 32), (uint32_t)(shift - 32), 8u);
    if (shift <= 24) return __builtin_amdgcn_ubfe((uint32_t)k, (uint32_t)shift, 8u);
    return (uint32_t)((k >> shift) & 0xFF);
}

template <int TILE>
__device__ __forceinline__ void radix_tile_span(const uint64_t* __restrict__ tab, uint32_t tile, uint64_t n,
                                                uint64_t& base, uint64_t& end);

template <bool FILTER, int TILE = kRadixTile>
__global__ void __launch_bounds__(256) k_radix_hist(const uint64_t* __restrict__ keys, uint64_t n, int shift,
                                                    uint32_t* __restrict__ counts, uint32_t nTiles,
                                                    const uint64_t* __restrict__ tab = nullptr) {
    __shared__ uint32_t hist[256];
    hist[threadIdx.x] = 0;
    __syncthreads();
    constexpr int kItems = TILE / kBlock;
    uint64_t base;
    radix_tile_span<TILE>(tab, blockIdx.x, n, base, n);
    uint64_t key[kItems];
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        const uint64_t i = base + (uint64_t)k * kBlock + threadIdx.x;
        key[k] = i < n ? keys[i] : kSentinel;
    }
#pragma unroll
    for (int k = 0; k < kItems; k++) {
        const uint64_t i = base + (uint64_t)k * kBlock + threadIdx.x;
        if (i < n && (!FILTER || key[k] != kSentinel)) atomicAdd(&hist[radix_digit(key[k], shift)], 1u);
    }
    __syncthreads();
    counts[(uint64_t)threadIdx.x * nTiles + blockIdx.x] = hist[threadIdx.x];
}

// The same histogram from a byte array of the pass's digits (written by the previous pass's scatter,
// or by the fused K1F for the first): 1 B read per key instead of 8.
// tab (nullable): tile t is [tab[t] >> 14, + (tab[t] & 0x3FFF)) instead of [t * kRadixTile, ...) up to n
// (the buckets of a binned K1F; starts are multiples of 16).
template <int TILE>
__device__ __forceinline__ void radix_tile_span(const uint64_t* __restrict__ tab, uint32_t tile, uint64_t n,
                                                uint64_t& base, uint64_t& end) {
    if (tab) {
        const uint64_t e = tab[tile];
        base = e >> 14;
        end = base + (e & 0x3FFFu);
    } else {
        base = (uint64_t)tile * TILE;
        end = n;
    }
}

template <int TILE = kRadixTile>
__global__ void __launch_bounds__(256) k_radix_hist_dig(const uint8_t* __restrict__ dig, uint64_t n,
                                                        uint32_t* __restrict__ counts, uint32_t nTiles,
                                                        const uint64_t* __restrict__ tab) {
    __shared__ uint32_t hist[256];
    hist[threadIdx.x] = 0;
    __syncthreads();
    uint64_t base, end;
    radix_tile_span<TILE>(tab, blockIdx.x, n, base, end);
    n = end;
    constexpr int kVec = TILE / kBlock / 16;  // uint4 loads per thread
    uint4 d[kVec];
    const bool full = base + TILE <= n;
#pragma unroll
    for (int k = 0; k < kVec; k++) {
        const uint64_t i = base + ((uint64_t)k * kBlock + threadIdx.x) * 16;
        d[k] = full ? reinterpret_cast<const uint4*>(dig + base)[k * kBlock + threadIdx.x] : make_uint4(0, 0, 0, 0);
        if (!full) {
            uint32_t w[4] = {0, 0, 0, 0};
            for (int b = 0; b < 16; b++)
                if (i + b < n) w[b >> 2] |= (uint32_t)dig[i + b] << (8 * (b & 3));
            d[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
#pragma unroll
    for (int k = 0; k < kVec; k++) {
        const uint64_t i = base + ((uint64_t)k * kBlock + threadIdx.x) * 16;
        const uint32_t w[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
#pragma unroll
        for (int b = 0; b < 16; b++)
            if (full || i + b < n) atomicAdd(&hist[(w[b >> 2] >> (8 * (b & 3))) & 0xFFu], 1u);
    }
    __syncthreads();
    counts[(uint64_t)threadIdx.x * nTiles + blockIdx.x] = hist[threadIdx.x];
}

// V: value type (64-bit payloads, or 32-bit slot indices). GEN: the values are the input positions
// (the first pass of a sort of slots), so none are read. digOut (nullable): the next pass's digit
// (bits [nextShift, nextShift + 8) of the key) of every written key, at its output position.
template <typename V, bool FILTER, bool GEN, int TILE = kRadixTile>
__global__ void __launch_bounds__(256) k_radix_scatter(const uint64_t* __restrict__ keysIn, const V* __restrict__ valsIn,
                                                       uint64_t n, int shift, const uint64_t* __restrict__ offs,
                                                       uint32_t nTiles, uint64_t* __restrict__ keysOut,
                                                       V* __restrict__ valsOut, uint8_t* __restrict__ digOut,
                                                       int nextShift, int xcdMap, const uint64_t* __restrict__ tab,
                                                       int atomicRank) {
    constexpr int kItems = TILE / kBlock, kSlice = 64 * kItems;
    __shared__ uint64_t sKV[TILE];  // keys, then (after they are written out) values
    __shared__ uint8_t sDig[TILE];
    __shared__ uint32_t waveHist[kWaves][256];
    __shared__ uint64_t sDst[256];  // global slot of this tile's first key of digit d, minus its tile offset
    __shared__ uint32_t sKept;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // XCD-aware tiles: blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one), so block b
    // takes tile (b mod 8)'s share start + b / 8: each XCD walks one contiguous eighth of the tiles in
    // order, and the digit-d runs of consecutive tiles — adjacent in the output — are written through
    // the same L2, which completes the lines a run leaves partial instead of two XCDs each writing
    // part of a line (speed only: any mapping is correct)
    uint32_t tile = blockIdx.x;
    if (xcdMap) {
        const uint32_t x = blockIdx.x & 7u, i = blockIdx.x >> 3, q = nTiles >> 3, r = nTiles & 7u;
        tile = x * q + min(x, r) + i;
    }
    uint64_t tBase, tEnd;
    radix_tile_span<TILE>(tab, tile, n, tBase, tEnd);
    n = tEnd;
    const uint64_t base = tBase + (uint64_t)w * kSlice;
    // the digit bases: one strided load per lane, issued first so its latency hides behind the
    // key loads (a dependent load per key in the write-out loop was the old bottleneck)
    const uint64_t digitBase = offs[(uint64_t)tid * nTiles + tile];
    for (int x = tid; x < kWaves * 256; x += kBlock) (&waveHist[0][0])[x] = 0;
    if (atomicRank & 4)
        for (int x = tid; x < kWaves * 256; x += kBlock) sKV[x] = 0;  // the digits' lane masks (below)
    __syncthreads();

    const unsigned long long ltMask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint64_t k[kItems];
    V v[kItems];
    uint32_t rk[kItems];  // digit << 16 | rank within this wave's slice; ~0 = not kept
    // all loads first (unguarded for the full tiles) so the 32 loads of a lane are in flight
    // together; interleaving them with the ranking serialised 16 memory round trips per tile
    if (tBase + TILE <= n) {
#pragma unroll
        for (int r = 0; r < kItems; r++) k[r] = keysIn[base + (uint64_t)r * 64 + lane];
#pragma unroll
        for (int r = 0; r < kItems; r++)
            v[r] = GEN ? (V)(base + (uint64_t)r * 64 + lane) : valsIn[base + (uint64_t)r * 64 + lane];
    } else {
#pragma unroll
        for (int r = 0; r < kItems; r++) {
            const uint64_t i = base + (uint64_t)r * 64 + lane;
            k[r] = i < n ? keysIn[i] : kSentinel;
            v[r] = GEN ? (V)i : (i < n ? valsIn[i] : (V)0);
        }
    }
    // atomicRank (an LSD sort's first pass, when its input order need not be kept): each key's rank
    // in its wave's slice from one LDS atomic on the wave's histogram — the order among a wave
    // instruction's lanes of one digit is the hardware's, so later passes, which must be stable,
    // keep the 8-ballot ranking (all three passes atomic: sort 15.8 -> 13.1-14.1 ms, but stability
    // would then rest on an undocumented lane order; profiles/r05/ab_radixatomic_allpasses.json). The
    // first pass alone measured even (ab_radixatomic_first.json): off by default (MTB_RADIX_ATOMIC_FIRST).
    // atomicRank & 4 (the default): the lane-mask ranking below, stable by construction, in place of the
    // nine ballots (sort 14.8 -> 14.2-14.3 ms same box, profiles/r05/ab_radix_orrank.json)
    if (atomicRank & 1) {
#pragma unroll
        for (int r = 0; r < kItems; r++) {
            const uint64_t i = base + (uint64_t)r * 64 + lane;
            const bool valid = i < n && (!FILTER || k[r] != kSentinel);
            const uint32_t d = valid ? radix_digit(k[r], shift) : 0u;
            rk[r] = valid ? (d << 16 | atomicAdd(&waveHist[w][d], 1u)) : ~0u;
        }
    } else if (atomicRank & 4) {
        // stable ranking from each digit's lane mask (sKV holds the masks until the keys are staged):
        // every lane ORs its bit into its digit's word — the result does not depend on the order the
        // lanes' ORs land in — and reads the word back (LDS operations of one wave complete in program
        // order); the digit's lowest lane advances the count and clears the word for the next key
        unsigned long long* sMask = reinterpret_cast<unsigned long long*>(sKV) + w * 256;
        // a full tile without sentinels (every tile of a sort but its last): no per-key validity
        // (MTB_RADIX_FULLTILE=0 for the A/B)
        if (!FILTER && !(atomicRank & 2) && tBase + TILE <= n) {
#pragma unroll
            for (int r = 0; r < kItems; r++) {
                const uint32_t d = radix_digit(k[r], shift);
                __hip_atomic_fetch_or(&sMask[d], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const unsigned long long peers = __hip_atomic_load(&sMask[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const uint32_t before = waveHist[w][d];
                const uint32_t rankInWave = (uint32_t)__popcll(peers & ltMask);
                if (rankInWave == 0) {
                    waveHist[w][d] = before + (uint32_t)__popcll(peers);
                    __hip_atomic_store(&sMask[d], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                rk[r] = d << 16 | (before + rankInWave);
            }
        } else
#pragma unroll
        for (int r = 0; r < kItems; r++) {
            const uint64_t i = base + (uint64_t)r * 64 + lane;
            const bool valid = i < n && (!FILTER || k[r] != kSentinel);
            const uint32_t d = valid ? radix_digit(k[r], shift) : 0u;
            if (valid) __hip_atomic_fetch_or(&sMask[d], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const unsigned long long peers =
                valid ? __hip_atomic_load(&sMask[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : 0ull;
            const uint32_t before = valid ? waveHist[w][d] : 0u;
            const uint32_t rankInWave = (uint32_t)__popcll(peers & ltMask);
            if (valid && rankInWave == 0) {
                waveHist[w][d] = before + (uint32_t)__popcll(peers);
                __hip_atomic_store(&sMask[d], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            rk[r] = valid ? (d << 16 | (before + rankInWave)) : ~0u;
        }
    } else if (!FILTER && !(atomicRank & 2) && tBase + TILE <= n) {
        // a full tile without sentinels (every tile of a sort but its last): every key is valid, so
        // the ranking drops the per-key bound checks and the validity terms of its nine ballots
#pragma unroll
        for (int r = 0; r < kItems; r++) {
            const uint32_t d = radix_digit(k[r], shift);
            unsigned long long peers = ~0ull;
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const unsigned long long m = __ballot((d >> b) & 1u);
                peers &= ((d >> b) & 1u) ? m : ~m;
            }
            const uint32_t before = waveHist[w][d];
            const uint32_t rankInWave = (uint32_t)__popcll(peers & ltMask);
            if (rankInWave == 0) waveHist[w][d] = before + (uint32_t)__popcll(peers);
            rk[r] = d << 16 | (before + rankInWave);
        }
    } else
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        const uint64_t i = base + (uint64_t)r * 64 + lane;
        const bool valid = i < n && (!FILTER || k[r] != kSentinel);
        const uint32_t d = valid ? radix_digit(k[r], shift) : 0u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            unsigned long long m = __ballot(valid && ((d >> b) & 1u));
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        // every peer reads the running count before the group's first lane advances it; LDS
        // operations of one wave complete in program order
        const uint32_t before = valid ? waveHist[w][d] : 0u;
        const uint32_t rankInWave = (uint32_t)__popcll(peers & ltMask);
        if (valid && rankInWave == 0) waveHist[w][d] = before + (uint32_t)__popcll(peers);
        rk[r] = valid ? (d << 16 | (before + rankInWave)) : ~0u;
    }
    __syncthreads();
    {
        uint32_t c[kWaves], sum = 0;
#pragma unroll
        for (int ww = 0; ww < kWaves; ww++) { c[ww] = waveHist[ww][tid]; sum += c[ww]; }
        unsigned long long tot;
        const uint32_t start = (uint32_t)block_exclusive_scan(sum, &tot);
        sDst[tid] = digitBase - start;
        if (tid == 0) sKept = (uint32_t)tot;
        uint32_t run = start;
#pragma unroll
        for (int ww = 0; ww < kWaves; ww++) { waveHist[ww][tid] = run; run += c[ww]; }
    }
    __syncthreads();
    // keys and values go through one LDS tile in two rounds (half the LDS of staging both, so
    // twice the resident blocks per CU to hide the ranking's dependency chains)
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        if (rk[r] == ~0u) continue;
        const uint32_t d = rk[r] >> 16;
        rk[r] = waveHist[w][d] + (rk[r] & 0xFFFFu);  // now the tile position
        sKV[rk[r]] = k[r];
        sDig[rk[r]] = (uint8_t)d;
    }
    __syncthreads();
    if (digOut) {
        for (uint32_t i = tid; i < sKept; i += kBlock) {
            const uint64_t o = sDst[sDig[i]] + i;
            keysOut[o] = sKV[i];
            digOut[o] = (uint8_t)radix_digit(sKV[i], nextShift);
        }
    } else {
        for (uint32_t i = tid; i < sKept; i += kBlock) keysOut[sDst[sDig[i]] + i] = sKV[i];
    }
    __syncthreads();
    V* sV = reinterpret_cast<V*>(sKV);
#pragma unroll
    for (int r = 0; r < kItems; r++)
        if (rk[r] != ~0u) sV[rk[r]] = v[r];
    __syncthreads();
    for (uint32_t i = tid; i < sKept; i += kBlock) valsOut[sDst[sDig[i]] + i] = sV[i];
}

// sized for the smallest tile radix_sort_pairs may take (MTB_RADIX_TILE=4096)
uint64_t radix_counts_elems(uint64_t n) { return 256ull * ((n + 4095) / 4096) + 1; }

// MTB_RADIX_TILE=4096 (A/B, read per sort): 4096-key tiles, 16 keys per lane (42 KB of LDS per block
// instead of 78: three resident blocks per CU instead of two), twice the tiles and histogram counts
static uint32_t radix_tile() {
    const char* e = getenv("MTB_RADIX_TILE");
    return e && atoi(e) == 4096 ? 4096u : (uint32_t)kRadixTile;
}


// Sorts n pairs by key bits [bitLo, bitHi). Returns the kept count (sentinels dropped when
// filter). Result ends in (keysA, valsA) if the number of passes is even, else in (keysB, valsB);
// *inB tells which. genVals: valsA is not read; the values are the input positions.
// every pass ranked from the digits' lane masks (default: profiles/r05/ab_radix_orrank.json);
// MTB_RADIX_ORRANK=0 (A/B, read per sort) ranks by the nine ballots
static int radix_or_rank() {
    const char* e = getenv("MTB_RADIX_ORRANK");
    return !e || atoi(e) ? 4 : 0;
}

template <typename V>
uint64_t radix_sort_pairs(uint64_t* keysA, V* valsA, uint64_t* keysB, V* valsB, uint64_t n, int bitLo, int bitHi,
                          bool filter, bool genVals, uint32_t* counts, uint64_t* offs, void* scanTmp, bool* inB,
                          hipStream_t s, uint8_t* digA, uint8_t* digB, bool unstableFirst) {
    uint64_t cur = n;
    uint64_t *ki = keysA, *ko = keysB;
    V *vi = valsA, *vo = valsB;
    uint8_t *di = digA, *dg = digB;  // digit side arrays: digA holds the first pass's digits (no filter)
    const bool digits = digA && digB && !filter;
    bool first = true;
    *inB = false;
    const uint32_t T = radix_tile();
    for (int shift = bitLo; shift < bitHi; shift += 8) {
        uint32_t nTiles = (uint32_t)((cur + T - 1) / T);
        if (nTiles == 0) break;
        const bool f = first && filter, g = first && genVals;
        if (T == 4096) {
            if (digits) k_radix_hist_dig<4096><<<nTiles, kBlock, 0, s>>>(di, cur, counts, nTiles, nullptr);
            else if (f) k_radix_hist<true, 4096><<<nTiles, kBlock, 0, s>>>(ki, cur, shift, counts, nTiles);
            else k_radix_hist<false, 4096><<<nTiles, kBlock, 0, s>>>(ki, cur, shift, counts, nTiles);
        } else if (digits) k_radix_hist_dig<<<nTiles, kBlock, 0, s>>>(di, cur, counts, nTiles, nullptr);
        else if (f) k_radix_hist<true><<<nTiles, kBlock, 0, s>>>(ki, cur, shift, counts, nTiles);
        else k_radix_hist<false><<<nTiles, kBlock, 0, s>>>(ki, cur, shift, counts, nTiles);
        exclusive_scan_u32(counts, 256ull * nTiles, offs, scanTmp, s);
        uint8_t* dOut = digits && shift + 8 < bitHi ? dg : nullptr;
        // MTB_RADIX_XCD=0 (A/B, read per sort): tiles in block order instead of one contiguous eighth per XCD
        const char* xe = getenv("MTB_RADIX_XCD");
        const int xcd = xe ? atoi(xe) : 1;
        const int ns = shift + 8;
        // MTB_RADIX_FULLTILE=0 (A/B, read per sort): full tiles ranked by the general path too
        const char* fe = getenv("MTB_RADIX_FULLTILE");
        const int ar = (first && unstableFirst ? 1 : 0) | (fe && atoi(fe) == 0 ? 2 : 0) | radix_or_rank();
        if (T == 4096) {
            if (f && g) k_radix_scatter<V, true, true, 4096><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
            else if (f) k_radix_scatter<V, true, false, 4096><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
            else if (g) k_radix_scatter<V, false, true, 4096><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
            else k_radix_scatter<V, false, false, 4096><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
        } else if (f && g) k_radix_scatter<V, true, true><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
        else if (f) k_radix_scatter<V, true, false><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
        else if (g) k_radix_scatter<V, false, true><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
        else k_radix_scatter<V, false, false><<<nTiles, kBlock, 0, s>>>(ki, vi, cur, shift, offs, nTiles, ko, vo, dOut, ns, xcd, nullptr, ar);
        std::swap(di, dg);
        if (f) {
            uint64_t kept = 0;
            hipMemcpyAsync(&kept, offs + 256ull * nTiles, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
            hipStreamSynchronize(s);
            cur = kept;
        }
        first = false;
        std::swap(ki, ko);
        std::swap(vi, vo);
        *inB = !*inB;
    }
    return cur;
}

// The tile table of a binned K1F's buckets (radix_sort_binned): one block, thread t walks digit t's 8
// regions (t * 8 .. t * 8 + 7: the regions in digit order), its tile count scanned over the block.
__global__ void __launch_bounds__(256) k_bin_tiles(const unsigned long long* __restrict__ binCnt, uint64_t rc,
                                                   uint64_t* __restrict__ tab) {
    uint64_t cnt[8], nt = 0;
#pragma unroll
    for (int x = 0; x < 8; x++) {
        cnt[x] = min((uint64_t)binCnt[threadIdx.x * 8 + x], rc);
        nt += (cnt[x] + kRadixTile - 1) / kRadixTile;
    }
    unsigned long long tot;
    uint64_t o = block_exclusive_scan(nt, &tot);
#pragma unroll
    for (int x = 0; x < 8; x++) {
        const uint64_t r0 = (uint64_t)(threadIdx.x * 8 + x) * rc;
        for (uint64_t i = 0; i < cnt[x]; i += kRadixTile) tab[o++] = (r0 + i) << 14 | min<uint64_t>(kRadixTile, cnt[x] - i);
    }
}

uint64_t radix_binned_tiles(const uint64_t* binHost, uint64_t rc) {
    uint64_t nt = 0;
    for (int r = 0; r < kSortBins; r++) nt += (std::min<uint64_t>(binHost[r], rc) + kRadixTile - 1) / kRadixTile;
    return nt;
}

template <typename V>
uint64_t radix_sort_binned(uint64_t* keysR, V* valsR, uint64_t* keysT, V* valsT, const uint64_t* binHost,
                           const unsigned long long* binDev, uint64_t rc, int bitLo, int bitHi, uint32_t* counts,
                           uint64_t* offs, void* scanTmp, uint64_t* tileTab, bool* inT, hipStream_t s, uint8_t* digR,
                           uint8_t* digT) {
    static_assert(kRadixTile < (1 << 14), "tile length in 14 bits");
    uint64_t Q = 0;
    for (int r = 0; r < kSortBins; r++) Q += binHost[r];
    const uint32_t nTiles = (uint32_t)radix_binned_tiles(binHost, rc);
    *inT = false;
    if (!nTiles) return Q;
    if (bitLo + 8 >= bitHi) {
        // one pass in all: K1F's buckets are already the sorted order, but gapped (bucket r at r * rc);
        // pack them into (keysT, valsT) slots [0, Q) as the caller reads them (never taken with
        // kQuerySortLo/Hi, which need three passes)
        uint64_t o = 0;
        for (int r = 0; r < kSortBins; r++) {
            const uint64_t n = std::min<uint64_t>(binHost[r], rc);
            if (!n) continue;
            hipMemcpyAsync(keysT + o, keysR + (uint64_t)r * rc, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, s);
            hipMemcpyAsync(valsT + o, valsR + (uint64_t)r * rc, n * sizeof(V), hipMemcpyDeviceToDevice, s);
            o += n;
        }
        *inT = true;
        return o;
    }
    // the second pass (bits bitLo + 8 ..) over the buckets in order -> (keysT, valsT) from slot 0
    k_bin_tiles<<<1, kBlock, 0, s>>>(binDev, rc, tileTab);
    const int shift = bitLo + 8, ns = shift + 8;
    if (digR) k_radix_hist_dig<<<nTiles, kBlock, 0, s>>>(digR, 0, counts, nTiles, tileTab);
    else k_radix_hist<false><<<nTiles, kBlock, 0, s>>>(keysR, 0, shift, counts, nTiles, tileTab);  // no K1F digits
    exclusive_scan_u32(counts, 256ull * nTiles, offs, scanTmp, s);
    const char* xe = getenv("MTB_RADIX_XCD");
    const int xcd = xe ? atoi(xe) : 1;
    k_radix_scatter<V, false, false><<<nTiles, kBlock, 0, s>>>(keysR, valsR, 0, shift, offs, nTiles, keysT, valsT,
                                                              ns < bitHi ? digT : nullptr, ns, xcd, tileTab,
                                                              radix_or_rank());
    *inT = true;
    if (ns < bitHi) {  // the rest: plain passes over the Q contiguous pairs
        bool inB = false;
        // (without K1F digits, digR is null: one remaining pass never writes the second digit array)
        uint8_t* dOther = digR ? digR : (ns + 8 >= bitHi ? digT : nullptr);
        radix_sort_pairs(keysT, valsT, keysR, valsR, Q, ns, bitHi, false, false, counts, offs, scanTmp, &inB, s, digT,
                         dOther);
        *inT = !inB;
    }
    return Q;
}

template uint64_t radix_sort_binned<uint32_t>(uint64_t*, uint32_t*, uint64_t*, uint32_t*, const uint64_t*,
                                              const unsigned long long*, uint64_t, int, int, uint32_t*, uint64_t*,
                                              void*, uint64_t*, bool*, hipStream_t, uint8_t*, uint8_t*);

template uint64_t radix_sort_pairs<uint64_t>(uint64_t*, uint64_t*, uint64_t*, uint64_t*, uint64_t, int, int, bool, bool,
                                             uint32_t*, uint64_t*, void*, bool*, hipStream_t, uint8_t*, uint8_t*, bool);
template uint64_t radix_sort_pairs<uint32_t>(uint64_t*, uint32_t*, uint64_t*, uint32_t*, uint64_t, int, int, bool, bool,
                                             uint32_t*, uint64_t*, void*, bool*, hipStream_t, uint8_t*, uint8_t*, bool);

// ------------------------------------------------------------------------------------------------
// K3 diffIdx decode (getNextTargetKmer, KmerMatcher.h:282-297) at DB open: terminator flags ->
// k-mer index by scan -> per-k-mer delta from its <= 5 15-bit groups -> values by 64-bit scan.
// ------------------------------------------------------------------------------------------------
__global__ void k_term_flags(const uint16_t* __restrict__ diff, uint64_t n, uint32_t* __restrict__ flag) {
    MTB_GRID_STRIDE(i, n) flag[i] = (diff[i] & 0x8000u) ? 1u : 0u;
}

__global__ void k_deltas(const uint16_t* __restrict__ diff, uint64_t n, const uint64_t* __restrict__ termIdx,
                         uint64_t* __restrict__ delta) {
    MTB_GRID_STRIDE(i, n) {
        if (!(diff[i] & 0x8000u)) continue;
        uint64_t d = diff[i] & 0x7FFFu;
        int sh = 15;
        for (uint64_t j = i; j > 0; j--) {
            uint16_t w = diff[j - 1];
            if (w & 0x8000u) break;
            d |= (uint64_t)w << sh;
            sh += 15;
        }
        delta[termIdx[i]] = d;
    }
}

__global__ void k_last_term(const uint32_t* __restrict__ flag, const uint64_t* __restrict__ idx, uint64_t n,
                            uint64_t last, uint64_t* __restrict__ out) {
    MTB_GRID_STRIDE(i, n) if (flag[i] && idx[i] == last) *out = i;
}

__global__ void k_add_carry(uint64_t* v, uint64_t carry) { v[0] += carry; }

// One chunk of diffIdx words that starts at a k-mer's first word: the values of the chunk's whole
// k-mers (their count is returned) continue from carry, the last value of the chunk before; a k-mer
// cut by the chunk's end is left to the next chunk, which starts at the word after *lastTerm (the
// chunk index of the last terminator). idxTmp: n + 2 u64; scanTmp: scan_tmp_elems(n) u64.
uint64_t decode_diff_chunk(const uint16_t* diff, uint64_t n, uint64_t carry, uint64_t* values, uint32_t* flagTmp,
                           uint64_t* idxTmp, void* scanTmp, uint64_t* lastTerm, uint64_t* lastValue, hipStream_t s) {
    *lastTerm = 0;
    if (n == 0) return 0;
    k_term_flags<<<stride_grid(n), 256, 0, s>>>(diff, n, flagTmp);
    exclusive_scan_u32(flagTmp, n, idxTmp, scanTmp, s);
    uint64_t terms = 0;
    hipMemcpyAsync(&terms, idxTmp + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (terms == 0) return 0;
    k_last_term<<<stride_grid(n), 256, 0, s>>>(flagTmp, idxTmp, n, terms - 1, idxTmp + n + 1);
    k_deltas<<<stride_grid(n), 256, 0, s>>>(diff, n, idxTmp, values);
    if (carry) k_add_carry<<<1, 1, 0, s>>>(values, carry);
    hipMemcpyAsync(lastTerm, idxTmp + n + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    // inclusive scan of deltas = exclusive scan shifted by one: scan into idxTmp then take [1..]
    exclusive_scan_u64(values, terms, idxTmp, scanTmp, s);
    hipMemcpyAsync(values, idxTmp + 1, terms * sizeof(uint64_t), hipMemcpyDeviceToDevice, s);
    hipMemcpyAsync(lastValue, values + terms - 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    return terms;
}

// ------------------------------------------------------------------------------------------------
// K4 merge-match (KmerMatcher::matchKmers, KmerMatcher.cpp:275-450; compareDna :1117-1146).
// The reference streams the whole diffIdx DB past each sorted query split. Here the decoded DB
// stays resident and a prefix directory built at open (below) maps the first L amino acids of a
// k-mer to its DB bucket, so each query finds its AA run with one directory read plus a short
// binary search inside the bucket. Candidates are the whole run except the DB's last k-mer (the
// reference's reader stops at diffIdxPos == numOfDiffIdx before loading it,
// KmerMatcher.cpp:363,378). Selected = hamming sum <= min(2*min, 7). COUNT pass: per-read match
// counts. EMIT pass: records into per-read segments.
// ------------------------------------------------------------------------------------------------
template <typename A>
__device__ __forceinline__ uint64_t lower_bound_u64(const A& a, uint64_t lo, uint64_t hi, uint64_t key) {
    while (lo < hi) {
        uint64_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// AA-prefix bucket of a resident k-mer: keys and DB values are held in rank form (the AA part is
// the base-21 rank of the 8 AA codes, see to_rank_form), so the first L AAs are rank / 21^(8-L).
__device__ __forceinline__ uint64_t aa_bucket(uint64_t v, const AADir& d) { return (v >> 24) / d.div; }

// Smallest k-mer value in bucket b.
__device__ __forceinline__ uint64_t aa_bucket_floor(uint64_t b, const AADir& d) { return (b * d.div) << 24; }

// Format 2 packs the 8 AA codes (0..20) as 5-bit fields; the resident form replaces that AA part
// with its base-21 rank (what format 1 stores already). The map is monotone, so sorted stays
// sorted, and the 24-bit DNA part, all the hamming and path code reads, is untouched; the AA part
// becomes 36 dense bits (fewer radix passes, plain division for the directory).
__host__ __device__ inline uint64_t to_rank_form(uint64_t v) {
    const uint64_t aa = v >> 24;
    uint64_t r = 0;
    for (int i = 7; i >= 0; i--) r = r * 21 + ((aa >> (5 * i)) & 31u);
    return (r << 24) | (v & 0xFFFFFFull);
}

__host__ __device__ inline uint64_t from_rank_form(uint64_t v) {
    uint64_t r = v >> 24, aa = 0;
    for (int i = 0; i < 8; i++) {
        aa |= (r % 21) << (5 * i);
        r /= 21;
    }
    return (aa << 24) | (v & 0xFFFFFFull);
}

__global__ void k_to_rank_form(uint64_t* __restrict__ v, uint64_t n) {
    MTB_GRID_STRIDE(i, n) v[i] = to_rank_form(v[i]);
}

__global__ void k_pack_db(const uint64_t* __restrict__ v, const uint32_t* __restrict__ tax, uint64_t n,
                          DbRec* __restrict__ out) {
    MTB_GRID_STRIDE(i, n) out[i] = DbRec{(uint32_t)v[i], (uint32_t)(v[i] >> 32), tax[i]};
}

__global__ void k_rec_rank_form(DbRec* __restrict__ db, uint64_t n) {
    MTB_GRID_STRIDE(i, n) {
        const uint64_t x = to_rank_form((uint64_t)db[i].hi << 32 | db[i].lo);
        db[i].lo = (uint32_t)x;
        db[i].hi = (uint32_t)(x >> 32);
    }
}

__global__ void k_rec_mask_info(DbRec* __restrict__ db, uint64_t n, uint32_t mask) {
    MTB_GRID_STRIDE(i, n) db[i].tax &= mask;
}

void launch_pack_db(const uint64_t* v, const uint32_t* tax, uint64_t n, DbRec* out, hipStream_t s) {
    if (n) k_pack_db<<<stride_grid(n), 256, 0, s>>>(v, tax, n, out);
}
void launch_rec_rank_form(DbRec* db, uint64_t n, hipStream_t s) {
    if (n) k_rec_rank_form<<<stride_grid(n), 256, 0, s>>>(db, n);
}
void launch_rec_mask_info(DbRec* db, uint64_t n, uint32_t mask, hipStream_t s) {
    // Skip_redundancy 1 (modern DBs) keeps every bit: nothing to do (a 12G-record pass was 50 ms)
    if (n && mask != ~0u) k_rec_mask_info<<<stride_grid(n), 256, 0, s>>>(db, n, mask);
}

void launch_to_rank_form(uint64_t* v, uint64_t n, hipStream_t s) {
    if (n) k_to_rank_form<<<stride_grid(n), 256, 0, s>>>(v, n);
}

uint64_t host_from_rank_form(uint64_t v) { return from_rank_form(v); }

__global__ void k_build_dir(const DbRec* __restrict__ db, uint64_t D, AADir d, uint64_t* __restrict__ dir) {
    const DbVal dbv{db};
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b > d.R) return;
    dir[b] = (b == d.R) ? D : lower_bound_u64(dbv, 0, D, aa_bucket_floor(b, d));
}

AADir make_aa_dir(uint64_t D, int kmerFormat) {
    AADir d{};
    d.fmt = kmerFormat;
    d.L = 1;
    uint64_t R = 21;
    while (d.L < 7 && R * 21 * 8 <= D) { R *= 21; d.L++; }
    d.R = R;
    d.div = 1;
    for (int i = d.L; i < 8; i++) d.div *= 21;
    return d;
}

void build_aa_dir(const DbRec* db, uint64_t D, const AADir& d, uint64_t* dir, hipStream_t s) {
    k_build_dir<<<(unsigned)((d.R + 1 + 255) / 256), 256, 0, s>>>(db, D, d, dir);
}

// Line heads: the DB index of the first k-mer of rank >= the line's first rank (lower bound inside
// the directory bucket of that rank); the end line holds D.
__global__ void k_line_base(const DbRec* __restrict__ db, uint64_t D, AADir d, ProbeLine* __restrict__ lines) {
    const DbVal dbv{db};
    const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= kProbeLines) return;
    const uint64_t r = l * kLineRanks;
    uint64_t base = D;
    if (r < kAARankEnd) {
        const uint64_t b = r / d.div;
        base = lower_bound_u64(dbv, d.dir[b], d.dir[b + 1], r << 24);
    }
    lines[l].base = base;
}

// Line heads as base | min(k-mers of the line, 2^24 - 1) << 40 (the probe bounds its searches
// with the count; a saturated count sends it to the next line's head).
__global__ void k_line_count(ProbeLine* __restrict__ lines) {
    const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l + 1 >= kProbeLines) return;
    // the next head may already carry its count (another thread's write): its low 40 bits do not change
    const uint64_t b = lines[l].base, n = (lines[l + 1].base & ((1ull << 40) - 1)) - b;
    lines[l].base = b | (min(n, (uint64_t)0xFFFFFFu) << 40);
}

// Membership bits: the first k-mer of each AA run sets its rank's bit.
__global__ void k_line_bits(const DbRec* __restrict__ db, uint64_t D, ProbeLine* __restrict__ lines) {
    const DbVal dbv{db};
    MTB_GRID_STRIDE(i, D) {
        const uint64_t r = dbv[i] >> 24;
        if (i > 0 && (dbv[i - 1] >> 24) == r) continue;
        uint32_t bit;
        const uint32_t* w = line_word(lines, r, bit);
        atomicOr(const_cast<uint32_t*>(w), 1u << bit);
    }
}

// The same bits a wave per line, with no global atomics: the line's DB records [base, next base)
// are read coalesced (consecutive lines are consecutive record ranges), each run start ORs its bit
// into the wave's 14 LDS words, and the wave stores the line's words once. k_line_bits above made
// one random global atomicOr per present AA rank (10.2G at GTDB scale: 361 ms).
constexpr int kLineWords = (int)(kLineRanks / 32);
__global__ void __launch_bounds__(256) k_line_bits_wave(const DbRec* __restrict__ db, uint64_t D,
                                                        ProbeLine* __restrict__ lines) {
    __shared__ uint32_t sW[4][kLineWords];
    const DbVal dbv{db};
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    for (uint64_t L = (uint64_t)blockIdx.x * 4 + wv; L < kProbeLines; L += (uint64_t)gridDim.x * 4) {
        if (lane < kLineWords) sW[wv][lane] = 0;
        const uint64_t b = lines[L].base & ((1ull << 40) - 1);
        const uint64_t e = L + 1 < kProbeLines ? lines[L + 1].base & ((1ull << 40) - 1) : D;
        const uint64_t r0 = L * kLineRanks;
        for (uint64_t i0 = b; i0 < e; i0 += 64) {
            const uint64_t i = i0 + lane;
            const uint64_t r = i < e ? dbv[i] >> 24 : ~0ull;
            // the previous record's rank: the lane below's, or (lane 0) the record before the chunk
            uint64_t prev = __shfl_up(r, 1, 64);
            if (lane == 0) prev = i > 0 ? dbv[i - 1] >> 24 : ~0ull;
            if (i < e && (i == 0 || prev != r)) {
                const uint32_t o = (uint32_t)(r - r0);
                atomicOr(&sW[wv][o >> 5], 1u << (o & 31u));
            }
        }
        // the wave's LDS writes are complete in program order; every lane reads its word after them
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        if (lane < kLineWords) lines[L].bits[lane] = sW[wv][lane];
        __builtin_amdgcn_wave_barrier();
    }
}

// Run index a wave per line too: the line's words in registers, each run start's present-rank
// index inside the line from the words' popcounts, its run start written at lineP[L] + that index.
__global__ void __launch_bounds__(256) k_run_offsets_wave(const DbRec* __restrict__ db, uint64_t D,
                                                          const ProbeLine* __restrict__ lines,
                                                          const uint64_t* __restrict__ lineP,
                                                          uint16_t* __restrict__ runOff) {
    __shared__ uint32_t sPre[4][kLineWords];  // present ranks in the line's words before word k
    __shared__ uint32_t sW[4][kLineWords];
    const DbVal dbv{db};
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    for (uint64_t L = (uint64_t)blockIdx.x * 4 + wv; L < kProbeLines; L += (uint64_t)gridDim.x * 4) {
        const uint64_t head = lines[L].base;
        const uint64_t b = head & ((1ull << 40) - 1);
        const uint64_t e = L + 1 < kProbeLines ? lines[L + 1].base & ((1ull << 40) - 1) : D;
        if ((head >> 40) > kRunIdxMax || e <= b) continue;  // not indexed (its queries gallop), or empty
        const uint32_t w = lane < kLineWords ? lines[L].bits[lane] : 0u;
        const uint32_t pc = (uint32_t)__popc(w);
        uint32_t inc = pc;  // inclusive scan of the word popcounts over lanes 0..13
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        if (lane < kLineWords) {
            sPre[wv][lane] = inc - pc;
            sW[wv][lane] = w;
        }
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        const uint64_t r0 = L * kLineRanks, p0 = lineP[L];
        for (uint64_t i0 = b; i0 < e; i0 += 64) {
            const uint64_t i = i0 + lane;
            const uint64_t r = i < e ? dbv[i] >> 24 : ~0ull;
            uint64_t prev = __shfl_up(r, 1, 64);
            if (lane == 0) prev = i > 0 ? dbv[i - 1] >> 24 : ~0ull;
            if (i < e && (i == 0 || prev != r)) {
                const uint32_t o = (uint32_t)(r - r0), k = o >> 5;
                const uint32_t before = sPre[wv][k] + (uint32_t)__popc(sW[wv][k] & ((1u << (o & 31u)) - 1u));
                runOff[p0 + before] = (uint16_t)(i - b);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

static unsigned line_wave_grid() { return (unsigned)std::min<uint64_t>((kProbeLines + 3) / 4, 1u << 20); }

// A present rank's run from its line's run-length codes xw (kExtRanks / 16 words): the codes' sum over
// the ranks before it (sum: its run start minus the line's base, minus before) and its own code (run
// length - 1); false when an escape (3) lies at or before it (the caller reads runOff instead).
__device__ __forceinline__ bool ext_run(const uint32_t* xw, uint32_t before, uint32_t& sum, uint32_t& code) {
    const uint32_t wq = before >> 4, f = before & 15u;
    uint32_t esc = 0;
    sum = 0;
    code = 0;
#pragma unroll
    for (uint32_t i = 0; i < kExtRanks / 16; i++) {
        const uint32_t w = xw[i];
        const uint32_t mLt = i < wq ? ~0u : (i == wq ? (1u << (2 * f)) - 1u : 0u);
        const uint32_t mLe = i < wq ? ~0u : (i == wq ? (f == 15u ? ~0u : (1u << (2 * f + 2)) - 1u) : 0u);
        const uint32_t wl = w & mLt, we = w & mLe;
        sum += (uint32_t)__popc(wl & 0x55555555u) + 2u * (uint32_t)__popc(wl & 0xAAAAAAAAu);
        esc |= we & (we >> 1) & 0x55555555u;
        if (i == wq) code = (w >> (2 * f)) & 3u;
    }
    return esc == 0;
}

// ext_run in a rolled loop over the words up to the rank's own (the wave join: fewer live registers)
__device__ __forceinline__ bool ext_run_rolled(const uint32_t* xw, uint32_t before, uint32_t& sum, uint32_t& code) {
    const uint32_t wq = before >> 4, f = before & 15u;
    uint32_t esc = 0, acc = 0;
#pragma nounroll
    for (uint32_t i = 0; i < wq; i++) {
        const uint32_t w = xw[i];
        acc += (uint32_t)__popc(w & 0x55555555u) + 2u * (uint32_t)__popc(w & 0xAAAAAAAAu);
        esc |= w & (w >> 1) & 0x55555555u;
    }
    const uint32_t w = xw[wq];
    const uint32_t mLt = (1u << (2 * f)) - 1u, mLe = f == 15u ? ~0u : (1u << (2 * f + 2)) - 1u;
    const uint32_t wl = w & mLt, we = w & mLe;
    sum = acc + (uint32_t)__popc(wl & 0x55555555u) + 2u * (uint32_t)__popc(wl & 0xAAAAAAAAu);
    esc |= we & (we >> 1) & 0x55555555u;
    code = (w >> (2 * f)) & 3u;
    return esc == 0;
}

// Every present rank of every indexed line against the run index (mtb_line_ext_check): out[0] the
// ranks within the run-length lines' reach, out[1] those they resolve, out[2] mismatches.
__global__ void __launch_bounds__(256) k_line_ext_check(const ProbeLine* __restrict__ lines, const uint64_t* __restrict__ lineP,
                                                        const uint16_t* __restrict__ runOff, const ProbeExt* __restrict__ ext,
                                                        unsigned long long* __restrict__ out) {
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    unsigned long long n = 0, ok = 0, bad = 0;
    for (uint64_t L = (uint64_t)blockIdx.x * 4 + wv; L + 1 < kProbeLines; L += (uint64_t)gridDim.x * 4) {
        const uint64_t cnt = lines[L].base >> 40, p0 = lineP[L];
        const uint32_t pc = (uint32_t)(lineP[L + 1] - p0);
        if (cnt > kRunIdxMax) continue;
        for (uint32_t k = (uint32_t)lane; k < min(pc, kExtRanks); k += 64) {
            n++;
            uint32_t sum, code;
            if (!ext_run(ext[L].w, k, sum, code)) continue;
            ok++;
            const uint32_t a = runOff[p0 + k], b = k + 1 < pc ? runOff[p0 + k + 1] : (uint32_t)cnt;
            bad += (k + sum != a || code + 1 != b - a) ? 1ull : 0ull;
        }
    }
    for (int d = 32; d > 0; d >>= 1) {
        n += __shfl_xor(n, d, 64);
        ok += __shfl_xor(ok, d, 64);
        bad += __shfl_xor(bad, d, 64);
    }
    if (lane == 0) {
        atomicAdd(out, n);
        atomicAdd(out + 1, ok);
        atomicAdd(out + 2, bad);
    }
}

void launch_line_ext_check(const ProbeLine* lines, const uint64_t* lineP, const uint16_t* runOff, const ProbeExt* ext,
                           unsigned long long* out, hipStream_t s) {
    k_line_ext_check<<<line_wave_grid(), 256, 0, s>>>(lines, lineP, runOff, ext, out);
}

// Run-length lines, a wave per line: lane l codes present ranks 4l .. 4l + 3 of the line from their
// run-index entries (the next rank's start, or the line's k-mer count for its last) into one byte.
__global__ void __launch_bounds__(256) k_line_ext(const ProbeLine* __restrict__ lines, const uint64_t* __restrict__ lineP,
                                                  const uint16_t* __restrict__ runOff, ProbeExt* __restrict__ ext) {
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    for (uint64_t L = (uint64_t)blockIdx.x * 4 + wv; L < kProbeLines; L += (uint64_t)gridDim.x * 4) {
        const uint64_t cnt = lines[L].base >> 40;
        const uint64_t p0 = lineP[L];
        const uint32_t pc = (uint32_t)(L + 1 < kProbeLines ? lineP[L + 1] - p0 : 0);
        uint32_t byte = 0xFFu;  // escapes: a line the run index does not cover
        if (cnt <= kRunIdxMax) {
            byte = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t k = 4u * (uint32_t)lane + (uint32_t)j;
                if (k >= pc) break;
                const uint32_t a = runOff[p0 + k], b = k + 1 < pc ? runOff[p0 + k + 1] : (uint32_t)cnt;
                byte |= min(b - a - 1u, 3u) << (2 * j);
            }
        }
        reinterpret_cast<uint8_t*>(ext + L)[lane] = (uint8_t)byte;
    }
}

void build_line_ext(const ProbeLine* lines, const uint64_t* lineP, const uint16_t* runOff, ProbeExt* ext,
                    hipStream_t s) {
    static_assert(kExtRanks == 4 * 64, "a byte of four codes per lane");
    k_line_ext<<<line_wave_grid(), 256, 0, s>>>(lines, lineP, runOff, ext);
}

static bool line_atomic_build() {  // MTB_LINE_BUILD=atomic (A/B): the per-k-mer atomic kernels
    const char* e = getenv("MTB_LINE_BUILD");
    return e && !strcmp(e, "atomic");
}

void build_probe_lines(const DbRec* db, uint64_t D, const AADir& dir, ProbeLine* lines, hipStream_t s) {
    k_line_base<<<(unsigned)((kProbeLines + 255) / 256), 256, 0, s>>>(db, D, dir, lines);
    k_line_count<<<(unsigned)((kProbeLines + 255) / 256), 256, 0, s>>>(lines);
    if (!D) return;
    if (line_atomic_build()) k_line_bits<<<stride_grid(D), 256, 0, s>>>(db, D, lines);
    else k_line_bits_wave<<<line_wave_grid(), 256, 0, s>>>(db, D, lines);
}

// Run index: the exact DB run of every present AA rank, for the unstaged K4 (a DB much larger than
// the query stream). lineP[L] = present ranks in the lines before L (exclusive scan of the lines'
// popcounts); runOff[lineP[L] + k] = DB index of the first k-mer of line L's k-th present rank
// minus the line's base. A query then finds its run [lo, hi) with one random 2-B read (two adjacent
// entries) instead of galloping from the line's lower bound through the DB values, a chain of
// dependent random reads. Lines of more than kRunIdxMax k-mers are not indexed: their queries
// gallop as before.
__global__ void k_line_pop(const ProbeLine* __restrict__ lines, uint32_t* __restrict__ pop) {
    const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= kProbeLines) return;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < (int)(kLineRanks / 32); i++) c += __popc(lines[l].bits[i]);
    pop[l] = c;
}

__global__ void k_run_offsets(const DbRec* __restrict__ db, uint64_t D, const ProbeLine* __restrict__ lines,
                              const uint64_t* __restrict__ lineP, uint16_t* __restrict__ runOff) {
    const DbVal dbv{db};
    MTB_GRID_STRIDE(i, D) {
        const uint64_t r = dbv[i] >> 24;
        if (i > 0 && (dbv[i - 1] >> 24) == r) continue;
        const uint64_t L = r / kLineRanks;
        const uint32_t o = (uint32_t)(r - L * kLineRanks);
        const uint64_t head = lines[L].base;
        if ((head >> 40) > kRunIdxMax) continue;
        const uint64_t before = line_lower_bound_at(lines + L, o) - (head & ((1ull << 40) - 1));
        runOff[lineP[L] + before] = (uint16_t)(i - (head & ((1ull << 40) - 1)));
    }
}

void build_line_prefix(const ProbeLine* lines, uint64_t* lineP, uint32_t* popTmp, void* scanTmp, hipStream_t s) {
    k_line_pop<<<(unsigned)((kProbeLines + 255) / 256), 256, 0, s>>>(lines, popTmp);
    exclusive_scan_u32(popTmp, kProbeLines, lineP, scanTmp, s);
}

// Bit r of the probe lines' membership bitmap.
__device__ __forceinline__ uint32_t probe_bit(const ProbeLine* __restrict__ lines, uint64_t r) {
    const uint64_t L = r / kLineRanks;
    const uint32_t o = (uint32_t)(r - L * kLineRanks);
    return (lines[L].bits[o >> 5] >> (o & 31u)) & 1u;
}

// One thread per AA 7-mer S: its 21 right extensions (ranks 21 S .. 21 S + 20, consecutive) and its 21
// left extensions (ranks x 21^7 + S: for each x the wave's lanes read consecutive ranks) from the
// probe lines, through the caches.
__global__ void __launch_bounds__(256) k_link_lines(const ProbeLine* __restrict__ lines, uint64_t* __restrict__ link) {
    MTB_GRID_STRIDE(S, kLinkSlots) {
        uint32_t right = 0, left = 0;
        for (uint32_t y = 0; y < 21; y++) right |= probe_bit(lines, 21 * S + y) << y;
        for (uint32_t x = 0; x < 21; x++) left |= probe_bit(lines, (uint64_t)x * kLinkSlots + S) << x;
        link[S] = (uint64_t)left << 32 | right;
    }
}

void build_link_lines(const ProbeLine* lines, uint64_t* link, hipStream_t s) {
    k_link_lines<<<stride_grid(kLinkSlots), 256, 0, s>>>(lines, link);
}

// mtb_link_check: every AA rank's membership bit against both link bits that stand for it — bit
// r % 21 of word r / 21 and bit 32 + r / 21^7 of word r % 21^7, by plain division (the definition,
// not the builder's loops). A thread per 32-rank bitmap word; out: ranks, present ranks, mismatches.
__global__ void __launch_bounds__(256) k_link_check(const ProbeLine* __restrict__ lines, const uint64_t* __restrict__ link,
                                                    unsigned long long* __restrict__ out) {
    constexpr uint32_t kWords = kLineRanks / 32;
    unsigned long long n = 0, present = 0, bad = 0;
    MTB_GRID_STRIDE(wi, (kProbeLines - 1) * kWords) {
        const uint64_t L = wi / kWords;
        const uint32_t k = (uint32_t)(wi - L * kWords);
        const uint32_t word = lines[L].bits[k];
        const uint64_t r0 = L * kLineRanks + 32ull * k;
        for (uint32_t b = 0; b < 32 && r0 + b < kAARankEnd; b++) {
            const uint64_t r = r0 + b;
            const uint32_t bit = (word >> b) & 1u;
            const uint32_t right = (uint32_t)(link[r / 21] >> (r % 21)) & 1u;
            const uint32_t left = (uint32_t)(link[r % kLinkSlots] >> (32 + r / kLinkSlots)) & 1u;
            n++;
            present += bit;
            bad += (right != bit) + (left != bit);
        }
    }
    for (int d = 32; d > 0; d >>= 1) {
        n += __shfl_xor(n, d, 64);
        present += __shfl_xor(present, d, 64);
        bad += __shfl_xor(bad, d, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], n);
        atomicAdd(&out[1], present);
        atomicAdd(&out[2], bad);
    }
}

void launch_link_check(const ProbeLine* lines, const uint64_t* link, unsigned long long* out, hipStream_t s) {
    k_link_check<<<stride_grid((kProbeLines - 1) * (kLineRanks / 32)), 256, 0, s>>>(lines, link, out);
}

void build_run_offsets(const DbRec* db, uint64_t D, const ProbeLine* lines, const uint64_t* lineP,
                       uint16_t* runOff, hipStream_t s) {
    if (!D) return;
    if (line_atomic_build()) k_run_offsets<<<stride_grid(D), 256, 0, s>>>(db, D, lines, lineP, runOff);
    else k_run_offsets_wave<<<line_wave_grid(), 256, 0, s>>>(db, D, lines, lineP, runOff);
}

// Query blocks: kMatchQ consecutive sorted queries span a narrow AA-rank range, so the DB values
// of that range (found with two directory lookups per block) are staged in LDS with coalesced
// loads and every query of the block searches LDS. A block whose range holds more than kMatchWin
// DB values (few queries against a large DB, or a very frequent AA k-mer) searches HBM through the
// directory instead.
constexpr int kMatchQ = 256;
constexpr int kMatchWin = 3072;
// D / Q above which K4 runs without LDS windows: a 256-query block's window (256 D / Q values) would
// pass the 3072-value LDS cap and search HBM through the directory anyway (round 4: 24 sent 3M-pair
// GTDB batches, D / Q = 17, through that path: join 35 -> 61 ms)
constexpr uint32_t kStageFreeRatio = 12;
constexpr int kFreePer = 1;               // queries per thread in the unstaged K4 (2: no gain with the run index; +1.6 ms before)
constexpr int kMatchLines = 256;          // probe lines a block of the unstaged K4 stages in LDS (16 KB)
constexpr int kExtLines = 128;            // run-length lines it stages beside them (MTB_LINE_EXT=1, A/B: 8 KB)
constexpr uint64_t kRankEnd = 37822859361ull;  // 21^8 AA k-mers

__device__ __forceinline__ uint64_t db_lower_bound(const DbVal& dbv, const AADir& d, uint64_t v) {
    const uint64_t b = aa_bucket(v, d);
    return lower_bound_u64(dbv, d.dir[b], d.dir[b + 1], v);
}

// One query's AA run [lo, hi) in vals (LDS window or the whole DB; vOff = DB index of vals[0],
// infos aligned with vals): the selection threshold min(2 * min hamming sum, 7) and the number
// of candidates within it, in one pass — sums <= 7 are tallied in the bytes of a 64-bit word
// (runs of more than 255 candidates take a second pass).
template <typename V>
__device__ __forceinline__ uint32_t run_select(const HamRows& hr, const V& vals, uint64_t vOff, uint64_t lo,
                                               uint64_t& hi, uint64_t D, uint32_t& thr) {
    if (hi + vOff > D - 1) hi = D - 1 - vOff;  // the last DB k-mer is never a candidate
    if (lo >= hi) return 0;
    uint32_t minSum = 255;
    uint64_t tally = 0;
    for (uint64_t t = lo; t < hi; t++) {
        const uint32_t s = hamming_sum_rows(hr, vals[t]);
        minSum = min(minSum, s);
        if (s <= 7) tally += 1ull << (8 * s);
    }
    thr = min(minSum * 2u, 7u);
    uint32_t c = 0;
    if (hi - lo <= 255) {
#pragma unroll
        for (uint32_t s = 0; s < 8; s++)
            if (s <= thr) c += (uint32_t)(tally >> (8 * s)) & 0xFFu;
    } else {
        for (uint64_t t = lo; t < hi; t++) c += hamming_sum_rows(hr, vals[t]) <= thr;
    }
    return c;
}

// One selected candidate (DB value tv, taxID tax, hamming sum hs) as a Match at out[w]
// (KmerMatcher.cpp:431-448); outRank (nullable) gets its rank inside its read's segment.
__device__ __forceinline__ void put_match(mtb_match* __restrict__ out, uint64_t w, const mtb_match& m) { out[w] = m; }
__device__ __forceinline__ void put_match(SegMatch* __restrict__ out, uint64_t w, const mtb_match& m) {
    out[w] = seg_pack(m);
}

template <typename O>
__device__ __forceinline__ void emit_match(uint64_t key, const HamRows& hr, uint64_t info, uint64_t tv, uint32_t tax,
                                           uint32_t hs, bool rev, const int32_t* __restrict__ spOf, uint32_t maxTax,
                                           O* __restrict__ out, uint32_t* __restrict__ outRank, uint64_t w,
                                           uint32_t rank, int* __restrict__ err) {
    const int32_t sp = tax <= maxTax ? spOf[tax] : 0;
    if (tax == 0 || sp <= 0) atomicExch(err, kErrTaxid);  // KmerMatcher.cpp:432-441 exits
    mtb_match m;
    m.qinfo = info;
    m.target_id = tax;
    m.species_id = (uint32_t)sp;
    m.dna_encoding = (uint32_t)(tv & 0xFFFFFFull);
    m.right_end_hamming = (uint16_t)hammings_rows(hr, key, tv, rev);
    m.hamming = (uint8_t)hs;
    m.pad = 0;
    if (outRank) outRank[w] = rank;
    put_match(out, w, m);
}

// Writes the run's selected candidates at out[w..wEnd); returns the next w (a selection that
// would pass wEnd sets err 4 and stops). outRank (nullable) gets each match's rank inside its
// read's segment, starting at `rank`.
template <typename V, typename T, typename O>
__device__ __forceinline__ uint64_t run_emit(uint64_t key, const HamRows& hr, uint64_t info, const V& vals,
                                             const T& infos, uint64_t lo, uint64_t hi, uint32_t thr,
                                             const int32_t* __restrict__ spOf, uint32_t maxTax, int kmerFormat,
                                             O* __restrict__ out, uint32_t* __restrict__ outRank, uint64_t w,
                                             uint64_t wEnd, uint32_t rank, int* __restrict__ err) {
    const bool rev = ((info_frame(info) < 3) != (kmerFormat == 2));
    for (uint64_t t = lo; t < hi; t++) {
        const uint64_t tv = vals[t];
        const uint32_t hs = hamming_sum_rows(hr, tv);
        if (hs > thr) continue;
        if (w >= wEnd) {
            atomicExch(err, kErrProbeCount);
            return w;
        }
        emit_match(key, hr, info, tv, infos[t], hs, rev, spOf, maxTax, out, outRank, w++, rank++, err);
    }
    return w;
}

// Both ends of an AA run in an LDS window of n sorted values: lower bounds of aa and aa + 2^24 by
// a fixed-trip binary search (the trip count depends only on n, so the two chains, and the
// chains of a thread's other queries, interleave instead of waiting on each other).
__device__ __forceinline__ void lds_run_bounds(const uint64_t* a, uint32_t n, uint32_t pow2, uint64_t aa,
                                               uint32_t& lo, uint32_t& hi) {
    const uint64_t aa2 = aa + (1ull << 24);
    uint32_t p1 = 0, p2 = 0;
    for (uint32_t step = pow2; step > 0; step >>= 1) {
        const uint32_t i1 = p1 + step, i2 = p2 + step;
        if (i1 <= n && a[i1 - 1] < aa) p1 = i1;
        if (i2 <= n && a[i2 - 1] < aa2) p2 = i2;
    }
    lo = p1;
    hi = p2;
}

// Window of each query block = DB values whose AA rank lies in the block's sort-prefix range
// (kQuerySortLo/Hi): [lower_bound(first prefix), lower_bound(last prefix + 1)). One thread per
// block boundary; computed once per batch and shared by the count and emit passes.
__global__ void k_match_windows(const uint64_t* __restrict__ qkey, uint64_t Q, const DbRec* __restrict__ db,
                                uint64_t D, AADir d, int kmerFormat, uint64_t nBlocks, uint64_t* __restrict__ win) {
    const DbVal dbv{db};
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * nBlocks) return;
    const uint64_t b = i >> 1;
    const uint32_t side = (uint32_t)(i & 1);
    const uint64_t q = side ? min((b + 1) * kMatchQ, Q) - 1 : b * kMatchQ;
    const int sh = kQuerySortLo - 24;
    const uint64_t r = (((qkey[q] >> 24) >> sh) + side) << sh;
    win[i] = r >= kRankEnd ? D : db_lower_bound(dbv, d, r << 24);
}

// Long AA runs (conserved AA 8-mers shared by hundreds to thousands of species): one query's run is
// scanned by its whole wave instead of serially by its lane (a lane looping over 10^4 candidates
// held its wave — and the block's other queries — for the whole scan). The wave takes the long
// queries of its lanes one after another: min Hamming sum and selected count by wave reductions
// over coalesced strides of the run, one rank reservation, and the selected candidates written at
// ballot-prefix positions (into the read's stretch, or spilled past it like the lane path's).
constexpr uint64_t kLongRun = 48;

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
    return v;
}

template <typename V, typename T>
__device__ __forceinline__ uint32_t wave_long_run(uint64_t key, uint32_t slot, uint64_t lo, uint64_t hi, const V& vals,
                                                  const T& infos, const uint64_t* __restrict__ unitInfo, uint32_t C,
                                                  const int32_t* __restrict__ spOf, uint32_t maxTax, int kmerFormat,
                                                  uint32_t* __restrict__ readCnt, unsigned long long* __restrict__ total,
                                                  mtb_match* __restrict__ buf, uint32_t* __restrict__ bufRank,
                                                  uint64_t region, int* __restrict__ err, SegMatch* __restrict__ direct,
                                                  const uint64_t* __restrict__ dirOff, int* __restrict__ overflow,
                                                  uint32_t capShift, int lane, unsigned long long* __restrict__ cnt64) {
    const HamRows hr = hamming_rows(key);
    uint32_t mn = 255;
    for (uint64_t t = lo + lane; t < hi; t += 64) mn = min(mn, hamming_sum_rows(hr, vals[t]));
    const uint32_t thr = min(wave_min_u32(mn) * 2u, 7u);
    uint32_t cnt = 0;
    for (uint64_t t = lo + lane; t < hi; t += 64) cnt += hamming_sum_rows(hr, vals[t]) <= thr;
    const uint32_t c = wave_sum_u32(cnt);
    if (c == 0) return 0;
    const uint64_t info = slot_info(slot, C, unitInfo, kmerFormat);
    const uint32_t r = info_seq(info) - 1;
    uint32_t rk = 0;
    // uniform units: the read's 64-bit counter (k_match's, count in the low word)
    if (lane == 0) rk = cnt64 ? (uint32_t)atomicAdd(&cnt64[r], (unsigned long long)c) : atomicAdd(&readCnt[r], c);
    rk = (uint32_t)__shfl((int)rk, 0, 64);
    // staged join (direct == nullptr): the block's staging stretch is claimed by the caller's count;
    // here only the direct join's long runs come (the staged path keeps them on the lane)
    const uint64_t o = dirOff[r] * C, cap = (dirOff[r + 1] * C - o) >> capShift;
    const bool spill = rk + c > cap;
    uint64_t w0 = rk;
    if (spill) {
        unsigned long long sp = 0;
        if (lane == 0) sp = atomicAdd(&total[0], (unsigned long long)c);
        sp = __shfl(sp, 0, 64);
        if (sp + c > region) {
            if (lane == 0) atomicExch(overflow, 1);
            return c;
        }
        w0 = sp;
    }
    const bool rev = ((info_frame(info) < 3) != (kmerFormat == 2));
    const uint64_t lt = (1ull << lane) - 1;
    uint64_t done = 0;
    for (uint64_t t0 = lo; t0 < hi; t0 += 64) {
        const uint64_t t = t0 + lane;
        uint64_t tv = 0;
        uint32_t hs = 255;
        if (t < hi) {
            tv = vals[t];
            hs = hamming_sum_rows(hr, tv);
        }
        const bool sel = hs <= thr;
        const uint64_t m = __ballot(sel);
        if (sel) {
            const uint64_t k = done + (uint64_t)__popcll(m & lt);
            if (spill)
                emit_match(key, hr, info, tv, infos[t], hs, rev, spOf, maxTax, buf, bufRank, w0 + k,
                           rk + (uint32_t)k, err);
            else
                emit_match(key, hr, info, tv, infos[t], hs, rev, spOf, maxTax, direct + o, (uint32_t*)nullptr,
                           w0 + k, 0, err);
        }
        done += (uint64_t)__popcll(m);
    }
    return c;
}

// The join in one pass. Each block selects its queries' candidates, counts them (per read with
// atomics, per thread for the block), claims one contiguous stretch of the staging buffer with a
// single atomic, and writes its matches there with the lanes' stretches adjacent. The buffer is
// kStageRegions regions of `region` slots, each with its own counter (block b uses b mod
// kStageRegions), so the claims do not all queue on one address. A later pass moves each match
// into its read's segment (k_match_transpose). A region that would overflow is not written; the
// caller grows the regions to the largest count and reruns.
// A/B only (MTB_AB_RANK_FREE): k_match takes a query's rank in its read's segment
// without the readCnt atomic (a wrong rank: the results are invalid), bounding what any scheme
// that removes the atomic could save in the join; 2: nor the read's stretch bounds (dirOff).
// Uniform units (round 6): 3 = no rank atomic (fixed lengths), 4 = nor the match writes.
__device__ int g_abRankFree = 0;
__device__ int g_matchXcd = 0;
__device__ int g_shareRuns = 0;
__device__ int g_pairRead = 0;
// MTB_MATCH_PREFETCH=<m> (A/B, lean join): while a query's run-index entry is in flight, read the record
// line its run most likely starts in — base + before + before * m / 256 (m ~ 256 * (records per
// present rank - 1): 45 at GTDB scale) — so the dependent record read that follows hits the L2 when
// the guess lands in the right line; 0: off
__device__ int g_prefetch = 0;
static int h_prefetch = 0;
void set_match_prefetch(int m) {
    h_prefetch = m;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_prefetch), &m, sizeof(int));
}

static int h_pairRead = 0, h_matchXcd = 0, h_abRankFree = 0;  // host copies: k_join_uniform runs only without them
void set_pair_read(int on) {
    h_pairRead = on;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_pairRead), &on, sizeof(int));
}

static int h_shareRuns = 0;  // host copy: the lean join (no sharing table) when off
void set_share_runs(int on) {
    h_shareRuns = on;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_shareRuns), &on, sizeof(int));
}

void set_match_xcd(int on) {
    h_matchXcd = on;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_matchXcd), &on, sizeof(int));
}

void set_ab_rank_free(int on) {
    h_abRankFree = on;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_abRankFree), &on, sizeof(int));
}

// The info of window p of uniform unit u (k_read_units: upr units per read, one per (mate, frame)), as
// unit_windows + unit_info_at compute it: read u / upr, mate and frame from u % upr, the frame's first
// window at its begin (KmerExtractor.cpp:374-378) plus the mate-2 offset (:341-345). L: the read's
// mate lengths (16 bits each), which k_match gets back from its rank atomic (the read's 64-bit counter
// carries them above the count), so a matched query reads no unit record and no length.
__device__ __forceinline__ uint64_t uniform_unit_info(uint32_t u, uint32_t p, uint32_t upr, uint32_t L,
                                                      int kmerFormat) {
    const uint32_t r = u / upr, local = u - r * upr;
    const uint32_t mate = local >= 6u ? 1u : 0u, frame = local - 6u * mate;
    const bool fwd = frame < 3u;
    const bool fromLeft = (kmerFormat == 2) ? fwd : !fwd;
    uint32_t pos0 = frame, posOffset = 0;
    if (mate || !fromLeft || !fwd) {
        const int len1 = (int)(L & 0xFFFFu), len = mate ? (int)(L >> 16) : len1;
        const int used = max_covered_length(len);
        int begin = (int)frame;
        if (!fwd) { begin = (len % 3) - ((int)frame % 3); if (begin < 0) begin += 3; }
        pos0 = fromLeft ? (uint32_t)begin : (uint32_t)(begin + used - 1 - 3 * 8 + 1);
        if (mate) posOffset = (uint32_t)max_covered_length(len1) + 3u;
    }
    return unit_info_at(pack_info(r + 1, pos0 + posOffset, frame), p, kmerFormat);
}

// kLean: the unstaged join without the A/B options' LDS (run-length lines, run sharing): 18 KB of LDS
// per block instead of 31, so LDS no longer caps the resident waves below what the VGPRs allow
template <bool kStage, int kPer, int kLeanWaves = 0, bool kPrefetch = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kLeanWaves ? kLeanWaves : 1))) k_match(const uint64_t* __restrict__ qkey, const uint32_t* __restrict__ qslot,
                                               const uint64_t* __restrict__ unitInfo, uint32_t C,
                                               uint64_t Q, const DbRec* __restrict__ db, uint64_t D, AADir d,
                                               const int32_t* __restrict__ spOf, uint32_t maxTax, int kmerFormat,
                                               uint32_t* __restrict__ readCnt, unsigned long long* __restrict__ total,
                                               mtb_match* __restrict__ buf, uint32_t* __restrict__ bufRank,
                                               uint64_t region, int* __restrict__ err, uint32_t winCap, const uint64_t* __restrict__ win,
                                               const ProbeLine* __restrict__ lines,
                                               const uint64_t* __restrict__ lineP, const uint16_t* __restrict__ runOff,
                                               int sortLo, unsigned long long* __restrict__ stats,
                                               SegMatch* __restrict__ direct, const uint64_t* __restrict__ dirOff,
                                               int* __restrict__ overflow, uint32_t capShift,
                                               LongRun* __restrict__ longList, uint32_t longCap,
                                               uint32_t* __restrict__ longCnt, const ProbeExt* __restrict__ lineExt,
                                               uint32_t upr, unsigned long long* __restrict__ cnt64) {
    constexpr bool kLean = kLeanWaves != 0;
    // without staging (a DB much larger than the query stream: windows over the LDS cap) the
    // kernel holds no LDS window, so twice as many blocks fit on a CU to overlap the random reads
    __shared__ uint64_t sDb[kStage ? kMatchWin : 1];
    __shared__ uint32_t sInfo[kStage ? kMatchWin : 1];
    // the block's probe lines (sorted queries) and, behind them, their run-length lines
    __shared__ uint4 sLineMem[kStage ? 1 : (kMatchLines + (kLean ? 0 : kExtLines)) * 4];
    ProbeLine* const sLines = reinterpret_cast<ProbeLine*>(sLineMem);
    const uint32_t* const sExt = reinterpret_cast<const uint32_t*>(sLineMem + (kStage ? 0 : kMatchLines * 4));
    __shared__ uint64_t sLineP[kStage ? 1 : kMatchLines];   // and their run-index bases
    __shared__ unsigned long long sTbl[kStage || kLean ? 1 : 512];  // run sharing: (AA rank + 1) << 8 | leader
    __shared__ unsigned long long sBase;
    static_assert(!kStage || kPer * 256 == kMatchQ, "staged blocks are the window blocks");
    const DbVal dbv{db};
    const DbTax dbtax{db};
    // g_matchXcd (MTB_MATCH_XCD=1, A/B): the unstaged join's blocks remapped so each XCD takes one
    // contiguous eighth of the sorted queries (neighbouring blocks' probe lines and records through one L2)
    uint32_t blk = blockIdx.x;
    if (!kStage && g_matchXcd) {
        const uint32_t x = blockIdx.x & 7u, i = blockIdx.x >> 3, q = gridDim.x >> 3, r = gridDim.x & 7u;
        blk = x * q + min(x, r) + i;
    }
    const uint64_t q0 = (uint64_t)blk * (256 * kPer);
    const uint64_t q1 = min(q0 + (uint64_t)(256 * kPer), Q);
    // every independent load of the block is issued up front (query keys and infos, the window
    // bounds, then the window) so their latencies overlap instead of adding up
    uint64_t key[kPer], info[kPer];
    uint32_t slot[kPer];
    bool live[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        const uint64_t q = q0 + threadIdx.x + (uint64_t)j * 256;
        live[j] = q < q1;
        key[j] = live[j] ? qkey[q] : 0;
        slot[j] = live[j] ? qslot[q] : 0;
    }
    const uint64_t winLo = kStage ? win[2 * blockIdx.x] : 0, winN = kStage ? win[2 * blockIdx.x + 1] - winLo : 0;
    const bool staged = kStage && winN <= (uint64_t)winCap;
    uint64_t lo[kPer], hi[kPer];
    uint32_t pfw = 0;      // MTB_MATCH_PREFETCH's speculative reads (kept live below, never used)
    uint32_t nGallop = 0;  // probe-line queries whose run the run index does not hold (gallop fallback)
    // Run sharing (the reference's same-AA reuse, KmerMatcher.cpp:315-353: a query whose AA part
    // equals the previous one's reuses its candidates): the block's queries with the same AA rank —
    // 13% of the queries of a uniform config-3 batch, 42% of a skewed-abundance one (MTB_DUP_STATS) —
    // elect one leader through an LDS hash table; only the leader reads the run index and the run's
    // first records, the followers take them from LDS. Each query still selects its own candidates.
    // Measured (round 5, same box): no gain — uniform 55.7 -> 57.3 ms, skewed 54.4 -> 55.7 ms per batch:
    // the repeated lookups hit the L2 already, and the barriers hold each block on its slowest leader.
    // Off by default (MTB_SHARE_RUNS=1: on).
    constexpr bool kShare = !kStage && kPer == 1 && !kLean;
    const bool share = kShare && g_shareRuns && lines != nullptr;
    bool follower = false;
    uint32_t leadT = threadIdx.x;
    if (share) {
        for (uint32_t i = threadIdx.x; i < 512; i += 256) sTbl[i] = 0ull;
        __syncthreads();
        if (live[0]) {
            const uint64_t rk = (key[0] & kAAMask) >> 24;
            const unsigned long long want = ((rk + 1) << 8) | threadIdx.x;
            uint32_t h = (uint32_t)((rk * 0x9E3779B97F4A7C15ull) >> 55);  // 9 bits
            while (true) {
                const unsigned long long old = atomicCAS(&sTbl[h], 0ull, want);
                if (old == 0ull) break;  // the rank's leader
                if ((old >> 8) == rk + 1) {
                    follower = true;
                    leadT = (uint32_t)(old & 255u);
                    break;
                }
                h = (h + 1) & 511u;
            }
        }
    }
    if (kStage && staged) {
        constexpr int kLoad = kMatchWin / 256;
        uint64_t v[kLoad];
        uint32_t tv[kLoad];
#pragma unroll
        for (int j = 0; j < kLoad; j++) {
            const uint32_t i = threadIdx.x + j * 256;
            v[j] = i < winN ? dbv[winLo + i] : 0;
            tv[j] = i < winN ? dbtax[winLo + i] : 0;
        }
#pragma unroll
        for (int j = 0; j < kLoad; j++) {
            const uint32_t i = threadIdx.x + j * 256;
            if (i < winN) {
                sDb[i] = v[j];
                sInfo[i] = tv[j];
            }
        }
        __syncthreads();
        const uint32_t n = (uint32_t)winN;
        uint32_t pow2 = 1;
        while (pow2 * 2 <= n) pow2 *= 2;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            uint32_t l, h;
            lds_run_bounds(sDb, n, pow2, key[j] & kAAMask, l, h);
            lo[j] = l;
            hi[j] = h;
        }
    } else if (lines) {  // HBM: the probe line names a lower bound of the run, a gallop finds its ends
        // sorted queries: the block's probe lines are one contiguous stretch (its sort-prefix range),
        // staged through LDS with coalesced loads unless it is long
        const int sh = sortLo - 24;
        const uint64_t L0 = ((qkey[q0] >> sortLo) << sh) / kLineRanks;
        const uint64_t L1 = ((((qkey[q1 - 1] >> sortLo) + 1) << sh) - 1) / kLineRanks;
        const bool inLds = !kStage && L1 - L0 < (uint64_t)kMatchLines;
        const bool extLds = !kLean && lineExt && inLds && L1 - L0 < (uint64_t)kExtLines;
        if (!kStage && inLds) {
            const uint32_t nv = (uint32_t)(L1 - L0 + 1) * 4;  // 4 x 16 B per line
            const uint4* src = reinterpret_cast<const uint4*>(lines + L0);
            uint4* dst = reinterpret_cast<uint4*>(sLines);
            for (uint32_t i = threadIdx.x; i < nv; i += 256) dst[i] = src[i];
            if (runOff)
                for (uint32_t i = threadIdx.x; i <= (uint32_t)(L1 - L0); i += 256) sLineP[i] = lineP[L0 + i];
            if (extLds) {
                const uint4* esrc = reinterpret_cast<const uint4*>(lineExt + L0);
                uint4* edst = sLineMem + kMatchLines * 4;
                for (uint32_t i = threadIdx.x; i < nv; i += 256) edst[i] = esrc[i];
            }
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const uint64_t aa = key[j] & kAAMask, x = aa >> 24, L = x / kLineRanks;
            const uint32_t o = (uint32_t)(x - L * kLineRanks);
            if (!live[j] || follower) {  // a follower takes its leader's run below
                lo[j] = hi[j] = 0;
                continue;
            }
            const ProbeLine* pl = inLds ? sLines + (L - L0) : lines + L;
            if (runOff) {  // exact run from the run index (indexed lines)
                uint32_t before, pc;
                bool present;
                const uint64_t head = line_scan(pl, o, before, pc, present);
                const uint64_t base = head & ((1ull << 40) - 1), cnt = head >> 40;
                if (cnt <= kRunIdxMax) {
                    if (!present) {  // an absent rank (not filtered: MTB_FILTER=0) has no run; runOff[p] may
                        lo[j] = hi[j] = base;  // be the next line's entry or the unset end entry
                        continue;
                    }
                    uint32_t sum, code;
                    if (extLds && before < kExtRanks && ext_run(sExt + (L - L0) * (kExtRanks / 16), before, sum, code)) {
                        lo[j] = base + before + sum;  // no run-index read
                        hi[j] = lo[j] + code + 1;
                        continue;
                    }
                    const uint64_t p = (inLds ? sLineP[L - L0] : lineP[L]) + before;
                    // both entries read unconditionally (p + 1 <= the index's end entry, allocated): no
                    // branch between the loads and the prefetch's issue
                    const uint32_t a = runOff[p], b1 = runOff[p + 1];
                    const uint32_t b = before + 1 < pc ? b1 : (uint32_t)cnt;
                    if (kPrefetch) {  // after the run-index reads, unconditionally: waiting for them leaves it in flight
                        const uint64_t gi = base + before + (((uint64_t)before * (uint32_t)g_prefetch) >> 8);
                        pfw |= reinterpret_cast<const uint32_t*>(db)[3 * min(gi, D) + 2];
                    }
                    lo[j] = base + a;
                    hi[j] = base + b;
                    continue;
                }
            }
            nGallop++;
            const uint64_t from = line_lower_bound_at(pl, o);
            lo[j] = gallop_lower1(dbv, from, aa);
            hi[j] = gallop_lower1(dbv, lo[j], aa + (1ull << 24));
        }
    } else {  // HBM through the AA-prefix directory (no probe lines: MTB_FORCE_GENERIC)
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const uint64_t aa = key[j] & kAAMask;
            const uint64_t b = aa_bucket(key[j], d);
            const uint64_t b1 = d.dir[b + 1];
            lo[j] = lower_bound_u64(dbv, d.dir[b], b1, aa);
            hi[j] = lower_bound_u64(dbv, lo[j], b1, aa + (1ull << 24));
        }
    }
    const uint64_t vOff = staged ? winLo : 0;  // DB index of the searched values' first entry
    // unstaged: a run at GTDB scale is 1-2 k-mers, so the run's first two records (value + taxID,
    // 24 contiguous bytes; the pad makes lo + 1 readable) are read at once
    uint64_t rv[kPer][2];
    uint32_t rt[kPer][2], rs[kPer][2];
    bool small[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        // a run start past the DB's end can only come from an inconsistent run index or probe line
        // (a run's lower bound is at most D): flagged, and the run taken as empty at the DB's end, so
        // the speculative two-record read below stays inside the 8 pad records (KmerMatcher.cpp:363,378:
        // the reader never runs past the DB)
        if (live[j] && lo[j] + vOff > D) {
            atomicExch(err, kErrRunOutsideDb);
            lo[j] = D - vOff;
        }
        if (hi[j] + vOff > D - 1) hi[j] = D - 1 - vOff;  // the last DB k-mer is never a candidate
        if (lo[j] > hi[j]) hi[j] = lo[j];
        small[j] = !staged && live[j] && hi[j] - lo[j] <= 2;
        if (small[j] && !follower) {
            // a random read moves a whole 128-B line (profiles/r05/random_fetch_calibration.json): the
            // second record is read only for a two-record run (g_pairRead = 0, A/B: always, as before
            // round 5), since it lies in the next line for ~1 in 10 records
            const bool two = g_pairRead || hi[j] - lo[j] == 2;
            const DbRec r0 = db[lo[j]], r1 = two ? db[lo[j] + 1] : DbRec{0, 0, 0};
            rv[j][0] = (uint64_t)r0.hi << 32 | r0.lo;
            rv[j][1] = (uint64_t)r1.hi << 32 | r1.lo;
            rt[j][0] = r0.tax;
            rt[j][1] = r1.tax;
        }
    }
    if (kShare && share) {  // the leaders' runs to their followers, through the (now free) line stage
        __syncthreads();    // every line scan of the block is done
        uint64_t* sLo = reinterpret_cast<uint64_t*>(sLines);
        uint64_t* sHi = sLo + 256;
        uint64_t* sRv = sHi + 256;
        uint32_t* sRt = reinterpret_cast<uint32_t*>(sRv + 512);
        static_assert(kStage || (256 * 8 * 4 + 512 * 4) <= sizeof(uint4) * (kMatchLines + kExtLines) * 4, "results fit the line stage");
        const uint32_t t = threadIdx.x;
        if (!follower) {
            sLo[t] = lo[0];
            sHi[t] = hi[0];
            if (small[0]) {
                sRv[2 * t] = rv[0][0];
                sRv[2 * t + 1] = rv[0][1];
                sRt[2 * t] = rt[0][0];
                sRt[2 * t + 1] = rt[0][1];
            }
        }
        __syncthreads();
        if (follower) {
            lo[0] = sLo[leadT];
            hi[0] = sHi[leadT];
            small[0] = live[0] && hi[0] - lo[0] <= 2;
            if (small[0]) {
                rv[0][0] = sRv[2 * leadT];
                rv[0][1] = sRv[2 * leadT + 1];
                rt[0][0] = sRt[2 * leadT];
                rt[0][1] = sRt[2 * leadT + 1];
            }
        }
    }
    // long runs (direct join): scanned by the whole wave below, not by the lane
    bool longq[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) longq[j] = longList && direct && !kStage && live[j] && hi[j] - lo[j] > kLongRun;
    uint32_t c[kPer], thr[kPer], rk[kPer], mine = 0;
    uint64_t stretch[kPer];
    const int abFree = g_abRankFree;
    HamRows hr[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        hr[j] = hamming_rows(key[j]);
        if (longq[j]) {
            c[j] = 0;
        } else if (small[j]) {  // run_select on the two registers
            const uint32_t n = (uint32_t)(hi[j] - lo[j]);
            rs[j][0] = n > 0 ? hamming_sum_rows(hr[j], rv[j][0]) : 255u;
            rs[j][1] = n > 1 ? hamming_sum_rows(hr[j], rv[j][1]) : 255u;
            thr[j] = min(min(rs[j][0], rs[j][1]) * 2u, 7u);
            c[j] = (uint32_t)(rs[j][0] <= thr[j]) + (uint32_t)(rs[j][1] <= thr[j]);
        } else {
            c[j] = !live[j] ? 0
                   : staged ? run_select(hr[j], sDb, vOff, lo[j], hi[j], D, thr[j])
                            : run_select(hr[j], dbv, vOff, lo[j], hi[j], D, thr[j]);
        }
        if (c[j] && upr && abFree >= 3) {  // A/B: the uniform path without its atomic (invalid results)
            uint32_t p;
            const uint32_t u = slot_unit(slot[j], C, p);
            const uint32_t r = u / upr;
            rk[j] = slot[j] & 7u;
            info[j] = uniform_unit_info(u, p, upr, 150u | 150u << 16, kmerFormat);
            stretch[j] = (uint64_t)r * upr | (uint64_t)upr << 40;
        } else if (c[j] && upr && !abFree) {
            // uniform units: the read and the segment bounds from the slot; one 64-bit atomic on the
            // read's counter reserves the ranks (low word) and returns its mate lengths (high word)
            uint32_t p;
            const uint32_t u = slot_unit(slot[j], C, p);
            const uint32_t r = u / upr;
            const unsigned long long old = atomicAdd(&cnt64[r], (unsigned long long)c[j]);
            rk[j] = (uint32_t)old;
            info[j] = uniform_unit_info(u, p, upr, (uint32_t)(old >> 32), kmerFormat);
            stretch[j] = (uint64_t)r * upr | (uint64_t)upr << 40;
        } else if (c[j]) {  // only matched queries need their info and their read's segment bounds (one 16-B load)
            uint32_t p;
            const ulonglong2 ur = reinterpret_cast<const ulonglong2*>(unitInfo)[slot_unit(slot[j], C, p)];
            info[j] = unit_info_at(ur.x, p, kmerFormat);
            stretch[j] = ur.y;
            // the returned count is the query's first rank inside its read's segment
            rk[j] = abFree ? (slot[j] & 7u) : atomicAdd(&readCnt[info_seq(info[j]) - 1], c[j]);
        } else {
            info[j] = 0;
            stretch[j] = 0;
            rk[j] = 0;
        }
        mine += c[j];
    }
    int hit = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        hit += c[j] != 0;
        const uint64_t lm = __ballot(longq[j]);
        if (lm) {  // the wave's long queries to the long-run list (one atomic per wave), for k_match_long
            const int lane = (int)(threadIdx.x & 63);
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(longCnt, (uint32_t)__popcll(lm));
            at = (uint32_t)__shfl((int)at, 0, 64) + (uint32_t)__popcll(lm & ((1ull << lane) - 1));
            if (longq[j] && at < longCap) longList[at] = LongRun{q0 + threadIdx.x + (uint64_t)j * 256, lo[j], hi[j]};
        }
    }
    if (kPrefetch && pfw == 0xFFFFFFFFu && key[0] == ~0ull) atomicAdd(&stats[kStatStripes], 0ull);  // keeps the prefetches
    const int blockHits = __syncthreads_count(hit >= 1) + (kPer > 1 ? __syncthreads_count(hit >= 2) : 0);
    // matched queries, on the block's stats stripe (one word for every block queued its atomics)
    if (threadIdx.x == 0 && blockHits) atomicAdd(&stats[blockIdx.x % kStatStripes], (unsigned long long)blockHits);
    if (!kStage && lines) {  // the fallback counter sits past the stripes (rare: a lane-0 atomic per wave)
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < kPer; j++) w += (uint32_t)__popcll(__ballot(nGallop > (uint32_t)j));
        if (w && (threadIdx.x & 63) == 0) atomicAdd(&stats[kStatStripes], (unsigned long long)w);
    }
    if (direct) {
        // each query's matches straight into its read's segment, at the ranks just reserved: the
        // read's stretch of C slots per K1 unit (slotOff) bounds it. A query whose ranks pass the
        // stretch's end spills its matches, with their ranks, to buf (total[0] counts them, `region`
        // bounds them; the caller scatters them after compacting the segments); a spill past that
        // bound sets the overflow flag and the caller reruns the batch with a larger one
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            if (!c[j] || abFree == 4) continue;
            const uint64_t o = abFree == 2 ? 0 : (stretch[j] & kStretchLoMask) * C;
            const uint64_t cap = abFree == 2 ? (1u << 20) : ((stretch[j] >> 40) * C) >> capShift;
            if (rk[j] + c[j] > cap) {
                const uint64_t sp = atomicAdd(&total[0], (unsigned long long)c[j]);
                if (sp + c[j] > region) {
                    atomicExch(overflow, 1);
                    continue;
                }
                if (small[j]) {
                    const bool rev = ((info_frame(info[j]) < 3) != (kmerFormat == 2));
                    uint64_t wj = sp;
                    uint32_t rj = rk[j];
#pragma unroll
                    for (int k = 0; k < 2; k++)
                        if (rs[j][k] <= thr[j])
                            emit_match(key[j], hr[j], info[j], rv[j][k], rt[j][k], rs[j][k], rev, spOf, maxTax, buf,
                                       bufRank, wj++, rj++, err);
                } else if (staged) {
                    run_emit(key[j], hr[j], info[j], sDb, sInfo, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, buf,
                             bufRank, sp, sp + c[j], rk[j], err);
                } else {
                    run_emit(key[j], hr[j], info[j], dbv, dbtax, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, buf,
                             bufRank, sp, sp + c[j], rk[j], err);
                }
                continue;
            }
            SegMatch* out = direct + o;
            if (small[j]) {
                const bool rev = ((info_frame(info[j]) < 3) != (kmerFormat == 2));
                uint64_t wj = rk[j];
#pragma unroll
                for (int k = 0; k < 2; k++)
                    if (rs[j][k] <= thr[j])
                        emit_match(key[j], hr[j], info[j], rv[j][k], rt[j][k], rs[j][k], rev, spOf, maxTax, out,
                                   nullptr, wj++, 0, err);
            } else if (staged) {
                run_emit(key[j], hr[j], info[j], sDb, sInfo, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, out,
                         nullptr, rk[j], rk[j] + c[j], 0, err);
            } else {
                run_emit(key[j], hr[j], info[j], dbv, dbtax, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, out,
                         nullptr, rk[j], rk[j] + c[j], 0, err);
            }
        }
        return;
    }
    unsigned long long blockTot;
    uint64_t w = block_exclusive_scan(mine, &blockTot);
    const uint32_t reg = blockIdx.x % kStageRegions;
    if (threadIdx.x == 0) sBase = blockTot ? atomicAdd(&total[reg], blockTot) : 0;
    __syncthreads();
    const uint64_t base = sBase;
    if (base + blockTot > region) return;  // region too small: the caller grows it and reruns
    w += base + (uint64_t)reg * region;
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        if (!c[j]) continue;
        if (small[j]) {
            const bool rev = ((info_frame(info[j]) < 3) != (kmerFormat == 2));
            uint64_t wj = w;
#pragma unroll
            for (int k = 0; k < 2; k++)
                if (rs[j][k] <= thr[j])
                    emit_match(key[j], hr[j], info[j], rv[j][k], rt[j][k], rs[j][k], rev, spOf, maxTax, buf, bufRank,
                               wj++, rk[j]++, err);
        } else if (staged) {
            run_emit(key[j], hr[j], info[j], sDb, sInfo, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, buf, bufRank,
                     w, w + c[j], rk[j], err);
        } else {
            run_emit(key[j], hr[j], info[j], dbv, dbtax, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, buf, bufRank,
                     w, w + c[j], rk[j], err);
        }
        w += c[j];
    }
}

// The production join alone (round 6): k_match's unstaged path for the one configuration the bench's
// batches take — run index, uniform units (the read's 64-bit counter), direct output, long-run list,
// none of the A/B options — with nothing else in the kernel, so its register peak is that path's:
// the run's two records, their taxa's species (read beside the rank atomic instead of after it)
// and the query's Hamming rows: 50 VGPRs and 18.7 KB of LDS, so 8 waves per SIMD (the hardware's most;
// k_match's lean form: 6). Same matches at the same ranks as k_match (KmerMatcher.cpp:360-448).
// kMode 1 (round 6, default; MTB_JOIN_WAVE=0: kMode 0, the block form): each wave stages its own 64
// queries' probe lines (≤ 16, one 16-B load per lane) and their run-index bases in a wave-private LDS
// stretch, and tallies its matched queries with a lane-0 atomic on a stats stripe: no block barrier,
// so the block's four waves run their dependent read chains (run index, records, rank atomic) out of
// step with each other (join 47.4 -> 42.9 ms per 3.33M-pair batch, profiles/r06/ab_k4_wave.json).
// kMode 2 / 3 (MTB_JOIN_WAVE=2 / 3, A/B: 7 / 6 waves per SIMD): resident waves walk their 64-query tiles with the next tile's probe
// lines and the tile after's keys loaded while the current tile joins, so a tile's chain starts at
// its run-index read.
constexpr int kWaveLines = 16;
template <int kMode>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kMode == 2 ? 7 : (kMode == 3 ? 6 : 8))))
k_join_uniform(const uint64_t* __restrict__ qkey, const uint32_t* __restrict__ qslot, uint32_t C, uint64_t Q,
               const DbRec* __restrict__ db, uint64_t D, const int32_t* __restrict__ spOf, uint32_t maxTax,
               int kmerFormat, unsigned long long* __restrict__ total, mtb_match* __restrict__ buf,
               uint32_t* __restrict__ bufRank, uint64_t region, int* __restrict__ err,
               const ProbeLine* __restrict__ lines, const uint64_t* __restrict__ lineP,
               const uint16_t* __restrict__ runOff, int sortLo, unsigned long long* __restrict__ stats,
               SegMatch* __restrict__ direct, int* __restrict__ overflow, uint32_t capShift,
               LongRun* __restrict__ longList, uint32_t longCap, uint32_t* __restrict__ longCnt, uint32_t upr,
               unsigned long long* __restrict__ cnt64, const ProbeExt* __restrict__ lineExt) {
    constexpr bool kWave = kMode != 0;
    constexpr bool kExt = kMode == 5;  // the wave form with run-length lines staged beside the probe lines
    constexpr int kStageLines = kWave ? kWaveLines : kMatchLines;  // (per wave / per block)
    __shared__ uint4 sLineMem[(kWave ? 4 : 1) * kStageLines * 4];
    __shared__ uint4 sExtMem[kExt ? 4 * kWaveLines * 4 : 1];
    uint4* const myExt4 = sExtMem + (kExt ? (threadIdx.x >> 6) * kWaveLines * 4 : 0);
    const uint32_t* const myExt = reinterpret_cast<const uint32_t*>(myExt4);
    __shared__ uint64_t sLineP[(kWave ? 4 : 1) * kStageLines];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    uint4* const myLines = sLineMem + (kWave ? wv * kStageLines * 4 : 0);
    uint64_t* const myLineP = sLineP + (kWave ? wv * kStageLines : 0);
    const ProbeLine* const sLines = reinterpret_cast<const ProbeLine*>(myLines);
    const DbVal dbv{db};
    const DbTax dbtax{db};
    const int sh = sortLo - 24;
    // the probe lines a stretch of sorted queries spans, from its first and last keys
    auto lineSpan = [&](uint64_t kFirst, uint64_t kLast, uint64_t& L0, uint64_t& L1) {
        L0 = ((kFirst >> sortLo) << sh) / kLineRanks;
        L1 = ((((kLast >> sortLo) + 1) << sh) - 1) / kLineRanks;
    };
    // one query: its run from the (staged) probe line and the run index, its records, selection, the
    // rank atomic, the matches into its read's segment (KmerMatcher.cpp:360-448)
    auto join = [&](const uint64_t q, const bool live, const uint64_t key, const uint32_t slot, const uint64_t L0,
                    const bool inLds, const uint32_t tile) {
        uint64_t lo = 0, hi = 0;
        bool gallop = false;
        if (live) {
            const uint64_t aa = key & kAAMask, x = aa >> 24, L = x / kLineRanks;
            const uint32_t o = (uint32_t)(x - L * kLineRanks);
            const ProbeLine* pl = inLds ? sLines + (L - L0) : lines + L;
            uint32_t before, pc;
            bool present;
            const uint64_t head = line_scan(pl, o, before, pc, present);
            const uint64_t base = head & ((1ull << 40) - 1), cnt = head >> 40;
            if (cnt > kRunIdxMax) {  // a line the run index does not hold: gallop from its lower bound
                gallop = true;
                lo = gallop_lower1(dbv, base + before, aa);
                hi = gallop_lower1(dbv, lo, aa + (1ull << 24));
            } else if (present) {
                uint32_t sum = 0, code = 0;
                if (kExt && inLds && before < kExtRanks && ext_run_rolled(myExt + (L - L0) * (kExtRanks / 16), before, sum, code)) {
                    lo = base + before + sum;  // no run-index read (the codes before it hold no escape)
                    hi = lo + code + 1;
                } else {
                    const uint64_t p = (inLds ? myLineP[L - L0] : lineP[L]) + before;
                    const uint32_t a = runOff[p], b1 = runOff[p + 1];
                    lo = base + a;
                    hi = base + (before + 1 < pc ? b1 : (uint32_t)cnt);
                }
            } else {
                lo = hi = base;
            }
            if (lo > D) {  // an inconsistent run index or probe line (k_match's check)
                atomicExch(err, kErrRunOutsideDb);
                lo = D;
            }
            if (hi > D - 1) hi = D - 1;  // the last DB k-mer is never a candidate
            if (lo > hi) hi = lo;
        }
        const uint64_t n = hi - lo;
        const bool longq = n > kLongRun;
        const bool small = live && n <= 2;
        uint64_t v0 = 0, v1 = 0;
        uint32_t t0 = 0, t1 = 0;
        if (small && n) {  // the run's records (a random read moves a 128-B line: the second only if present)
            const DbRec r0 = db[lo], r1 = n == 2 ? db[lo + 1] : DbRec{0, 0, 0};
            v0 = (uint64_t)r0.hi << 32 | r0.lo;
            v1 = (uint64_t)r1.hi << 32 | r1.lo;
            t0 = r0.tax;
            t1 = r1.tax;
        }
        const HamRows hr = hamming_rows(key);
        uint32_t c = 0, thr = 0, s0 = 255, s1 = 255;
        if (small) {
            s0 = n > 0 ? hamming_sum_rows(hr, v0) : 255u;
            s1 = n > 1 ? hamming_sum_rows(hr, v1) : 255u;
            thr = min(min(s0, s1) * 2u, 7u);
            c = (uint32_t)(s0 <= thr) + (uint32_t)(s1 <= thr);
        } else if (live && !longq) {
            c = run_select(hr, dbv, 0, lo, hi, D, thr);
        }
        // the selected records' species (L2-resident spOf) in flight with the rank atomic below
        const bool e0 = small && s0 <= thr, e1 = small && s1 <= thr;
        const int32_t sp0 = e0 ? (t0 <= maxTax ? spOf[t0] : 0) : 0;
        const int32_t sp1 = e1 ? (t1 <= maxTax ? spOf[t1] : 0) : 0;
        uint32_t rk = 0, r = 0;
        uint64_t info = 0;
        if (c) {
            uint32_t p;
            const uint32_t u = slot_unit(slot, C, p);
            r = u / upr;
            const unsigned long long old = atomicAdd(&cnt64[r], (unsigned long long)c);
            rk = (uint32_t)old;
            info = uniform_unit_info(u, p, upr, (uint32_t)(old >> 32), kmerFormat);
        }
        const uint64_t lm = __ballot(longq && live);
        if (lm) {  // the wave's long queries to the long-run list (one atomic per wave), for k_match_long
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(longCnt, (uint32_t)__popcll(lm));
            at = (uint32_t)__shfl((int)at, 0, 64) + (uint32_t)__popcll(lm & ((1ull << lane) - 1));
            if (longq && live && at < longCap) longList[at] = LongRun{q, lo, hi};
        }
        if (kMode != 0) {  // matched queries: a lane-0 atomic per wave on its stripe
            const uint64_t hw = __ballot(c != 0);
            if (lane == 0 && hw) atomicAdd(&stats[tile % kStatStripes], (unsigned long long)__popcll(hw));
        } else {
            const int blockHits = __syncthreads_count(c != 0);
            if (threadIdx.x == 0 && blockHits) atomicAdd(&stats[blockIdx.x % kStatStripes], (unsigned long long)blockHits);
        }
        const uint64_t gw = __ballot(gallop);
        if (gw && (threadIdx.x & 63) == 0) atomicAdd(&stats[kStatStripes], (unsigned long long)__popcll(gw));
        if (!c) return;
        const bool rev = ((info_frame(info) < 3) != (kmerFormat == 2));
        // the read's stretch of upr units (C slots each) bounds its segment; ranks past it spill to buf
        const uint64_t cap = ((uint64_t)upr * C) >> capShift;
        const bool spill = rk + c > cap;
        uint64_t w = rk;
        if (spill) {
            const uint64_t sp = atomicAdd(&total[0], (unsigned long long)c);
            if (sp + c > region) {
                atomicExch(overflow, 1);
                return;
            }
            w = sp;
        }
        SegMatch* const out = direct + (uint64_t)r * upr * C;
        if (small) {
    #pragma unroll
            for (int k = 0; k < 2; k++) {
                if (!(k ? e1 : e0)) continue;
                const uint64_t tv = k ? v1 : v0;
                const uint32_t tax = k ? t1 : t0, hs = k ? s1 : s0;
                const int32_t sp = k ? sp1 : sp0;
                if (tax == 0 || sp <= 0) atomicExch(err, kErrTaxid);  // KmerMatcher.cpp:432-441 exits
                mtb_match m;
                m.qinfo = info;
                m.target_id = tax;
                m.species_id = (uint32_t)sp;
                m.dna_encoding = (uint32_t)(tv & 0xFFFFFFull);
                m.right_end_hamming = (uint16_t)hammings_rows(hr, key, tv, rev);
                m.hamming = (uint8_t)hs;
                m.pad = 0;
                if (spill) {
                    bufRank[w] = rk++;
                    buf[w] = m;
                } else {
                    out[w] = seg_pack(m);
                }
                w++;
            }
        } else if (spill) {
            run_emit(key, hr, info, dbv, dbtax, lo, hi, thr, spOf, maxTax, kmerFormat, buf, bufRank, w, w + c, rk, err);
        } else {
            run_emit(key, hr, info, dbv, dbtax, lo, hi, thr, spOf, maxTax, kmerFormat, out, (uint32_t*)nullptr, w, w + c, 0,
                     err);
        }
    };
    if constexpr (kMode < 2 || kMode >= 5) {
        // the wave's first query (kMode 1 runs with 256- or 64-thread blocks: MTB_JOIN_WAVE=4, A/B).
        // kMode 7 (MTB_JOIN_WAVE=7, A/B): blocks dealt round-robin over the 8 XCDs walk contiguous
        // eighths of the sorted queries, so neighbouring tiles share one L2
        uint64_t blk = blockIdx.x;
        if (kMode == 7) {
            const uint64_t x = blk & 7u, i = blk >> 3, qn = gridDim.x >> 3, rn = gridDim.x & 7u;
            blk = x * qn + min(x, rn) + i;
        }
        const uint64_t waveId = (blk * blockDim.x + threadIdx.x) >> 6;
        const uint64_t q0 = kWave ? waveId * 64 : (uint64_t)blockIdx.x * 256;
        if (kWave && q0 >= Q) return;  // a wave past the queries (no block barrier below in this form)
        const uint64_t q1 = min(q0 + (kWave ? 64 : 256), Q);
        const uint64_t q = q0 + (kWave ? (uint64_t)lane : threadIdx.x);
        const bool live = q < q1;
        const uint64_t key = live ? qkey[q] : 0;
        const uint32_t slot = live ? qslot[q] : 0;
        // the block's (wave's) probe lines (one contiguous stretch: sorted queries) and their run-index
        // bases in LDS
        uint64_t L0, L1;
        lineSpan(kWave ? (uint64_t)__shfl((long long)key, 0, 64) : qkey[q0],
                 kWave ? (uint64_t)__shfl((long long)key, (int)(q1 - q0 - 1), 64) : qkey[q1 - 1], L0, L1);
        const bool inLds = L1 - L0 < (uint64_t)kStageLines;
        if (inLds) {
            const uint32_t nv = (uint32_t)(L1 - L0 + 1) * 4;
            const uint4* src = reinterpret_cast<const uint4*>(lines + L0);
            if (kWave) {  // one 16-B load per lane and a base per line, both in flight together
                uint4 v{0, 0, 0, 0}, xv{0, 0, 0, 0};
                uint64_t lp = 0;
                if ((uint32_t)lane < nv) v = src[lane];
                if (kExt && (uint32_t)lane < nv) xv = reinterpret_cast<const uint4*>(lineExt + L0)[lane];
                if ((uint32_t)lane <= (uint32_t)(L1 - L0)) lp = lineP[L0 + lane];
                if ((uint32_t)lane < nv) myLines[lane] = v;
                if (kExt && (uint32_t)lane < nv) myExt4[lane] = xv;
                if ((uint32_t)lane <= (uint32_t)(L1 - L0)) myLineP[lane] = lp;
                // the wave's LDS writes complete in program order before any lane reads them back
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_wave_barrier();
            } else {
                for (uint32_t i = threadIdx.x; i < nv; i += 256) myLines[i] = src[i];
                for (uint32_t i = threadIdx.x; i <= (uint32_t)(L1 - L0); i += 256) myLineP[i] = lineP[L0 + i];
                __syncthreads();
            }
        }
        join(q, live, key, slot, L0, inLds, (uint32_t)waveId);
    } else {
        // resident waves: tile t = 64 sorted queries; wave w takes tiles w, w + W, w + 2W, ...
        const uint64_t nT = (Q + 63) / 64, W = (uint64_t)gridDim.x * 4;
        uint64_t t = (uint64_t)blockIdx.x * 4 + (uint64_t)wv;
        if (t >= nT) return;
        auto tileKeys = [&](uint64_t tt, uint64_t& k) {
            const uint64_t qq = tt * 64 + (uint64_t)lane;
            k = (tt < nT && qq < Q) ? qkey[qq] : 0;
        };
        auto tileSpan = [&](uint64_t tt, uint64_t k, uint64_t& L0, uint64_t& L1) {
            const uint64_t qa = tt * 64, qb = min(qa + 64, Q);
            lineSpan((uint64_t)__shfl((long long)k, 0, 64), (uint64_t)__shfl((long long)k, (int)(qb - qa - 1), 64), L0,
                     L1);
        };
        auto stageLoad = [&](uint64_t L0, uint64_t L1, uint4& v, uint64_t& lp) {
            v = uint4{0, 0, 0, 0};
            lp = 0;
            if (L1 - L0 < (uint64_t)kWaveLines) {
                if ((uint32_t)lane < (uint32_t)(L1 - L0 + 1) * 4) v = reinterpret_cast<const uint4*>(lines + L0)[lane];
                if ((uint32_t)lane <= (uint32_t)(L1 - L0)) lp = lineP[L0 + lane];
            }
        };
        auto stageStore = [&](uint64_t L0, uint64_t L1, const uint4& v, uint64_t lp) {
            if (L1 - L0 < (uint64_t)kWaveLines) {
                if ((uint32_t)lane < (uint32_t)(L1 - L0 + 1) * 4) myLines[lane] = v;
                if ((uint32_t)lane <= (uint32_t)(L1 - L0)) myLineP[lane] = lp;
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the LDS writes done; loads stay in flight
            __builtin_amdgcn_wave_barrier();
        };
        uint64_t kc, kn, L0c, L1c;
        tileKeys(t, kc);
        tileKeys(t + W, kn);
        tileSpan(t, kc, L0c, L1c);
        {
            uint4 v;
            uint64_t lp;
            stageLoad(L0c, L1c, v, lp);
            stageStore(L0c, L1c, v, lp);
        }
        for (;;) {
            const bool more = t + W < nT;
            uint64_t L0n = 0, L1n = 0, kk;
            uint4 v{0, 0, 0, 0};
            uint64_t lp = 0;
            if (more) {  // the next tile's probe lines in flight (its keys arrived during the last tile)
                tileSpan(t + W, kn, L0n, L1n);
                stageLoad(L0n, L1n, v, lp);
            }
            tileKeys(t + 2 * W, kk);  // the keys of the tile after it
            const uint64_t q = t * 64 + (uint64_t)lane;
            const uint32_t sc = q < Q ? qslot[q] : 0;  // needed at the rank atomic: in flight with the run index
            join(q, q < Q, kc, sc, L0c, L1c - L0c < (uint64_t)kWaveLines, (uint32_t)t);
            if (!more) break;
            stageStore(L0n, L1n, v, lp);
            t += W;
            kc = kn;
            kn = kk;
            L0c = L0n;
            L1c = L1n;
        }
    }
}

// k_join_uniform's wave form with two queries per lane (MTB_JOIN_WAVE=6, A/B): a wave takes 128 sorted
// queries (lane l: queries l and l + 64) and stages their ≤ 32 probe lines; each phase of the chain
// (run index, records, rank atomic) issues both queries' requests before waiting, so a SIMD keeps two
// chains in flight per lane. K4 is bound by the chains in flight (8 / 6 / 4 waves per SIMD: 41.6 /
// 46-49.5 / 56 ms per batch, profiles/r06/ab_k4_occ.json). Same matches at the same ranks.
constexpr int kPairLines = 32;
template <int kW>  // waves per SIMD the registers are held to (MTB_JOIN_WAVE=6 / 7 / 8)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kW)))
k_join_pair(const uint64_t* __restrict__ qkey, const uint32_t* __restrict__ qslot, uint32_t C, uint64_t Q,
            const DbRec* __restrict__ db, uint64_t D, const int32_t* __restrict__ spOf, uint32_t maxTax,
            int kmerFormat, unsigned long long* __restrict__ total, mtb_match* __restrict__ buf,
            uint32_t* __restrict__ bufRank, uint64_t region, int* __restrict__ err,
            const ProbeLine* __restrict__ lines, const uint64_t* __restrict__ lineP,
            const uint16_t* __restrict__ runOff, int sortLo, unsigned long long* __restrict__ stats,
            SegMatch* __restrict__ direct, int* __restrict__ overflow, uint32_t capShift,
            LongRun* __restrict__ longList, uint32_t longCap, uint32_t* __restrict__ longCnt, uint32_t upr,
            unsigned long long* __restrict__ cnt64) {
    __shared__ uint4 sLineMem[4 * kPairLines * 4];
    __shared__ uint64_t sLineP[4 * kPairLines];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    uint4* const myLines = sLineMem + wv * kPairLines * 4;
    uint64_t* const myLineP = sLineP + wv * kPairLines;
    const ProbeLine* const sLines = reinterpret_cast<const ProbeLine*>(myLines);
    const DbVal dbv{db};
    const DbTax dbtax{db};
    const uint64_t waveId = (uint64_t)blockIdx.x * 4 + (uint64_t)wv;
    const uint64_t q0 = waveId * 128;
    if (q0 >= Q) return;
    const uint64_t q1 = min(q0 + 128, Q);
    uint64_t q[2], key[2];
    uint32_t slot[2];
    bool live[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        q[j] = q0 + (uint64_t)(64 * j + lane);
        live[j] = q[j] < q1;
        key[j] = live[j] ? qkey[q[j]] : 0;
        slot[j] = live[j] ? qslot[q[j]] : 0;
    }
    const int sh = sortLo - 24;
    const int last = (int)(q1 - q0 - 1);
    const uint64_t kFirst = (uint64_t)__shfl((long long)key[0], 0, 64);
    const uint64_t kLast = (uint64_t)(last < 64 ? __shfl((long long)key[0], last, 64) : __shfl((long long)key[1], last - 64, 64));
    const uint64_t L0 = ((kFirst >> sortLo) << sh) / kLineRanks;
    const uint64_t L1 = ((((kLast >> sortLo) + 1) << sh) - 1) / kLineRanks;
    const bool inLds = L1 - L0 < (uint64_t)kPairLines;
    if (inLds) {  // two 16-B loads per lane and a base per line, all in flight together
        const uint32_t nv = (uint32_t)(L1 - L0 + 1) * 4;
        const uint4* src = reinterpret_cast<const uint4*>(lines + L0);
        uint4 v0{0, 0, 0, 0}, v1{0, 0, 0, 0};
        uint64_t lp = 0;
        if ((uint32_t)lane < nv) v0 = src[lane];
        if ((uint32_t)lane + 64 < nv) v1 = src[lane + 64];
        if ((uint32_t)lane <= (uint32_t)(L1 - L0)) lp = lineP[L0 + lane];
        if ((uint32_t)lane < nv) myLines[lane] = v0;
        if ((uint32_t)lane + 64 < nv) myLines[lane + 64] = v1;
        if ((uint32_t)lane <= (uint32_t)(L1 - L0)) myLineP[lane] = lp;
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
    }
    // the runs: line scans from LDS, then both run-index reads
    uint64_t lo[2] = {0, 0}, hi[2] = {0, 0};
    bool gallop[2] = {false, false};
    uint64_t rp[2] = {0, 0}, rbase[2] = {0, 0};
    uint32_t rcnt[2] = {0, 0}, rlast[2] = {0, 0};
    bool needIdx[2] = {false, false};
#pragma unroll
    for (int j = 0; j < 2; j++) {
        if (!live[j]) continue;
        const uint64_t aa = key[j] & kAAMask, x = aa >> 24, L = x / kLineRanks;
        const uint32_t o = (uint32_t)(x - L * kLineRanks);
        const ProbeLine* pl = inLds ? sLines + (L - L0) : lines + L;
        uint32_t before, pc;
        bool present;
        const uint64_t head = line_scan(pl, o, before, pc, present);
        const uint64_t base = head & ((1ull << 40) - 1), cnt = head >> 40;
        if (cnt > kRunIdxMax) {  // a line the run index does not hold: gallop from its lower bound
            gallop[j] = true;
            lo[j] = gallop_lower1(dbv, base + before, aa);
            hi[j] = gallop_lower1(dbv, lo[j], aa + (1ull << 24));
        } else if (present) {
            needIdx[j] = true;
            rp[j] = (inLds ? myLineP[L - L0] : lineP[L]) + before;
            rbase[j] = base;
            rcnt[j] = (uint32_t)cnt;
            rlast[j] = before + 1 < pc ? 0u : 1u;
        } else {
            lo[j] = hi[j] = base;
        }
    }
    uint32_t ra[2] = {0, 0}, rb[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 2; j++)
        if (needIdx[j]) {
            ra[j] = runOff[rp[j]];
            rb[j] = runOff[rp[j] + 1];
        }
#pragma unroll
    for (int j = 0; j < 2; j++) {
        if (needIdx[j]) {
            lo[j] = rbase[j] + ra[j];
            hi[j] = rbase[j] + (rlast[j] ? rcnt[j] : rb[j]);
        }
        if (live[j]) {
            if (lo[j] > D) {  // an inconsistent run index or probe line (k_match's check)
                atomicExch(err, kErrRunOutsideDb);
                lo[j] = D;
            }
            if (hi[j] > D - 1) hi[j] = D - 1;  // the last DB k-mer is never a candidate
            if (lo[j] > hi[j]) hi[j] = lo[j];
        }
    }
    // the runs' records, both queries' in flight together
    bool small[2], longq[2];
    uint64_t v0[2] = {0, 0}, v1[2] = {0, 0};
    uint32_t t0[2] = {0, 0}, t1[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const uint64_t n = hi[j] - lo[j];
        longq[j] = live[j] && n > kLongRun;
        small[j] = live[j] && n <= 2;
        if (small[j] && n) {
            const DbRec r0 = db[lo[j]], r1 = n == 2 ? db[lo[j] + 1] : DbRec{0, 0, 0};
            v0[j] = (uint64_t)r0.hi << 32 | r0.lo;
            v1[j] = (uint64_t)r1.hi << 32 | r1.lo;
            t0[j] = r0.tax;
            t1[j] = r1.tax;
        }
    }
    uint32_t c[2] = {0, 0}, thr[2] = {0, 0}, s0[2] = {255, 255}, s1[2] = {255, 255};
    int32_t sp0[2] = {0, 0}, sp1[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const HamRows hr = hamming_rows(key[j]);
        const uint64_t n = hi[j] - lo[j];
        if (small[j]) {
            s0[j] = n > 0 ? hamming_sum_rows(hr, v0[j]) : 255u;
            s1[j] = n > 1 ? hamming_sum_rows(hr, v1[j]) : 255u;
            thr[j] = min(min(s0[j], s1[j]) * 2u, 7u);
            c[j] = (uint32_t)(s0[j] <= thr[j]) + (uint32_t)(s1[j] <= thr[j]);
        } else if (live[j] && !longq[j]) {
            c[j] = run_select(hr, dbv, 0, lo[j], hi[j], D, thr[j]);
        }
        const bool e0 = small[j] && s0[j] <= thr[j], e1 = small[j] && s1[j] <= thr[j];
        sp0[j] = e0 ? (t0[j] <= maxTax ? spOf[t0[j]] : 0) : 0;
        sp1[j] = e1 ? (t1[j] <= maxTax ? spOf[t1[j]] : 0) : 0;
    }
    // both rank atomics in flight together
    uint32_t rk[2] = {0, 0}, rr[2] = {0, 0};
    uint64_t info[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 2; j++)
        if (c[j]) {
            uint32_t p;
            const uint32_t u = slot_unit(slot[j], C, p);
            rr[j] = u / upr;
            const unsigned long long old = atomicAdd(&cnt64[rr[j]], (unsigned long long)c[j]);
            rk[j] = (uint32_t)old;
            info[j] = uniform_unit_info(u, p, upr, (uint32_t)(old >> 32), kmerFormat);
        }
    uint32_t hits = 0, gal = 0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const uint64_t lm = __ballot(longq[j]);
        if (lm) {  // the wave's long queries to the long-run list (one atomic per wave), for k_match_long
            uint32_t at = 0;
            if (lane == 0) at = atomicAdd(longCnt, (uint32_t)__popcll(lm));
            at = (uint32_t)__shfl((int)at, 0, 64) + (uint32_t)__popcll(lm & ((1ull << lane) - 1));
            if (longq[j] && at < longCap) longList[at] = LongRun{q[j], lo[j], hi[j]};
        }
        hits += (uint32_t)__popcll(__ballot(c[j] != 0));
        gal += (uint32_t)__popcll(__ballot(gallop[j]));
    }
    if (lane == 0 && hits) atomicAdd(&stats[waveId % kStatStripes], (unsigned long long)hits);
    if (lane == 0 && gal) atomicAdd(&stats[kStatStripes], (unsigned long long)gal);
    const uint64_t cap = ((uint64_t)upr * C) >> capShift;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        if (!c[j]) continue;
        const bool rev = ((info_frame(info[j]) < 3) != (kmerFormat == 2));
        // the read's stretch of upr units (C slots each) bounds its segment; ranks past it spill to buf
        const bool spill = rk[j] + c[j] > cap;
        uint64_t w = rk[j];
        if (spill) {
            const uint64_t sp = atomicAdd(&total[0], (unsigned long long)c[j]);
            if (sp + c[j] > region) {
                atomicExch(overflow, 1);
                continue;
            }
            w = sp;
        }
        SegMatch* const out = direct + (uint64_t)rr[j] * upr * C;
        if (small[j]) {
            const HamRows hr = hamming_rows(key[j]);
            uint32_t rkj = rk[j];
#pragma unroll
            for (int k = 0; k < 2; k++) {
                if (!(k ? s1[j] <= thr[j] : s0[j] <= thr[j])) continue;
                const uint64_t tv = k ? v1[j] : v0[j];
                const uint32_t tax = k ? t1[j] : t0[j], hs = k ? s1[j] : s0[j];
                const int32_t sp = k ? sp1[j] : sp0[j];
                if (tax == 0 || sp <= 0) atomicExch(err, kErrTaxid);  // KmerMatcher.cpp:432-441 exits
                mtb_match m;
                m.qinfo = info[j];
                m.target_id = tax;
                m.species_id = (uint32_t)sp;
                m.dna_encoding = (uint32_t)(tv & 0xFFFFFFull);
                m.right_end_hamming = (uint16_t)hammings_rows(hr, key[j], tv, rev);
                m.hamming = (uint8_t)hs;
                m.pad = 0;
                if (spill) {
                    bufRank[w] = rkj++;
                    buf[w] = m;
                } else {
                    out[w] = seg_pack(m);
                }
                w++;
            }
        } else {
            const HamRows hr = hamming_rows(key[j]);
            if (spill)
                run_emit(key[j], hr, info[j], dbv, dbtax, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, buf, bufRank, w,
                         w + c[j], rk[j], err);
            else
                run_emit(key[j], hr, info[j], dbv, dbtax, lo[j], hi[j], thr[j], spOf, maxTax, kmerFormat, out,
                         (uint32_t*)nullptr, w, w + c[j], 0, err);
        }
    }
}

// The long-run list of the direct join: one wave per long query (wave_long_run).
__global__ void __launch_bounds__(64) k_match_long(const LongRun* __restrict__ list, const uint64_t* __restrict__ qkey,
                                                   const uint32_t* __restrict__ qslot,
                                                   const uint64_t* __restrict__ unitInfo, uint32_t C,
                                                   const DbRec* __restrict__ db, uint64_t D,
                                                   const int32_t* __restrict__ spOf, uint32_t maxTax, int kmerFormat,
                                                   uint32_t* __restrict__ readCnt,
                                                   unsigned long long* __restrict__ total, mtb_match* __restrict__ buf,
                                                   uint32_t* __restrict__ bufRank, uint64_t region, int* __restrict__ err,
                                                   SegMatch* __restrict__ direct, const uint64_t* __restrict__ dirOff,
                                                   int* __restrict__ overflow, uint32_t capShift,
                                                   unsigned long long* __restrict__ stats,
                                                   unsigned long long* __restrict__ cnt64) {
    const LongRun lr = list[blockIdx.x];
    if (lr.lo > lr.hi || lr.hi > D - 1) {  // the producers clamp runs to [0, D - 1]: never read past the DB
        if (threadIdx.x == 0) atomicExch(err, kErrRunOutsideDb);
        return;
    }
    const uint32_t got = wave_long_run(qkey[lr.q], qslot[lr.q], lr.lo, lr.hi, DbVal{db}, DbTax{db}, unitInfo, C, spOf,
                                       maxTax, kmerFormat, readCnt, total, buf, bufRank, region, err, direct, dirOff,
                                       overflow, capShift, (int)threadIdx.x, cnt64);
    if (threadIdx.x == 0 && got) atomicAdd(&stats[blockIdx.x % kStatStripes], 1ull);  // a matched query
}

void launch_match_long(const LongRun* list, uint32_t n, const uint64_t* qkey, const uint32_t* qslot,
                       const uint64_t* unitInfo, uint32_t C, const DbRec* db, uint64_t D, const int32_t* spOf,
                       uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total, mtb_match* buf,
                       uint32_t* bufRank, uint64_t region, int* err, SegMatch* direct, const uint64_t* dirOff,
                       int* overflow, uint32_t capShift, unsigned long long* stats, hipStream_t s,
                       unsigned long long* cnt64) {
    if (n) k_match_long<<<n, 64, 0, s>>>(list, qkey, qslot, unitInfo, C, db, D, spOf, maxTax, kmerFormat, readCnt, total, buf,
                                         bufRank, region, err, direct, dirOff, overflow, capShift, stats, cnt64);
}

// Uniform units' read counters (k_match): count 0 in the low word, the mate lengths above it.
__global__ void k_cnt64_init(const uint32_t* __restrict__ readLens, uint32_t n, unsigned long long* __restrict__ cnt64) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) cnt64[i] = (unsigned long long)readLens[i] << 32;
}
// ... and the counts back into the per-read u32 counts every later stage reads.
__global__ void k_cnt64_counts(const unsigned long long* __restrict__ cnt64, uint32_t n, uint32_t* __restrict__ readCnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) readCnt[i] = (uint32_t)cnt64[i];
}
void launch_cnt64_init(const uint32_t* readLens, uint32_t n, unsigned long long* cnt64, hipStream_t s) {
    if (n) k_cnt64_init<<<(n + 255) / 256, 256, 0, s>>>(readLens, n, cnt64);
}
void launch_cnt64_counts(const unsigned long long* cnt64, uint32_t n, uint32_t* readCnt, hipStream_t s) {
    if (n) k_cnt64_counts<<<(n + 255) / 256, 256, 0, s>>>(cnt64, n, readCnt);
}

// Each staged match into its read's segment at the rank the join reserved for it (no atomics);
// the order inside a segment is settled by K5.
__global__ void k_match_transpose(const mtb_match* __restrict__ buf, const uint32_t* __restrict__ bufRank,
                                  uint64_t region, const unsigned long long* __restrict__ total,
                                  const uint64_t* __restrict__ readOff, uint32_t nReads,
                                  mtb_match* __restrict__ out, int* __restrict__ err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= region * kStageRegions || i % region >= total[i / region]) return;
    const mtb_match m = buf[i];
    const uint32_t r = info_seq(m.qinfo) - 1;
    if (r >= nReads) {  // cannot happen for staged matches; never write out of bounds
        atomicExch(err, kErrStagedRead);
        return;
    }
    const uint64_t o = readOff[r] + bufRank[i];
    if (o >= readOff[r + 1]) {
        atomicExch(err, kErrStagedRead);
        return;
    }
    out[o] = m;
}

// ------------------------------------------------------------------------------------------------
// K1F membership filter: a query k-mer whose AA 8-mer is absent from the DB can match nothing
// (matchKmers compares AA parts for equality first), so only the present ones go on. One thread
// per 16 slots, all 16 keys and then all 16 probe-line words in flight at once (one random 4-B
// read per window, the pass's whole cost); each block packs its present windows and claims their
// output stretch with one atomic. For the probe join (FROM) a present window also gets its DB
// lower bound: the line's base plus the present ranks before it in the line (each holds >= 1
// DB k-mer), from the rest of the same line.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t line_base(uint64_t h) { return h & ((1ull << 40) - 1); }

constexpr int kFilterPer = 16;

template <bool FROM>
__global__ void __launch_bounds__(256) k_filter(const uint64_t* __restrict__ keys, uint64_t R,
                                                const ProbeLine* __restrict__ lines, uint64_t* __restrict__ qkey,
                                                uint32_t* __restrict__ qslot, uint64_t* __restrict__ qfrom,
                                                unsigned long long* __restrict__ counter, uint64_t rankLo,
                                                uint64_t rankHi) {
    __shared__ unsigned long long sBase;
    const uint64_t base = (uint64_t)blockIdx.x * (256 * kFilterPer) + threadIdx.x;
    uint64_t k[kFilterPer];
    uint32_t word[kFilterPer];
#pragma unroll
    for (int j = 0; j < kFilterPer; j++) k[j] = base + 256ull * j < R ? keys[base + 256ull * j] : kSentinel;
#pragma unroll
    for (int j = 0; j < kFilterPer; j++) {
        word[j] = 0;
        const uint64_t xr = k[j] >> 24;
        if (k[j] != kSentinel && xr >= rankLo && xr < rankHi) {  // outside a DB part's range: no probe
            const uint64_t x = xr, L = x / kLineRanks;
            const uint32_t o = (uint32_t)(x - L * kLineRanks);
            word[j] = (lines[L].bits[o >> 5] >> (o & 31u)) & 1u;
        }
    }
    uint32_t mask = 0, emitted = 0;
#pragma unroll
    for (int j = 0; j < kFilterPer; j++) {
        mask |= word[j] << j;
        emitted += k[j] != kSentinel;
    }
    // one scan carries both counts: present windows (the output offset) in the low 32 bits, emitted
    // (non-blank) windows in the high 32 bits — the reference's "Query k-mer number"
    // (KmerMatcher.cpp:143-152) counts every non-blank query k-mer, before any AA test
    unsigned long long tot;
    const unsigned long long off =
        block_exclusive_scan((unsigned long long)__popc(mask) | ((unsigned long long)emitted << 32), &tot) &
        0xFFFFFFFFull;
    if (threadIdx.x == 0) {
        const unsigned long long present = tot & 0xFFFFFFFFull;
        sBase = present ? atomicAdd(counter, present) : 0;
        if (tot >> 32) atomicAdd(counter + 1, tot >> 32);
    }
    __syncthreads();
    uint64_t pos = sBase + off;
#pragma unroll
    for (int j = 0; j < kFilterPer; j++) {
        if (!((mask >> j) & 1u)) continue;
        qkey[pos] = k[j];
        qslot[pos] = (uint32_t)(base + 256ull * j);
        if (FROM) qfrom[pos] = line_lower_bound(lines, k[j] >> 24);
        pos++;
    }
}

// K1 + K1F fused (the sort-merge join's default): each thread scans its unit's windows as k_extract
// does, 16 at a time, probes the 16 keys' lines together and packs the present ones (block-wide,
// one counter atomic per block and group; below) — the window keys never go through HBM. The block's
// threads share the group loop up to the block's longest unit (a unit past its windows, or a padding
// unit, contributes sentinels). The emitted-window count goes to the counter once per wave at the
// end: same-address atomics are what the kernel waits on when it has no probes to make (round 4:
// a per-wave-per-group counter atomic tripled the probe-free pass, `MTB_AB_FILTER=1`). Output: qkey /
// qslot as k_filter's (slot = the window's K1 slot).
constexpr uint32_t kBinStage = 2560;  // binned K1F: windows per group staged in LDS (a group keeps ~1.9k at GTDB scale)
// kLink: window pairs through the link lines — 3: at the registers the code takes (3 waves per SIMD),
// 4: held to 128 VGPRs (4 waves, a few spills); 0: one probe-line read per window. kSplit: the group's
// probes issued after its scan instead of as each window's (pair's) key is known. kSeqLds (uniform units
// only): the block's reads' bases staged in LDS first, so the scan loads nothing from HBM — a load's
// wait counter drains in issue order, and a base load issued behind a probe waits for that probe
constexpr uint32_t kSeqStage = 10240;  // >= 23 read pairs (or 44 single reads) of <= 219 bp: a uniform batch's block
// kWavePack (MTB_K1F_WAVEPACK=1, A/B): each wave packs its own present windows with its own counter
// atomic per group — no block barrier per group (the K4 finding: a block's waves held at a barrier
// wait for its slowest lane's random reads)
template <int kPer, bool kJMajor, bool kBinned = false, int kLink = 0, bool kSplit = false, bool kSeqLds = false,
          bool kWavePack = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kLink == 4 ? 4 : 1))) k_extract_filter(const uint8_t* __restrict__ seq1, const uint64_t* __restrict__ off1,
                                                        const uint8_t* __restrict__ seq2, const uint64_t* __restrict__ off2,
                                                        const ReadMeta* __restrict__ meta, const uint64_t* __restrict__ uOff,
                                                        const uint32_t* __restrict__ unitRead, uint64_t nUnits, uint32_t C,
                                                        ExtractTables tabs, int kmerFormat, int syncmer, int smerLen,
                                                        uint64_t* __restrict__ unitInfo, const ProbeLine* __restrict__ lines,
                                                        uint64_t* __restrict__ qkey, uint32_t* __restrict__ qslot,
                                                        unsigned long long* __restrict__ counter, uint64_t rankLo,
                                                        uint64_t rankHi, uint64_t cap, uint8_t* __restrict__ qdig,
                                                        unsigned long long* __restrict__ binCnt, uint64_t binRc,
                                                        uint32_t upr, const uint64_t* __restrict__ link,
                                                        int emitPerBlock = 0) {
    static_assert(kLink == 0 || kPer % 2 == 0, "windows probed in pairs");
    __shared__ uint8_t sBase[256];
    __shared__ uint32_t sBin[256];
    __shared__ uint32_t sBinBase[256];
    // binned output's LDS stage (below): dynamic, launched only with binRc, so the packed form keeps
    // its occupancy
    extern __shared__ uint64_t sStageKey[];  // kBinStage keys, then kBinStage slots (as u32 at 2 kBinStage + i)
    __shared__ int8_t sAA[64], sNum[64];
    __shared__ unsigned long long sOut;
    __shared__ uint32_t sMaxWin, sCnt[kPer * kWaves], sEx[kWaves][64];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    const unsigned long long ltMask = (1ull << lane) - 1;
    if (threadIdx.x == 0) sMaxWin = 0;
    load_extract_tables(tabs, sBase, sAA, sNum);  // syncs
    const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t slotBase = (u >> 6) * 64ull * C + (u & 63u);
    const UnitWindows w = unit_windows(u, nUnits, C, seq1, off1, seq2, off2, meta, uOff, unitRead, kmerFormat, upr);
    if (w.nWin > 0) {
        reinterpret_cast<ulonglong2*>(unitInfo)[u] = make_ulonglong2(w.info0, w.stretch);
        atomicMax(&sMaxWin, (uint32_t)w.nWin);
    }
    __shared__ uint8_t sSeq[kSeqLds ? kSeqStage : 1];
    // the scanner's bases: in HBM, or (kSeqLds) always an LDS address, so its loads are LDS reads (a
    // pointer that may be either is a flat load, which waits on the probes' counter too)
    const uint8_t* seqAt = kSeqLds ? sSeq : w.seq;
    if constexpr (kSeqLds) {
        // the block's reads r0..r1 (upr units each): mate 1's bases, then mate 2's, copied with
        // coalesced byte loads
        const uint64_t u0 = (uint64_t)blockIdx.x * blockDim.x, uL = min(u0 + blockDim.x, nUnits) - 1;
        const uint64_t r0 = u0 / upr, r1 = uL / upr;
        const uint64_t a1 = off1[r0], n1 = off1[r1 + 1] - a1;
        const uint64_t a2 = seq2 ? off2[r0] : 0, n2 = seq2 ? off2[r1 + 1] - a2 : 0;
        if (n1 + n2 <= kSeqStage) {
            for (uint32_t i = threadIdx.x; i < n1; i += blockDim.x) sSeq[i] = seq1[a1 + i];
            for (uint32_t i = threadIdx.x; i < n2; i += blockDim.x) sSeq[n1 + i] = seq2[a2 + i];
            if (w.nWin > 0) {
                const uint64_t r = u / upr;
                seqAt = (u - r * upr) >= 6u ? sSeq + n1 + (off2[r] - a2) : sSeq + (off1[r] - a1);
            }
        } else if (threadIdx.x == 0) {
            // cannot happen in a uniform batch (mates <= 219 bp); flagged in the emitted count, never silent
            atomicOr(counter + 1, 1ull << 63);
        }
    }
    __syncthreads();
    WinScanner sc(w, sBase, sAA, sNum, syncmer, smerLen, seqAt);  // loads nothing for a unit without windows
    __syncthreads();
    const uint32_t gEnd = min(C, sMaxWin);
    uint32_t emitted = 0;
    for (uint32_t g = 0; g < gEnd; g += kPer) {
        // each probe's word index (u32 offsets into the link lines, < 2 * 21^7, or the probe lines,
        // < 16 * kProbeLines; 0 for a window without a probe: a shared, cached word), its read issued at
        // once, or (kSplit) with the group's others after the scan: a load's wait counter drains in issue
        // order, so a probe issued between two windows makes the next window's base loads wait for it
        const uint32_t* const src = kLink ? reinterpret_cast<const uint32_t*>(link) : reinterpret_cast<const uint32_t*>(lines);
        uint64_t k[kPer];
        uint32_t word[kPer], sh[kPer];
        uint32_t f0 = 0, t0 = 0, h0 = 0, y0 = 0;
        bool ok0 = false;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            k[j] = (int)(g + j) < w.nWin ? sc.next() : kSentinel;
            if constexpr (kLink) {
                // the scanner's split of the window's rank r = 21 h + y = f 21^7 + t (no division)
                const uint64_t r = k[j] >> 24;
                const bool ok = k[j] != kSentinel && r >= rankLo && r < rankHi;
                const uint32_t h = sc.first7, y = sc.lastAA, f = sc.firstAA;
                if (!(j & 1)) {
                    f0 = f, h0 = h, y0 = y, ok0 = ok;
                    t0 = (uint32_t)(r - (uint64_t)f * kLinkSlots);
                    continue;
                }
                // windows j - 1 and j: consecutive windows of the frame (the last seven AAs of the first
                // are the first seven of the second) read the two halves of their shared 7-mer's word —
                // one 8-B stretch, one memory request; else each window the right half of its own first
                // seven's
                const bool shared = ok0 && ok && t0 == h;
                word[j - 1] = !ok0 ? 0u : (shared ? 2u * t0 + 1u : 2u * h0);
                word[j] = !ok ? 0u : 2u * h;
                sh[j - 1] = !ok0 ? 32u : (shared ? f0 : y0);
                sh[j] = !ok ? 32u : y;
                if constexpr (!kSplit) {
                    word[j - 1] = src[word[j - 1]];
                    word[j] = src[word[j]];
                }
            } else {
                word[j] = 0;
                sh[j] = 32;
                const uint64_t xr = k[j] >> 24;
                if (k[j] != kSentinel && xr >= rankLo && xr < rankHi) {
                    const uint64_t L = xr / kLineRanks;
                    const uint32_t o = (uint32_t)(xr - L * kLineRanks);
                    word[j] = (uint32_t)(L * (sizeof(ProbeLine) / 4) + 2 + (o >> 5));  // bits[o / 32] of line L
                    sh[j] = o & 31u;
                }
                if constexpr (!kSplit) word[j] = src[word[j]];
            }
        }
        if constexpr (kSplit) {
            asm volatile("" ::: "memory");  // the probes stay behind the scan's base loads
#pragma unroll
            for (int j = 0; j < kPer; j++) word[j] = src[word[j]];
        }
        uint32_t mask = 0;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            mask |= (sh[j] < 32u ? (word[j] >> sh[j]) & 1u : 0u) << j;
            emitted += k[j] != kSentinel;
        }
        if constexpr (!kJMajor) {  // A/B (MTB_FILTER_PACK=thread): thread-major order, round 3's packing
            const uint32_t pc = (uint32_t)__popc(mask);
            const uint32_t inc = (uint32_t)wave_inclusive_scan((unsigned long long)pc);
            if (lane == 63) sCnt[wv] = inc;
            __syncthreads();
            uint32_t off = inc - pc, tot = 0;
#pragma unroll
            for (int i = 0; i < kWaves; i++) {
                off += i < wv ? sCnt[i] : 0u;
                tot += sCnt[i];
            }
            if (threadIdx.x == 0) sOut = tot ? atomicAdd(counter, (unsigned long long)tot) : 0;
            __syncthreads();
            uint64_t pos = sOut + off;
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                if (!((mask >> j) & 1u)) continue;
                if (pos < cap) {
                    qkey[pos] = k[j];
                    qslot[pos] = (uint32_t)(slotBase + 64ull * (g + j));
                    if (qdig) qdig[pos] = (uint8_t)(k[j] >> kQuerySortLo);
                }
                pos++;
            }
            continue;
        }
        // the block's present windows packed in (window j, wave, lane) order — the output needs no
        // order: K2 sorts it and K5 puts each read's matches in compareMatches order — so every store
        // instruction writes one contiguous stretch. Per group: a ballot per window j, each wave's 16
        // counts to LDS, an exclusive scan of the block's 16 x kWaves counts by every wave (one entry
        // per lane), one counter atomic, two barriers (the counts of the next group are written after
        // this group's second barrier, by which every thread has read them; sOut after the next
        // group's first, by which every thread has read it)
        static_assert(kPer * kWaves <= 64, "one count per lane");
        if constexpr (kBinned) {
            // binned output (K2's first pass folded in): each present window goes straight into the
            // bucket of its first sort digit d (key bits kQuerySortLo..+8) — region d * 8 + XCD of
            // binRc slots, digit-major, so the regions in order are the first pass's output; the
            // order inside a region is free (the first LSD pass need not be stable). Per group: a
            // block histogram of the digits, one space reservation per non-empty bucket, three
            // barriers. Blocks are dealt
            // round-robin over the 8 XCDs, so a region's consecutive reservations come from one L2,
            // which completes the lines the short runs leave partial. A bucket past binRc is counted
            // only (the caller reruns the batch unbinned). The side digit written is the second
            // pass's (bits kQuerySortLo + 8..).
            const uint32_t xcd = blockIdx.x & 7u;
            sBin[threadIdx.x] = 0;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kPer; j++)
                if ((mask >> j) & 1u) atomicAdd(&sBin[(uint32_t)(k[j] >> kQuerySortLo) & 0xFFu], 1u);
            __syncthreads();
            // the reservation, then the block scan of the bucket counts while it is in flight; then
            // each window takes a slot of its digit's run in an LDS stage, and the stage leaves in
            // digit order — consecutive threads write consecutive slots of one bucket, so a store
            // instruction covers a few short runs instead of 64 lines (the unstaged form cost the
            // fused kernel 10 ms per 3.33M-pair batch). Windows past the stage are written directly.
            const uint32_t nb = sBin[threadIdx.x];
            const uint32_t gb = nb ? (uint32_t)atomicAdd(binCnt + threadIdx.x * 8u + xcd, (unsigned long long)nb) : 0u;
            unsigned long long tot;
            const uint32_t st = (uint32_t)block_exclusive_scan(nb, &tot);
            sBin[threadIdx.x] = st;  // the digit's stage cursor
            // bucket slot of stage entry i of digit d: sBinBase[d] + i (mod 2^32). When the whole group
            // fits the stage (block-uniform), it is stored after the staging, so the reservation's
            // round trip overlaps it; else before, for the windows written directly
            const bool fits = tot <= kBinStage;
            if (!fits) sBinBase[threadIdx.x] = gb - st;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                if (!((mask >> j) & 1u)) continue;
                const uint32_t d = (uint32_t)(k[j] >> kQuerySortLo) & 0xFFu;
                const uint32_t p = atomicAdd(&sBin[d], 1u);
                const uint32_t slot = (uint32_t)(slotBase + 64ull * (g + j));
                if (p < kBinStage) {
                    sStageKey[p] = k[j];
                    reinterpret_cast<uint32_t*>(sStageKey)[2 * kBinStage + p] = slot;
                } else {
                    const uint32_t at = sBinBase[d] + p;
                    if (at < binRc) {
                        const uint64_t pos = (uint64_t)(d * 8u + xcd) * binRc + at;
                        qkey[pos] = k[j];
                        qslot[pos] = slot;
                        if (qdig) qdig[pos] = (uint8_t)(k[j] >> (kQuerySortLo + 8));
                    }
                }
            }
            if (fits) sBinBase[threadIdx.x] = gb - st;
            __syncthreads();
            const uint32_t nst = min((uint32_t)tot, (uint32_t)kBinStage);
            for (uint32_t i = threadIdx.x; i < nst; i += blockDim.x) {
                const uint64_t key = sStageKey[i];
                const uint32_t d = (uint32_t)(key >> kQuerySortLo) & 0xFFu;
                const uint32_t at = sBinBase[d] + i;
                if (at < binRc) {
                    const uint64_t pos = (uint64_t)(d * 8u + xcd) * binRc + at;
                    qkey[pos] = key;
                    qslot[pos] = reinterpret_cast<const uint32_t*>(sStageKey)[2 * kBinStage + i];
                    if (qdig) qdig[pos] = (uint8_t)(key >> (kQuerySortLo + 8));
                }
            }
            // sBin / sBinBase / the stage are rewritten after the next group's first barrier, by which
            // every thread has read them
            continue;
        }
        uint32_t myCnt = 0;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const unsigned long long b = __ballot((mask >> j) & 1u);
            if (lane == j) myCnt = (uint32_t)__popcll(b);
        }
        if constexpr (kWavePack) {  // the wave's present windows in (window j, lane) order
            const uint32_t inc = (uint32_t)wave_inclusive_scan((unsigned long long)myCnt);
            const uint32_t tot = (uint32_t)__shfl((int)inc, 63, 64);
            unsigned long long wb = 0;
            if (lane == 0 && tot) wb = atomicAdd(counter, (unsigned long long)tot);
            const uint64_t base = (uint64_t)__shfl((long long)wb, 0, 64);
            const uint32_t ex = inc - myCnt;  // lane j: window j's offset in the wave's stretch
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const unsigned long long b = __ballot((mask >> j) & 1u);
                const uint32_t exj = (uint32_t)__shfl((int)ex, j, 64);
                if (!((mask >> j) & 1u)) continue;
                const uint64_t pos = base + exj + (uint32_t)__popcll(b & ltMask);
                if (pos < cap) {  // past the output's capacity: counted only (the caller grows it and reruns)
                    qkey[pos] = k[j];
                    qslot[pos] = (uint32_t)(slotBase + 64ull * (g + j));
                    if (qdig) qdig[pos] = (uint8_t)(k[j] >> kQuerySortLo);
                }
            }
            continue;
        }
        if (lane < kPer) sCnt[lane * kWaves + wv] = myCnt;
        __syncthreads();
        const uint32_t c = lane < kPer * kWaves ? sCnt[lane] : 0u;
        const uint32_t inc = (uint32_t)wave_inclusive_scan((unsigned long long)c);
        const uint32_t tot = (uint32_t)__shfl((int)inc, 63, 64);
        sEx[wv][lane] = inc - c;  // the wave's own copy of the offsets: read back per window below
        if (threadIdx.x == 0) sOut = tot ? atomicAdd(counter, (unsigned long long)tot) : 0;
        __syncthreads();
        const uint64_t base = sOut;
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const unsigned long long b = __ballot((mask >> j) & 1u);  // recomputed: no 16 live ballots
            if (!((mask >> j) & 1u)) continue;
            const uint64_t pos = base + sEx[wv][j * kWaves + wv] + (uint32_t)__popcll(b & ltMask);
            if (pos < cap) {  // past the output's capacity: counted only (the caller grows it and reruns)
                qkey[pos] = k[j];
                qslot[pos] = (uint32_t)(slotBase + 64ull * (g + j));
                if (qdig) qdig[pos] = (uint8_t)(k[j] >> kQuerySortLo);  // the sort's first digit (K2's side array)
            }
        }
    }
    // the reference's "Query k-mer number" (KmerMatcher.cpp:143-152) counts every non-blank query
    // k-mer, before any AA test: one atomic per wave, or (emitPerBlock, the default for the production
    // form) per block — the count shares its line with the output counter the groups' atomics wait on,
    // and same-line atomics are served one at a time
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) emitted += (uint32_t)__shfl_xor((int)emitted, d, 64);
    if (emitPerBlock) {
        __shared__ uint32_t sEmit[kWaves];
        if ((threadIdx.x & 63) == 0) sEmit[wv] = emitted;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t e = 0;
#pragma unroll
            for (int i = 0; i < kWaves; i++) e += sEmit[i];
            if (e) atomicAdd(counter + 1, (unsigned long long)e);
        }
        return;
    }
    if ((threadIdx.x & 63) == 0 && emitted) atomicAdd(counter + 1, (unsigned long long)emitted);
}

uint64_t launch_extract_filter(const uint8_t* seq1, const uint64_t* off1, const uint8_t* seq2, const uint64_t* off2,
                               const ReadMeta* meta, const uint64_t* uOff, const uint32_t* unitRead, uint64_t nUnits,
                               uint32_t C, const HostTables& t, int kmerFormat, int syncmer, int smerLen,
                               uint64_t* unitInfo, const ProbeLine* lines, uint64_t* qkey, uint32_t* qslot,
                               unsigned long long* counter, uint64_t rankLo, uint64_t rankHi, uint64_t* emitted,
                               uint64_t cap, bool threadMajor, hipStream_t s, uint8_t* qdig,
                               unsigned long long* binCnt, uint64_t binRc, uint64_t* binHost, uint32_t upr,
                               const uint64_t* link) {
    if (binRc) {
        // binned output: the writes go to 2048 regions of binRc slots; the bucket counts come back
        threadMajor = false;
        hipMemsetAsync(binCnt, 0, kSortBins * sizeof(unsigned long long), s);
    }
    hipMemsetAsync(counter, 0, 2 * sizeof(unsigned long long), s);
    if (nUnits) {
        const uint64_t threads = (nUnits + 63) / 64 * 64;
        // MTB_FILTER_PER (A/B): windows per probe group (16: the default; 8: fewer registers, more waves)
        static const int per = getenv("MTB_FILTER_PER") && atoi(getenv("MTB_FILTER_PER")) == 8 ? 8 : 16;
        const bool jMajor = !threadMajor;
        const unsigned blocks = (unsigned)((threads + 255) / 256);
        const size_t lds = binRc ? kBinStage * (sizeof(uint64_t) + sizeof(uint32_t)) : 0;
#define MTB_EF(P, J)                                                                                                  \
    k_extract_filter<P, J, false, 0, true><<<blocks, 256, lds, s>>>(seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits, C, \
                                                  extract_tables(t), kmerFormat, syncmer, smerLen, unitInfo, lines, qkey, \
                                                  qslot, counter, rankLo, rankHi, cap, qdig, binCnt, binRc, upr, nullptr)
        if (binRc) {
            k_extract_filter<kFilterPer, true, true><<<blocks, 256, lds, s>>>(
                seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits, C, extract_tables(t), kmerFormat, syncmer, smerLen,
                unitInfo, lines, qkey, qslot, counter, rankLo, rankHi, cap, qdig, binCnt, binRc, upr, nullptr);
        } else if (link && jMajor) {  // window pairs through the link lines (the default when the context has them)
            // MTB_LINK_FORM (A/B, read per batch): w<waves><s|i>[8] — 4 or 3 waves per SIMD, probes issued
            // after the group's scan (s) or interleaved (i), groups of 8 windows instead of 16
            const char* lf = getenv("MTB_LINK_FORM");
            const std::string f = lf ? lf : "w4i";
#define MTB_EFL(P, W, S)                                                                                            \
    k_extract_filter<P, true, false, W, S><<<blocks, 256, lds, s>>>(                                                \
        seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits, C, extract_tables(t), kmerFormat, syncmer, smerLen,   \
        unitInfo, lines, qkey, qslot, counter, rankLo, rankHi, cap, qdig, binCnt, binRc, upr, link)
            // MTB_K1F_EMIT_BLOCK=0 (A/B, read per batch): the emitted count by one atomic per wave
            const char* eb = getenv("MTB_K1F_EMIT_BLOCK");
            const int emitBlock = !eb || atoi(eb) != 0;
#define MTB_EFLS(P, W, S)                                                                                           \
    k_extract_filter<P, true, false, W, S, true><<<blocks, 256, lds, s>>>(                                          \
        seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits, C, extract_tables(t), kmerFormat, syncmer, smerLen,   \
        unitInfo, lines, qkey, qslot, counter, rankLo, rankHi, cap, qdig, binCnt, binRc, upr, link, emitBlock)
            const char* wp = getenv("MTB_K1F_WAVEPACK");  // A/B, read per batch
            const bool wavePack = wp && atoi(wp) != 0;
            // the bases staged in LDS (uniform batches; MTB_K1F_SEQ_LDS=0, A/B: read from HBM)
            const char* sl = getenv("MTB_K1F_SEQ_LDS");
            const bool seqLds = upr && (!sl || atoi(sl) != 0);
            if (seqLds && wavePack && f == "w4i")
                k_extract_filter<16, true, false, 4, false, true, true><<<blocks, 256, lds, s>>>(
                    seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits, C, extract_tables(t), kmerFormat, syncmer,
                    smerLen, unitInfo, lines, qkey, qslot, counter, rankLo, rankHi, cap, qdig, binCnt, binRc, upr, link);
            else if (seqLds && f == "w3i") MTB_EFLS(16, 3, false);
            else if (seqLds && f == "w3i8") MTB_EFLS(8, 3, false);
            else if (seqLds) MTB_EFLS(16, 4, false);
            else if (f == "w3i") MTB_EFL(16, 3, false);
            else if (f == "w3s") MTB_EFL(16, 3, true);
            else if (f == "w4s") MTB_EFL(16, 4, true);
            else if (f == "w3i8") MTB_EFL(8, 3, false);
            else if (f == "w3s8") MTB_EFL(8, 3, true);
            else MTB_EFL(16, 4, false);
#undef MTB_EFLS
#undef MTB_EFL
        } else if (per == 8) {
            if (jMajor) MTB_EF(8, true);
            else MTB_EF(8, false);
        } else {
            if (jMajor) MTB_EF(kFilterPer, true);
            else MTB_EF(kFilterPer, false);
        }
#undef MTB_EF
    }
    unsigned long long Q[2] = {0, 0};
    hipMemcpyAsync(Q, counter, sizeof(Q), hipMemcpyDeviceToHost, s);
    if (binRc) hipMemcpyAsync(binHost, binCnt, kSortBins * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (Q[1] >> 63) {  // a block's bases past the LDS stage (kSeqLds): never expected in a uniform batch
        fprintf(stderr, "[mtb] internal error: K1F sequence stage overflow\n");
        Q[1] &= ~(1ull << 63);
        *emitted = ~0ull;
        return ~0ull;
    }
    *emitted = Q[1];
    if (binRc) {
        Q[0] = 0;
        for (int r = 0; r < kSortBins; r++) Q[0] += binHost[r];
    }
    // MTB_AB_FILTER=1 (diagnostics; results unaffected): after the real pass, two timed passes that
    // write no output (cap 0) and count into a scratch word — with the probes, and with none (an empty
    // rank range) — to split the kernel's time between the probe-line reads, the scan and the packing
    static const bool abDiag = getenv("MTB_AB_FILTER") && atoi(getenv("MTB_AB_FILTER")) == 1;
    if (abDiag && nUnits) {
        const unsigned blocks = (unsigned)(((nUnits + 63) / 64 * 64 + 255) / 256);
        unsigned long long* sc = nullptr;
        hipEvent_t ev[3];
        if (hipMalloc((void**)&sc, 2 * sizeof(unsigned long long)) == hipSuccess) {
            for (auto& e : ev) hipEventCreate(&e);
            hipMemsetAsync(sc, 0, 2 * sizeof(unsigned long long), s);
            // the form the batch ran (link lines: without probes every window reads word 0, from the cache)
            hipEventRecord(ev[0], s);
            for (int pass = 0; pass < 2; pass++) {
                const uint64_t lo = pass ? 0 : rankLo, hi = pass ? 0 : rankHi;
                if (link)
                    k_extract_filter<kFilterPer, true, false, 4><<<blocks, 256, 0, s>>>(
                        seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits, C, extract_tables(t), kmerFormat, syncmer,
                        smerLen, unitInfo, lines, qkey, qslot, sc, lo, hi, 0, nullptr, nullptr, 0, upr, link);
                else
                    k_extract_filter<kFilterPer, true, false, 0, true><<<blocks, 256, 0, s>>>(
                        seq1, off1, seq2, off2, meta, uOff, unitRead, nUnits, C, extract_tables(t), kmerFormat, syncmer,
                        smerLen, unitInfo, lines, qkey, qslot, sc, lo, hi, 0, nullptr, nullptr, 0, upr, nullptr);
                hipEventRecord(ev[pass + 1], s);
            }
            hipStreamSynchronize(s);
            float a = 0, b = 0;
            hipEventElapsedTime(&a, ev[0], ev[1]);
            hipEventElapsedTime(&b, ev[1], ev[2]);
            fprintf(stderr, "[mtb ab filter] windows %llu present %llu: probes, no output %.3f ms; no probes %.3f ms\n",
                    (unsigned long long)Q[1], (unsigned long long)Q[0], a, b);
            for (auto& e : ev) hipEventDestroy(e);
            hipFree(sc);
        }
    }
    return Q[0];
}

uint64_t launch_filter(const uint64_t* keys, uint64_t R, const ProbeLine* lines, uint64_t* qkey, uint32_t* qslot,
                       uint64_t* qfrom, unsigned long long* counter, uint64_t rankLo, uint64_t rankHi,
                       uint64_t* emitted, hipStream_t s) {
    hipMemsetAsync(counter, 0, 2 * sizeof(unsigned long long), s);
    const uint64_t blocks = (R + 256 * kFilterPer - 1) / (256 * kFilterPer);
    if (blocks) {
        if (qfrom) k_filter<true><<<(unsigned)blocks, 256, 0, s>>>(keys, R, lines, qkey, qslot, qfrom, counter, rankLo, rankHi);
        else k_filter<false><<<(unsigned)blocks, 256, 0, s>>>(keys, R, lines, qkey, qslot, qfrom, counter, rankLo, rankHi);
    }
    unsigned long long Q[2] = {0, 0};
    hipMemcpyAsync(Q, counter, sizeof(Q), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    *emitted = Q[1];
    return Q[0];
}

// ------------------------------------------------------------------------------------------------
// K4P probe join (the default): instead of sorting the present query k-mers and streaming the DB
// past them (sort + k_match), each one reads its run directly: 8 DB values and taxIDs from its
// lower bound (K1F), which almost always hold the whole run (longer runs: exponential + binary
// search). One thread per query, dense. Selection, per-read counting, staging and the transpose
// that follows are k_match's, so the matches are identical.
// ------------------------------------------------------------------------------------------------
// First index >= lo with a[i] >= key (an answer exists below D + kDbPad: the pad is ~0).
// First index >= lo with a[i] >= key, by galloping from lo in steps 1, 2, 4, ... (runs at GTDB
// scale are 1-2 k-mers: the first probes stay in lo's line).
template <typename A>
__device__ __forceinline__ uint64_t gallop_lower1(const A& a, uint64_t lo, uint64_t key) {
    uint64_t step = 1, hi = lo;
    while (a[hi] < key) {
        lo = hi + 1;
        hi += step;
        step *= 2;
    }
    return lower_bound_u64(a, lo, hi, key);
}

template <typename A>
__device__ __forceinline__ uint64_t gallop_lower(const A& a, uint64_t lo, uint64_t key) {
    uint64_t step = 8, hi = lo;
    while (a[hi] < key) {
        lo = hi + 1;
        hi += step;
        step *= 2;
    }
    return lower_bound_u64(a, lo, hi, key);
}

__global__ void __launch_bounds__(256) k_probe(const uint64_t* __restrict__ qkey, const uint32_t* __restrict__ qslot,
                                               const uint64_t* __restrict__ qfrom, uint64_t Q,
                                               const uint64_t* __restrict__ unitInfo, uint32_t C,
                                               const DbRec* __restrict__ db,
                                               uint64_t D, const int32_t* __restrict__ spOf, uint32_t maxTax,
                                               int kmerFormat, uint32_t* __restrict__ readCnt,
                                               unsigned long long* __restrict__ total, mtb_match* __restrict__ buf,
                                               uint32_t* __restrict__ bufRank, uint64_t region, int* __restrict__ err,
                                               unsigned long long* __restrict__ stats) {
    const DbVal dbv{db};
    const DbTax dbtax{db};
    __shared__ unsigned long long sBase;
    const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = q < Q;
    const uint64_t key = live ? qkey[q] : 0, from = live ? qfrom[q] : 0;
    const uint32_t slot = live ? qslot[q] : 0;
    uint64_t v[8];
    uint32_t tax[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        v[k] = dbv[from + k];
        tax[k] = dbtax[from + k];
    }
    const uint64_t x = key >> 24;
    uint32_t below = 0, in = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        below += (v[k] >> 24) < x;
        in += (v[k] >> 24) == x;
    }
    const HamRows hr = hamming_rows(key);
    const bool inReg = below + in < 8 || from + 8 >= D;
    uint64_t lo, hi;
    uint32_t thr = 0, c = 0;
    uint32_t sums[8];
    if (inReg) {
        lo = from + below;
        hi = min(lo + in, D - 1);  // the last DB k-mer is never a candidate (run_select)
        uint32_t minSum = 255;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const bool in_run = from + k >= lo && from + k < hi;
            sums[k] = in_run ? hamming_sum_rows(hr, v[k]) : 255u;
            minSum = min(minSum, sums[k]);
        }
        thr = min(minSum * 2u, 7u);
#pragma unroll
        for (int k = 0; k < 8; k++) c += sums[k] <= thr;
    } else {
        lo = below < 8 ? from + below : gallop_lower(dbv, from + 8, x << 24);
        hi = gallop_lower(dbv, max(lo, from + 8), (x + 1) << 24);
        c = run_select(hr, dbv, 0, lo, hi, D, thr);
    }
    if (!live) c = 0;
    const uint64_t info = c ? slot_info(slot, C, unitInfo, kmerFormat) : 0;
    // The query's first rank inside its read's segment. Queries arrive in K1 slot order, so a
    // wave's queries come from a few reads: one atomic per (wave, read) with the group's sum,
    // the lanes' ranks from a scan inside the group (per-query atomics would queue on one address).
    uint32_t rk = 0;
    {
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t r = c ? info_seq(info) - 1 : 0xFFFFFFFFu;
        unsigned long long todo = __ballot(c != 0);
        while (todo) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
            const uint32_t r0 = __shfl(r, leader);
            const unsigned long long grp = __ballot(r == r0);
            const uint32_t mine = r == r0 ? c : 0u;
            const uint32_t pre = (uint32_t)wave_inclusive_scan(mine) - mine;
            const uint32_t sum = __shfl(pre + mine, 63);
            uint32_t b = 0;
            if (lane == leader) b = atomicAdd(&readCnt[r0], sum);
            b = __shfl(b, leader);
            if (r == r0) rk = b + pre;
            todo &= ~grp;
        }
    }
    const int blockHits = __syncthreads_count(c != 0);
    if (threadIdx.x == 0 && blockHits)
        atomicAdd(&stats[blockIdx.x % kStatStripes], (unsigned long long)blockHits);  // matched queries
    unsigned long long blockTot;
    uint64_t w = block_exclusive_scan(c, &blockTot);
    const uint32_t reg = blockIdx.x % kStageRegions;
    if (threadIdx.x == 0) sBase = blockTot ? atomicAdd(&total[reg], blockTot) : 0;
    __syncthreads();
    const uint64_t base = sBase;
    if (base + blockTot > region || !c) return;  // region too small: the caller grows it and reruns
    w += base + (uint64_t)reg * region;
    if (!inReg) {
        run_emit(key, hr, info, dbv, dbtax, lo, hi, thr, spOf, maxTax, kmerFormat, buf, bufRank, w, w + c, rk, err);
        return;
    }
    const bool rev = ((info_frame(info) < 3) != (kmerFormat == 2));
    uint32_t rank = rk;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (sums[k] > thr) continue;
        const uint32_t t = tax[k];
        const int32_t sp = t <= maxTax ? spOf[t] : 0;
        if (t == 0 || sp <= 0) atomicExch(err, kErrTaxid);  // KmerMatcher.cpp:432-441 exits
        mtb_match m;
        m.qinfo = info;
        m.target_id = t;
        m.species_id = (uint32_t)sp;
        m.dna_encoding = (uint32_t)(v[k] & 0xFFFFFFull);
        m.right_end_hamming = (uint16_t)hammings_rows(hr, key, v[k], rev);
        m.hamming = (uint8_t)sums[k];
        m.pad = 0;
        bufRank[w] = rank++;
        buf[w++] = m;
    }
}

void launch_probe(const uint64_t* qkey, const uint32_t* qslot, const uint64_t* qfrom, uint64_t Q,
                  const uint64_t* unitInfo, uint32_t C, const DbRec* db, uint64_t D,
                  const int32_t* spOf, uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total,
                  mtb_match* buf, uint32_t* bufRank, uint64_t region, int* err, unsigned long long* stats,
                  hipStream_t s) {
    if (Q == 0 || D < 2) return;
    k_probe<<<(unsigned)((Q + 255) / 256), 256, 0, s>>>(qkey, qslot, qfrom, Q, unitInfo, C, db, D, spOf, maxTax,
                                                        kmerFormat, readCnt, total, buf, bufRank, region, err, stats);
}

bool unstaged_join(bool lines, uint64_t D, uint64_t Q, uint32_t winCap) {
    // MTB_STAGE_FREE_RATIO (experiments): the D / Q ratio above which K4 goes unstaged
    static const uint64_t ratio = [] {
        const char* e = getenv("MTB_STAGE_FREE_RATIO");
        return e ? (uint64_t)strtoull(e, nullptr, 10) : (uint64_t)kStageFreeRatio;
    }();
    return lines && (D > ratio * Q || winCap == 0);
}

// mtb_hamming: the device's Hamming functions on given pairs — the row-cached forms K4 emits with
// (hamming_sum_rows, hammings_rows) next to the plain forms (hamming_sum, hammings); bad counts
// the pairs where the two disagree.
__global__ void k_hamming_check(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint64_t n,
                                uint8_t* __restrict__ sum, uint16_t* __restrict__ fwd, uint16_t* __restrict__ rev,
                                unsigned long long* __restrict__ bad) {
    MTB_GRID_STRIDE(i, n) {
        const HamRows hr = hamming_rows(a[i]);
        const uint32_t s = hamming_sum_rows(hr, b[i]);
        const uint32_t f = hammings_rows(hr, a[i], b[i], false), r = hammings_rows(hr, a[i], b[i], true);
        if (s != hamming_sum(a[i], b[i]) || f != hammings(a[i], b[i], false) || r != hammings(a[i], b[i], true))
            atomicAdd(bad, 1ull);
        sum[i] = (uint8_t)s;
        fwd[i] = (uint16_t)f;
        rev[i] = (uint16_t)r;
    }
}

void launch_hamming_check(const uint64_t* a, const uint64_t* b, uint64_t n, uint8_t* sum, uint16_t* fwd, uint16_t* rev,
                          unsigned long long* bad, hipStream_t s) {
    if (n) k_hamming_check<<<stride_grid(n), 256, 0, s>>>(a, b, n, sum, fwd, rev, bad);
}

// MTB_DUP_STATS=1 (diagnostic): how much of the reference's identical-query and same-AA reuse
// (KmerMatcher.cpp:277-353: a query equal to the previous one replays its matches; one with the
// same AA part re-runs compareDna on the cached candidates) the join's blocks could exploit. Per
// block of 256 sorted queries (K4's unstaged block): the keys bitonic-sorted in LDS, then out[0] +=
// queries whose AA rank equals an earlier one's in the block (a run lookup another query of the
// block already made), out[1] += queries whose whole key (AA + DNA) does (identical queries).
__global__ void __launch_bounds__(256) k_dup_stats(const uint64_t* __restrict__ qkey, uint64_t Q,
                                                   unsigned long long* __restrict__ out) {
    __shared__ uint64_t sk[256];
    const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    sk[threadIdx.x] = q < Q ? qkey[q] : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= 256; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t i = threadIdx.x, l = i ^ j;
            if (l > i) {
                const uint64_t a = sk[i], b = sk[l];
                if (((i & k) == 0) == (a > b)) {
                    sk[i] = b;
                    sk[l] = a;
                }
            }
            __syncthreads();
        }
    const uint32_t i = threadIdx.x;
    const bool valid = sk[i] != ~0ull && i > 0;
    const uint32_t aa = valid && (sk[i] >> 24) == (sk[i - 1] >> 24), same = valid && sk[i] == sk[i - 1];
    const int nAa = __syncthreads_count(aa), nSame = __syncthreads_count(same);
    if (threadIdx.x == 0) {
        if (nAa) atomicAdd(&out[0], (unsigned long long)nAa);
        if (nSame) atomicAdd(&out[1], (unsigned long long)nSame);
    }
}

void launch_dup_stats(const uint64_t* qkey, uint64_t Q, unsigned long long* out, hipStream_t s) {
    if (Q) k_dup_stats<<<(unsigned)((Q + 255) / 256), 256, 0, s>>>(qkey, Q, out);
}

uint64_t match_window_elems(uint64_t Q) { return 2 * ((Q + kMatchQ - 1) / kMatchQ); }

void launch_match_windows(const uint64_t* qkey, uint64_t Q, const DbRec* db, uint64_t D, const AADir& dir,
                          int kmerFormat, uint64_t* win, hipStream_t s) {
    if (Q == 0 || D < 2) return;
    const uint64_t nb = (Q + kMatchQ - 1) / kMatchQ;
    k_match_windows<<<(unsigned)((2 * nb + 255) / 256), 256, 0, s>>>(qkey, Q, db, D, dir, kmerFormat, nb, win);
}

void launch_match(const uint64_t* qkey, const uint32_t* qslot, const uint64_t* unitInfo, uint32_t C, uint64_t Q,
                  const DbRec* db, uint64_t D, const AADir& dir, const int32_t* spOf,
                  uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total, mtb_match* buf,
                  uint32_t* bufRank, uint64_t region, int* err, uint32_t winCap, const uint64_t* win,
                  const ProbeLine* lines, const uint64_t* lineP, const uint16_t* runOff, int sortLo,
                  unsigned long long* stats, SegMatch* direct, const uint64_t* dirOff, int* overflow,
                  uint32_t capShift, LongRun* longList, uint32_t longCap, uint32_t* longCnt, hipStream_t s,
                  const ProbeExt* lineExt, uint32_t upr, unsigned long long* cnt64) {
    if (Q == 0 || D < 2) return;
    winCap = std::min<uint32_t>(winCap, kMatchWin);
    // a block's window holds ~256 * D / Q values: far past the LDS cap, every block would take the
    // HBM path anyway
    if (unstaged_join(lines != nullptr, D, Q, winCap)) {
        const unsigned blocks = (unsigned)((Q + 256 * kFreePer - 1) / (256 * kFreePer));
        // MTB_MATCH_LEAN=0 (A/B, read per batch): the full-LDS form even without run-length lines or sharing
        const char* le = getenv("MTB_MATCH_LEAN");
        const bool leanOk = !le || atoi(le) != 0;
        // MTB_MATCH_WAVES (A/B, read per batch): the lean form's waves per SIMD — 6 (80 VGPRs, no
        // spills; the default), 7 or 8 (72 / 64 VGPRs with scratch spills)
        const char* we = getenv("MTB_MATCH_WAVES");
        const int waves = we ? atoi(we) : 6;
#define MTB_K4_LEAN(W)                                                                                             \
    k_match<false, kFreePer, W, false><<<blocks, 256, 0, s>>>(qkey, qslot, unitInfo, C, Q, db, D, dir, spOf, maxTax, kmerFormat, \
                                                       readCnt, total, buf, bufRank, region, err, winCap, win, lines,   \
                                                       lineP, runOff, sortLo, stats, direct, dirOff, overflow, capShift, \
                                                       longList, longCap, longCnt, nullptr, upr, cnt64)
        // MTB_JOIN_FAST=0 (A/B, read per batch): the production configuration through k_match's lean form
        // instead of k_join_uniform
        const char* fe = getenv("MTB_JOIN_FAST");
        const char* wfe = getenv("MTB_JOIN_WAVE");  // run-length lines: only the wave form (mode 5) reads them
        const bool fastOk = (!fe || atoi(fe) != 0) && leanOk && lines && runOff &&
                            (!lineExt || !wfe || atoi(wfe) == 1) && direct && longList &&
                            upr && cnt64 && !h_shareRuns && !h_prefetch && !h_pairRead && !h_matchXcd &&
                            !h_abRankFree;
        if (fastOk) {
            // MTB_JOIN_WAVE=1 (A/B, read per batch): the per-wave staging form
            const char* wf = getenv("MTB_JOIN_WAVE");
            const int wmode = wf ? atoi(wf) : 1;
            unsigned grid = (unsigned)((Q + 255) / 256);
#define MTB_K4_JOIN(M)                                                                                              \
    k_join_uniform<M><<<grid, 256, 0, s>>>(qkey, qslot, C, Q, db, D, spOf, maxTax, kmerFormat, total, buf, bufRank,  \
                                           region, err, lines, lineP, runOff, sortLo, stats, direct, overflow,      \
                                           capShift, longList, longCap, longCnt, upr, cnt64, lineExt)
            if (wmode == 2 || wmode == 3) {  // resident waves: 7 (6) blocks of 4 waves per CU
                int dev = 0, cus = 256;
                if (hipGetDevice(&dev) == hipSuccess)
                    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
                grid = std::min<unsigned>(grid, (unsigned)std::max(cus, 1) * (wmode == 2 ? 7u : 6u));
                if (wmode == 2) MTB_K4_JOIN(2);
                else MTB_K4_JOIN(3);
            } else if (wmode == 4) {  // a wave per block: a finished wave frees its slot at once
                k_join_uniform<1><<<(unsigned)((Q + 63) / 64), 64, 0, s>>>(
                    qkey, qslot, C, Q, db, D, spOf, maxTax, kmerFormat, total, buf, bufRank, region, err, lines, lineP,
                    runOff, sortLo, stats, direct, overflow, capShift, longList, longCap, longCnt, upr, cnt64, nullptr);
            } else if (lineExt) {  // MTB_LINE_EXT=1 with the wave form: runs from the staged run-length lines
                MTB_K4_JOIN(5);
            } else if (wmode >= 6 && wmode <= 8) {  // two queries per lane
#define MTB_K4_PAIR(W)                                                                                              \
    k_join_pair<W><<<(unsigned)((Q + 511) / 512), 256, 0, s>>>(qkey, qslot, C, Q, db, D, spOf, maxTax, kmerFormat,   \
                                                              total, buf, bufRank, region, err, lines, lineP, runOff, \
                                                              sortLo, stats, direct, overflow, capShift, longList,    \
                                                              longCap, longCnt, upr, cnt64)
                if (wmode == 6) MTB_K4_PAIR(6);
                else if (wmode == 7) MTB_K4_PAIR(7);
                else MTB_K4_PAIR(8);
#undef MTB_K4_PAIR
            } else if (wmode == 1 && getenv("MTB_JOIN_PAD")) {
                // A/B diagnostic: dynamic LDS reserved per block (unused) to cap the waves per SIMD
                k_join_uniform<1><<<grid, 256, (size_t)atoi(getenv("MTB_JOIN_PAD")), s>>>(
                    qkey, qslot, C, Q, db, D, spOf, maxTax, kmerFormat, total, buf, bufRank, region, err, lines, lineP,
                    runOff, sortLo, stats, direct, overflow, capShift, longList, longCap, longCnt, upr, cnt64, lineExt);
            } else if (wmode == 7) {
                MTB_K4_JOIN(7);
            } else if (wmode == 1) {
                MTB_K4_JOIN(1);
            } else {
                MTB_K4_JOIN(0);
            }
#undef MTB_K4_JOIN
        } else
        if (leanOk && !(runOff && lineExt) && !h_shareRuns && h_prefetch && runOff) {
            k_match<false, kFreePer, 6, true><<<blocks, 256, 0, s>>>(qkey, qslot, unitInfo, C, Q, db, D, dir, spOf, maxTax,
                                                                     kmerFormat, readCnt, total, buf, bufRank, region,
                                                                     err, winCap, win, lines, lineP, runOff, sortLo,
                                                                     stats, direct, dirOff, overflow, capShift, longList,
                                                                     longCap, longCnt, nullptr, upr, cnt64);
        } else if (leanOk && !(runOff && lineExt) && !h_shareRuns) {
            if (waves == 8) MTB_K4_LEAN(8);
            else if (waves == 7) MTB_K4_LEAN(7);
            else MTB_K4_LEAN(6);
        } else
#undef MTB_K4_LEAN
            k_match<false, kFreePer><<<blocks, 256, 0, s>>>(qkey, qslot, unitInfo, C, Q, db, D, dir, spOf, maxTax,
                                                            kmerFormat, readCnt, total, buf, bufRank, region, err, winCap,
                                                            win, lines, lineP, runOff, sortLo, stats, direct, dirOff,
                                                            overflow, capShift, longList, longCap, longCnt,
                                                            runOff ? lineExt : nullptr, upr, cnt64);
    } else {
        const unsigned blocks = (unsigned)((Q + kMatchQ - 1) / kMatchQ);
        k_match<true, kMatchQ / 256><<<blocks, 256, 0, s>>>(qkey, qslot, unitInfo, C, Q, db, D, dir, spOf,
                                                            maxTax, kmerFormat, readCnt, total, buf, bufRank, region,
                                                            err, winCap, win, lines, nullptr, nullptr, kQuerySortLo,
                                                            stats, direct, dirOff, overflow, capShift, nullptr, 0,
                                                            longCnt, nullptr, upr, cnt64);
    }
}

// Direct join output -> compact per-read segments: read r's n = readOff[r + 1] - readOff[r]
// matches from its reserved stretch (dirOff[r] * C), expanded to mtb_match, to readOff[r]. One wave
// per read, coalesced.
__global__ void __launch_bounds__(256) k_compact_segments(const SegMatch* __restrict__ in,
                                                          const uint64_t* __restrict__ dirOff, uint32_t C,
                                                          const uint64_t* __restrict__ readOff, uint32_t nReads,
                                                          mtb_match* __restrict__ out, uint32_t capShift, int mode) {
    const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= nReads) return;
    const uint64_t src = dirOff[r] * C, dst = readOff[r];
    const uint64_t cap = ((dirOff[r + 1] - dirOff[r]) * C) >> capShift;
    // mode 1: only the reads that overflowed their stretch (K5 reads the others in place); mode 2:
    // all but those (compacted with their spills already, by a mode-1 pass + k_spill_scatter)
    const bool over = readOff[r + 1] - dst > cap;
    if ((mode == 1 && !over) || (mode == 2 && over)) return;
    const uint64_t n = min(readOff[r + 1] - dst, cap);  // ranks past it: spilled
    for (uint64_t i = lane; i < n; i += 64) out[dst + i] = seg_expand(in[src + i], (uint64_t)(r + 1) << 32);
}

// The direct join's spilled matches (queries whose ranks passed their read's stretch) to their
// ranks in the compacted segments, after k_compact_segments (which leaves those ranks stale).
__global__ void k_spill_scatter(const mtb_match* __restrict__ spill, const uint32_t* __restrict__ spillRank,
                                const unsigned long long* __restrict__ total, const uint64_t* __restrict__ readOff,
                                uint32_t nReads, mtb_match* __restrict__ out, int* __restrict__ err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total[0]) return;
    const mtb_match m = spill[i];
    const uint32_t r = info_seq(m.qinfo) - 1;
    if (r >= nReads || readOff[r] + spillRank[i] >= readOff[r + 1]) {  // never write out of bounds
        atomicExch(err, kErrStagedRead);
        return;
    }
    out[readOff[r] + spillRank[i]] = m;
}

void launch_spill_scatter(const mtb_match* spill, const uint32_t* spillRank, const unsigned long long* total,
                          uint64_t nSpill, const uint64_t* readOff, uint32_t nReads, mtb_match* out, int* err,
                          hipStream_t s) {
    if (nSpill) k_spill_scatter<<<(unsigned)((nSpill + 255) / 256), 256, 0, s>>>(spill, spillRank, total, readOff, nReads,
                                                                               out, err);
}

void launch_compact_segments(const SegMatch* in, const uint64_t* dirOff, uint32_t C, const uint64_t* readOff,
                             uint32_t nReads, mtb_match* out, uint32_t capShift, hipStream_t s, int mode) {
    if (nReads)
        k_compact_segments<<<(nReads + 3) / 4, 256, 0, s>>>(in, dirOff, C, readOff, nReads, out, capShift, mode);
}

void launch_match_transpose(const mtb_match* buf, const uint32_t* bufRank, uint64_t region,
                            const unsigned long long* total, const uint64_t* readOff, uint32_t nReads, mtb_match* out,
                            int* err, hipStream_t s) {
    const uint64_t slots = region * kStageRegions;
    if (slots)
        k_match_transpose<<<(unsigned)((slots + 255) / 256), 256, 0, s>>>(buf, bufRank, region, total, readOff,
                                                                          nReads, out, err);
}

__global__ void k_mask_info(uint32_t* info, uint64_t n, uint32_t mask) {
    MTB_GRID_STRIDE(i, n) info[i] &= mask;
}

void launch_mask_info(uint32_t* info, uint64_t n, uint32_t mask, hipStream_t s) {
    if (n && mask != ~0u) k_mask_info<<<stride_grid(n), 256, 0, s>>>(info, n, mask);
}

// ------------------------------------------------------------------------------------------------
// K4S DB-sweep join (MTB_JOIN=sweep): the reference's own shape — matchKmers streams the whole
// diffIdx past each sorted query split (KmerMatcher.cpp:363-406) — as one pass over the resident
// records in DB order. The DB is cut once into tiles of ~kSweepNom records that end at sort-prefix
// bucket bounds (value >> kQuerySortLo: the query keys' sort prefix), so a tile's queries are one
// contiguous stretch of the sorted query array (qStart, per batch). A block stages its tile in LDS
// with coalesced 16-B loads (every load in flight before the first LDS write), then each of the
// tile's queries finds its AA run by a fixed-trip binary search in LDS and selects / emits as the
// random-access join does. A tile without queries costs two loads and no DB bytes. No run index,
// no probe lines, no per-query random DB reads.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kSweepCap = 4096;  // records a tile stages in LDS (48 KB); a longer tile searches HBM
constexpr uint64_t kSweepPrefixes = 1ull << (kQuerySortHi - kQuerySortLo);

__device__ __forceinline__ uint32_t key_prefix(uint64_t v) { return (uint32_t)(v >> kQuerySortLo); }

// starts[p] = first index i of the sorted array with prefix(a[i]) >= p, for p in [0, 2^24]: each
// element that opens a prefix writes its index there (the rest hold ~0 from a memset), then a
// suffix minimum fills the prefixes no element has (the gaps are unbounded for a small array)
template <typename A, typename S>
__global__ void k_prefix_firsts(A a, uint64_t n, S* __restrict__ starts) {
    MTB_GRID_STRIDE(i, n + 1) {
        if (i == n) {
            starts[kSweepPrefixes] = (S)n;
        } else {
            const uint32_t p = key_prefix(a[i]);
            if (i == 0 || key_prefix(a[i - 1]) != p) starts[p] = (S)i;
        }
    }
}

constexpr int kSufTile = 1024;  // entries per block of the suffix minimum (4 per thread)

template <typename S>
__global__ void __launch_bounds__(256) k_suffix_min_tiles(S* __restrict__ x, uint64_t n, S* __restrict__ tileMin) {
    __shared__ S sm[256];
    const uint64_t t0 = (uint64_t)blockIdx.x * kSufTile;
    S v[4];
    S m = (S)~(S)0;
#pragma unroll
    for (int k = 3; k >= 0; k--) {  // each thread's 4 entries, suffix min within them
        const uint64_t i = t0 + threadIdx.x * 4 + k;
        v[k] = i < n ? x[i] : (S)~(S)0;
        m = min(m, v[k]);
        v[k] = m;
    }
    sm[threadIdx.x] = m;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {  // suffix min over the threads (Hillis-Steele)
        const S o = threadIdx.x + d < 256 ? sm[threadIdx.x + d] : (S)~(S)0;
        __syncthreads();
        sm[threadIdx.x] = min(sm[threadIdx.x], o);
        __syncthreads();
    }
    const S after = threadIdx.x + 1 < 256 ? sm[threadIdx.x + 1] : (S)~(S)0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t i = t0 + threadIdx.x * 4 + k;
        if (i < n) x[i] = min(v[k], after);
    }
    if (threadIdx.x == 0) tileMin[blockIdx.x] = sm[0];
}

// tileMin[t] <- the minimum over the tiles after t (one 1024-thread block, a chunk of tiles per thread)
template <typename S>
__global__ void __launch_bounds__(1024) k_suffix_min_carry(S* __restrict__ tileMin, uint64_t nTiles) {
    __shared__ S sm[1024];
    const uint64_t per = (nTiles + 1023) / 1024, b = threadIdx.x * per, e = min(nTiles, b + per);
    S m = (S)~(S)0;
    for (uint64_t t = b; t < e; t++) m = min(m, tileMin[t]);
    sm[threadIdx.x] = m;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const S o = threadIdx.x + d < 1024 ? sm[threadIdx.x + d] : (S)~(S)0;
        __syncthreads();
        sm[threadIdx.x] = min(sm[threadIdx.x], o);
        __syncthreads();
    }
    S after = threadIdx.x + 1 < 1024 ? sm[threadIdx.x + 1] : (S)~(S)0;
    for (uint64_t t = e; t-- > b;) {
        const S v = tileMin[t];
        tileMin[t] = after;
        after = min(after, v);
    }
}

template <typename S>
__global__ void k_suffix_min_apply(S* __restrict__ x, uint64_t n, const S* __restrict__ carry) {
    MTB_GRID_STRIDE(i, n) x[i] = min(x[i], carry[i / kSufTile]);
}

template <typename A, typename S>
static void prefix_starts(A a, uint64_t n, S* starts, S* tmp, hipStream_t s) {
    const uint64_t m = kSweepPrefixes + 1, nT = (m + kSufTile - 1) / kSufTile;
    hipMemsetAsync(starts, 0xFF, sizeof(S) * m, s);
    k_prefix_firsts<<<stride_grid(n + 1), 256, 0, s>>>(a, n, starts);
    k_suffix_min_tiles<<<(unsigned)nT, 256, 0, s>>>(starts, m, tmp);
    k_suffix_min_carry<<<1, 1024, 0, s>>>(tmp, nT);
    k_suffix_min_apply<<<stride_grid(m), 256, 0, s>>>(starts, m, tmp);
}

struct KeyArr {
    const uint64_t* __restrict__ k;
    __device__ __forceinline__ uint64_t operator[](uint64_t i) const { return k[i]; }
};

// tile j = DB records [tileRec[j], tileRec[j + 1]) = prefix buckets [tilePre[j], tilePre[j + 1]): the
// nominal start j * nom snapped down to the start of its bucket (a bucket longer than nom leaves
// empty tiles behind it, which no query names)
__global__ void k_sweep_tiles(const DbRec* __restrict__ db, uint64_t D, const uint64_t* __restrict__ pstart,
                              uint64_t nTiles, uint32_t nom, uint64_t* __restrict__ tileRec,
                              uint32_t* __restrict__ tilePre) {
    MTB_GRID_STRIDE(j, nTiles + 1) {
        if (j == nTiles) {
            tileRec[j] = D;
            tilePre[j] = (uint32_t)kSweepPrefixes;
        } else {
            const uint32_t p = key_prefix((uint64_t)db[j * nom].hi << 32 | db[j * nom].lo);
            tileRec[j] = pstart[p];
            tilePre[j] = p;
        }
    }
}

// One query of a tile against the tile's records (LDS or HBM view; vOff = DB index of view[0]); its
// key, slot and unit record are loaded by the caller (the first query of a thread while its tile is
// still in flight).
template <typename V, typename T>
__device__ __forceinline__ bool sweep_query(uint64_t q, uint64_t key, uint32_t slot, ulonglong2 ur, const V& vals,
                                            const T& taxs, uint32_t n, uint32_t pow2, uint64_t vOff, uint32_t C,
                                            uint64_t D, const int32_t* __restrict__ spOf, uint32_t maxTax,
                                            int kmerFormat, uint32_t* __restrict__ readCnt,
                                            unsigned long long* __restrict__ total, mtb_match* __restrict__ buf,
                                            uint32_t* __restrict__ bufRank, uint64_t region, int* __restrict__ err,
                                            SegMatch* __restrict__ direct, int* __restrict__ overflow, uint32_t capShift,
                                            LongRun* __restrict__ longList, uint32_t longCap,
                                            uint32_t* __restrict__ longCnt) {
    const uint64_t aa = key & kAAMask, aa2 = aa + (1ull << 24);
    uint32_t p1 = 0, p2 = 0;  // lower bounds of aa and aa2: two fixed-trip searches, interleaved
    for (uint32_t step = pow2; step > 0; step >>= 1) {
        const uint32_t i1 = p1 + step, i2 = p2 + step;
        if (i1 <= n && vals[i1 - 1] < aa) p1 = i1;
        if (i2 <= n && vals[i2 - 1] < aa2) p2 = i2;
    }
    uint64_t lo = p1, hi = p2;
    if (lo + vOff > D) {  // a tile past the DB's end (inconsistent tiles): flagged, the run taken as empty
        atomicExch(err, kErrRunOutsideDb);
        lo = D - vOff;
    }
    if (hi + vOff > D - 1) hi = D - 1 - vOff;  // the last DB k-mer is never a candidate
    if (lo > hi) hi = lo;
    if (hi - lo > kLongRun) {  // a long run: scanned by a wave of its own (k_match_long), from HBM
        const uint32_t at = atomicAdd(longCnt, 1u);
        if (at < longCap) longList[at] = LongRun{q, lo + vOff, hi + vOff};
        return false;
    }
    const HamRows hr = hamming_rows(key);
    uint32_t thr = 0;
    const uint32_t c = run_select(hr, vals, vOff, lo, hi, D, thr);
    if (!c) return false;
    uint32_t pu;
    (void)slot_unit(slot, C, pu);
    const uint64_t info = unit_info_at(ur.x, pu, kmerFormat);
    const uint32_t rk = atomicAdd(&readCnt[info_seq(info) - 1], c);
    const uint64_t o = (ur.y & kStretchLoMask) * C, cap = ((ur.y >> 40) * C) >> capShift;
    if (rk + c > cap) {  // past the read's stretch: spilled with the ranks (scattered after compaction)
        const uint64_t sp = atomicAdd(&total[0], (unsigned long long)c);
        if (sp + c > region) {
            atomicExch(overflow, 1);
            return true;
        }
        run_emit(key, hr, info, vals, taxs, lo, hi, thr, spOf, maxTax, kmerFormat, buf, bufRank, sp, sp + c, rk, err);
        return true;
    }
    run_emit(key, hr, info, vals, taxs, lo, hi, thr, spOf, maxTax, kmerFormat, direct + o, (uint32_t*)nullptr,
             (uint64_t)rk, (uint64_t)rk + c, 0, err);
    return true;
}

__device__ int g_abSweepCount = 0;  // MTB_AB_SWEEP_COUNT=1 (A/B only): k_sweep_ws without emission
void set_ab_sweep_count(int on) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_abSweepCount), &on, sizeof(int)); }

// tileQ[t] = the first sorted query of tile t's buckets (per batch: one coalesced pass, so a sweep
// block reads its query range and its records' range in one round trip)
__global__ void k_tile_queries(const uint32_t* __restrict__ tilePre, uint64_t nTiles, const uint32_t* __restrict__ qStart,
                               uint32_t* __restrict__ tileQ) {
    MTB_GRID_STRIDE(t, nTiles + 1) tileQ[t] = qStart[tilePre[t]];
}

template <uint32_t kCap>
__global__ void __launch_bounds__(256) k_sweep(const uint64_t* __restrict__ tileRec, const uint32_t* __restrict__ tileQ,
                                               const uint64_t* __restrict__ qkey,
                                               const uint32_t* __restrict__ qslot, const uint64_t* __restrict__ unitInfo,
                                               uint32_t C, const DbRec* __restrict__ db, uint64_t D,
                                               const int32_t* __restrict__ spOf, uint32_t maxTax, int kmerFormat,
                                               uint32_t* __restrict__ readCnt, unsigned long long* __restrict__ total,
                                               mtb_match* __restrict__ buf, uint32_t* __restrict__ bufRank,
                                               uint64_t region, int* __restrict__ err,
                                               unsigned long long* __restrict__ stats, SegMatch* __restrict__ direct,
                                               int* __restrict__ overflow, uint32_t capShift,
                                               LongRun* __restrict__ longList, uint32_t longCap,
                                               uint32_t* __restrict__ longCnt, uint32_t ldsCap) {
    constexpr uint32_t kVec = kCap * 12 / 16 + 1;  // 16-B vectors of a full tile (+1: unaligned start)
    constexpr int kLoad = (int)((kVec + 255) / 256);
    __shared__ uint4 sRaw[kVec];
    const uint64_t t = blockIdx.x;
    const uint32_t q0 = tileQ[t], q1 = tileQ[t + 1];
    const uint64_t r0 = tileRec[t], r1 = tileRec[t + 1];
    if (q0 >= q1) return;  // no query in the tile's buckets: its records are not read
    const uint32_t n = (uint32_t)(r1 - r0);
    uint32_t pow2 = 1;
    while (pow2 * 2 <= n) pow2 *= 2;
    // the thread's first query: key and slot, then its unit record, loaded while the tile streams in
    const uint64_t qa = q0 + threadIdx.x;
    const bool has0 = qa < q1;
    uint64_t key0 = 0;
    uint32_t slot0 = 0;
    if (has0) {
        key0 = qkey[qa];
        slot0 = qslot[qa];
    }
    uint32_t hits = 0;
    auto unit_of = [&](uint32_t slot) {
        uint32_t p;
        return reinterpret_cast<const ulonglong2*>(unitInfo)[slot_unit(slot, C, p)];
    };
    auto run = [&](const auto& vals, const auto& taxs, ulonglong2 ur0) {
        if (has0)
            hits += sweep_query(qa, key0, slot0, ur0, vals, taxs, n, pow2, r0, C, D, spOf, maxTax, kmerFormat, readCnt,
                                total, buf, bufRank, region, err, direct, overflow, capShift, longList, longCap, longCnt);
        for (uint64_t q = qa + 256; q < q1; q += 256) {
            const uint32_t slot = qslot[q];
            hits += sweep_query(q, qkey[q], slot, unit_of(slot), vals, taxs, n, pow2, r0, C, D, spOf, maxTax,
                                kmerFormat, readCnt, total, buf, bufRank, region, err, direct, overflow, capShift,
                                longList, longCap, longCnt);
        }
    };
    if (n <= ldsCap && n <= kCap) {
        const uint64_t b0 = (r0 * 12) & ~15ull;
        const uint32_t nv = (uint32_t)((r1 * 12 - b0 + 15) >> 4);  // the pad records make the tail readable
        const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(db) + b0);
        uint4 v[kLoad];
#pragma unroll
        for (int j = 0; j < kLoad; j++) {  // every load in flight before the first LDS write
            const uint32_t i = threadIdx.x + (uint32_t)j * 256;
            v[j] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
        }
        ulonglong2 ur0 = make_ulonglong2(0, 0);
        if (has0) ur0 = unit_of(slot0);
#pragma unroll
        for (int j = 0; j < kLoad; j++) {
            const uint32_t i = threadIdx.x + (uint32_t)j * 256;
            if (i < nv) sRaw[i] = v[j];
        }
        __syncthreads();
        const DbRec* rec = reinterpret_cast<const DbRec*>(reinterpret_cast<const char*>(sRaw) + (r0 * 12 - b0));
        run(DbVal{rec}, DbTax{rec}, ur0);
    } else {  // one sort-prefix bucket longer than an LDS tile (heavily shared AA 8-mers): from HBM
        run(DbVal{db + r0}, DbTax{db + r0}, has0 ? unit_of(slot0) : make_ulonglong2(0, 0));
    }
    const uint32_t w = wave_sum_u32(hits);
    if ((threadIdx.x & 63) == 0 && w) atomicAdd(&stats[t % kStatStripes], (unsigned long long)w);
    if (threadIdx.x == 0) atomicAdd(&stats[kStatStripes + 1 + t % kStatStripes], (unsigned long long)n);
}

// Persistent form of the sweep: a block walks tiles blockIdx.x, + gridDim.x, ... and keeps the next
// tile's records in flight (in registers) while it searches the current one's queries from LDS, so a
// CU's HBM requests do not stop during the query phases (the rank atomics and unit-record loads are
// round trips). Tile descriptors (query range, record range) are loaded one tile further ahead.
struct SweepDesc {
    uint32_t q0, q1;
    uint64_t r0, r1;
};
__device__ __forceinline__ SweepDesc sweep_desc(const uint64_t* __restrict__ tileRec, const uint32_t* __restrict__ tileQ,
                                                uint64_t t, uint64_t nTiles) {
    if (t >= nTiles) return SweepDesc{0, 0, 0, 0};
    return SweepDesc{tileQ[t], tileQ[t + 1], tileRec[t], tileRec[t + 1]};
}

template <uint32_t kCap>
__global__ void __launch_bounds__(256) k_sweep_p(const uint64_t* __restrict__ tileRec, const uint32_t* __restrict__ tileQ,
                                                 uint64_t nTiles, const uint64_t* __restrict__ qkey,
                                                 const uint32_t* __restrict__ qslot, const uint64_t* __restrict__ unitInfo,
                                                 uint32_t C, const DbRec* __restrict__ db, uint64_t D,
                                                 const int32_t* __restrict__ spOf, uint32_t maxTax, int kmerFormat,
                                                 uint32_t* __restrict__ readCnt, unsigned long long* __restrict__ total,
                                                 mtb_match* __restrict__ buf, uint32_t* __restrict__ bufRank,
                                                 uint64_t region, int* __restrict__ err,
                                                 unsigned long long* __restrict__ stats, SegMatch* __restrict__ direct,
                                                 int* __restrict__ overflow, uint32_t capShift,
                                                 LongRun* __restrict__ longList, uint32_t longCap,
                                                 uint32_t* __restrict__ longCnt, uint32_t ldsCap) {
    constexpr uint32_t kVec = kCap * 12 / 16 + 1;
    constexpr int kLoad = (int)((kVec + 255) / 256);
    __shared__ uint4 sRaw[kVec];
    const uint64_t G = gridDim.x;
    uint64_t t = blockIdx.x;
    SweepDesc cur = sweep_desc(tileRec, tileQ, t, nTiles);
    SweepDesc nxt = sweep_desc(tileRec, tileQ, t + G, nTiles);
    auto staged = [&](const SweepDesc& d) { return d.q0 < d.q1 && d.r1 - d.r0 <= (uint64_t)min(ldsCap, kCap); };
    uint4 v[kLoad];
    auto issue = [&](const SweepDesc& d) {  // the tile's 16-B vectors into registers (all in flight)
        const uint64_t b0 = (d.r0 * 12) & ~15ull;
        const uint32_t nv = (uint32_t)((d.r1 * 12 - b0 + 15) >> 4);
        const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(db) + b0);
#pragma unroll
        for (int j = 0; j < kLoad; j++) {
            const uint32_t i = threadIdx.x + (uint32_t)j * 256;
            v[j] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
        }
    };
    if (staged(cur)) issue(cur);
    uint32_t hits = 0;
    uint64_t recs = 0;
    while (t < nTiles) {
        const bool st = staged(cur);
        if (st) {
            const uint64_t b0 = (cur.r0 * 12) & ~15ull;
            const uint32_t nv = (uint32_t)((cur.r1 * 12 - b0 + 15) >> 4);
            __syncthreads();  // the previous tile's searches are done with the LDS
#pragma unroll
            for (int j = 0; j < kLoad; j++) {
                const uint32_t i = threadIdx.x + (uint32_t)j * 256;
                if (i < nv) sRaw[i] = v[j];
            }
            __syncthreads();
        }
        // the next tile streams in while this one's queries are searched
        const SweepDesc after = sweep_desc(tileRec, tileQ, t + 2 * G, nTiles);
        if (staged(nxt)) issue(nxt);
        if (cur.q0 < cur.q1) {
            const uint32_t n = (uint32_t)(cur.r1 - cur.r0);
            uint32_t pow2 = 1;
            while (pow2 * 2 <= n) pow2 *= 2;
            recs += n;
            auto run = [&](const auto& vals, const auto& taxs) {
                for (uint64_t q = cur.q0 + threadIdx.x; q < cur.q1; q += 256) {
                    const uint32_t slot = qslot[q];
                    uint32_t p;
                    const ulonglong2 ur = reinterpret_cast<const ulonglong2*>(unitInfo)[slot_unit(slot, C, p)];
                    hits += sweep_query(q, qkey[q], slot, ur, vals, taxs, n, pow2, cur.r0, C, D, spOf, maxTax,
                                        kmerFormat, readCnt, total, buf, bufRank, region, err, direct, overflow,
                                        capShift, longList, longCap, longCnt);
                }
            };
            if (st) {
                const uint64_t b0 = (cur.r0 * 12) & ~15ull;
                const DbRec* rec = reinterpret_cast<const DbRec*>(reinterpret_cast<const char*>(sRaw) + (cur.r0 * 12 - b0));
                run(DbVal{rec}, DbTax{rec});
            } else {  // a bucket longer than an LDS tile: from HBM
                run(DbVal{db + cur.r0}, DbTax{db + cur.r0});
            }
        }
        t += G;
        cur = nxt;
        nxt = after;
    }
    const uint32_t w = wave_sum_u32(hits);
    if ((threadIdx.x & 63) == 0 && w) atomicAdd(&stats[blockIdx.x % kStatStripes], (unsigned long long)w);
    if (threadIdx.x == 0 && recs) atomicAdd(&stats[kStatStripes + 1 + blockIdx.x % kStatStripes], (unsigned long long)recs);
}

// Warp-specialised sweep (the default): a 512-thread block whose first four waves only stream tiles
// (global -> registers -> one of two LDS buffers) and whose other four only search queries. The
// vector-memory counter is per wave and in order, so in one wave a tile prefetch would hold up every
// later query load and rank atomic until the whole tile arrived (the persistent form measured ~10 us
// per tile); split over waves the two streams overlap. Lock-step iterations: in iteration k the
// loaders write tile k (loaded during iteration k-1) into buffer k & 1 and issue tile k+1's loads,
// while the searchers work on tile k-1 in the other buffer; one barrier ends the iteration.
template <uint32_t kCap>
__global__ void __launch_bounds__(512) k_sweep_ws(const uint64_t* __restrict__ tileRec, const uint32_t* __restrict__ tileQ,
                                                  uint64_t nTiles, const uint64_t* __restrict__ qkey,
                                                  const uint32_t* __restrict__ qslot,
                                                  const uint64_t* __restrict__ unitInfo, uint32_t C,
                                                  const DbRec* __restrict__ db, uint64_t D,
                                                  const int32_t* __restrict__ spOf, uint32_t maxTax, int kmerFormat,
                                                  uint32_t* __restrict__ readCnt, unsigned long long* __restrict__ total,
                                                  mtb_match* __restrict__ buf, uint32_t* __restrict__ bufRank,
                                                  uint64_t region, int* __restrict__ err,
                                                  unsigned long long* __restrict__ stats, SegMatch* __restrict__ direct,
                                                  int* __restrict__ overflow, uint32_t capShift,
                                                  LongRun* __restrict__ longList, uint32_t longCap,
                                                  uint32_t* __restrict__ longCnt, uint32_t ldsCap) {
    constexpr uint32_t kVec = kCap * 12 / 16 + 1;
    constexpr int kLoad = (int)((kVec + 255) / 256);
    __shared__ uint4 sBuf[2][kVec];
    __shared__ SweepDesc sDesc[2];
    const bool loader = threadIdx.x < 256;
    const uint32_t lt = threadIdx.x & 255;
    const uint64_t G = gridDim.x, t0 = blockIdx.x;
    const uint64_t m = t0 < nTiles ? (nTiles - t0 + G - 1) / G : 0;  // this block's tiles
    const uint32_t cap = min(ldsCap, kCap);
    auto staged = [&](const SweepDesc& d) { return d.q0 < d.q1 && d.r1 - d.r0 <= (uint64_t)cap; };
    uint4 v[kLoad];
    SweepDesc dCur{0, 0, 0, 0}, dAhead{0, 0, 0, 0};
    auto issue = [&](const SweepDesc& d) {
        const uint64_t b0 = (d.r0 * 12) & ~15ull;
        const uint32_t nv = (uint32_t)((d.r1 * 12 - b0 + 15) >> 4);
        const uint4* src = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(db) + b0);
#pragma unroll
        for (int j = 0; j < kLoad; j++) {
            const uint32_t i = lt + (uint32_t)j * 256;
            v[j] = i < nv ? src[i] : make_uint4(0, 0, 0, 0);
        }
    };
    if (loader && m) {
        dCur = sweep_desc(tileRec, tileQ, t0, nTiles);
        if (staged(dCur)) issue(dCur);
        dAhead = sweep_desc(tileRec, tileQ, t0 + G, nTiles);
    }
    uint32_t hits = 0;
    uint64_t recs = 0;
    for (uint64_t k = 0; k <= m; k++) {
        if (loader) {
            if (k < m) {  // tile k into buffer k & 1, then tile k + 1's loads
                if (staged(dCur)) {
                    const uint64_t b0 = (dCur.r0 * 12) & ~15ull;
                    const uint32_t nv = (uint32_t)((dCur.r1 * 12 - b0 + 15) >> 4);
#pragma unroll
                    for (int j = 0; j < kLoad; j++) {
                        const uint32_t i = lt + (uint32_t)j * 256;
                        if (i < nv) sBuf[k & 1][i] = v[j];
                    }
                }
                if (lt == 0) sDesc[k & 1] = dCur;
                dCur = dAhead;
                if (k + 1 < m && staged(dCur)) issue(dCur);
                dAhead = sweep_desc(tileRec, tileQ, t0 + (k + 2) * G, nTiles);
            }
        } else if (k >= 1) {  // tile k - 1 from buffer (k - 1) & 1
            const SweepDesc d = sDesc[(k - 1) & 1];
            if (d.q0 < d.q1) {
                const uint32_t n = (uint32_t)(d.r1 - d.r0);
                uint32_t pow2 = 1;
                while (pow2 * 2 <= n) pow2 *= 2;
                recs += n;
                auto run = [&](const auto& vals, const auto& taxs) {
                    for (uint64_t q = d.q0 + lt; q < d.q1; q += 256) {
                        if (g_abSweepCount) {  // A/B only: the sweep's LDS work alone (no emission: invalid results)
                            const uint64_t key = qkey[q], aa = key & kAAMask, aa2 = aa + (1ull << 24);
                            uint32_t p1 = 0, p2 = 0;
                            for (uint32_t step = pow2; step > 0; step >>= 1) {
                                const uint32_t i1 = p1 + step, i2 = p2 + step;
                                if (i1 <= n && vals[i1 - 1] < aa) p1 = i1;
                                if (i2 <= n && vals[i2 - 1] < aa2) p2 = i2;
                            }
                            uint64_t hi = p2;
                            uint32_t thr = 0;
                            hits += run_select(hamming_rows(key), vals, d.r0, (uint64_t)p1, hi, D, thr) != 0;
                            continue;
                        }
                        const uint32_t slot = qslot[q];
                        uint32_t p;
                        const ulonglong2 ur = reinterpret_cast<const ulonglong2*>(unitInfo)[slot_unit(slot, C, p)];
                        hits += sweep_query(q, qkey[q], slot, ur, vals, taxs, n, pow2, d.r0, C, D, spOf, maxTax,
                                            kmerFormat, readCnt, total, buf, bufRank, region, err, direct, overflow,
                                            capShift, longList, longCap, longCnt);
                    }
                };
                if (staged(d)) {
                    const uint64_t b0 = (d.r0 * 12) & ~15ull;
                    const DbRec* rec = reinterpret_cast<const DbRec*>(
                        reinterpret_cast<const char*>(sBuf[(k - 1) & 1]) + (d.r0 * 12 - b0));
                    run(DbVal{rec}, DbTax{rec});
                } else {  // a bucket longer than an LDS tile: from HBM
                    run(DbVal{db + d.r0}, DbTax{db + d.r0});
                }
            }
        }
        __syncthreads();
    }
    if (!loader) {
        const uint32_t w = wave_sum_u32(hits);
        if ((threadIdx.x & 63) == 0 && w) atomicAdd(&stats[blockIdx.x % kStatStripes], (unsigned long long)w);
        if (lt == 0 && recs) atomicAdd(&stats[kStatStripes + 1 + blockIdx.x % kStatStripes], (unsigned long long)recs);
    }
}

uint64_t sweep_tiles(uint64_t D, uint32_t nom) { return D ? (D + nom - 1) / nom : 0; }

void build_sweep_tiles(const DbRec* db, uint64_t D, uint32_t nom, uint64_t* pstartTmp, uint64_t* tileRec,
                       uint32_t* tilePre, hipStream_t s) {
    prefix_starts(DbVal{db}, D, pstartTmp, pstartTmp + kSweepStarts, s);
    const uint64_t nT = sweep_tiles(D, nom);
    k_sweep_tiles<<<stride_grid(nT + 1), 256, 0, s>>>(db, D, pstartTmp, nT, nom, tileRec, tilePre);
}

void build_query_starts(const uint64_t* qkey, uint64_t Q, uint32_t* qStart, const uint32_t* tilePre, uint64_t nTiles,
                        uint32_t* tileQ, hipStream_t s) {
    prefix_starts(KeyArr{qkey}, Q, qStart, qStart + kSweepStarts, s);
    k_tile_queries<<<stride_grid(nTiles + 1), 256, 0, s>>>(tilePre, nTiles, qStart, tileQ);
}

void launch_sweep(const uint64_t* tileRec, const uint32_t* tileQ, uint64_t nTiles, const uint64_t* qkey,
                  const uint32_t* qslot, const uint64_t* unitInfo, uint32_t C, const DbRec* db, uint64_t D,
                  const int32_t* spOf, uint32_t maxTax, int kmerFormat, uint32_t* readCnt, unsigned long long* total,
                  mtb_match* buf, uint32_t* bufRank, uint64_t region, int* err, unsigned long long* stats,
                  SegMatch* direct, int* overflow, uint32_t capShift, LongRun* longList, uint32_t longCap,
                  uint32_t* longCnt, uint32_t ldsCap, bool small, int persist, hipStream_t s) {
    if (!nTiles || D < 2) return;
    if (persist == 2) {  // warp-specialised: 24-KB tiles, two LDS buffers, 2 blocks of 512 threads per CU (121 VGPRs)
        int cus = 256;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        const uint64_t g = std::min<uint64_t>(nTiles, (uint64_t)cus * 2);
        k_sweep_ws<2048><<<(unsigned)g, 512, 0, s>>>(tileRec, tileQ, nTiles, qkey, qslot, unitInfo, C, db, D, spOf,
                                                     maxTax, kmerFormat, readCnt, total, buf, bufRank, region, err,
                                                     stats, direct, overflow, capShift, longList, longCap, longCnt,
                                                     ldsCap);
        return;
    }
    if (persist) {  // blocks resident on every CU (3 per CU at 48-KB tiles), each walking its tiles
        int cus = 256;
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
        // resident blocks per CU: 3 for 48-KB tiles (LDS, and 145 VGPRs), 4 for 24-KB tiles (109 VGPRs)
        const uint64_t g = std::min<uint64_t>(nTiles, (uint64_t)cus * (small ? 4 : 3) * persist);
        if (small)
            k_sweep_p<2048><<<(unsigned)g, 256, 0, s>>>(tileRec, tileQ, nTiles, qkey, qslot, unitInfo, C, db, D, spOf,
                                                        maxTax, kmerFormat, readCnt, total, buf, bufRank, region, err,
                                                        stats, direct, overflow, capShift, longList, longCap, longCnt,
                                                        ldsCap);
        else
            k_sweep_p<kSweepCap><<<(unsigned)g, 256, 0, s>>>(tileRec, tileQ, nTiles, qkey, qslot, unitInfo, C, db, D,
                                                             spOf, maxTax, kmerFormat, readCnt, total, buf, bufRank,
                                                             region, err, stats, direct, overflow, capShift, longList,
                                                             longCap, longCnt, ldsCap);
        return;
    }
    if (small)  // 24-KB tiles: twice the blocks per CU (tiles of more than 2048 records search HBM)
        k_sweep<2048><<<(unsigned)nTiles, 256, 0, s>>>(tileRec, tileQ, qkey, qslot, unitInfo, C, db, D, spOf, maxTax,
                                                       kmerFormat, readCnt, total, buf, bufRank, region, err, stats,
                                                       direct, overflow, capShift, longList, longCap, longCnt, ldsCap);
    else
        k_sweep<kSweepCap><<<(unsigned)nTiles, 256, 0, s>>>(tileRec, tileQ, qkey, qslot, unitInfo, C, db, D, spOf,
                                                            maxTax, kmerFormat, readCnt, total, buf, bufRank, region,
                                                            err, stats, direct, overflow, capShift, longList, longCap,
                                                            longCnt, ldsCap);
}

}  // namespace mtb
