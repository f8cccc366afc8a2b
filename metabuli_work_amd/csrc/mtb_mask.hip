// K0M: low-complexity masking of the query reads (--mask-residues 1): KmerExtractor::processSequence
// (KmerExtractor.cpp:328-335) runs SeqIterator::maskLowComplexityRegions (SeqIterator.cpp:154-175)
// on every read before the scanners see it: NucleotideMatrix letter codes, tantan::maskSequences
// (maxCycleLength 50, repeatProb 0.005, repeatEndProb 0.05, repeatOffsetProbDecay 0.9, no gaps,
// minMaskProb = maskProb), then every position whose code is the hard-mask code becomes 'N'.
// tantan is MMseqs2's (un-vendored): restated from its published algorithm, PARITY UNPINNED
// (DESIGN.md §2); the tables are built by make_tantan_tables (mtb_host.cpp).
//
// One thread per mate runs the HMM's forward-backward serially along its read (a read's letters
// depend on each other through the 51 states; reads are independent): the 50 repeat-state
// probabilities live in registers (fully unrolled), the last 50 letter codes in a packed 13-word
// register window, the per-letter forward values (float) and the scale factors (every 16 letters)
// in scratch. Double precision, -ffp-contract=off and the reference's operation order: the masks
// equal the oracle's restatement bit for bit.
#include <hip/hip_runtime.h>

#include "mtb_host.h"
#include "mtb_launch.h"

namespace mtb {

namespace {

constexpr int kW = kTantanOffsets;  // 50
constexpr int kWords = (kW + 3) / 4;  // packed window: 4 codes per 32-bit word
constexpr int kStep = 16;             // rescaling step

__device__ __forceinline__ uint32_t letter_code(uint8_t c) {
    const uint32_t u = c & 0xDFu;  // lower case -> upper case for letters (only bit 5 differs)
    return u == 'A' ? 0u : u == 'C' ? 1u : u == 'G' ? 2u : (u == 'T' || u == 'U') ? 3u : 4u;
}

__device__ __forceinline__ double pick(uint32_t c, double r0, double r1, double r2, double r3, double r4) {
    return c == 0 ? r0 : c == 1 ? r1 : c == 2 ? r2 : c == 3 ? r3 : r4;
}

// row x of the likelihood-ratio table with compile-time indices only (the tables stay in the
// kernel-argument segment: scalar loads, no private copy)
__device__ __forceinline__ void lr_row(const TantanTables& tt, uint32_t x, double& r0, double& r1, double& r2,
                                       double& r3, double& r4) {
    r0 = pick(x, tt.lr[0], tt.lr[5], tt.lr[10], tt.lr[15], tt.lr[20]);
    r1 = pick(x, tt.lr[1], tt.lr[6], tt.lr[11], tt.lr[16], tt.lr[21]);
    r2 = pick(x, tt.lr[2], tt.lr[7], tt.lr[12], tt.lr[17], tt.lr[22]);
    r3 = pick(x, tt.lr[3], tt.lr[8], tt.lr[13], tt.lr[18], tt.lr[23]);
    r4 = pick(x, tt.lr[4], tt.lr[9], tt.lr[14], tt.lr[19], tt.lr[24]);
}

__global__ void __launch_bounds__(64) k_tantan(const uint8_t* __restrict__ seq, const uint64_t* __restrict__ off,
                                               uint32_t n, TantanTables tt, float* __restrict__ prob,
                                               double* __restrict__ scaleBuf, uint8_t* __restrict__ out) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const uint64_t beg = off[r];
    const int len = (int)(off[r + 1] - beg);
    const uint8_t* s = seq + beg;
    float* pr = prob + beg;
    double* sc = scaleBuf + beg / kStep + r;  // disjoint per read (see launch_tantan_mask)
    uint8_t* o = out + beg;
    const double b2b = tt.b2b, f2b = tt.f2b, f2f = tt.f2f;
    double fg[kW];
#pragma unroll
    for (int i = 0; i < kW; i++) fg[i] = 0.0;
    uint32_t win[kWords];  // byte i = code of letter p - 1 - i
#pragma unroll
    for (int k = 0; k < kWords; k++) win[k] = 0x04040404u;
    double bg = 1.0;
    // forward: transition into letter p, then its emission
    for (int p = 0; p < len; p++) {
        const uint32_t x = letter_code(s[p]);
        double r0, r1, r2, r3, r4;
        lr_row(tt, x, r0, r1, r2, r3, r4);
        const int m = p < kW ? p : kW;
        double from = 0.0;
#pragma unroll
        for (int i = 0; i < kW; i++) {
            const double f = fg[i];
            from += f;  // fg[i] is 0 for i >= m
            const uint32_t c = (win[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            const double nf = (bg * tt.b2f[i] + f * f2f) * pick(c, r0, r1, r2, r3, r4);
            fg[i] = i < m ? nf : f;
        }
        bg = bg * b2b + from * f2b;
        if (p % kStep == kStep - 1) {
            const double sf = 1 / bg;
            sc[p / kStep] = sf;
            bg *= sf;
#pragma unroll
            for (int i = 0; i < kW; i++) fg[i] *= sf;
        }
        pr[p] = (float)bg;
#pragma unroll
        for (int k = kWords - 1; k > 0; k--) win[k] = (win[k] << 8) | (win[k - 1] >> 24);
        win[0] = (win[0] << 8) | x;
    }
    double fs = 0.0;
#pragma unroll
    for (int i = 0; i < kW; i++) fs += fg[i];
    const double z = bg + fs * f2b;  // to the end through the background state
    // backward: the background state's posterior at p, then back over letter p's emission
    bg = 1.0;
#pragma unroll
    for (int i = 0; i < kW; i++) fg[i] = f2b;
#pragma unroll
    for (int k = 0; k < kWords; k++) win[k] = 0x04040404u;
#pragma unroll
    for (int i = 0; i < kW; i++) {  // byte i = code of letter len - 2 - i
        const int q = len - 2 - i;
        if (q >= 0) win[i >> 2] = (win[i >> 2] & ~(0xFFu << (8 * (i & 3)))) | (letter_code(s[q]) << (8 * (i & 3)));
    }
    for (int p = len - 1; p >= 0; p--) {
        const uint8_t letter = s[p];
        const uint32_t x = letter_code(letter);
        const double nonRepeat = (double)pr[p] * bg / z;
        const float rp = (float)(1 - nonRepeat);
        o[p] = ((double)rp >= tt.minMask || x == 4u) ? (uint8_t)'N' : letter;
        if (p % kStep == kStep - 1) {
            const double sf = sc[p / kStep];
            bg *= sf;
#pragma unroll
            for (int i = 0; i < kW; i++) fg[i] *= sf;
        }
        double r0, r1, r2, r3, r4;
        lr_row(tt, x, r0, r1, r2, r3, r4);
        const int m = p < kW ? p : kW;
        const double toBg = f2b * bg;
        double toFg = 0.0;
#pragma unroll
        for (int i = 0; i < kW; i++) {
            const uint32_t c = (win[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            const double f = fg[i] * pick(c, r0, r1, r2, r3, r4);
            if (i < m) {
                toFg += f * tt.b2f[i];
                fg[i] = toBg + f2f * f;
            }
        }
        bg = b2b * bg + toFg;
        // window for letter p - 1: byte i = code of letter p - 2 - i
#pragma unroll
        for (int k = 0; k < kWords - 1; k++) win[k] = (win[k] >> 8) | (win[k + 1] << 24);
        win[kWords - 1] >>= 8;
        const int q = p - 1 - kW;  // the letter entering at byte kW - 1
        const uint32_t cq = q >= 0 ? letter_code(s[q]) : 4u;
        constexpr int kb = kW - 1;
        win[kb >> 2] = (win[kb >> 2] & ~(0xFFu << (8 * (kb & 3)))) | (cq << (8 * (kb & 3)));
    }
}

}  // namespace

uint64_t tantan_scale_elems(uint64_t bases, uint32_t n) { return bases / kStep + n + 2; }

void launch_tantan_mask(const uint8_t* seq, const uint64_t* off, uint32_t n, const TantanTables& tt, float* prob,
                        double* scale, uint8_t* out, hipStream_t s) {
    // a read's scale factors: scale[off[r] / 16 + r + p / 16], p < len: read r + 1 starts past them,
    // since off[r+1] / 16 + r + 1 > (off[r] + len - 1) / 16 + r
    if (n) k_tantan<<<(n + 63) / 64, 64, 0, s>>>(seq, off, n, tt, prob, scale, out);
}

}  // namespace mtb
