// ORACLE — test infrastructure only (see orc_core.h header).
// Low-complexity masking of query reads (--mask-residues 1, par.maskMode): KmerExtractor::
// processSequence (KmerExtractor.cpp:328-335) passes each read through
// SeqIterator::maskLowComplexityRegions (SeqIterator.cpp:154-175): letters -> NucleotideMatrix codes,
// tantan::maskSequences(maxCycleLength 50, repeatProb 0.005, repeatEndProb 0.05,
// repeatOffsetProbDecay 0.9, no gaps, minMaskProb = maskProb, hardMaskTable), then every position
// whose code equals hardMaskTable[0] becomes 'N' and the others keep their letter.
//
// tantan and the nucleotide scoring matrix live in MMseqs2 (lib/mmseqs, an un-vendored submodule
// absent from /root/reference; its pinned SHA is not in the mount either). This restates tantan's
// published algorithm (M. C. Frith, "A new repeat-masking method enables specific detection of
// homologous sequences", NAR 2011: an HMM with one background state and one repeat state per offset
// 1..maxCycleLength, forward-backward posteriors, rescaled every 16 positions) — PARITY UNPINNED.
// Assumptions (documented in DESIGN.md §2): letter codes A=0 C=1 G=2 T/U=3, every other byte N=4
// (hardMaskTable maps every code to N's); likelihood ratios exp(lambda * s) for s = +2 match / -3
// mismatch over ACGT and -1 against N, lambda solved for uniform base frequencies.
#include <cmath>
#include <vector>

#include "orc_internal.h"

namespace orc {

namespace {

constexpr int kMaxOffset = 50;          // options.maxCycleLength (SeqIterator.cpp:163)
constexpr double kRepeatProb = 0.005;   // options.repeatProb
constexpr double kRepeatEndProb = 0.05; // options.repeatEndProb
constexpr double kDecay = 0.9;          // options.repeatOffsetProbDecay
constexpr int kScaleStep = 16;
constexpr int kCodeN = 4;

struct MaskTables {
    int code[256];
    double lr[5][5];
    double b2f[kMaxOffset];
    MaskTables() {
        for (int c = 0; c < 256; c++) code[c] = kCodeN;
        code['A'] = code['a'] = 0;
        code['C'] = code['c'] = 1;
        code['G'] = code['g'] = 2;
        code['T'] = code['t'] = code['U'] = code['u'] = 3;
        // lambda of the +2 / -3 scoring at uniform frequencies: 0.25 e^{2l} + 0.75 e^{-3l} = 1
        double lo = 0.1, hi = 2.0;
        for (int it = 0; it < 200; it++) {
            const double mid = 0.5 * (lo + hi);
            if (0.25 * std::exp(2 * mid) + 0.75 * std::exp(-3 * mid) > 1.0) hi = mid; else lo = mid;
        }
        const double lambda = 0.5 * (lo + hi);
        for (int a = 0; a < 5; a++)
            for (int b = 0; b < 5; b++) {
                const int s = (a == kCodeN || b == kCodeN) ? -1 : (a == b ? 2 : -3);
                lr[a][b] = std::exp(lambda * s);
            }
        // background -> repeat offset k (k = 1..50): repeatProb * (1 - d) d^(k-1) / (1 - d^50)
        const double first = kRepeatProb * (1 - kDecay) / (1 - std::pow(kDecay, kMaxOffset));
        double p = first;
        for (int i = 0; i < kMaxOffset; i++) {
            b2f[i] = p;
            p *= kDecay;
        }
    }
};

const MaskTables& tables() {
    static const MaskTables t;
    return t;
}

}  // namespace

// tantan's per-letter repeat probabilities (calcRepeatProbs) of a coded sequence.
void tantanRepeatProbs(const unsigned char* x, int n, float* prob) {
    const MaskTables& T = tables();
    const double b2b = 1 - kRepeatProb, f2b = kRepeatEndProb, f2f = 1 - kRepeatEndProb;
    std::vector<double> fg(kMaxOffset, 0.0), scale(n / kScaleStep + 1, 1.0);
    double bg = 1.0;
    for (int p = 0; p < n; p++) {  // forward: transition into p, then emission of letter p
        const int m = p < kMaxOffset ? p : kMaxOffset;
        const double* row = T.lr[x[p]];
        double from = 0;
        for (int i = 0; i < m; i++) {
            const double f = fg[i];
            from += f;
            fg[i] = (bg * T.b2f[i] + f * f2f) * row[x[p - i - 1]];
        }
        bg = bg * b2b + from * f2b;
        if (p % kScaleStep == kScaleStep - 1) {
            const double s = 1 / bg;
            scale[p / kScaleStep] = s;
            bg *= s;
            for (double& f : fg) f *= s;
        }
        prob[p] = (float)bg;
    }
    double z = bg;  // to the end through the background state
    {
        double fs = 0;
        for (double f : fg) fs += f;
        z = bg + fs * f2b;
    }
    bg = 1.0;
    for (double& f : fg) f = f2b;
    for (int p = n - 1; p >= 0; p--) {  // backward: posterior of the background state at p
        const double nonRepeat = (double)prob[p] * bg / z;
        prob[p] = (float)(1 - nonRepeat);
        if (p % kScaleStep == kScaleStep - 1) {
            const double s = scale[p / kScaleStep];
            bg *= s;
            for (double& f : fg) f *= s;
        }
        const int m = p < kMaxOffset ? p : kMaxOffset;
        const double* row = T.lr[x[p]];
        const double toBg = f2b * bg;
        double toFg = 0;
        for (int i = 0; i < m; i++) {
            const double f = fg[i] * row[x[p - i - 1]];
            toFg += f * T.b2f[i];
            fg[i] = toBg + f2f * f;
        }
        bg = b2b * bg + toFg;
    }
}

// SeqIterator::maskLowComplexityRegions for one read: out[i] = 'N' where masked (or where the
// letter's code is N's already), else seq[i].
void maskLowComplexityRegions(const char* seq, int n, float maskProb, char* out) {
    const MaskTables& T = tables();
    std::vector<unsigned char> x(n);
    std::vector<float> prob(n);
    for (int i = 0; i < n; i++) x[i] = (unsigned char)T.code[(unsigned char)seq[i]];
    tantanRepeatProbs(x.data(), n, prob.data());
    for (int i = 0; i < n; i++) {
        const bool masked = prob[i] >= (double)maskProb || x[i] == kCodeN;
        out[i] = masked ? 'N' : seq[i];
    }
}

}  // namespace orc
