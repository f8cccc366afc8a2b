// ORACLE — test infrastructure only. CPU restatement of the Metabuli `classify` hot path used as the
// parity checker for the HIP path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load it; the product (metabuli_work_amd/) never links or calls anything under oracle/.
//
// Parity status: PARTIALLY PINNED. The genetic-code / IUPAC tables are pinned against the
// reference's own GeneticCode.h compiled in place (oracle/_ref, tests/golden/genetic_code.json).
// Everything else is a restatement of the reference sources cited per function; the reference
// cannot be built here (lib/mmseqs is an empty submodule) and ships no golden vectors, so the
// rest of the oracle is "parity unpinned" (see DESIGN.md §Oracle).
#pragma once
#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "../include/mtb_gpu.h"

namespace orc {

// IUPAC -> base char and reverse complement (common.cpp:13-23). Built from the same 64-char
// row the reference uses for bytes 64..127; every other byte maps to '.'.
struct CharTables {
    unsigned char atcg[256];
    unsigned char iRCT[256];
    CharTables() {
        const char* row_atcg = ".AGCG..GT..G.CN...ACTG.A.T.......agcg..gt..g.cn...actg.a.t......";
        const char* row_irct = ".TVGH..CD..M.KN...YSAABW.R.......tvgh..cd..m.kn...ysaabw.r......";
        for (int i = 0; i < 256; i++) { atcg[i] = '.'; iRCT[i] = '.'; }
        for (int i = 0; i < 64; i++) {
            atcg[64 + i] = (unsigned char)row_atcg[i];
            iRCT[64 + i] = (unsigned char)row_irct[i];
        }
    }
};
extern const CharTables kChars;

// nuc2int (GeneticCode.h:6): A->0, C->1, T->2, G->3, everything else (N, '.') -> 7.
inline int nuc2int(unsigned char x) { return (x & 14u) >> 1u; }

// Standard genetic code over the reference AA alphabet "ARNDCQEGHILKMFPSTWYVX" (X = stop = 20)
// and the 3-bit synonymous-codon code (GeneticCode.h:32-194). Indices are nuc2int codes.
struct GeneticCode {
    int nuc2aa[8][8][8];
    int nuc2num[8][8][8];
    GeneticCode() {
        // Codon table in TCAG order, restated from the standard code.
        const char* bases = "TCAG";
        const char* aa64 = "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
        const char* alphabet = "ARNDCQEGHILKMFPSTWYV";
        auto code = [](char b) { return b == 'A' ? 0 : b == 'C' ? 1 : b == 'T' ? 2 : 3; };
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++)
                for (int k = 0; k < 8; k++) { nuc2aa[i][j][k] = -1; nuc2num[i][j][k] = -1; }
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 4; k++) {
                    char a = aa64[i * 16 + j * 4 + k];
                    int idx = 20;
                    if (a != '*') idx = (int)(strchr(alphabet, a) - alphabet);
                    int c1 = code(bases[i]), c2 = code(bases[j]), c3 = code(bases[k]);
                    nuc2aa[c1][c2][c3] = idx;
                    nuc2num[c1][c2][c3] = c3;  // default: third-base code
                }
        nuc2num[0][3][3] = 4;  // AGG (Arg)
        nuc2num[0][3][0] = 5;  // AGA (Arg)
        nuc2num[2][2][3] = 4;  // TTG (Leu)
        nuc2num[2][2][0] = 5;  // TTA (Leu)
        nuc2num[0][3][2] = 6;  // AGT (Ser)
        nuc2num[0][3][1] = 7;  // AGC (Ser)
        nuc2num[2][3][0] = 5;  // TGA (stop)
    }
    int getAA(unsigned char a, unsigned char b, unsigned char c) const {
        return nuc2aa[nuc2int(a)][nuc2int(b)][nuc2int(c)];
    }
    int getCodon(unsigned char a, unsigned char b, unsigned char c) const {
        return nuc2num[nuc2int(a)][nuc2int(b)][nuc2int(c)];
    }
};
extern const GeneticCode kCode;

struct ScanKmer {
    uint64_t value;
    uint32_t pos;
};

// KmerScanner base state (KmerScanner.h:11-47).
struct Scanner {
    const char* seq = nullptr;
    uint32_t seqStart = 0, seqEnd = 0, seqLen = 0;
    int loadedCharCnt = 0, posStart = 0, kmerSize = 8;
    bool isForward = true;
    virtual ~Scanner() {}
    virtual void init(const char* s, size_t start, size_t end, bool fwd) {
        seq = s; seqStart = (uint32_t)start; seqEnd = (uint32_t)end; seqLen = seqEnd - seqStart + 1;
        loadedCharCnt = 0; posStart = 0; isForward = fwd;
    }
    virtual ScanKmer next() = 0;
    unsigned char at(int i) const { return (unsigned char)seq[i]; }
    int fwdAA(int ci) const { return kCode.getAA(kChars.atcg[at(ci)], kChars.atcg[at(ci + 1)], kChars.atcg[at(ci + 2)]); }
    int fwdCodon(int ci) const { return kCode.getCodon(kChars.atcg[at(ci)], kChars.atcg[at(ci + 1)], kChars.atcg[at(ci + 2)]); }
    int revAA(int ci) const {
        return kCode.getAA(kChars.iRCT[kChars.atcg[at(ci)]], kChars.iRCT[kChars.atcg[at(ci - 1)]], kChars.iRCT[kChars.atcg[at(ci - 2)]]);
    }
    int revCodon(int ci) const {
        return kCode.getCodon(kChars.iRCT[kChars.atcg[at(ci)]], kChars.iRCT[kChars.atcg[at(ci - 1)]], kChars.iRCT[kChars.atcg[at(ci - 2)]]);
    }
};

// MetamerScanner (format 2): 5-bit AA x 8 | 3-bit codon x 8 (KmerScanner.h:49-118).
struct MetamerScanner : Scanner {
    int aaLen = 0;
    uint64_t dnaPart = 0, aaPart = 0;
    static constexpr uint64_t dnaMask = (1ULL << 24) - 1;
    void init(const char* s, size_t start, size_t end, bool fwd) override {
        Scanner::init(s, start, end, fwd);
        aaLen = (int)(seqLen / 3); dnaPart = 0; aaPart = 0;
    }
    ScanKmer next() override {
        int aa = 0, codon = 0;
        while (posStart <= aaLen - 8) {
            bool sawN = false;
            loadedCharCnt -= (loadedCharCnt == 8);
            while (loadedCharCnt < 8) {
                if (isForward) {
                    int ci = (int)seqStart + (posStart + loadedCharCnt) * 3;
                    aa = fwdAA(ci); codon = fwdCodon(ci);
                } else {
                    int ci = (int)seqEnd - (posStart + loadedCharCnt) * 3;
                    aa = revAA(ci); codon = revCodon(ci);
                }
                if (aa < 0) { sawN = true; break; }
                dnaPart = (dnaPart << 3) | (uint64_t)codon;
                aaPart = (aaPart << 5) | (uint64_t)aa;
                loadedCharCnt++;
            }
            if (sawN) { posStart += loadedCharCnt + 1; dnaPart = aaPart = 0; loadedCharCnt = 0; continue; }
            if (isForward) return {(aaPart << 24) | (dnaPart & dnaMask), seqStart + (uint32_t)(posStart++) * 3};
            return {(aaPart << 24) | (dnaPart & dnaMask), seqEnd - (uint32_t)((posStart++) + 8) * 3 + 1};
        }
        return {UINT64_MAX, 0};
    }
};

// OldMetamerScanner (format 1): base-21 AA, window read right-to-left (KmerScanner.h:120-182).
// The deque of scaled AA contributions is kept exactly as the reference keeps it.
struct OldMetamerScanner : MetamerScanner {
    std::deque<size_t> dq;
    void init(const char* s, size_t start, size_t end, bool fwd) override {
        MetamerScanner::init(s, start, end, fwd);
        dq.clear();
    }
    ScanKmer next() override {
        int aa = 0, codon = 0;
        while (posStart <= aaLen - 8) {
            bool sawN = false;
            loadedCharCnt -= (loadedCharCnt == 8);
            while (loadedCharCnt < 8) {
                if (isForward) {
                    int ci = (int)seqEnd - (posStart + loadedCharCnt) * 3;
                    aa = fwdAA(ci - 2); codon = fwdCodon(ci - 2);
                } else {
                    int ci = (int)seqStart + (posStart + loadedCharCnt) * 3;
                    aa = revAA(ci + 2); codon = revCodon(ci + 2);
                }
                if (aa < 0) { sawN = true; break; }
                if (dq.size() == 8) { aaPart = aaPart - dq.back(); dq.pop_back(); }
                for (auto& x : dq) x *= 21;
                dq.emplace_front(aa);
                aaPart = aaPart * 21 + aa;
                dnaPart = (dnaPart << 3) | (uint64_t)codon;
                loadedCharCnt++;
            }
            if (sawN) { posStart += loadedCharCnt + 1; dnaPart = aaPart = 0; loadedCharCnt = 0; dq.clear(); continue; }
            if (isForward) return {(aaPart << 24) | (dnaPart & dnaMask), seqEnd - (uint32_t)((posStart++) + 8) * 3 + 1};
            return {(aaPart << 24) | (dnaPart & dnaMask), seqStart + (uint32_t)(posStart++) * 3};
        }
        return {UINT64_MAX, 0};
    }
};

// SyncmerScanner (format 2 + closed syncmer): monotone deque of s-mers, lazy accumulator
// extension (SyncmerScanner.h:9-103).
struct SyncmerScanner : MetamerScanner {
    int smerLen;
    uint64_t smerMask;
    struct DqItem { uint64_t value; uint32_t pos; };
    std::deque<DqItem> dq;
    int smerCnt = 0;
    uint64_t smer = 0;
    int prevPos = -8;
    explicit SyncmerScanner(int s) : smerLen(s), smerMask((1ULL << (5 * s)) - 1) {}
    void init(const char* s, size_t start, size_t end, bool fwd) override {
        MetamerScanner::init(s, start, end, fwd);
        dq.clear(); smerCnt = 0; smer = 0; prevPos = -8;
    }
    ScanKmer next() override {
        bool found = false;
        int aa = 0;
        while (posStart <= aaLen - 8 && !found) {
            bool sawN = false;
            smerCnt -= (smerCnt > 0);
            while (smerCnt < 8 - smerLen + 1) {
                loadedCharCnt -= (loadedCharCnt == smerLen);
                while (loadedCharCnt < smerLen) {
                    if (isForward) aa = fwdAA((int)seqStart + (posStart + smerCnt + loadedCharCnt) * 3);
                    else aa = revAA((int)seqEnd - (posStart + smerCnt + loadedCharCnt) * 3);
                    if (aa < 0) { sawN = true; break; }
                    smer = (smer << 5) | (uint64_t)aa;
                    loadedCharCnt++;
                }
                if (sawN) break;
                smer &= smerMask;
                while (!dq.empty() && dq.back().value > smer) dq.pop_back();
                dq.push_back({smer, (uint32_t)(posStart + smerCnt)});
                smerCnt++;
            }
            if (sawN) {
                posStart += smerCnt + loadedCharCnt + 1;
                prevPos = posStart - 8;
                dq.clear(); smerCnt = loadedCharCnt = 0; smer = 0;
                continue;
            }
            if (!dq.empty() && dq.front().pos < (uint32_t)posStart) dq.pop_front();
            uint32_t anchor1 = (uint32_t)posStart;
            uint32_t anchor2 = (uint32_t)(posStart + (kmerSize - smerLen));
            if (!dq.empty() && (dq.front().pos == anchor1 || dq.front().pos == anchor2)) {
                int shifts = posStart - prevPos;
                for (int i = 0; i < shifts; ++i) {
                    if (isForward) {
                        int ci = (int)seqStart + (prevPos + 8 + i) * 3;
                        aaPart = (aaPart << 5) | (uint64_t)fwdAA(ci);
                        dnaPart = (dnaPart << 3) | (uint64_t)fwdCodon(ci);
                    } else {
                        int ci = (int)seqEnd - (prevPos + 8 + i) * 3;
                        aaPart = (aaPart << 5) | (uint64_t)revAA(ci);
                        dnaPart = (dnaPart << 3) | (uint64_t)revCodon(ci);
                    }
                }
                prevPos = posStart;
                found = true;
            }
            ++posStart;
        }
        if (found) {
            if (isForward) return {(aaPart << 24) | (dnaPart & dnaMask), seqStart + (uint32_t)prevPos * 3};
            return {(aaPart << 24) | (dnaPart & dnaMask), seqEnd - (uint32_t)(prevPos + 8) * 3 + 1};
        }
        return {UINT64_MAX, 0};
    }
};

// getMaxCoveredLength / getQueryKmerNumber (LocalUtil.h:45-59).
inline int maxCoveredLength(int len) {
    if (len % 3 == 2) return len - 2;
    if (len % 3 == 1) return len - 4;
    return len - 3;
}
inline int queryKmerNumber(int len, int k = 8, int spaceNum = 0) { return (maxCoveredLength(len) / 3 - k - spaceNum + 1) * 6; }

// QueryKmerInfo bitfield (Kmer.h:11-16): pos [0,32), seqID [32,61), frame [61,64).
inline uint64_t packInfo(uint32_t seqId, uint32_t pos, uint32_t frame) {
    return (uint64_t)pos | ((uint64_t)(seqId & 0x1FFFFFFFu) << 32) | ((uint64_t)(frame & 7u) << 61);
}
inline uint32_t infoPos(uint64_t x) { return (uint32_t)x; }
inline uint32_t infoSeq(uint64_t x) { return (uint32_t)((x >> 32) & 0x1FFFFFFFu); }
inline uint32_t infoFrame(uint64_t x) { return (uint32_t)(x >> 61); }

// Hamming tables (KmerMatcher.h:66-158). hammingLookup is the per-codon distance of two 3-bit
// synonymous-codon codes; the per-codon 2-bit fields keep a distance of 4 as 0, except the
// field-7 table (HAMMING_LUT7) whose rows 4-5, columns 6-7 are 1.
static const uint8_t kHammingLookup[8][8] = {
    {0, 1, 1, 1, 2, 1, 3, 3}, {1, 0, 1, 1, 2, 2, 3, 2}, {1, 1, 0, 1, 2, 2, 2, 3}, {1, 1, 1, 0, 1, 2, 3, 3},
    {2, 2, 2, 1, 0, 1, 4, 4}, {1, 2, 2, 2, 1, 0, 4, 4}, {3, 3, 2, 3, 4, 4, 0, 1}, {3, 2, 3, 3, 4, 4, 1, 0}};
inline uint16_t codonField(int q, int t, int field) {
    uint8_t h = kHammingLookup[q][t];
    if (field == 7 && (q == 4 || q == 5) && (t == 6 || t == 7)) return 1;
    return h == 4 ? 0 : h;
}
inline uint8_t hammingSum(uint64_t a, uint64_t b) {  // getHammingDistanceSum (KmerMatcher.h:348-360)
    uint8_t s = 0;
    for (int i = 0; i < 8; i++) s += kHammingLookup[(a >> (3 * i)) & 7][(b >> (3 * i)) & 7];
    return s;
}
inline uint16_t hammings(uint64_t a, uint64_t b) {  // getHammings (KmerMatcher.h:386-400)
    uint16_t h = 0;
    for (int i = 0; i < 8; i++) h |= codonField((a >> (3 * i)) & 7, (b >> (3 * i)) & 7, i) << (2 * i);
    return h;
}
inline uint16_t hammingsReverse(uint64_t a, uint64_t b) {  // getHammings_reverse (:402-416)
    uint16_t h = 0;
    for (int i = 0; i < 8; i++) h |= codonField((a >> (3 * i)) & 7, (b >> (3 * i)) & 7, 7 - i) << (2 * (7 - i));
    return h;
}

}  // namespace orc
