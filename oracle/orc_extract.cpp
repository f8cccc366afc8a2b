// ORACLE — test infrastructure only (see orc_core.h header).
// Query k-mer extraction: KmerExtractor.cpp:52-81 (extractQueryKmers), :312-353 (processSequence),
// :355-386 (fillQueryKmerBuffer), :442-494 (loadChunkOfReads), LocalUtil.h:45-59.
#include <algorithm>
#include <memory>

#include "orc_internal.h"
#ifdef _OPENMP
#include <omp.h>
#include <parallel/algorithm>
#endif

namespace orc {

const CharTables kChars;
const GeneticCode kCode;

static std::unique_ptr<Scanner> makeScanner(const mtb_params& par) {
    // KmerExtractor::KmerExtractor (KmerExtractor.cpp:11-35)
    if (par.kmer_format == 1) return std::unique_ptr<Scanner>(new OldMetamerScanner());
    if (par.syncmer) return std::unique_ptr<Scanner>(new SyncmerScanner(par.smer_len));
    return std::unique_ptr<Scanner>(new MetamerScanner());
}

// fillQueryKmerBuffer (KmerExtractor.cpp:355-386)
static size_t fillQueryKmerBuffer(Scanner& sc, const char* seq, int seqLen, mtb_kmer* out, uint32_t seqID,
                                  uint32_t offset) {
    int usedLen = maxCoveredLength(seqLen);
    size_t w = 0;
    for (int frame = 0; frame < 6; frame++) {
        bool fwd = frame < 3;
        int begin;
        if (fwd) {
            begin = frame % 3;
        } else {
            begin = (seqLen % 3) - (frame % 3);
            if (begin < 0) begin += 3;
        }
        sc.init(seq, begin, begin + usedLen - 1, fwd);
        for (ScanKmer k = sc.next(); k.value != UINT64_MAX; k = sc.next())
            out[w++] = {k.value, packInfo(seqID, k.pos + offset, (uint32_t)frame)};
    }
    return w;
}

void extractQueryKmers(const mtb_params& par, const Reads& reads, std::vector<mtb_kmer>& buf,
                       std::vector<Query>& queries, bool sort) {
    const bool paired = par.seq_mode == 2;
    queries.assign(reads.n, Query());
    std::vector<char> empty(reads.n, 0);
    // loadChunkOfReads: lengths, k-mer counts and the shared empty flag (KmerExtractor.cpp:442-494)
    std::vector<uint64_t> reserveOff(reads.n + 1, 0);
    for (uint32_t i = 0; i < reads.n; i++) {
        int len1 = (int)(reads.off1[i + 1] - reads.off1[i]);
        Query& q = queries[i];
        q.queryLength = maxCoveredLength(len1);
        int kc = queryKmerNumber(len1);
        if (kc < 1) { empty[i] = 1; q.kmerCnt = 0; } else { q.kmerCnt = kc; }
        if (paired) {
            int len2 = (int)(reads.off2[i + 1] - reads.off2[i]);
            q.queryLength2 = maxCoveredLength(len2);
            if (!empty[i]) {
                int kc2 = queryKmerNumber(len2);
                if (kc2 < 1) { empty[i] = 1; q.kmerCnt2 = 0; } else { q.kmerCnt2 = kc2; }
            }
        }
        uint64_t reserve = 0;
        if (!empty[i]) reserve = (uint64_t)q.kmerCnt + (paired ? (uint64_t)q.kmerCnt2 : 0);
        reserveOff[i + 1] = reserveOff[i] + reserve;
    }
    // Buffer::init zero-fills the reserved buffer (common.h:176-181).
    buf.assign(reserveOff[reads.n], mtb_kmer{0, 0});
#pragma omp parallel
    {
        std::unique_ptr<Scanner> sc = makeScanner(par);
        std::vector<char> m1, m2;  // masked copies (processSequence, KmerExtractor.cpp:328-335)
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < (int64_t)reads.n; i++) {
            if (empty[i]) continue;  // processSequence (KmerExtractor.cpp:324)
            const Query& q = queries[i];
            mtb_kmer* out = buf.data() + reserveOff[i];
            const char* s1 = reads.seq1 + reads.off1[i];
            const int l1 = (int)(reads.off1[i + 1] - reads.off1[i]);
            if (par.mask_mode) {
                m1.resize(l1 + 1);
                maskLowComplexityRegions(s1, l1, par.mask_prob, m1.data());
                s1 = m1.data();
            }
            fillQueryKmerBuffer(*sc, s1, l1, out, (uint32_t)i + 1, 0);
            if (paired) {
                const char* s2 = reads.seq2 + reads.off2[i];
                if (par.mask_mode) {
                    const int l2 = (int)(reads.off2[i + 1] - reads.off2[i]);
                    m2.resize(l2 + 1);
                    maskLowComplexityRegions(s2, l2, par.mask_prob, m2.data());
                    s2 = m2.data();
                }
                fillQueryKmerBuffer(*sc, s2, (int)(reads.off2[i + 1] - reads.off2[i]), out + q.kmerCnt,
                                    (uint32_t)i + 1, (uint32_t)q.queryLength + 3);
            }
        }
    }
    if (sort) {
        // SORT_PARALLEL(..., Kmer::compareQueryKmer) (KmerExtractor.cpp:79, Kmer.h:89-94); MMseqs2's
        // SORT_PARALLEL is __gnu_parallel::sort under OpenMP
        __gnu_parallel::sort(buf.begin(), buf.end(), [](const mtb_kmer& a, const mtb_kmer& b) {
            if (a.value != b.value) return a.value < b.value;
            return infoSeq(a.info) < infoSeq(b.info);
        });
    }
}

}  // namespace orc
