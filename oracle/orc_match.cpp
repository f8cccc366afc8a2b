// ORACLE — test infrastructure only (see orc_core.h header).
// KmerMatcher::matchKmers restated over in-memory DB files (KmerMatcher.cpp:123-481),
// getNextTargetKmer (KmerMatcher.h:282-297), compareDna (KmerMatcher.cpp:1117-1146),
// sortMatches/compareMatches (:1071-1078, :1149-1166), loadTaxIdList (:56-120).
#include <algorithm>
#include <parallel/algorithm>

#include "orc_internal.h"
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

static const uint64_t DNA_MASK = ~(uint64_t)16777215;  // AMINO_ACID_PART (KmerMatcher.h:22)
static const uint64_t AA_MASK = 0xffffffULL;

bool Db::buildSpeciesMap(std::string* err) {
    // KmerMatcher::loadTaxIdList, non-contamination branch (KmerMatcher.cpp:92-117)
    taxId2speciesId.clear();
    for (TaxID taxId : taxIdList) {
        if (!tax.nodeExists(taxId)) { *err = "taxID_list entry not in taxonomy"; return false; }
        TaxID speciesTaxID = tax.getTaxIdAtRank(taxId, "species");
        const TaxonNode* taxon = tax.taxonNode(taxId);
        if (taxId != taxon->taxId) taxId2speciesId[taxId] = speciesTaxID;
        int guard = 0;
        while (taxon->taxId != speciesTaxID) {
            taxId2speciesId[taxon->taxId] = speciesTaxID;
            taxon = tax.taxonNode(taxon->parentTaxId);
            if (++guard > 1000) { *err = "taxID_list entry has no species ancestor"; return false; }
        }
        taxId2speciesId[speciesTaxID] = speciesTaxID;
    }
    return true;
}

static inline uint64_t nextTargetKmer(uint64_t looking, const uint16_t* diff, size_t& idx, size_t& totalPos) {
    uint64_t d = 0;
    uint16_t f = diff[idx++];
    totalPos++;
    while (!(f & 0x8000)) {
        d |= f;
        d <<= 15u;
        f = diff[idx++];
        totalPos++;
    }
    d |= (f & 0x7FFF);
    return d + looking;
}

uint64_t decodeDiffIdx(const uint16_t* diff, uint64_t nWords, uint64_t* values) {
    size_t idx = 0, totalPos = 0;
    uint64_t v = 0, k = 0;
    while (idx < nWords) {
        v = nextTargetKmer(v, diff, idx, totalPos);
        values[k++] = v;
    }
    return k;
}

struct QueryKmerSplit {
    size_t start, end;
    DiffIdxSplit split;
};

static void compareDna(uint64_t query, const std::vector<uint64_t>& targets, std::vector<uint8_t>& hd,
                       std::vector<size_t>& sel, std::vector<uint8_t>& selSum, std::vector<uint16_t>& selHam,
                       size_t& selCnt, uint8_t frame, int kmerFormat) {
    hd.resize(targets.size());
    uint8_t minSum = UINT8_MAX;
    for (size_t i = 0; i < targets.size(); i++) {
        hd[i] = hammingSum(query, targets[i]);
        minSum = std::min(minSum, hd[i]);
    }
    selCnt = 0;
    uint8_t maxH = (uint8_t)std::min(minSum * 2, 7);
    for (size_t h = 0; h < targets.size(); h++) {
        if (hd[h] <= maxH) {
            selSum[selCnt] = hd[h];
            selHam[selCnt] = !((frame < 3) ^ (kmerFormat == 2)) ? hammings(query, targets[h]) : hammingsReverse(query, targets[h]);
            sel[selCnt++] = h;
        }
    }
}

bool matchKmers(const Db& db, const mtb_params& par, const mtb_kmer* queryKmerList, size_t queryKmerNum,
                std::vector<mtb_match>& out, std::string* err) {
    out.clear();
    const size_t numOfDiffIdx = db.diffIdx.size();
    size_t blankCnt = 0;
    for (size_t i = 0; i < queryKmerNum; i++) {
        if (infoSeq(queryKmerList[i].info) == 0) blankCnt++; else break;
    }
    queryKmerNum -= blankCnt;
    if (queryKmerNum == 0 || numOfDiffIdx == 0) return true;

    std::vector<DiffIdxSplit> splits = db.split;
    size_t numSplits = splits.size();
    size_t numUse = numSplits;
    for (size_t i = 1; i < numSplits; i++) {
        if (splits[i].ADkmer == 0 || splits[i].ADkmer == UINT64_MAX) {
            splits[i] = {UINT64_MAX, UINT64_MAX, UINT64_MAX};
            numUse--;
        }
    }
    if (numUse < 2) { *err = "DB has fewer than one split (reference indexes split[use-2])"; return false; }

    size_t threads = par.threads > 0 ? (size_t)par.threads : 1;
    std::vector<QueryKmerSplit> querySplits;
    size_t quotient = queryKmerNum / threads, remainder = queryKmerNum % threads;
    size_t startIdx = blankCnt, endIdx = 0;
    for (size_t i = 0; i < threads; i++) {
        endIdx = startIdx + quotient - 1;
        if (remainder > 0) { endIdx++; remainder--; }
        if (endIdx + 1 <= startIdx) continue;  // empty range (fewer queries than threads)
        bool needLast = true;
        uint64_t queryAA = queryKmerList[startIdx].value & DNA_MASK;
        for (size_t j = 0; j < numUse; j++) {
            if (queryAA <= (splits[j].ADkmer & DNA_MASK)) {
                j = j - (j != 0);
                querySplits.push_back({startIdx, endIdx, splits[j]});
                needLast = false;
                break;
            }
        }
        if (needLast) querySplits.push_back({startIdx, endIdx, splits[numUse - 2]});
        startIdx = endIdx + 1;
    }

    const int redundancyStored = (par.skip_redundancy == 0);
    const unsigned int mask = ~((unsigned int)redundancyStored << 31);
    const int kmerFormat = par.kmer_format;
    std::vector<std::vector<mtb_match>> perSplit(querySplits.size());
    bool fatal = false;

#pragma omp parallel num_threads((int)threads)
    {
        std::vector<uint64_t> candidateTargetKmers;
        std::vector<TaxID> candidateKmerInfos;
        std::vector<uint8_t> hammingDists;
        std::vector<uint8_t> selectedHammingSum(1024);
        std::vector<size_t> selectedMatches(1024);
        std::vector<uint16_t> selectedHammings(1024);
        size_t selectedMatchCnt = 0;

#pragma omp for schedule(dynamic, 1)
        for (size_t i = 0; i < querySplits.size(); i++) {
            std::vector<mtb_match>& matches = perSplit[i];
            const QueryKmerSplit& qs = querySplits[i];
            uint64_t currentTargetKmer = qs.split.ADkmer;
            size_t diffIdxBufferIdx = qs.split.diffIdxOffset;
            size_t kmerInfoBufferIdx = qs.split.infoIdxOffset - (qs.split.ADkmer != 0);
            size_t diffIdxPos = qs.split.diffIdxOffset;
            const uint16_t* diff = db.diffIdx.data();
            if (qs.split.ADkmer == 0 && qs.split.diffIdxOffset == 0 && qs.split.infoIdxOffset == 0)
                currentTargetKmer = nextTargetKmer(currentTargetKmer, diff, diffIdxBufferIdx, diffIdxPos);

            uint64_t currentQuery = UINT64_MAX, currentQueryAA = UINT64_MAX;
            uint64_t currentQueryInfo = 0;
            auto emit = [&](size_t j) {
                for (size_t k = 0; k < selectedMatchCnt; k++) {
                    size_t idx = selectedMatches[k];
                    TaxID t = candidateKmerInfos[idx];
                    auto it = db.taxId2speciesId.find(t);
                    TaxID sp = it == db.taxId2speciesId.end() ? 0 : it->second;
                    if (t == 0 || sp == 0) { fatal = true; return; }  // KmerMatcher.cpp:432-441 exit(1)
                    mtb_match m;
                    m.qinfo = queryKmerList[j].info;
                    m.target_id = (uint32_t)t;
                    m.species_id = (uint32_t)sp;
                    m.dna_encoding = (uint32_t)(candidateTargetKmers[idx] & AA_MASK);
                    m.right_end_hamming = selectedHammings[k];
                    m.hamming = selectedHammingSum[k];
                    m.pad = 0;
                    matches.push_back(m);
                }
            };
            for (size_t j = qs.start; j < qs.end + 1; j++) {
                const uint64_t qv = queryKmerList[j].value;
                const uint32_t qframe = infoFrame(queryKmerList[j].info);
                // Reuse when the query is identical and on the same strand class (:277-311)
                if (currentQuery == qv && (infoFrame(currentQueryInfo) / 3 == qframe / 3)) {
                    emit(j);
                    continue;
                }
                selectedMatchCnt = 0;
                // Same AA part: reuse the candidate list (:315-353)
                if (currentQueryAA == (qv & DNA_MASK)) {
                    compareDna(qv, candidateTargetKmers, hammingDists, selectedMatches, selectedHammingSum,
                               selectedHammings, selectedMatchCnt, (uint8_t)qframe, kmerFormat);
                    emit(j);
                    currentQuery = qv;
                    currentQueryAA = qv & DNA_MASK;
                    currentQueryInfo = queryKmerList[j].info;
                    continue;
                }
                candidateTargetKmers.clear();
                candidateKmerInfos.clear();
                currentQuery = qv;
                currentQueryAA = qv & DNA_MASK;
                currentQueryInfo = queryKmerList[j].info;
                // Skip target k-mers not matching at the AA level (:363-371)
                while (diffIdxPos != numOfDiffIdx && currentQueryAA > (currentTargetKmer & DNA_MASK)) {
                    currentTargetKmer = nextTargetKmer(currentTargetKmer, diff, diffIdxBufferIdx, diffIdxPos);
                    kmerInfoBufferIdx++;
                }
                if (currentQueryAA != (currentTargetKmer & DNA_MASK)) continue;
                // Load the AA-equal run (:378-406); the last DB k-mer is never loaded.
                while (diffIdxPos != numOfDiffIdx && currentQueryAA == (currentTargetKmer & DNA_MASK)) {
                    candidateTargetKmers.push_back(currentTargetKmer);
                    candidateKmerInfos.push_back((TaxID)(db.info[kmerInfoBufferIdx] & mask));
                    currentTargetKmer = nextTargetKmer(currentTargetKmer, diff, diffIdxBufferIdx, diffIdxPos);
                    kmerInfoBufferIdx++;
                }
                if (candidateTargetKmers.size() > selectedMatches.size()) {
                    selectedMatches.resize(candidateTargetKmers.size());
                    selectedHammingSum.resize(candidateTargetKmers.size());
                    selectedHammings.resize(candidateTargetKmers.size());
                }
                compareDna(currentQuery, candidateTargetKmers, hammingDists, selectedMatches, selectedHammingSum,
                           selectedHammings, selectedMatchCnt, (uint8_t)qframe, kmerFormat);
                emit(j);
            }
        }
    }
    if (fatal) { *err = "k-mer with taxID 0 or without species (reference exits)"; return false; }
    size_t total = 0;
    for (auto& v : perSplit) total += v.size();
    out.reserve(total);
    for (auto& v : perSplit) out.insert(out.end(), v.begin(), v.end());
    return true;
}

bool compareMatches(const mtb_match& a, const mtb_match& b) {
    uint32_t sa = infoSeq(a.qinfo), sb = infoSeq(b.qinfo);
    if (sa != sb) return sa < sb;
    if (a.species_id != b.species_id) return (int)a.species_id < (int)b.species_id;
    uint32_t fa = infoFrame(a.qinfo), fb = infoFrame(b.qinfo);
    if (fa != fb) return fa < fb;
    uint32_t pa = infoPos(a.qinfo), pb = infoPos(b.qinfo);
    if (pa != pb) return pa < pb;
    if (a.hamming != b.hamming) return a.hamming < b.hamming;
    return a.dna_encoding < b.dna_encoding;
}

void sortMatches(std::vector<mtb_match>& m) { __gnu_parallel::sort(m.begin(), m.end(), compareMatches); }

}  // namespace orc
