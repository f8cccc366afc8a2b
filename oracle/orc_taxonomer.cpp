// ORACLE — test infrastructure only (see orc_core.h header).
// Classifier::assignTaxonomy (Classifier.cpp:166-208) and Taxonomer (Taxonomer.cpp:12-713,
// Taxonomer.h:15-59), Match score helpers (Match.h:32-86).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include "orc_internal.h"
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

static inline int get2(uint32_t x) { return (int)(x & 3u); }

// Match::getScore / getRightPartScore / getLeftPartScore / *HammingDist (Match.h:32-86)
static float matchScore(const mtb_match& m) {
    float score = 0.0f;
    for (int cnt = 0; cnt < 8; cnt++) {
        int h = get2(m.right_end_hamming >> (cnt * 2));
        score += (h == 0) ? 3.0f : 2.0f - 0.5f * h;
    }
    return score;
}
static float rightPartScore(const mtb_match& m, int range) {
    float score = 0.0f;
    for (int cnt = 0; cnt < range; cnt++) {
        int h = get2(m.right_end_hamming >> (cnt * 2));
        score += (h == 0) ? 3.0f : 2.0f - 0.5f * h;
    }
    return score;
}
static float leftPartScore(const mtb_match& m, int range) {
    float score = 0.0f;
    for (int cnt = 0; cnt < range; cnt++) {
        int h = get2(m.right_end_hamming >> (14 - cnt * 2));
        score += (h == 0) ? 3.0f : 2.0f - 0.5f * h;
    }
    return score;
}
static int rightPartHamming(const mtb_match& m, int range) {
    int s = 0;
    for (int i = 0; i < range; i++) s += get2(m.right_end_hamming >> (i * 2));
    return s;
}
static int leftPartHamming(const mtb_match& m, int range) {
    int s = 0;
    for (int i = 0; i < range; i++) s += get2(m.right_end_hamming >> (14 - i * 2));
    return s;
}

// The Taxonomer constructor's shape parameters (Taxonomer.cpp:34-58; reducedAA is refused by the path,
// so 3-bit codons): dnaShift, maxCodonShift, denominator, bitsPerCodon, totalDnaBits, lastCodonMask.
struct TaxShape {
    int dnaShift, maxCodonShift, denominator, bitsPerCodon, totalDnaBits;
    uint32_t lastCodonMask;
};
static TaxShape taxShape(const mtb_params& par) {
    TaxShape t;
    if (par.syncmer) { t.dnaShift = (8 - par.smer_len) * 3; t.maxCodonShift = 8 - par.smer_len; }
    else { t.dnaShift = 3; t.maxCodonShift = 1; }
    t.denominator = (par.seq_mode == 1 || par.seq_mode == 2) ? 100 : 1000;
    t.bitsPerCodon = 3; t.totalDnaBits = 24; t.lastCodonMask = 0x1FFFFF;
    return t;
}

// calScoreIncrement / calHammingDistIncrement (Taxonomer.cpp:650-669)
static float scoreIncrement(uint16_t h, int shift) {
    float inc = 0;
    for (int i = 0; i < shift; i++) {
        uint8_t x = (h >> (i * 2)) & 3;
        inc += (x == 0) ? 3.0f : 2.0f - 0.5f * x;
    }
    return inc;
}
static int hammingIncrement(uint16_t h, int shift) {
    int inc = 0;
    for (int i = 0; i < shift; i++) inc += (h >> (i * 2)) & 3;
    return inc;
}
// isConsecutive / isConsecutive2 of two DNA encodings (Taxonomer.cpp:677-699)
static bool consecutive1(uint32_t a, uint32_t b, int shift, int bitsPerCodon, int totalDnaBits) {
    return (a >> (bitsPerCodon * shift)) == (b & ((1U << (totalDnaBits - bitsPerCodon * shift)) - 1));
}
static bool consecutive2(uint32_t a, uint32_t b, int shift, int bitsPerCodon, int totalDnaBits) {
    return (a & ((1U << (totalDnaBits - bitsPerCodon * shift)) - 1)) == (b >> (bitsPerCodon * shift));
}

struct TaxonScore {
    TaxID taxId = 0;
    float score = 0.0f;
    int hammingDist = 0;
    bool LCA = false;
};

struct MatchPath {  // Taxonomer.h:35-59
    int start = 0, end = 0;
    float score = 0.f;
    int hammingDist = 0, depth = 0;
    const mtb_match* startMatch = nullptr;
    const mtb_match* endMatch = nullptr;
    MatchPath() {}
    explicit MatchPath(const mtb_match* m)
        : start((int)infoPos(m->qinfo)), end((int)infoPos(m->qinfo) + 23), score(matchScore(*m)),
          hammingDist(m->hamming), depth(1), startMatch(m), endMatch(m) {}
};

class Taxonomer {
public:
    Taxonomer(const Db& db, const mtb_params& par) : db(db), par(par), tax(db.tax) {
        minConsCnt = par.min_cons_cnt;
        minConsCntEuk = par.min_cons_cnt_euk;
        eukaryotaTaxId = tax.eukaryotaTaxID;
        tieRatio = par.tie_ratio;
        accessionLevel = par.accession_level;
        kmerFormat = par.kmer_format;
        const TaxShape t = taxShape(par);
        dnaShift = t.dnaShift;
        maxCodonShift = t.maxCodonShift;
        denominator = t.denominator;
        bitsPerCodon = t.bitsPerCodon;
        totalDnaBits = t.totalDnaBits;
    }

    void chooseBestTaxon(uint32_t currentQuery, size_t offset, size_t end, const mtb_match* matchList,
                         std::vector<Query>& queryList);

    // pin hook (orc_pin_combine): combineMatchPaths over the caller's paths alone
    float combineForPin(std::vector<MatchPath>& paths, std::vector<MatchPath>& out, int readLength) {
        matchPaths.swap(paths);
        combinedMatchPaths.clear();
        const float s = combineMatchPaths(0, 0, readLength);
        out = combinedMatchPaths;
        matchPaths.swap(paths);
        return s;
    }

private:
    const Db& db;
    const mtb_params& par;
    const Taxonomy& tax;
    int minConsCnt, minConsCntEuk, eukaryotaTaxId, accessionLevel, kmerFormat;
    float tieRatio;
    int dnaShift, maxCodonShift, denominator, bitsPerCodon, totalDnaBits;
    std::vector<MatchPath> matchPaths, combinedMatchPaths, localMatchPaths;
    std::vector<bool> connectedToNext;
    std::vector<TaxID> maxSpecies;
    std::unordered_map<TaxID, unsigned int> taxCnt;
    std::unordered_map<TaxID, TaxonCounts> cladeCnt;
    std::vector<const mtb_match*> bestMatchForQuotient;
    std::vector<TaxID> bestMatchTaxIdForQuotient;
    std::vector<uint8_t> minHammingForQuotient;

    TaxonScore getBestSpeciesMatches(std::pair<size_t, size_t>& range, const mtb_match* ml, size_t end,
                                     size_t offset, Query& q);
    float combineMatchPaths(size_t pathStart, size_t combStart, int readLength);
    void trimMatchPath(MatchPath& p1, const MatchPath& p2, int overlap);
    void getMatchPaths(const mtb_match* ml, size_t start, size_t end, TaxID speciesId);
    void filterRedundantMatches(const mtb_match* ml, const std::pair<size_t, size_t>& range, int queryLength);
    TaxID lowerRankClassification(TaxID spTaxId, int queryLength);
    void getSpeciesCladeCounts(TaxID speciesTaxID);
    TaxID BFS(TaxID root, unsigned int maxCnt);

    float calScoreIncrement(uint16_t h, int shift) const { return scoreIncrement(h, shift); }
    int calHammingDistIncrement(uint16_t h, int shift) const { return hammingIncrement(h, shift); }
    bool isConsecutive(const mtb_match* a, const mtb_match* b, int shift) const {  // Taxonomer.cpp:677-683
        return consecutive1(a->dna_encoding, b->dna_encoding, shift, bitsPerCodon, totalDnaBits);
    }
    bool isConsecutive2(const mtb_match* a, const mtb_match* b, int shift) const {  // :692-699
        return consecutive2(a->dna_encoding, b->dna_encoding, shift, bitsPerCodon, totalDnaBits);
    }
};

void Taxonomer::chooseBestTaxon(uint32_t currentQuery, size_t offset, size_t end, const mtb_match* matchList,
                                std::vector<Query>& queryList) {
    Query& q = queryList[currentQuery];
    std::pair<size_t, size_t> bestSpeciesRange(0, 0);
    TaxonScore speciesScore = getBestSpeciesMatches(bestSpeciesRange, matchList, end, offset, q);
    if (speciesScore.score == 0 || speciesScore.score < par.min_score) {
        q.isClassified = false; q.classification = 0; q.score = speciesScore.score;
        q.hammingDist = speciesScore.hammingDist; q.newSpecies = false;
        return;
    }
    if (speciesScore.LCA) {
        q.isClassified = true; q.classification = speciesScore.taxId; q.score = speciesScore.score;
        q.hammingDist = speciesScore.hammingDist;
        return;
    }
    taxCnt.clear();
    filterRedundantMatches(matchList, bestSpeciesRange, q.queryLength + q.queryLength2);
    for (auto& t : taxCnt) q.taxCnt[t.first] = (int)t.second;
    if (speciesScore.score < par.min_sp_score) {
        q.isClassified = true;
        q.classification = tax.taxonNode(tax.getTaxIdAtRank(speciesScore.taxId, "species"))->parentTaxId;
        q.score = speciesScore.score; q.hammingDist = speciesScore.hammingDist;
        return;
    }
    q.isClassified = true; q.score = speciesScore.score; q.hammingDist = speciesScore.hammingDist;
    q.newSpecies = false;
    q.classification = par.em ? speciesScore.taxId  // :193-201
                              : lowerRankClassification(speciesScore.taxId, q.queryLength + q.queryLength2);
}

void Taxonomer::filterRedundantMatches(const mtb_match* ml, const std::pair<size_t, size_t>& range,
                                       int queryLength) {  // Taxonomer.cpp:205-241
    size_t maxQuotient = (size_t)((queryLength + 3) / dnaShift);
    bestMatchForQuotient.assign(maxQuotient + 1, nullptr);
    bestMatchTaxIdForQuotient.assign(maxQuotient + 1, 0);
    minHammingForQuotient.assign(maxQuotient + 1, std::numeric_limits<uint8_t>::max());
    for (size_t i = range.first; i < range.second; i++) {
        size_t qt = infoPos(ml[i].qinfo) / (uint32_t)dnaShift;
        uint8_t h = ml[i].hamming;
        if (bestMatchForQuotient[qt] == nullptr) {
            bestMatchForQuotient[qt] = ml + i; bestMatchTaxIdForQuotient[qt] = (TaxID)ml[i].target_id;
            minHammingForQuotient[qt] = h;
        } else if (h < minHammingForQuotient[qt]) {
            bestMatchForQuotient[qt] = ml + i; bestMatchTaxIdForQuotient[qt] = (TaxID)ml[i].target_id;
            minHammingForQuotient[qt] = h;
        } else if (h == minHammingForQuotient[qt]) {
            bestMatchTaxIdForQuotient[qt] = tax.LCA(bestMatchTaxIdForQuotient[qt], (TaxID)ml[i].target_id);
        }
    }
    for (size_t i = 0; i <= maxQuotient; ++i)
        if (bestMatchForQuotient[i] != nullptr) taxCnt[bestMatchTaxIdForQuotient[i]]++;
}

TaxID Taxonomer::lowerRankClassification(TaxID spTaxId, int queryLength) {  // :252-271
    unsigned int minSubSpeciesMatch = (unsigned int)((queryLength - 1) / denominator);
    cladeCnt.clear();
    getSpeciesCladeCounts(spTaxId);
    if (accessionLevel == 2) {
        std::vector<TaxID> keys;
        for (auto& kv : cladeCnt) keys.push_back(kv.first);
        for (TaxID k : keys) {
            const TaxonNode* taxon = tax.taxonNode(k);
            if (taxon->rank == "" || taxon->rank == "accession") {
                auto& ch = cladeCnt[taxon->parentTaxId].children;
                ch.erase(std::find(ch.begin(), ch.end(), k));
            }
        }
    }
    return BFS(spTaxId, minSubSpeciesMatch);
}

void Taxonomer::getSpeciesCladeCounts(TaxID speciesTaxID) {  // :273-290
    for (auto it = taxCnt.begin(); it != taxCnt.end(); ++it) {
        const TaxonNode* taxon = tax.taxonNode(it->first);
        cladeCnt[taxon->taxId].taxCount = it->second;
        cladeCnt[taxon->taxId].cladeCount += it->second;
        while (taxon->taxId != speciesTaxID) {
            auto& ch = cladeCnt[taxon->parentTaxId].children;
            if (std::find(ch.begin(), ch.end(), taxon->taxId) == ch.end()) ch.push_back(taxon->taxId);
            cladeCnt[taxon->parentTaxId].cladeCount += it->second;
            taxon = tax.taxonNode(taxon->parentTaxId);
        }
    }
}

TaxID Taxonomer::BFS(TaxID root, unsigned int maxCnt) {  // :292-314
    unsigned int maxCnt2 = maxCnt;
    if (cladeCnt.at(root).children.empty()) return root;
    std::vector<TaxID> best;
    for (TaxID c : cladeCnt.at(root).children) {
        unsigned int cur = cladeCnt.at(c).cladeCount;
        if (cur > maxCnt) { best.clear(); best.push_back(c); maxCnt = cur; }
        else if (cur == maxCnt) best.push_back(c);
    }
    if (best.size() == 1) return BFS(best[0], maxCnt2);
    return root;
}

TaxonScore Taxonomer::getBestSpeciesMatches(std::pair<size_t, size_t>& bestSpeciesRange, const mtb_match* ml,
                                            size_t end, size_t offset, Query& query) {  // :316-408
    matchPaths.clear();
    combinedMatchPaths.clear();
    std::vector<std::pair<TaxID, float>> sp2score;
    int queryLength = query.queryLength + query.queryLength2;
    TaxonScore bestScore;
    float bestSpScore = 0;
    size_t i = offset;
    size_t meaningfulSpecies = 0;
    while (i < end + 1) {
        TaxID currentSpecies = (TaxID)ml[i].species_id;
        size_t start = i;
        size_t previousPathSize = matchPaths.size();
        while ((i < end + 1) && currentSpecies == (TaxID)ml[i].species_id) {
            uint32_t curFrame = infoFrame(ml[i].qinfo);
            size_t fstart = i;
            while ((i < end + 1) && currentSpecies == (TaxID)ml[i].species_id && curFrame == infoFrame(ml[i].qinfo)) i++;
            if (i - fstart > 1) getMatchPaths(ml, fstart, i, currentSpecies);
        }
        size_t pathSize = matchPaths.size();
        if (pathSize > previousPathSize) {
            float score = combineMatchPaths(previousPathSize, combinedMatchPaths.size(), queryLength);
            score = std::min(score, 1.0f);
            if (score < par.min_score) continue;
            sp2score.emplace_back(currentSpecies, score);
            if (score > 0.f) meaningfulSpecies++;
            if (score > bestSpScore) { bestSpScore = score; bestSpeciesRange = std::make_pair(start, i); }
        }
    }
    if (meaningfulSpecies == 0) { bestScore.score = 0; return bestScore; }
    if (par.em && !sp2score.empty()) {  // :377-386
        std::sort(sp2score.begin(), sp2score.end(),
                  [](const std::pair<TaxID, float>& a, const std::pair<TaxID, float>& b) { return a.second > b.second; });
        query.topSpeciesId = sp2score[0].first;
        for (size_t k = 0; k < 10 && k < sp2score.size(); k++)
            query.species2Score.emplace_back(sp2score[k].first, sp2score[k].second * sp2score[k].second);
    }
    maxSpecies.clear();
    for (size_t k = 0; k < sp2score.size(); k++) {
        if (sp2score[k].second >= bestSpScore * tieRatio) {
            maxSpecies.push_back(sp2score[k].first);
            bestScore.score += sp2score[k].second;
        }
    }
    if (maxSpecies.size() > 1) {
        bestScore.LCA = true;
        bestScore.taxId = tax.LCA(maxSpecies)->taxId;
        bestScore.score /= maxSpecies.size();
        return bestScore;
    }
    bestScore.taxId = maxSpecies[0];
    return bestScore;
}

float Taxonomer::combineMatchPaths(size_t matchPathStart, size_t combMatchPathStart, int readLength) {  // :410-468
    std::sort(matchPaths.begin() + matchPathStart, matchPaths.end(), [](const MatchPath& a, const MatchPath& b) {
        if (a.score != b.score) return a.score > b.score;
        if (a.hammingDist != b.hammingDist) return a.hammingDist < b.hammingDist;
        return a.start > b.start;
    });
    float score = 0;
    for (size_t i = matchPathStart; i < matchPaths.size(); i++) {
        if (combMatchPathStart == combinedMatchPaths.size()) {
            combinedMatchPaths.push_back(matchPaths[i]);
            score += matchPaths[i].score;
        } else {
            bool isOverlapped = false;
            for (size_t j = combMatchPathStart; j < combinedMatchPaths.size(); j++) {
                MatchPath& p = matchPaths[i];
                const MatchPath& c = combinedMatchPaths[j];
                if (!((p.end < c.start) || (c.end < p.start))) {
                    int overlappedLength = std::min(p.end, c.end) - std::max(p.start, c.start) + 1;
                    if (overlappedLength == p.end - p.start + 1) { isOverlapped = true; break; }
                    if (overlappedLength < 24) { trimMatchPath(p, c, overlappedLength); continue; }
                    isOverlapped = true;
                    break;
                }
            }
            if (!isOverlapped) {
                combinedMatchPaths.push_back(matchPaths[i]);
                score += matchPaths[i].score;
            }
        }
    }
    return score / readLength;
}

void Taxonomer::trimMatchPath(MatchPath& p1, const MatchPath& p2, int overlap) {  // :475-485
    if (p1.start < p2.start) {
        p1.end = p2.start - 1;
        p1.hammingDist = std::max(0, p1.hammingDist - rightPartHamming(*p1.endMatch, overlap / 3));
        p1.score = p1.score - rightPartScore(*p1.endMatch, overlap / 3) - (overlap % 3);
    } else {
        p1.start = p2.end + 1;
        p1.hammingDist = std::max(0, p1.hammingDist - leftPartHamming(*p1.startMatch, overlap / 3));
        p1.score = p1.score - leftPartScore(*p1.startMatch, overlap / 3) - (overlap % 3);
    }
}

void Taxonomer::getMatchPaths(const mtb_match* ml, size_t start, size_t end, TaxID speciesId) {  // :487-648
    size_t i = start;
    size_t currPos = infoPos(ml[start].qinfo);
    uint64_t frame = infoFrame(ml[start].qinfo);
    int MIN_DEPTH = minConsCnt;
    if (tax.IsAncestor(eukaryotaTaxId, speciesId)) MIN_DEPTH = minConsCntEuk;
    connectedToNext.assign(end - start + 1, false);
    localMatchPaths.clear();
    localMatchPaths.resize(end - start + 1);
    const bool fwd = frame < 3;

    size_t curPosMatchStart = i;
    while (i < end && infoPos(ml[i].qinfo) == currPos) { localMatchPaths[i - start] = MatchPath(ml + i); ++i; }
    size_t curPosMatchEnd = i;
    while (i < end) {
        uint32_t nextPos = infoPos(ml[i].qinfo);
        size_t nextPosMatchStart = i;
        while (i < end && nextPos == infoPos(ml[i].qinfo)) { localMatchPaths[i - start] = MatchPath(ml + i); ++i; }
        size_t nextPosMatchEnd = i;
        int shift = (int)((nextPos - currPos) / 3);
        if (shift > 0 && shift <= maxCodonShift) {
            for (size_t nextIdx = nextPosMatchStart; nextIdx < nextPosMatchEnd; nextIdx++) {
                float scoreIncrement = calScoreIncrement(ml[nextIdx].right_end_hamming, shift);
                const MatchPath* bestPath = nullptr;
                float bestScore = 0;
                for (size_t curIdx = curPosMatchStart; curIdx < curPosMatchEnd; ++curIdx) {
                    bool cons;
                    if (kmerFormat == 2) cons = fwd ? isConsecutive2(ml + curIdx, ml + nextIdx, shift)
                                                    : isConsecutive2(ml + nextIdx, ml + curIdx, shift);
                    else cons = fwd ? isConsecutive(ml + curIdx, ml + nextIdx, shift)
                                    : isConsecutive(ml + nextIdx, ml + curIdx, shift);
                    if (cons) {
                        connectedToNext[curIdx - start] = true;
                        if (localMatchPaths[curIdx - start].score > bestScore) {
                            bestPath = &localMatchPaths[curIdx - start];
                            bestScore = localMatchPaths[curIdx - start].score;
                        }
                    }
                }
                if (bestPath != nullptr) {
                    MatchPath& np = localMatchPaths[nextIdx - start];
                    np.start = bestPath->start;
                    np.score = bestPath->score + scoreIncrement;
                    np.hammingDist = bestPath->hammingDist + calHammingDistIncrement(ml[nextIdx].right_end_hamming, shift);
                    np.depth = bestPath->depth + shift;
                    np.startMatch = bestPath->startMatch;
                }
            }
        }
        for (size_t curIdx = curPosMatchStart; curIdx < curPosMatchEnd; ++curIdx)
            if (!connectedToNext[curIdx - start] && localMatchPaths[curIdx - start].depth >= MIN_DEPTH)
                matchPaths.push_back(localMatchPaths[curIdx - start]);
        if (i == end)
            for (size_t nextIdx = nextPosMatchStart; nextIdx < nextPosMatchEnd; ++nextIdx)
                if (localMatchPaths[nextIdx - start].depth >= MIN_DEPTH) matchPaths.push_back(localMatchPaths[nextIdx - start]);
        curPosMatchStart = nextPosMatchStart;
        curPosMatchEnd = nextPosMatchEnd;
        currPos = nextPos;
    }
}

void assignTaxonomy(const Db& db, const mtb_params& par, const mtb_match* matchList, size_t numOfMatches,
                    std::vector<Query>& queryList) {
    struct Block { size_t start, end; uint32_t id; };
    std::vector<Block> blocks;
    size_t matchIdx = 0;
    while (matchIdx < numOfMatches) {  // Classifier.cpp:178-185
        uint32_t cur = infoSeq(matchList[matchIdx].qinfo);
        Block b{matchIdx, 0, cur};
        while (matchIdx < numOfMatches && cur == infoSeq(matchList[matchIdx].qinfo)) ++matchIdx;
        b.end = matchIdx - 1;
        blocks.push_back(b);
    }
#pragma omp parallel
    {
        Taxonomer t(db, par);
#pragma omp for schedule(dynamic, 1)
        for (size_t i = 0; i < blocks.size(); ++i)
            t.chooseBestTaxon(blocks[i].id - 1, blocks[i].start, blocks[i].end, matchList, queryList);
    }
}

}  // namespace orc

namespace orc {

void emReassign(const Db& db, const mtb_em_map* maps, size_t n, size_t totalQueryCnt, EmOut& out) {
    // countUniqueKmerPerSpecies (Classifier.cpp:388-431): every info entry's species
    std::unordered_map<TaxID, uint32_t> sp2uniq;
    for (uint32_t t : db.info) {
        if (t == 0) break;  // ReadBuffer<TaxID>::getNext() == 0 ends the loop
        auto it = db.taxId2speciesId.find((TaxID)t);
        if (it != db.taxId2speciesId.end() && it->second) sp2uniq[it->second]++;
    }
    auto lengthFactor = [&](TaxID sp) {
        auto it = sp2uniq.find(sp);
        return (it != sp2uniq.end() && it->second > 0) ? 1.0 / log((double)it->second) : 0.0;
    };
    std::vector<std::pair<size_t, size_t>> queryRanges;  // :224-233
    for (size_t idx = 0; idx < n;) {
        const uint32_t cur = maps[idx].query_id;
        const size_t start = idx;
        while (idx < n && maps[idx].query_id == cur) idx++;
        queryRanges.emplace_back(start, idx);
    }
    std::map<TaxID, double> taxProbs, Fnew;  // species ascending (the reference's unordered_set order is arbitrary)
    std::vector<TaxID> spList;
    for (auto& r : queryRanges) taxProbs[maps[r.first].species_id] = 0;  // topSpeciesSet
    for (auto& kv : taxProbs) spList.push_back(kv.first);
    for (TaxID sp : spList) { taxProbs[sp] = 1.0 / spList.size(); Fnew[sp] = 0.0; }
    auto prob = [&](TaxID sp) { auto it = taxProbs.find(sp); return it == taxProbs.end() ? 0.0 : it->second; };
    size_t queryCount = 0;
    for (size_t iter = 0; iter < 1000; ++iter) {  // :247-309
        for (auto& kv : Fnew) kv.second = 0.0;
        queryCount = 0;
        for (auto& r : queryRanges) {
            double denom = 0.0;
            for (size_t j = r.first; j < r.second; ++j)
                denom += maps[j].score * prob(maps[j].species_id) * lengthFactor(maps[j].species_id);
            if (denom == 0.0) continue;
            queryCount++;
            for (size_t j = r.first; j < r.second; ++j)
                Fnew[maps[j].species_id] +=
                    (maps[j].score * prob(maps[j].species_id) * lengthFactor(maps[j].species_id)) / denom;
        }
        for (TaxID sp : spList) Fnew[sp] /= queryCount;
        double delta = 0.0;
        for (TaxID sp : spList) {
            delta += fabs(Fnew[sp] - taxProbs[sp]);
            if (iter > 10 && Fnew[sp] < 1e-5) Fnew[sp] = 0.0;
        }
        taxProbs.swap(Fnew);
        out.iterations = (uint32_t)iter + 1;
        if (delta < 1e-6) break;
    }
    size_t explained = 0;  // :312-318
    for (TaxID sp : spList) {
        out.probs[sp] = taxProbs[sp];
        out.emTaxCounts[sp] = (unsigned int)(taxProbs[sp] * queryCount);
        explained += out.emTaxCounts[sp];
    }
    out.emTaxCounts[0] = (unsigned int)(totalQueryCnt - explained);
    out.queryCount = queryCount;
    out.reads.assign(totalQueryCnt, mtb_em_read{0, 0, 0.0});
    for (auto& r : queryRanges) {  // reclassify (:326-372)
        const uint32_t q = maps[r.first].query_id;
        double denom = 0.0;
        std::vector<std::pair<TaxID, double>> sp2prob;
        for (size_t j = r.first; j < r.second; ++j) {
            const double sc = prob(maps[j].species_id) * maps[j].score * lengthFactor(maps[j].species_id);
            denom += sc;
            sp2prob.emplace_back(maps[j].species_id, sc);
        }
        if (denom == 0.0) { out.reads[q] = mtb_em_read{0, 2, 0.0}; continue; }
        for (auto& sp : sp2prob) sp.second /= denom;
        std::sort(sp2prob.begin(), sp2prob.end(),
                  [](const std::pair<TaxID, double>& a, const std::pair<TaxID, double>& b) { return a.second > b.second; });
        double sum = 0.0;
        std::vector<TaxID> cand;
        for (size_t j = 0; j < sp2prob.size() && sum < 0.5; ++j) {
            sum += sp2prob[j].second;
            cand.push_back(sp2prob[j].first);
        }
        out.reads[q] = mtb_em_read{db.tax.LCA(cand)->taxId, 1, sum};
    }
}

}  // namespace orc

// Pin hook (test infrastructure: tests/test_oracle.py checks these restatements against
// tests/golden/ref_functions.json, which the reference's own function bodies computed): the
// dependency-free helpers above on caller vectors, fn = MTB_PIN_* (include/mtb_gpu.h).
extern "C" int orc_pin_eval(int fn, const int64_t* param, const uint64_t* a, const uint64_t* b, uint64_t n,
                            int64_t* out, uint64_t* n_out) {
    using namespace orc;
    auto fbits = [](float f) { uint32_t u; memcpy(&u, &f, 4); return (int64_t)u; };
    *n_out = n;
    if (fn == MTB_PIN_DECODE_DIFF_IDX) {
        std::vector<uint16_t> w(n);
        for (uint64_t i = 0; i < n; i++) w[i] = (uint16_t)a[i];
        std::vector<uint64_t> v(n);
        *n_out = decodeDiffIdx(w.data(), n, v.data());
        for (uint64_t i = 0; i < *n_out; i++) out[i] = (int64_t)v[i];
        return MTB_OK;
    }
    const TaxShape t = taxShape(mtb_params{});
    for (uint64_t i = 0; i < n; i++) {
        const int p = (int)param[i];
        mtb_match m{};
        m.right_end_hamming = (uint16_t)a[i];
        switch (fn) {
            case MTB_PIN_SCORE_INCREMENT: out[i] = fbits(scoreIncrement((uint16_t)a[i], p)); break;
            case MTB_PIN_HAMMING_INCREMENT: out[i] = hammingIncrement((uint16_t)a[i], p); break;
            case MTB_PIN_IS_CONSECUTIVE:  // shift 0: the shift-less form (one codon, lastCodonMask)
                out[i] = consecutive1((uint32_t)a[i], (uint32_t)b[i], p ? p : 1, t.bitsPerCodon, t.totalDnaBits); break;
            case MTB_PIN_IS_CONSECUTIVE2:
                out[i] = consecutive2((uint32_t)a[i], (uint32_t)b[i], p ? p : 1, t.bitsPerCodon, t.totalDnaBits); break;
            case MTB_PIN_MATCH_SCORE: out[i] = fbits(matchScore(m)); break;
            case MTB_PIN_RIGHT_PART_SCORE: out[i] = fbits(rightPartScore(m, p)); break;
            case MTB_PIN_LEFT_PART_SCORE: out[i] = fbits(leftPartScore(m, p)); break;
            case MTB_PIN_RIGHT_PART_HAMMING: out[i] = rightPartHamming(m, p); break;
            case MTB_PIN_LEFT_PART_HAMMING: out[i] = leftPartHamming(m, p); break;
            case MTB_PIN_MAX_COVERED_LENGTH: out[i] = maxCoveredLength((int)a[i]); break;
            case MTB_PIN_QUERY_KMER_NUMBER: out[i] = queryKmerNumber((int)a[i], 8, p); break;
            case MTB_PIN_TAXONOMER_SHAPE: {
                mtb_params par{};
                par.syncmer = (int)(a[i] >> 16);
                par.smer_len = (int)(a[i] & 0xFF);
                par.seq_mode = (int)b[i];
                const TaxShape q = taxShape(par);
                const int64_t v[6] = {q.dnaShift, q.maxCodonShift, q.denominator, q.bitsPerCodon, q.totalDnaBits,
                                      (int64_t)q.lastCodonMask};
                for (int k = 0; k < 6; k++) out[6 * i + k] = v[k];
                break;
            }
            default: return MTB_ERR_ARG;
        }
    }
    return MTB_OK;
}

// Pin hook (tests/test_ref_paths.py against tests/golden/ref_paths.npz, which the reference's own
// combineMatchPaths / trimMatchPath / isMatchPathOverlapped / MatchPath produced): one species run's
// paths — start, end, score, hammingDist, and the rightEndHamming of their start and end matches —
// combined. Returns the score (score / readLength); comb_out gets (start, end, hammingDist, score bits)
// per kept path.
extern "C" int orc_pin_combine(const int32_t* start, const int32_t* end, const float* score, const int32_t* hd,
                               const uint16_t* reh_start, const uint16_t* reh_end, uint64_t n, int read_length,
                               float* score_out, int32_t* comb_out, uint64_t* n_comb) {
    using namespace orc;
    static const Db db;
    static const mtb_params par{};
    Taxonomer t(db, par);
    std::vector<mtb_match> ms(2 * n);
    std::vector<MatchPath> paths(n), out;
    for (uint64_t i = 0; i < n; i++) {
        ms[2 * i] = mtb_match{};
        ms[2 * i + 1] = mtb_match{};
        ms[2 * i].right_end_hamming = reh_start[i];
        ms[2 * i + 1].right_end_hamming = reh_end[i];
        MatchPath& p = paths[i];
        p.start = start[i];
        p.end = end[i];
        p.score = score[i];
        p.hammingDist = hd[i];
        p.depth = 1;
        p.startMatch = &ms[2 * i];
        p.endMatch = &ms[2 * i + 1];
    }
    *score_out = t.combineForPin(paths, out, read_length);
    *n_comb = out.size();
    for (size_t i = 0; i < out.size(); i++) {
        comb_out[4 * i] = out[i].start;
        comb_out[4 * i + 1] = out[i].end;
        comb_out[4 * i + 2] = out[i].hammingDist;
        memcpy(&comb_out[4 * i + 3], &out[i].score, 4);
    }
    return MTB_OK;
}
