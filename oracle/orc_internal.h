// ORACLE — test infrastructure only (see orc_core.h header).
#pragma once
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "orc_core.h"
#include "orc_taxonomy.h"

namespace orc {

struct DiffIdxSplit {  // Kmer.h:111-119
    uint64_t ADkmer;
    uint64_t diffIdxOffset;
    uint64_t infoIdxOffset;
};

// A reference DB held in memory: the on-disk files of SURVEY Appendix B plus the loaded taxonomy
// and the taxId2speciesId map built by KmerMatcher::loadTaxIdList (KmerMatcher.cpp:56-120).
struct Db {
    std::vector<uint16_t> diffIdx;
    std::vector<uint32_t> info;
    std::vector<DiffIdxSplit> split;
    std::vector<TaxID> taxIdList;
    Taxonomy tax;
    std::unordered_map<TaxID, TaxID> taxId2speciesId;
    bool buildSpeciesMap(std::string* err);
};

// Query (common.h:95-128), restricted to the fields the path writes.
struct Query {
    int queryLength = 0, queryLength2 = 0, kmerCnt = 0, kmerCnt2 = 0;
    int classification = 0;
    float score = 0;
    int hammingDist = 0;
    bool isClassified = false;
    bool newSpecies = false;
    std::map<TaxID, int> taxCnt;
    TaxID topSpeciesId = 0;                             // --em (common.h:104,110)
    std::vector<std::pair<TaxID, float>> species2Score;
};

struct Reads {
    const char* seq1; const uint64_t* off1;
    const char* seq2; const uint64_t* off2;
    uint32_t n;
};

// getNextTargetKmer (KmerMatcher.h:282-297) over a whole diffIdx word stream from 0: the values of its
// whole k-mers in order; returns their number (orc_match.cpp; the pin hook, orc_pin_eval).
uint64_t decodeDiffIdx(const uint16_t* diff, uint64_t nWords, uint64_t* values);

// KmerExtractor::extractQueryKmers (KmerExtractor.cpp:52-81): fills the reserved buffer exactly as
// the reference does (unused reserved slots stay {0,0}) and sorts it by compareQueryKmer.
void extractQueryKmers(const mtb_params& par, const Reads& reads, std::vector<mtb_kmer>& buf,
                       std::vector<Query>& queries, bool sort);

// SeqIterator::maskLowComplexityRegions (SeqIterator.cpp:154-175) of one read (orc_mask.cpp), and
// tantan's per-letter repeat probabilities of a coded sequence.
void maskLowComplexityRegions(const char* seq, int n, float maskProb, char* out);
void tantanRepeatProbs(const unsigned char* x, int n, float* prob);

// KmerMatcher::matchKmers (KmerMatcher.cpp:123-481) over in-memory files.
bool matchKmers(const Db& db, const mtb_params& par, const mtb_kmer* kmers, size_t nKmers,
                std::vector<mtb_match>& matches, std::string* err);
void sortMatches(std::vector<mtb_match>& matches);  // KmerMatcher.cpp:1071-1078
bool compareMatches(const mtb_match& a, const mtb_match& b);

// Classifier::assignTaxonomy (Classifier.cpp:166-208) with Taxonomer::chooseBestTaxon.
void assignTaxonomy(const Db& db, const mtb_params& par, const mtb_match* matches, size_t n,
                    std::vector<Query>& queries);

// --em (Classifier.cpp:209-386) over the mappings of all batches (MappingRes = mtb_em_map), one
// thread: the reference's OpenMP sums in the order a single thread takes them.
struct EmOut {
    std::vector<mtb_em_read> reads;  // per read
    std::map<TaxID, double> probs;   // top species -> final abundance
    std::map<TaxID, unsigned int> emTaxCounts;
    uint64_t queryCount = 0;
    uint32_t iterations = 0;
};
void emReassign(const Db& db, const mtb_em_map* maps, size_t n, size_t totalReads, EmOut& out);

// Synthetic reference DB writer (IndexCreator restatement, orc_dbwriter.cpp).
struct BuildInput {
    const char* seq; const uint64_t* off; uint32_t nGenomes; const int32_t* genomeTaxId;
    const int32_t* blkGenome; const int32_t* blkStart; const int32_t* blkEnd; const int32_t* blkStrand; uint64_t nBlocks;
    int splitNum;
};
bool buildDb(const mtb_params& par, const Taxonomy& tax, const BuildInput& in, Db& db, std::string* err);
bool writeDbFiles(const Db& db, const mtb_params& par, const std::string& dir, std::string* err);

}  // namespace orc
