// ORACLE — test infrastructure only (see orc_core.h header).
//
// Restatement of the taxonomy services the path uses. They live in MMseqs2's NcbiTaxonomy
// (dependency lib/mmseqs = github.com/jaebeom-kim/MMseqs2, an un-vendored submodule; no pinned
// SHA in the mount) plus Metabuli's TaxonomyWrapper (src/commons/TaxonomyWrapper.{h,cpp}).
// Restated from MMseqs2's published NcbiTaxonomy.cpp algorithm (Euler tour E/L/H + sparse-table
// RMQ LCA, nodes.dmp/merged.dmp loading, the NcbiRanks rank table) — parity unpinned: no
// fixture or test in the reference exercises it.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace orc {

typedef int TaxID;

struct TaxonNode {
    int id;
    TaxID taxId;
    TaxID parentTaxId;
    std::string rank;
    std::string name;
};

struct TaxonCounts {  // MMseqs2 NcbiTaxonomy.h
    unsigned int taxCount = 0;
    unsigned int cladeCount = 0;
    std::vector<TaxID> children;
};

class Taxonomy {
public:
    std::vector<TaxonNode> nodes;  // node index = row of nodes.dmp
    std::vector<int> D;            // taxID -> node index, -1 if absent
    TaxID maxTaxID = 0;
    TaxID eukaryotaTaxID = 0;
    std::vector<int> E, L, H;
    std::vector<std::vector<int>> M;

    // NcbiTaxonomy(names, nodes, merged) non-internal path (TaxonomyWrapper.cpp:67-118).
    bool loadDmp(const std::string& dir, std::string* err);
    // TaxonomyWrapper::unserialize (TaxonomyWrapper.cpp:363-421) of a taxonomyDB file, with the
    // MMseqs2 TaxonNode / StringBlock<unsigned int> layouts (unpinned). Returns false with *err
    // empty when the serialization version differs (the reference then falls back to the dmp
    // files, common.cpp:71-85), with *err set on a malformed file.
    bool loadTaxonomyDb(const std::string& path, std::string* err);
    static const int kSerializationVersion = 2;  // NcbiTaxonomy::SERIALIZATION_VERSION (MMseqs2)
    bool useInternalTaxID = false;
    std::vector<int> internal2orgTaxId;  // TaxonomyWrapper::internal2orgTaxId
    TaxID getOriginalTaxID(TaxID t) const {  // TaxonomyWrapper.h:70-79
        if (!useInternalTaxID) return t;
        return (t >= 0 && t <= maxTaxID) ? internal2orgTaxId[t] : t;
    }
    bool fromArrays(const int32_t* taxid, const int32_t* parent, size_t n, const std::vector<std::string>& ranks,
                    const std::vector<std::string>& names, const int32_t* mergedOld, const int32_t* mergedNew,
                    size_t nMerged, std::string* err);

    bool nodeExists(TaxID t) const { return t >= 0 && t <= maxTaxID && D[t] != -1; }
    int nodeId(TaxID t) const { return D[t]; }
    const TaxonNode* taxonNode(TaxID t) const { return &nodes[D[t]]; }
    TaxID LCA(TaxID a, TaxID b) const;                     // NcbiTaxonomy::LCA(TaxID, TaxID)
    const TaxonNode* LCA(const std::vector<TaxID>& v) const;  // NcbiTaxonomy::LCA(vector)
    bool IsAncestor(TaxID ancestor, TaxID child) const;    // NcbiTaxonomy::IsAncestor
    TaxID getTaxIdAtRank(int taxId, const std::string& rank) const;  // TaxonomyWrapper.cpp:479-498
    static int findRankIndex(const std::string& rank);

private:
    void finish();
    int lcaHelper(int i, int j) const;
    int rmq(int i, int j) const;
};

}  // namespace orc
