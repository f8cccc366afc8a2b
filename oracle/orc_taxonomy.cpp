// ORACLE — test infrastructure only (see orc_core.h header).
#include "orc_taxonomy.h"

#include <cassert>
#include <cstring>
#include <iterator>
#include <fstream>
#include <functional>

namespace orc {

static std::vector<std::string> splitBy(const std::string& s, const std::string& delim, int maxCol) {
    // TaxonomyWrapper::splitByDelimiter (TaxonomyWrapper.cpp:26-39)
    std::vector<std::string> out;
    size_t prev = 0, pos = 0;
    int i = 0;
    do {
        pos = s.find(delim, prev);
        if (pos == std::string::npos) pos = s.length();
        out.emplace_back(s.substr(prev, pos - prev));
        prev = pos + delim.length();
        i++;
    } while (pos < s.length() && prev < s.length() && i < maxCol);
    return out;
}

bool Taxonomy::loadDmp(const std::string& dir, std::string* err) {
    std::ifstream nodesIn(dir + "/nodes.dmp");
    if (!nodesIn) { *err = "nodes.dmp not found in " + dir; return false; }
    std::vector<int32_t> tax, par;
    std::vector<std::string> ranks;
    std::string line;
    while (std::getline(nodesIn, line)) {
        auto r = splitBy(line, "\t|\t", 3);
        if (r.size() < 3) continue;
        tax.push_back((int32_t)strtol(r[0].c_str(), nullptr, 10));
        par.push_back((int32_t)strtol(r[1].c_str(), nullptr, 10));
        ranks.push_back(r[2]);
    }
    std::vector<int32_t> mo, mn;
    std::ifstream mergedIn(dir + "/merged.dmp");
    while (mergedIn && std::getline(mergedIn, line)) {
        auto r = splitBy(line, "\t|\t", 2);
        if (r.size() != 2) { *err = "invalid merged entry"; return false; }
        mo.push_back((int32_t)strtoul(r[0].c_str(), nullptr, 10));
        mn.push_back((int32_t)strtoul(r[1].c_str(), nullptr, 10));
    }
    std::vector<std::string> names(tax.size());
    std::ifstream namesIn(dir + "/names.dmp");
    std::unordered_map<int, size_t> row;
    for (size_t i = 0; i < tax.size(); i++) row[tax[i]] = i;
    while (namesIn && std::getline(namesIn, line)) {
        if (line.find("scientific name") == std::string::npos) continue;
        auto r = splitBy(line, "\t|\t", 2);
        int t = (int)strtol(r[0].c_str(), nullptr, 10);
        auto it = row.find(t);
        if (it == row.end()) { *err = "names.dmp taxon not in nodes.dmp"; return false; }
        names[it->second] = r.size() > 1 ? r[1] : "";
    }
    return fromArrays(tax.data(), par.data(), tax.size(), ranks, names, mo.data(), mn.data(), mo.size(), err);
}

bool Taxonomy::fromArrays(const int32_t* taxid, const int32_t* parent, size_t n, const std::vector<std::string>& ranks,
                          const std::vector<std::string>& names, const int32_t* mergedOld, const int32_t* mergedNew,
                          size_t nMerged, std::string* err) {
    nodes.clear();
    maxTaxID = 0;
    for (size_t i = 0; i < n; i++) {
        nodes.push_back({(int)i, taxid[i], parent[i], ranks[i], i < names.size() ? names[i] : ""});
        if (taxid[i] > maxTaxID) maxTaxID = taxid[i];
    }
    D.assign((size_t)maxTaxID + 1, -1);
    for (size_t i = 0; i < n; i++) D[taxid[i]] = (int)i;
    for (auto& nd : nodes)
        if (!nodeExists(nd.parentTaxId)) { *err = "inconsistent nodes.dmp: missing parent"; return false; }
    for (size_t i = 0; i < nMerged; i++) {  // NcbiTaxonomy::loadMerged
        int o = mergedOld[i], m = mergedNew[i];
        if (o >= 0 && o <= maxTaxID && !nodeExists(o) && nodeExists(m)) D[o] = D[m];
    }
    eukaryotaTaxID = 0;  // TaxonomyWrapper::setEukaryoteTaxID (TaxonomyWrapper.h:89-100)
    for (auto& nd : nodes)
        if (nd.name == "Eukaryota") { eukaryotaTaxID = nd.taxId; break; }
    if (!nodeExists(1)) { *err = "taxonomy has no root taxID 1"; return false; }
    finish();
    return true;
}

void Taxonomy::finish() {
    // TaxonomyWrapper::initTaxonomy (TaxonomyWrapper.cpp:116-146): Euler tour from taxID 1,
    // first occurrences H, sparse table M over levels L.
    size_t maxNodes = nodes.size();
    H.assign(maxNodes, 0);
    std::vector<std::vector<TaxID>> children(maxNodes);
    for (size_t i = 0; i < maxNodes; ++i)
        if (nodes[i].parentTaxId != nodes[i].taxId) children[nodeId(nodes[i].parentTaxId)].push_back(nodes[i].taxId);
    E.clear(); L.clear();
    E.reserve(maxNodes * 2); L.reserve(maxNodes * 2);
    std::function<void(TaxID, int)> elh = [&](TaxID t, int level) {  // NcbiTaxonomy::elh
        int id = nodeId(t);
        if (H[id] == 0) H[id] = (int)E.size();
        E.push_back(id); L.push_back(level);
        for (TaxID c : children[id]) elh(c, level + 1);
        E.push_back(nodeId(nodes[id].parentTaxId)); L.push_back(level - 1);
    };
    elh(1, 0);
    E.resize(maxNodes * 2, 0); L.resize(maxNodes * 2, 0);
    size_t N = maxNodes * 2;
    int k = 0;
    while ((1ul << (k + 1)) <= N) k++;
    M.assign(N, std::vector<int>(k + 1, 0));
    for (size_t i = 0; i < N; ++i) M[i][0] = (int)i;  // NcbiTaxonomy::computeSparseTable
    for (unsigned j = 1; (1ul << j) <= N; ++j)
        for (size_t i = 0; i + (1ul << j) - 1 < N; ++i) {
            int a = M[i][j - 1], b = M[i + (1ul << (j - 1))][j - 1];
            M[i][j] = (L[a] < L[b]) ? a : b;
        }
}

bool Taxonomy::loadTaxonomyDb(const std::string& path, std::string* err) {
    std::ifstream in(path, std::ios::binary);
    if (!in) { *err = "cannot open " + path; return false; }
    std::vector<char> mem((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    const char* p = mem.data();
    const char* end = p + mem.size();
    auto take = [&](void* dst, size_t bytes) {
        if ((size_t)(end - p) < bytes) return false;
        memcpy(dst, p, bytes);
        p += bytes;
        return true;
    };
    err->clear();
    int version = 0;
    if (!take(&version, sizeof(int))) { *err = "taxonomyDB truncated"; return false; }
    if (version != kSerializationVersion) return false;  // outdated: dmp fallback
    size_t internalUsed = 0;  // read as size_t; only the value 1 means "internal IDs" (:372-381)
    if ((size_t)(end - p) < sizeof(size_t)) { *err = "taxonomyDB truncated"; return false; }
    memcpy(&internalUsed, p, sizeof(size_t));
    useInternalTaxID = internalUsed == 1;
    if (useInternalTaxID) p += sizeof(size_t);
    size_t maxNodes = 0;
    int maxTax = 0;
    if (!take(&maxNodes, sizeof(size_t)) || !take(&maxTax, sizeof(int)) || maxTax < 0) {
        *err = "taxonomyDB truncated"; return false;
    }
    struct RawNode { int id; int taxId; int parentTaxId; size_t rankIdx; size_t nameIdx; };  // MMseqs2 TaxonNode
    static_assert(sizeof(RawNode) == 32, "TaxonNode layout");
    std::vector<RawNode> raw(maxNodes);
    std::vector<int> d((size_t)maxTax + 1);
    if (!take(raw.data(), maxNodes * sizeof(RawNode)) || !take(d.data(), d.size() * sizeof(int))) {
        *err = "taxonomyDB truncated"; return false;
    }
    internal2orgTaxId.clear();
    if (useInternalTaxID) {
        internal2orgTaxId.resize((size_t)maxTax + 1);
        if (!take(internal2orgTaxId.data(), internal2orgTaxId.size() * sizeof(int))) { *err = "taxonomyDB truncated"; return false; }
    }
    const size_t N = maxNodes * 2;
    size_t K = 0;  // (int)flog2(N) + 1 columns
    while ((2ul << K) <= N) K++;
    K += 1;
    E.assign(N, 0); L.assign(N, 0); H.assign(maxNodes, 0);
    std::vector<int> flatM(N * K);
    if (!take(E.data(), N * sizeof(int)) || !take(L.data(), N * sizeof(int)) || !take(H.data(), maxNodes * sizeof(int)) ||
        !take(flatM.data(), flatM.size() * sizeof(int))) {
        *err = "taxonomyDB truncated"; return false;
    }
    M.assign(N, std::vector<int>(K));
    for (size_t i = 0; i < N; i++)
        for (size_t k = 0; k < K; k++) M[i][k] = flatM[i * K + k];
    // StringBlock<unsigned int>: byteCapacity, entryCapacity, entryCount, bytes, offsets
    unsigned int byteCap = 0, entryCap = 0, entryCount = 0;
    if (!take(&byteCap, 4) || !take(&entryCap, 4) || !take(&entryCount, 4)) { *err = "taxonomyDB truncated"; return false; }
    std::vector<char> bytes(byteCap);
    std::vector<unsigned int> offs(entryCap);
    if (!take(bytes.data(), byteCap) || !take(offs.data(), (size_t)entryCap * 4)) { *err = "taxonomyDB truncated"; return false; }
    auto str = [&](size_t idx) -> std::string {  // StringBlock::getString: NULL past entryCount
        if (idx >= entryCount || offs[idx] >= byteCap) return "";
        return std::string(bytes.data() + offs[idx], strnlen(bytes.data() + offs[idx], byteCap - offs[idx]));
    };
    nodes.clear();
    for (size_t i = 0; i < maxNodes; i++)
        nodes.push_back({raw[i].id, raw[i].taxId, raw[i].parentTaxId, str(raw[i].rankIdx), str(raw[i].nameIdx)});
    maxTaxID = maxTax;
    D = d;
    eukaryotaTaxID = 0;  // setEukaryoteTaxID (TaxonomyWrapper.h:89-100): nodes with nameIdx 0 skipped
    for (size_t i = 0; i < maxNodes; i++)
        if (raw[i].nameIdx != 0 && nodes[i].name == "Eukaryota") { eukaryotaTaxID = nodes[i].taxId; break; }
    return true;
}

int Taxonomy::rmq(int i, int j) const {  // NcbiTaxonomy::RangeMinimumQuery
    int k = 0;
    while ((1 << (k + 1)) <= (j - i + 1)) k++;
    int A = M[i][k], B = M[j - (1 << k) + 1][k];
    return (L[A] <= L[B]) ? A : B;
}

int Taxonomy::lcaHelper(int i, int j) const {  // NcbiTaxonomy::lcaHelper
    if (i == 0 || j == 0) return 0;
    if (i == j) return i;
    int v1 = H[i], v2 = H[j];
    if (v1 > v2) std::swap(v1, v2);
    return E[rmq(v1, v2)];
}

TaxID Taxonomy::LCA(TaxID a, TaxID b) const {
    if (!nodeExists(a)) return b;
    if (!nodeExists(b)) return a;
    return nodes[lcaHelper(nodeId(a), nodeId(b))].taxId;
}

const TaxonNode* Taxonomy::LCA(const std::vector<TaxID>& v) const {
    auto it = v.begin();
    while (it != v.end() && !nodeExists(*it)) ++it;
    if (it == v.end()) return nullptr;
    int red = nodeId(*it++);
    for (; it != v.end(); ++it)
        if (nodeExists(*it)) red = lcaHelper(red, nodeId(*it));
    return &nodes[red];
}

bool Taxonomy::IsAncestor(TaxID ancestor, TaxID child) const {
    if (ancestor == child) return true;
    if (ancestor == 0 || child == 0) return false;
    if (!nodeExists(child) || !nodeExists(ancestor)) return false;
    return lcaHelper(nodeId(child), nodeId(ancestor)) == nodeId(ancestor);
}

int Taxonomy::findRankIndex(const std::string& rank) {
    // MMseqs2 NcbiRanks table, with "domain" as TaxonomyWrapper::findRankIndex2 maps it.
    static const std::map<std::string, int> ranks = {
        {"forma", 1}, {"varietas", 2}, {"subspecies", 3}, {"species", 4}, {"species subgroup", 5},
        {"species group", 6}, {"subgenus", 7}, {"genus", 8}, {"subtribe", 9}, {"tribe", 10},
        {"subfamily", 11}, {"family", 12}, {"superfamily", 13}, {"parvorder", 14}, {"infraorder", 15},
        {"suborder", 16}, {"order", 17}, {"superorder", 18}, {"infraclass", 19}, {"subclass", 20},
        {"class", 21}, {"superclass", 22}, {"subphylum", 23}, {"phylum", 24}, {"superphylum", 25},
        {"subkingdom", 26}, {"kingdom", 27}, {"superkingdom", 28}, {"domain", 28}};
    auto it = ranks.find(rank);
    return it == ranks.end() ? -1 : it->second;
}

TaxID Taxonomy::getTaxIdAtRank(int taxId, const std::string& rank) const {
    if (taxId == 0 || !nodeExists(taxId) || taxId == 1) return 0;
    int rankIndex = findRankIndex(rank);
    const TaxonNode* cur = taxonNode(taxId);
    int cnt = 0;
    while (cnt < 30 && findRankIndex(cur->rank) < rankIndex) {
        cur = taxonNode(cur->parentTaxId);
        cnt++;
    }
    if (cnt == 30) return taxId;
    return cur->taxId;
}

}  // namespace orc
