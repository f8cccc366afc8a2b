// ORACLE — test infrastructure only (see orc_core.h header).
//
// Restatement of Reporter::writeReportFile / writeReport (src/commons/Reporter.cpp:175-190,
// :217-244) and of the MMseqs2 NcbiTaxonomy services they call, getParentToChildren and
// getCladeCounts (un-vendored lib/mmseqs; restated from MMseqs2's published NcbiTaxonomy.cpp —
// parity unpinned, no reference fixture exercises the report). The Krona chart
// (Reporter::kronaReport) needs MMseqs2's krona_prelude_html and is not restated.
#include <algorithm>
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#include "orc_internal.h"

namespace orc {

// NcbiTaxonomy::getParentToChildren: every node but the root (its own parent) under its parent,
// in nodes.dmp order.
static std::unordered_map<TaxID, std::vector<TaxID>> parentToChildren(const Taxonomy& t) {
    std::unordered_map<TaxID, std::vector<TaxID>> out;
    for (const TaxonNode& n : t.nodes)
        if (n.parentTaxId != n.taxId) out[n.parentTaxId].push_back(n.taxId);
    return out;
}

// NcbiTaxonomy::getCladeCounts: a taxon's reads count for itself and for each ancestor.
static std::unordered_map<TaxID, TaxonCounts> cladeCounts(const Taxonomy& t,
                                                          const std::unordered_map<TaxID, unsigned>& taxCnt,
                                                          const std::unordered_map<TaxID, std::vector<TaxID>>& p2c) {
    std::unordered_map<TaxID, TaxonCounts> cc;
    for (const auto& kv : taxCnt) {
        cc[kv.first].taxCount = kv.second;
        cc[kv.first].cladeCount += kv.second;
        if (!t.nodeExists(kv.first)) continue;
        const TaxonNode* n = &t.nodes[t.D[kv.first]];
        while (n->parentTaxId != n->taxId && t.nodeExists(n->parentTaxId)) {
            n = &t.nodes[t.D[n->parentTaxId]];
            cc[n->taxId].cladeCount += kv.second;
        }
    }
    for (auto& kv : cc) {
        auto it = p2c.find(kv.first);
        if (it != p2c.end()) kv.second.children = it->second;
    }
    return cc;
}

static unsigned cladeOf(const std::unordered_map<TaxID, TaxonCounts>& cc, TaxID t) {
    auto it = cc.find(t);
    return it == cc.end() ? 0 : it->second.cladeCount;
}

// Reporter::writeReport: unclassified first, then depth-first from the root; children by clade
// count, descending (SORT_SERIAL = std::sort), stopping at the first child without counts.
static void writeReport(FILE* fp, const Taxonomy& t, const std::unordered_map<TaxID, TaxonCounts>& cc,
                        unsigned long total, TaxID taxId, int depth) {
    auto it = cc.find(taxId);
    const unsigned clade = it == cc.end() ? 0 : it->second.cladeCount;
    const unsigned taxc = it == cc.end() ? 0 : it->second.taxCount;
    if (taxId == 0) {
        if (clade > 0)
            fprintf(fp, "%.4f\t%i\t%i\tno rank\t0\tunclassified\n", 100 * clade / double(total), clade, taxc);
        writeReport(fp, t, cc, total, 1, 0);
        return;
    }
    if (clade == 0) return;
    const TaxonNode& n = t.nodes[t.D[taxId]];
    fprintf(fp, "%.4f\t%i\t%i\t%s\t%i\t%s%s\n", 100 * clade / double(total), clade, taxc, n.rank.c_str(),
            t.getOriginalTaxID(taxId),
            std::string(2 * depth, ' ').c_str(), n.name.c_str());
    std::vector<TaxID> ch = it->second.children;
    std::sort(ch.begin(), ch.end(), [&](TaxID a, TaxID b) { return cladeOf(cc, a) > cladeOf(cc, b); });
    for (TaxID c : ch) {
        if (!cc.count(c)) break;
        writeReport(fp, t, cc, total, c, depth + 1);
    }
}

}  // namespace orc

using namespace orc;

extern "C" int orc_write_report(void* dbp, const char* path, int numOfQuery, const int32_t* ids, const uint32_t* cnt,
                                uint64_t n) {
    const Db* db = static_cast<const Db*>(dbp);
    std::unordered_map<TaxID, unsigned> taxCnt;
    for (uint64_t i = 0; i < n; i++) taxCnt[ids[i]] += cnt[i];
    const auto p2c = parentToChildren(db->tax);
    const auto cc = cladeCounts(db->tax, taxCnt, p2c);
    FILE* fp = fopen(path, "w");
    if (!fp) return -1;
    fprintf(fp, "#clade_proportion\tclade_count\ttaxon_count\trank\ttaxID\tname\n");
    writeReport(fp, db->tax, cc, (unsigned long)numOfQuery, 0, 0);
    return fclose(fp) == 0 ? 0 : -1;
}
