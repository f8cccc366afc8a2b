// Host side of the C-ABI library: classify parameters, DB file loading and taxonomy
// preprocessing. Replaces the state the reference builds in its constructors:
// Classifier::Classifier (Classifier.cpp:6-32), loadDbParameters (common.cpp:88-133),
// loadTaxonomy (common.cpp:50-86), KmerMatcher::loadTaxIdList (KmerMatcher.cpp:56-120), and the
// MMseqs2 NcbiTaxonomy services those use (LCA / IsAncestor / findRankIndex / loadMerged).
#include "mtb_host.h"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <unordered_map>

namespace mtb {

static thread_local std::string g_error;
void set_error(const std::string& msg) { g_error = msg; }

// Genetic code (GeneticCode.h:33-194) restated from the standard table over the reference's AA
// alphabet "ARNDCQEGHILKMFPSTWYVX" (stop = 20); base codes are nuc2int(atcg[c]) (common.cpp:13-17).
HostTables make_tables() {
    HostTables t;
    const char* row = ".AGCG..GT..G.CN...ACTG.A.T.......agcg..gt..g.cn...actg.a.t......";
    for (int i = 0; i < 256; i++) {
        unsigned char c = (i >= 64 && i < 128) ? (unsigned char)row[i - 64] : (unsigned char)'.';
        t.base[i] = (uint8_t)((c & 14u) >> 1u);
    }
    const char* bases = "TCAG";
    const char* aa64 = "FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG";
    const char* alphabet = "ARNDCQEGHILKMFPSTWYV";
    auto code = [](char b) { return b == 'A' ? 0 : b == 'C' ? 1 : b == 'T' ? 2 : 3; };
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 4; k++) {
                char a = aa64[i * 16 + j * 4 + k];
                int aa = a == '*' ? 20 : (int)(strchr(alphabet, a) - alphabet);
                int c1 = code(bases[i]), c2 = code(bases[j]), c3 = code(bases[k]);
                t.aa[c1 << 4 | c2 << 2 | c3] = (int8_t)aa;
                t.num[c1 << 4 | c2 << 2 | c3] = (int8_t)c3;
            }
    t.num[0 << 4 | 3 << 2 | 3] = 4;  // AGG
    t.num[0 << 4 | 3 << 2 | 0] = 5;  // AGA
    t.num[2 << 4 | 2 << 2 | 3] = 4;  // TTG
    t.num[2 << 4 | 2 << 2 | 0] = 5;  // TTA
    t.num[0 << 4 | 3 << 2 | 2] = 6;  // AGT
    t.num[0 << 4 | 3 << 2 | 1] = 7;  // AGC
    t.num[2 << 4 | 3 << 2 | 0] = 5;  // TGA
    return t;
}

int HostTaxonomy::rankIndex(const std::string& r) {
    // MMseqs2 NcbiRanks (findRankIndex) plus "domain" as TaxonomyWrapper::findRankIndex2 has it.
    static const std::map<std::string, int> ranks = {
        {"forma", 1}, {"varietas", 2}, {"subspecies", 3}, {"species", 4}, {"species subgroup", 5},
        {"species group", 6}, {"subgenus", 7}, {"genus", 8}, {"subtribe", 9}, {"tribe", 10},
        {"subfamily", 11}, {"family", 12}, {"superfamily", 13}, {"parvorder", 14}, {"infraorder", 15},
        {"suborder", 16}, {"order", 17}, {"superorder", 18}, {"infraclass", 19}, {"subclass", 20},
        {"class", 21}, {"superclass", 22}, {"subphylum", 23}, {"phylum", 24}, {"superphylum", 25},
        {"subkingdom", 26}, {"kingdom", 27}, {"superkingdom", 28}, {"domain", 28}};
    auto it = ranks.find(r);
    return it == ranks.end() ? -1 : it->second;
}

int HostTaxonomy::lcaNode(int i, int j) const {  // lcaHelper: node 0 short-circuits
    if (i == 0 || j == 0) return 0;
    while (i != j) {
        int di = depth[i], dj = depth[j];
        if (di >= dj) i = parent[i];
        if (dj >= di) j = parent[j];
    }
    return i;
}

int32_t HostTaxonomy::taxIdAtRank(int32_t taxId, const std::string& r) const {
    if (taxId == 0 || !exists(taxId) || taxId == 1) return 0;
    int target = rankIndex(r);
    int node = nodeOf[taxId];
    int cnt = 0;
    while (cnt < 30 && rankIndex(rank[node]) < target) {
        node = parent[node];
        cnt++;
    }
    if (cnt == 30) return taxId;
    return nodeTax[node];
}

bool build_taxonomy(const int32_t* taxid, const int32_t* par, uint64_t n, const std::vector<std::string>& ranks,
                    const std::vector<std::string>& names, const int32_t* mergedOld, const int32_t* mergedNew,
                    uint64_t nMerged, HostTaxonomy& T) {
    T = HostTaxonomy();
    if (n == 0) { set_error("empty taxonomy"); return false; }
    for (uint64_t i = 0; i < n; i++) {
        if (taxid[i] < 0) { set_error("negative taxID in nodes.dmp"); return false; }
        T.maxTax = std::max(T.maxTax, taxid[i]);
    }
    T.nodeOf.assign((size_t)T.maxTax + 1, -1);
    T.nodeTax.assign(taxid, taxid + n);
    T.rank = ranks;
    T.name = names;
    T.name.resize(n);
    for (uint64_t i = 0; i < n; i++) T.nodeOf[taxid[i]] = (int32_t)i;
    T.parent.assign(n, 0);
    for (uint64_t i = 0; i < n; i++) {
        if (!T.exists(par[i])) { set_error("inconsistent nodes.dmp: missing parent " + std::to_string(par[i])); return false; }
        T.parent[i] = T.nodeOf[par[i]];
    }
    for (uint64_t i = 0; i < nMerged; i++) {  // NcbiTaxonomy::loadMerged
        int32_t o = mergedOld[i], m = mergedNew[i];
        if (o >= 0 && o <= T.maxTax && !T.exists(o) && T.exists(m)) T.nodeOf[o] = T.nodeOf[m];
    }
    if (!T.exists(1)) { set_error("taxonomy has no root taxID 1"); return false; }
    const int root = T.nodeOf[1];
    T.parent[root] = root;
    T.depth.assign(n, -1);
    T.depth[root] = 0;
    std::vector<int> chain;
    for (uint64_t i = 0; i < n; i++) {
        int x = (int)i;
        chain.clear();
        while (T.depth[x] < 0) {
            chain.push_back(x);
            if (chain.size() > n) { set_error("taxonomy does not reach taxID 1 (cycle)"); return false; }
            x = T.parent[x];
        }
        int d = T.depth[x];
        for (size_t k = chain.size(); k-- > 0;) T.depth[chain[k]] = ++d;
    }
    T.eukaryota = 0;  // TaxonomyWrapper::setEukaryoteTaxID
    for (uint64_t i = 0; i < n; i++)
        if (T.name[i] == "Eukaryota") { T.eukaryota = taxid[i]; break; }
    T.flags.assign(n, 0);
    T.spParent.assign(n, 0);
    const int eukNode = T.exists(T.eukaryota) ? T.nodeOf[T.eukaryota] : -1;
    for (uint64_t i = 0; i < n; i++) {
        int32_t t = taxid[i];
        bool euk;  // NcbiTaxonomy::IsAncestor(eukaryota, t)
        if (T.eukaryota == t) euk = true;
        else if (T.eukaryota == 0 || t == 0) euk = false;
        else if (eukNode < 0) euk = false;
        else euk = T.lcaNode((int)i, eukNode) == eukNode;
        uint8_t f = euk ? 1 : 0;
        if (T.rank[i].empty() || T.rank[i] == "accession") f |= 2;
        T.flags[i] = f;
        int32_t s = T.taxIdAtRank(t, "species");
        T.spParent[i] = T.exists(s) ? T.nodeTax[T.parent[T.nodeOf[s]]] : 0;
    }
    return true;
}

static std::vector<std::string> split_field(const std::string& s, const std::string& delim, int maxCol) {
    std::vector<std::string> out;  // TaxonomyWrapper::splitByDelimiter semantics
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

bool load_dmp(const std::string& dir, HostTaxonomy& out) {
    std::ifstream nodes(dir + "/nodes.dmp");
    if (!nodes) { set_error("cannot open " + dir + "/nodes.dmp"); return false; }
    std::vector<int32_t> tax, par, mo, mn;
    std::vector<std::string> ranks;
    std::string line;
    while (std::getline(nodes, line)) {
        auto f = split_field(line, "\t|\t", 3);
        if (f.size() < 3) continue;
        tax.push_back((int32_t)strtol(f[0].c_str(), nullptr, 10));
        par.push_back((int32_t)strtol(f[1].c_str(), nullptr, 10));
        ranks.push_back(f[2]);
    }
    std::unordered_map<int32_t, size_t> row;
    for (size_t i = 0; i < tax.size(); i++) row[tax[i]] = i;
    std::vector<std::string> names(tax.size());
    std::ifstream nm(dir + "/names.dmp");
    while (nm && std::getline(nm, line)) {
        if (line.find("scientific name") == std::string::npos) continue;
        auto f = split_field(line, "\t|\t", 2);
        auto it = row.find((int32_t)strtol(f[0].c_str(), nullptr, 10));
        if (it == row.end()) { set_error("names.dmp taxon not present in nodes.dmp"); return false; }
        names[it->second] = f.size() > 1 ? f[1] : "";
    }
    std::ifstream mg(dir + "/merged.dmp");
    while (mg && std::getline(mg, line)) {
        auto f = split_field(line, "\t|\t", 2);
        if (f.size() != 2) { set_error("invalid merged.dmp entry"); return false; }
        mo.push_back((int32_t)strtoul(f[0].c_str(), nullptr, 10));
        mn.push_back((int32_t)strtoul(f[1].c_str(), nullptr, 10));
    }
    return build_taxonomy(tax.data(), par.data(), tax.size(), ranks, names, mo.data(), mn.data(), mo.size(), out);
}

bool build_species_map(HostDb& db) {
    // KmerMatcher::loadTaxIdList, non-contamination branch (KmerMatcher.cpp:92-117).
    const HostTaxonomy& T = db.tax;
    db.speciesOf.assign((size_t)T.maxTax + 1, 0);
    for (int32_t taxId : db.taxIdList) {
        if (!T.exists(taxId)) { set_error("taxID_list entry " + std::to_string(taxId) + " not in taxonomy"); return false; }
        int32_t sp = T.taxIdAtRank(taxId, "species");
        int node = T.nodeOf[taxId];
        if (taxId != T.nodeTax[node]) db.speciesOf[taxId] = sp;
        int guard = 0;
        while (T.nodeTax[node] != sp) {
            db.speciesOf[T.nodeTax[node]] = sp;
            node = T.parent[node];
            if (++guard > 4096) { set_error("taxID_list entry without a species ancestor"); return false; }
        }
        if (sp >= 0 && sp <= T.maxTax) db.speciesOf[sp] = sp;
    }
    return true;
}

template <typename T>
static bool read_file(const std::string& path, std::vector<T>& out) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize((size_t)sz / sizeof(T));
    size_t got = out.empty() ? 0 : fread(out.data(), sizeof(T), out.size(), f);
    fclose(f);
    return got == out.size();
}

bool load_db_files(const std::string& dir, HostDb& db) {
    if (!read_file(dir + "/diffIdx", db.diffIdx) || !read_file(dir + "/info", db.info)) {
        set_error("cannot read " + dir + "/diffIdx or /info");
        return false;
    }
    read_file(dir + "/split", db.split);
    std::ifstream tl(dir + "/taxID_list");
    if (!tl) { set_error("cannot read " + dir + "/taxID_list"); return false; }
    std::string line;
    while (std::getline(tl, line))
        if (!line.empty()) db.taxIdList.push_back((int32_t)std::stoul(line));
    // taxonomyDB (MMseqs2 serialization) is not supported: loadTaxonomy's dmp fallback only.
    if (!load_dmp(dir + "/taxonomy", db.tax)) return false;
    return build_species_map(db);
}

bool check_db(const HostDb& db) {
    // validateDatabase.cpp:78-131: terminal 0x8000 fragments == info entries.
    uint64_t terms = 0;
    for (uint16_t w : db.diffIdx) terms += (w & 0x8000u) ? 1 : 0;
    if (terms != db.info.size()) {
        set_error("diffIdx k-mer count " + std::to_string(terms) + " != info entries " + std::to_string(db.info.size()));
        return false;
    }
    if (!db.diffIdx.empty() && !(db.diffIdx.back() & 0x8000u)) { set_error("diffIdx ends mid k-mer"); return false; }
    return true;
}

}  // namespace mtb

using namespace mtb;

extern "C" {

void mtb_default_params(mtb_params* p) {  // setClassifyDefaults (classify.cpp:10-37)
    memset(p, 0, sizeof(*p));
    p->seq_mode = 2;
    p->kmer_format = 1;
    p->syncmer = 0;
    p->smer_len = 5;
    p->reduced_aa = 0;
    p->skip_redundancy = 0;
    p->min_score = 0.0f;
    p->min_sp_score = 0.0f;
    p->min_cons_cnt = 4;
    p->min_cons_cnt_euk = 9;
    p->tie_ratio = 0.95f;
    p->accession_level = 0;
    p->em = 0;
    p->threads = 1;
    p->mask_mode = 0;
}

int mtb_load_db_parameters(const char* dir, mtb_params* par) {  // loadDbParameters (common.cpp:88-133)
    std::ifstream f(std::string(dir) + "/db.parameters");
    if (!f) return 0;
    std::string line;
    while (std::getline(f, line)) {
        size_t tab = line.find('\t');
        std::string k = line.substr(0, tab), v = tab == std::string::npos ? "" : line.substr(tab + 1);
        if (k == "Reduced_alphabet") par->reduced_aa = atoi(v.c_str());
        else if (k == "Accession_level") {
            if (v == "0" && par->accession_level == 1) par->accession_level = 0;
            if (v == "1" && par->accession_level == 0) par->accession_level = 2;
        } else if (k == "Skip_redundancy") {
            if (v == "1") par->skip_redundancy = 1;
        } else if (k == "Syncmer") {
            if (v == "1" && par->syncmer == 0) par->syncmer = 1;
        } else if (k == "S-mer_len") {  // the writer emits "Syncmer_len", which this key misses
            par->smer_len = atoi(v.c_str());
        } else if (k == "Kmer_format") {
            par->kmer_format = atoi(v.c_str());
        }
    }
    return 1;
}

const char* mtb_last_error(void) { return g_error.c_str(); }

// Restated tables, for the CPU test that pins them against tests/golden/genetic_code.json.
void mtb_debug_tables(uint8_t* base256, int8_t* aa64, int8_t* num64) {
    HostTables t = make_tables();
    memcpy(base256, t.base, 256);
    memcpy(aa64, t.aa, 64);
    memcpy(num64, t.num, 64);
}

}  // extern "C"
