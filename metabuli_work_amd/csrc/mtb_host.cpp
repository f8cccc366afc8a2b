// Host side of the C-ABI library: classify parameters, DB file loading and taxonomy
// preprocessing. Replaces the state the reference builds in its constructors:
// Classifier::Classifier (Classifier.cpp:6-32), loadDbParameters (common.cpp:88-133),
// loadTaxonomy (common.cpp:50-86), KmerMatcher::loadTaxIdList (KmerMatcher.cpp:56-120), and the
// MMseqs2 NcbiTaxonomy services those use (LCA / IsAncestor / findRankIndex / loadMerged).
#include "mtb_host.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <functional>
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

// TaxonomyWrapper::unserialize (TaxonomyWrapper.cpp:363-421) over a taxonomyDB file: version,
// [size_t 1 = internal taxIDs], size_t maxNodes, int maxTaxID, MMseqs2 TaxonNode[maxNodes]
// {int id, taxId, parentTaxId; size_t rankIdx, nameIdx}, int D[maxTaxID + 1], [internal2orgTaxId],
// E, L (2 maxNodes ints), H (maxNodes), the sparse table M, StringBlock<unsigned int>. The Euler
// tour / sparse table are skipped: the device LCA is built from the parent links. The TaxonNode and
// StringBlock layouts are MMseqs2's (submodule absent: unpinned). Returns 0 = loaded, 1 = other
// serialization version (the reference falls back to the dmp files, common.cpp:71-85), -1 = error.
int load_taxonomy_db(const std::string& path, HostTaxonomy& out) {
    std::vector<char> mem;
    if (!read_file(path, mem)) { set_error("cannot read " + path); return -1; }
    const char* p = mem.data();
    const char* end = p + mem.size();
    auto take = [&](void* dst, size_t bytes) {
        if ((size_t)(end - p) < bytes) return false;
        if (dst) memcpy(dst, p, bytes);
        p += bytes;
        return true;
    };
    const std::string bad = path + ": truncated or malformed taxonomyDB";
    int32_t version = 0;
    if (!take(&version, 4)) { set_error(bad); return -1; }
    if (version != kTaxonomyDbVersion) return 1;
    uint64_t internalUsed = 0;
    if ((size_t)(end - p) < 8) { set_error(bad); return -1; }
    memcpy(&internalUsed, p, 8);  // read as size_t; only 1 means internal IDs (TaxonomyWrapper.cpp:372-381)
    const bool internal = internalUsed == 1;
    if (internal) p += 8;
    uint64_t maxNodes = 0;
    int32_t maxTax = 0;
    if (!take(&maxNodes, 8) || !take(&maxTax, 4) || maxTax < 0 || maxNodes == 0 ||
        maxNodes > (uint64_t)(end - p) / 32) { set_error(bad); return -1; }
    struct RawNode { int32_t id, taxId, parentTaxId; uint64_t rankIdx, nameIdx; };
    static_assert(sizeof(RawNode) == 32, "MMseqs2 TaxonNode layout");
    std::vector<RawNode> raw(maxNodes);
    std::vector<int32_t> D((size_t)maxTax + 1), i2o;
    if (!take(raw.data(), maxNodes * 32) || !take(D.data(), D.size() * 4)) { set_error(bad); return -1; }
    if (internal) {
        i2o.resize((size_t)maxTax + 1);
        if (!take(i2o.data(), i2o.size() * 4)) { set_error(bad); return -1; }
    }
    const uint64_t N = 2 * maxNodes;
    uint64_t K = 0;  // (int)flog2(N) + 1 sparse-table columns
    while ((2ull << K) <= N) K++;
    K += 1;
    if (!take(nullptr, (2 * N + maxNodes + N * K) * 4)) { set_error(bad); return -1; }  // E, L, H, M
    uint32_t byteCap = 0, entryCap = 0, entryCount = 0;
    if (!take(&byteCap, 4) || !take(&entryCap, 4) || !take(&entryCount, 4)) { set_error(bad); return -1; }
    const char* bytes = p;
    if (!take(nullptr, byteCap)) { set_error(bad); return -1; }
    std::vector<uint32_t> offs(entryCap);
    if (!take(offs.data(), (size_t)entryCap * 4)) { set_error(bad); return -1; }
    auto str = [&](uint64_t idx) -> std::string {  // StringBlock::getString (NULL past entryCount)
        if (idx >= entryCount || offs[idx] >= byteCap) return std::string();
        return std::string(bytes + offs[idx], strnlen(bytes + offs[idx], byteCap - offs[idx]));
    };
    std::vector<int32_t> tax(maxNodes), par(maxNodes), mo, mn;
    std::vector<std::string> ranks(maxNodes), names(maxNodes);
    for (uint64_t i = 0; i < maxNodes; i++) {
        tax[i] = raw[i].taxId;
        par[i] = raw[i].parentTaxId;
        ranks[i] = str(raw[i].rankIdx);
        names[i] = raw[i].nameIdx == 0 ? std::string() : str(raw[i].nameIdx);  // setEukaryoteTaxID skips index 0
        if (tax[i] < 0 || tax[i] > maxTax) { set_error(bad); return -1; }
    }
    for (int32_t t = 0; t <= maxTax; t++) {  // D entries of IDs that are not a node's own: merged IDs
        const int32_t d = D[t];
        if (d < 0) continue;
        if ((uint64_t)d >= maxNodes) { set_error(bad); return -1; }
        if (tax[d] != t) { mo.push_back(t); mn.push_back(tax[d]); }
    }
    if (!build_taxonomy(tax.data(), par.data(), maxNodes, ranks, names, mo.data(), mn.data(), mo.size(), out))
        return -1;
    // internal IDs unused by any node still map (getOriginalTaxID indexes the full table)
    if (out.maxTax < maxTax) out.nodeOf.resize((size_t)maxTax + 1, -1), out.maxTax = maxTax;
    out.internal2org = i2o;
    return 0;
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

bool load_db_files(const std::string& dir, HostDb& db, bool stream) {
    if (stream) {
        struct stat a, b;
        if (stat((dir + "/diffIdx").c_str(), &a) != 0 || stat((dir + "/info").c_str(), &b) != 0) {
            set_error("cannot read " + dir + "/diffIdx or /info");
            return false;
        }
        db.diffFile = dir + "/diffIdx";
        db.infoFile = dir + "/info";
        db.nDiff = (uint64_t)a.st_size / sizeof(uint16_t);
        db.nInfo = (uint64_t)b.st_size / sizeof(uint32_t);
    } else if (!read_file(dir + "/diffIdx", db.diffIdx) || !read_file(dir + "/info", db.info)) {
        set_error("cannot read " + dir + "/diffIdx or /info");
        return false;
    } else {
        db.use_vectors();
    }
    read_file(dir + "/split", db.split);
    std::ifstream tl(dir + "/taxID_list");
    if (!tl) { set_error("cannot read " + dir + "/taxID_list"); return false; }
    std::string line;
    while (std::getline(tl, line))
        if (!line.empty()) db.taxIdList.push_back((int32_t)std::stoul(line));
    // loadTaxonomy (common.cpp:50-86): the taxonomyDB binary when present and of the current
    // serialization version, else taxonomy/{nodes,names,merged}.dmp (original taxIDs)
    int rc = 1;
    if (std::ifstream(dir + "/taxonomyDB").good()) rc = load_taxonomy_db(dir + "/taxonomyDB", db.tax);
    if (rc < 0) return false;
    if (rc == 1 && !load_dmp(dir + "/taxonomy", db.tax)) return false;
    return build_species_map(db);
}

bool check_db(const HostDb& db) {
    // validateDatabase.cpp:78-131: terminal 0x8000 fragments == info entries (a streamed DB is
    // checked on the device, before its decode writes by k-mer index: decode_diff_idx)
    if (!db.diffP) {
        if (db.nDiff == 0 && db.nInfo > 0) { set_error("diffIdx is empty but info is not"); return false; }
        return true;
    }
    // the k-mer count and the last word are checked by the decode itself (decode_db_chunked), chunk
    // by chunk on the device, instead of a serial host pass over ~30G words at GTDB scale
    if (db.nDiff && !(db.diffP[db.nDiff - 1] & 0x8000u)) { set_error("diffIdx ends mid k-mer"); return false; }
    return true;
}

// `bytes` into device memory through pinned staging buffers: up to 8 threads, each filling one of
// its two 32-MB buffers (fill(buf, at, len): bytes [at, at + len) of the source) while the other
// uploads. what names the source in the error message.
StageLanes::StageLanes(int device) : dev(device) {
    hipSetDevice(dev);
    for (Lane& l : lane) {
        bool good = hipStreamCreateWithFlags(&l.st, hipStreamNonBlocking) == hipSuccess;
        for (int k = 0; k < 2 && good; k++)
            good = hipHostMalloc((void**)&l.buf[k], kChunk, hipHostMallocDefault) == hipSuccess &&
                   hipEventCreateWithFlags(&l.done[k], hipEventDisableTiming) == hipSuccess;
        ok = ok && good;
    }
}

StageLanes::~StageLanes() {
    hipSetDevice(dev);
    for (Lane& l : lane) {
        if (l.st) hipStreamSynchronize(l.st);
        for (int k = 0; k < 2; k++) {
            if (l.buf[k]) hipHostFree(l.buf[k]);
            if (l.done[k]) hipEventDestroy(l.done[k]);
        }
        if (l.st) hipStreamDestroy(l.st);
    }
}

// `bytes` into device memory through pinned staging buffers: up to kLanes threads, each filling one
// of its two 32-MB buffers (fill(buf, at, len): bytes [at, at + len) of the source) while the other
// uploads. what names the source in the error message. lanes: buffers and streams reused across
// calls (an open's chunked decode makes ~50 of them; each call pinning its own 16 buffers was most
// of the GTDB-scale open's upload time), or none (made for this call).
static bool stage_to_device(const std::function<bool(char*, uint64_t, uint64_t)>& fill, void* dst, uint64_t bytes,
                            const std::string& what, StageLanes* lanes) {
    int dev = 0;
    hipGetDevice(&dev);
    std::unique_ptr<StageLanes> own;
    if (!lanes || lanes->dev != dev) {
        own.reset(new StageLanes(dev));
        lanes = own.get();
    }
    if (!lanes->ok) { set_error("cannot pin staging buffers for " + what); return false; }
    constexpr uint64_t kChunk = StageLanes::kChunk;
    const unsigned nThreads = (unsigned)std::min<uint64_t>(StageLanes::kLanes, (bytes + kChunk - 1) / kChunk);
    std::atomic<uint64_t> next{0};
    std::atomic<bool> ok{true};
    auto work = [&](unsigned t) {
        hipSetDevice(dev);
        StageLanes::Lane& l = lanes->lane[t];
        bool good = true;
        for (int k = 0; good && ok;) {  // alternate two buffers: read one while the other uploads
            const uint64_t at = next.fetch_add(kChunk);
            if (at >= bytes) break;
            const uint64_t len = std::min(kChunk, bytes - at);
            if (hipEventSynchronize(l.done[k]) != hipSuccess) { good = false; break; }
            good = fill(l.buf[k], at, len);
            good = good && hipMemcpyAsync((char*)dst + at, l.buf[k], len, hipMemcpyHostToDevice, l.st) == hipSuccess &&
                   hipEventRecord(l.done[k], l.st) == hipSuccess;
            k ^= 1;
        }
        good = hipStreamSynchronize(l.st) == hipSuccess && good;
        if (!good) ok = false;
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nThreads; t++) th.emplace_back(work, t);
    if (nThreads) work(0);
    for (auto& t : th) t.join();
    if (!ok) set_error("cannot read or upload " + what);
    return ok;
}

bool read_to_device(const std::string& path, void* dst, uint64_t bytes, uint64_t fileOff, StageLanes* lanes) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) { set_error("cannot read " + path); return false; }
    const bool ok = stage_to_device(
        [&](char* buf, uint64_t at, uint64_t len) {
            for (uint64_t got = 0; got < len;) {
                const ssize_t r = pread(fd, buf + got, len - got, (off_t)(fileOff + at + got));
                if (r <= 0) return false;
                got += (uint64_t)r;
            }
            return true;
        },
        dst, bytes, path, lanes);
    close(fd);
    return ok;
}

bool upload_to_device(const void* src, void* dst, uint64_t bytes, StageLanes* lanes) {
    return stage_to_device(
        [&](char* buf, uint64_t at, uint64_t len) {
            std::memcpy(buf, (const char*)src + at, len);
            return true;
        },
        dst, bytes, "host arrays", lanes);
}

// ---- range partition of the DB at split entries -------------------------
// Split entry j (j >= 1) is written right after the first k-mer of a new AA group past each
// (D / (splitNum-1)) mark: {value of that k-mer, diffIdx offset of the NEXT k-mer, its info index
// + 1} (IndexCreator.cpp:843-851). The reader starts a thread at value ADkmer, info index
// infoIdxOffset - 1 and diffIdx offset diffIdxOffset (KmerMatcher.cpp:255-271). Entry 0 is
// {0, 0, 0} (decode from the start); unused entries stay 0 (KmerMatcher.cpp:134-141).
bool partition_bounds(const uint64_t* split, uint64_t nSplit, uint64_t D, int parts, std::vector<uint64_t>& start,
                      std::vector<uint64_t>& entry) {
    if (parts < 1 || D == 0) { set_error("partition: need >= 1 part and a non-empty DB"); return false; }
    std::vector<std::pair<uint64_t, uint64_t>> usable;  // (first k-mer index, split entry)
    for (uint64_t j = 1; j < nSplit; j++) {
        const uint64_t* e = split + 3 * j;
        if (e[0] == 0 || e[0] == UINT64_MAX || e[2] == 0 || e[2] > D) continue;
        if (!usable.empty() && e[2] - 1 <= usable.back().first) continue;
        usable.emplace_back(e[2] - 1, j);
    }
    start.assign(1, 0);
    entry.assign(1, 0);
    size_t u = 0;
    for (int p = 1; p < parts; p++) {
        const double target = (double)D * p / parts;
        size_t best = SIZE_MAX;
        for (; u < usable.size(); u++) {  // first usable boundary at or past the target, or the one just before
            if ((double)usable[u].first >= target) break;
        }
        for (size_t cand : {u ? u - 1 : SIZE_MAX, u}) {
            if (cand >= usable.size() || usable[cand].first <= start.back()) continue;
            if (usable.size() - cand < (size_t)(parts - p)) continue;  // leave one boundary per later part
            if (best == SIZE_MAX ||
                std::abs((double)usable[cand].first - target) < std::abs((double)usable[best].first - target))
                best = cand;
        }
        if (best == SIZE_MAX) {
            set_error("partition: the split table has too few AA-aligned entries for " + std::to_string(parts) +
                      " parts");
            return false;
        }
        start.push_back(usable[best].first);
        entry.push_back(usable[best].second);
        u = best + 1;
    }
    start.push_back(D);
    return true;
}

// Keep part `part` of `parts`: k-mers [s_p, s_{p+1}) plus, for every part but the last, the first
// k-mer of the next part, which is the part's last resident k-mer and so never a candidate (the
// reference reader stops before the DB's last k-mer, KmerMatcher.cpp:363,378; the next part's AA
// run holds it instead). diffIdx of the part = the varint of its first value (a delta from 0, as
// IndexCreator's getDiffIdx writes it, IndexCreator.cpp:811-835) + the file's words from the split's
// diffIdxOffset up to the next boundary's, so the device decode runs unchanged.
bool slice_db_part(HostDb& db, int part, int parts) {
    if (parts <= 1) return true;
    if (part < 0 || part >= parts) { set_error("db_part out of range"); return false; }
    if (db.split.size() < 6) { set_error("partitioned DB needs the split file"); return false; }
    if (db.diffIdx.size() != db.nDiff) { set_error("internal: a partitioned open needs the host diffIdx"); return false; }
    const uint64_t D = db.info.size(), nSplit = db.split.size() / 3;
    std::vector<uint64_t> start, entry;
    if (!partition_bounds(db.split.data(), nSplit, D, parts, start, entry)) return false;
    const uint64_t s0 = start[part], s1 = start[part + 1];
    const bool last = part == parts - 1;
    const uint64_t* e0 = db.split.data() + 3 * entry[part];
    const uint64_t dBeg = part == 0 ? 0 : e0[1];
    const uint64_t dEnd = last ? db.diffIdx.size() : db.split[3 * entry[part + 1] + 1];
    std::vector<uint16_t> diff;
    if (part > 0) {  // getDiffIdx(lastKmer = 0, ADkmer)
        uint64_t v = e0[0];
        uint16_t buf[5];
        int idx = 3;
        buf[4] = (uint16_t)(0x8000u | (v & 0x7FFF));
        v >>= 15;
        while (v) {
            buf[idx--] = (uint16_t)(v & 0x7FFF);
            v >>= 15;
        }
        for (int i = idx + 1; i <= 4; i++) diff.push_back(buf[i]);
    }
    diff.insert(diff.end(), db.diffIdx.begin() + dBeg, db.diffIdx.begin() + dEnd);
    const uint64_t iEnd = last ? D : s1 + 1;
    std::vector<uint32_t> info(db.info.begin() + s0, db.info.begin() + iEnd);
    db.diffIdx.swap(diff);
    db.info.swap(info);
    db.use_vectors();
    return check_db(db);  // terminal words == info entries
}

}  // namespace mtb

namespace mtb {

// tantan's parameters as SeqIterator::maskLowComplexityRegions passes them (SeqIterator.cpp:160-172)
// and the nucleotide likelihood ratios exp(lambda * score): +2 match, -3 mismatch over ACGT, -1
// against N, lambda of that scoring at uniform base frequencies (MMseqs2's NucleotideMatrix /
// ProbabilityMatrix are not in the mount: an assumption).
TantanTables make_tantan_tables(float maskProb) {
    TantanTables t{};
    const double repeatProb = 0.005, repeatEndProb = 0.05, decay = 0.9;
    double lo = 0.1, hi = 2.0;  // 0.25 e^{2 lambda} + 0.75 e^{-3 lambda} = 1
    for (int it = 0; it < 200; it++) {
        const double mid = 0.5 * (lo + hi);
        if (0.25 * std::exp(2 * mid) + 0.75 * std::exp(-3 * mid) > 1.0) hi = mid; else lo = mid;
    }
    const double lambda = 0.5 * (lo + hi);
    for (int a = 0; a < 5; a++)
        for (int b = 0; b < 5; b++) {
            const int sc = (a == 4 || b == 4) ? -1 : (a == b ? 2 : -3);
            t.lr[5 * a + b] = std::exp(lambda * sc);
        }
    double p = repeatProb * (1 - decay) / (1 - std::pow(decay, kTantanOffsets));  // firstRepeatOffsetProb
    for (int i = 0; i < kTantanOffsets; i++) {
        t.b2f[i] = p;
        p *= decay;
    }
    t.b2b = 1 - repeatProb;
    t.f2b = repeatEndProb;
    t.f2f = 1 - repeatEndProb;
    t.minMask = (double)maskProb;
    return t;
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
    p->mask_prob = 0.9f;
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

int mtb_partition_bounds(const uint64_t* split, uint64_t n_split, uint64_t n_kmers, int n_parts, uint64_t* kmer_start,
                         uint64_t* split_index) {
    if (!split || !kmer_start) { set_error("null argument"); return MTB_ERR_ARG; }
    std::vector<uint64_t> start, entry;
    if (!partition_bounds(split, n_split, n_kmers, n_parts, start, entry)) return MTB_ERR_DB;
    for (int p = 0; p <= n_parts; p++) kmer_start[p] = start[p];
    if (split_index)
        for (int p = 0; p < n_parts; p++) split_index[p] = entry[p];
    return MTB_OK;
}

// Restated tables, for the CPU test that pins them against tests/golden/genetic_code.json.
void mtb_debug_tables(uint8_t* base256, int8_t* aa64, int8_t* num64) {
    HostTables t = make_tables();
    memcpy(base256, t.base, 256);
    memcpy(aa64, t.aa, 64);
    memcpy(num64, t.num, 64);
}

}  // extern "C"
