// ORACLE — test infrastructure only (see orc_core.h header).
// extern "C" surface of the oracle for ctypes (tests/, smoke(), bench.py cpu_baseline only).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "orc_internal.h"
#ifdef _OPENMP
#include <omp.h>
#endif

using namespace orc;

static void setErr(char* err, int len, const std::string& msg) {
    if (err && len > 0) { strncpy(err, msg.c_str(), (size_t)len - 1); err[len - 1] = 0; }
}

template <typename T>
static bool readFile(const std::string& path, std::vector<T>& out) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) return false;
    std::streamsize sz = f.tellg();
    f.seekg(0);
    out.resize((size_t)sz / sizeof(T));
    return (bool)f.read(reinterpret_cast<char*>(out.data()), (std::streamsize)(out.size() * sizeof(T)));
}

extern "C" {

// loadDbParameters (common.cpp:88-133) — "S-mer_len" is read, the writer's "Syncmer_len" is not.
int orc_load_db_parameters(const char* dir, mtb_params* par) {
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
        } else if (k == "Skip_redundancy") { if (v == "1") par->skip_redundancy = 1; }
        else if (k == "Syncmer") { if (v == "1" && par->syncmer == 0) par->syncmer = 1; }
        else if (k == "S-mer_len") par->smer_len = atoi(v.c_str());
        else if (k == "Kmer_format") par->kmer_format = atoi(v.c_str());
    }
    return 1;
}

void* orc_db_open(const char* dir, char* err, int errlen) {
    Db* db = new Db();
    std::string d(dir), e;
    std::vector<uint64_t> split;
    if (!readFile(d + "/diffIdx", db->diffIdx) || !readFile(d + "/info", db->info) || !readFile(d + "/split", split)) {
        setErr(err, errlen, "cannot read diffIdx/info/split in " + d);
        delete db;
        return nullptr;
    }
    for (size_t i = 0; i + 2 < split.size(); i += 3) db->split.push_back({split[i], split[i + 1], split[i + 2]});
    std::ifstream tl(d + "/taxID_list");
    std::string line;
    while (std::getline(tl, line)) if (!line.empty()) db->taxIdList.push_back((TaxID)std::stoul(line));
    // loadTaxonomy (common.cpp:50-86): the taxonomyDB binary when present and current, else the dmp
    // files under taxonomy/
    bool haveTax = false;
    if (std::ifstream(d + "/taxonomyDB").good()) {
        haveTax = db->tax.loadTaxonomyDb(d + "/taxonomyDB", &e);
        if (!haveTax && !e.empty()) {
            setErr(err, errlen, e);
            delete db;
            return nullptr;
        }
    }
    if ((!haveTax && !db->tax.loadDmp(d + "/taxonomy", &e)) || !db->buildSpeciesMap(&e)) {
        setErr(err, errlen, e);
        delete db;
        return nullptr;
    }
    return db;
}

void* orc_db_open_host(const mtb_db_host* h, char* err, int errlen) {
    Db* db = new Db();
    std::string e;
    db->diffIdx.assign(h->diff_idx, h->diff_idx + h->n_diff_idx);
    db->info.assign(h->info, h->info + h->n_info);
    for (uint64_t i = 0; i < h->n_split; i++) db->split.push_back({h->split[3 * i], h->split[3 * i + 1], h->split[3 * i + 2]});
    db->taxIdList.assign(h->taxid_list, h->taxid_list + h->n_taxid_list);
    std::vector<std::string> ranks(h->n_nodes), names(h->n_nodes);
    for (uint64_t i = 0; i < h->n_nodes; i++) {
        ranks[i] = std::string(h->rank_pool + h->rank_off[i]);
        if (h->name_pool) names[i] = std::string(h->name_pool + h->name_off[i]);
    }
    if (!db->tax.fromArrays(h->node_taxid, h->node_parent, h->n_nodes, ranks, names, h->merged_old, h->merged_new,
                            h->n_merged, &e) ||
        !db->buildSpeciesMap(&e)) {
        setErr(err, errlen, e);
        delete db;
        return nullptr;
    }
    return db;
}

// A DB whose diffIdx / info / split the caller fills in place (bench: the GTDB-scale DB lives on the
// GPU and is encoded straight into these buffers, no second host copy). Taxonomy + taxID_list from h.
void* orc_db_new(const mtb_db_host* h, uint64_t n_diff, uint64_t n_info, uint64_t n_split, void** diff, void** info,
                 void** split, char* err, int errlen) {
    mtb_db_host t = *h;
    t.diff_idx = nullptr, t.n_diff_idx = 0, t.info = nullptr, t.n_info = 0, t.split = nullptr, t.n_split = 0;
    Db* db = static_cast<Db*>(orc_db_open_host(&t, err, errlen));
    if (!db) return nullptr;
    db->diffIdx.resize(n_diff);
    db->info.resize(n_info);
    db->split.resize(n_split);
    *diff = db->diffIdx.data();
    *info = db->info.data();
    *split = db->split.data();
    return db;
}

void orc_db_close(void* db) { delete static_cast<Db*>(db); }

uint64_t orc_db_kmers(void* db) { return static_cast<Db*>(db)->info.size(); }

// Synthetic reference DB: writes diffIdx, info, split, taxID_list, db.parameters into out_dir
// (the taxonomy/ directory must already hold the dmp files given in tax_dir).
int orc_db_build(const char* out_dir, const char* tax_dir, const mtb_params* par, const char* seq, const uint64_t* off,
                 uint32_t n_genomes, const int32_t* genome_taxid, const int32_t* blk_genome, const int32_t* blk_start,
                 const int32_t* blk_end, const int32_t* blk_strand, uint64_t n_blocks, int split_num, char* err,
                 int errlen) {
    Taxonomy tax;
    std::string e;
    if (!tax.loadDmp(tax_dir, &e)) { setErr(err, errlen, e); return MTB_ERR_IO; }
    BuildInput in{seq, off, n_genomes, genome_taxid, blk_genome, blk_start, blk_end, blk_strand, n_blocks, split_num};
    Db db;
    if (!buildDb(*par, tax, in, db, &e) || !writeDbFiles(db, *par, out_dir, &e)) { setErr(err, errlen, e); return MTB_ERR_IO; }
    return MTB_OK;
}

// Query extraction (+ optional compareQueryKmer sort). Returns every reserved slot, blanks included.
int orc_extract(const mtb_params* par, const char* seq1, const uint64_t* off1, const char* seq2, const uint64_t* off2,
                uint32_t n, int sort, mtb_kmer* out, uint64_t cap, uint64_t* n_out, uint32_t* qlen1, uint32_t* qlen2) {
    Reads r{seq1, off1, seq2, off2, n};
    std::vector<mtb_kmer> buf;
    std::vector<Query> q;
    extractQueryKmers(*par, r, buf, q, sort != 0);
    *n_out = buf.size();
    for (uint32_t i = 0; i < n; i++) {
        if (qlen1) qlen1[i] = (uint32_t)q[i].queryLength;
        if (qlen2) qlen2[i] = (uint32_t)q[i].queryLength2;
    }
    if (buf.size() > cap) return MTB_RETRY;
    memcpy(out, buf.data(), buf.size() * sizeof(mtb_kmer));
    return MTB_OK;
}

// SeqIterator::maskLowComplexityRegions over a batch of reads (test entry point): masked bases and,
// if probs is non-NULL, tantan's per-letter repeat probabilities.
void orc_tantan(const char* seq, const uint64_t* off, uint32_t n, float mask_prob, char* out, float* probs) {
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        const int len = (int)(off[i + 1] - off[i]);
        maskLowComplexityRegions(seq + off[i], len, mask_prob, out + off[i]);
        if (probs) {
            std::vector<unsigned char> x(len);
            for (int k = 0; k < len; k++) {
                const char c = seq[off[i] + k];
                x[k] = (c == 'A' || c == 'a') ? 0 : (c == 'C' || c == 'c') ? 1 : (c == 'G' || c == 'g') ? 2
                     : (c == 'T' || c == 't' || c == 'U' || c == 'u') ? 3 : 4;
            }
            tantanRepeatProbs(x.data(), len, probs + off[i]);
        }
    }
}

int orc_match(void* dbp, const mtb_params* par, const mtb_kmer* kmers, uint64_t n, mtb_match* out, uint64_t cap,
              uint64_t* n_out, char* err, int errlen) {
    std::vector<mtb_match> m;
    std::string e;
    if (!matchKmers(*static_cast<Db*>(dbp), *par, kmers, n, m, &e)) { setErr(err, errlen, e); return MTB_ERR_DB; }
    *n_out = m.size();
    if (m.size() > cap) return MTB_RETRY;
    memcpy(out, m.data(), m.size() * sizeof(mtb_match));
    return MTB_OK;
}

void orc_sort_matches(mtb_match* m, uint64_t n) {
    std::vector<mtb_match> v(m, m + n);
    sortMatches(v);
    memcpy(m, v.data(), n * sizeof(mtb_match));
}

// --em: the last assignment's mappings (Reporter::writeMappings, Reporter.h:80-92), batch read indices
static std::vector<mtb_em_map> g_lastMaps;

static int exportResults(const std::vector<Query>& q, mtb_result* out, mtb_taxcnt* tc, uint64_t cap, uint64_t* n_tc) {
    g_lastMaps.clear();
    for (size_t i = 0; i < q.size(); i++)
        if (q[i].isClassified)
            for (auto& sp : q[i].species2Score) g_lastMaps.push_back(mtb_em_map{(uint32_t)i, sp.first, sp.second});
    uint64_t w = 0;
    bool overflow = false;
    for (size_t i = 0; i < q.size(); i++) {
        mtb_result& r = out[i];
        memset(&r, 0, sizeof(r));
        r.classification = q[i].classification;
        r.score = q[i].score;
        r.hamming_dist = q[i].hammingDist;
        r.query_length = (uint32_t)(q[i].queryLength + q[i].queryLength2);
        r.is_classified = q[i].isClassified ? 1 : 0;
        r.taxcnt_offset = (uint32_t)w;
        r.taxcnt_len = (uint32_t)q[i].taxCnt.size();
        for (auto& kv : q[i].taxCnt) {
            if (w < cap) tc[w] = {kv.first, (uint32_t)kv.second}; else overflow = true;
            w++;
        }
    }
    *n_tc = w;
    return overflow ? MTB_RETRY : MTB_OK;
}

int orc_assign(void* dbp, const mtb_params* par, const mtb_match* m, uint64_t n, const uint32_t* ql1,
               const uint32_t* ql2, uint32_t n_reads, mtb_result* out, mtb_taxcnt* tc, uint64_t cap, uint64_t* n_tc) {
    std::vector<Query> q(n_reads);
    for (uint32_t i = 0; i < n_reads; i++) { q[i].queryLength = (int)ql1[i]; q[i].queryLength2 = ql2 ? (int)ql2[i] : 0; }
    assignTaxonomy(*static_cast<Db*>(dbp), *par, m, n, q);
    return exportResults(q, out, tc, cap, n_tc);
}

// Whole path for one QuerySplit (Classifier.cpp:81-124). stage_s: extract+sort, search,
// match sort, analysis (the reference's own phase prints). counts: query k-mers, matches.
int orc_classify(void* dbp, const mtb_params* par, const char* seq1, const uint64_t* off1, const char* seq2,
                 const uint64_t* off2, uint32_t n, mtb_result* out, mtb_taxcnt* tc, uint64_t cap, uint64_t* n_tc,
                 double* stage_s, uint64_t* counts, char* err, int errlen) {
    using clk = std::chrono::steady_clock;
    Db& db = *static_cast<Db*>(dbp);
    Reads r{seq1, off1, seq2, off2, n};
    std::vector<mtb_kmer> buf;
    std::vector<Query> q;
    auto t0 = clk::now();
    extractQueryKmers(*par, r, buf, q, true);
    auto t1 = clk::now();
    std::vector<mtb_match> m;
    std::string e;
    if (!matchKmers(db, *par, buf.data(), buf.size(), m, &e)) { setErr(err, errlen, e); return MTB_ERR_DB; }
    auto t2 = clk::now();
    sortMatches(m);
    auto t3 = clk::now();
    assignTaxonomy(db, *par, m.data(), m.size(), q);
    auto t4 = clk::now();
    if (stage_s) {
        stage_s[0] = std::chrono::duration<double>(t1 - t0).count();
        stage_s[1] = std::chrono::duration<double>(t2 - t1).count();
        stage_s[2] = std::chrono::duration<double>(t3 - t2).count();
        stage_s[3] = std::chrono::duration<double>(t4 - t3).count();
    }
    if (counts) {
        uint64_t blank = 0;
        while (blank < buf.size() && infoSeq(buf[blank].info) == 0) blank++;
        counts[0] = buf.size() - blank;
        counts[1] = m.size();
    }
    return exportResults(q, out, tc, cap, n_tc);
}

// The last orc_classify / orc_assign's mappings (read indices of that batch).
int orc_last_em_maps(mtb_em_map* out, uint64_t cap, uint64_t* n) {
    *n = g_lastMaps.size();
    if (g_lastMaps.size() > cap) return MTB_RETRY;
    if (!g_lastMaps.empty()) memcpy(out, g_lastMaps.data(), g_lastMaps.size() * sizeof(mtb_em_map));
    return MTB_OK;
}

// Classifier::em + reclassify: reads_out (total_reads), the top species' final abundance and
// emTaxCounts (ascending taxID; cap entries), stats[0] = queryCount, stats[1] = iterations.
int orc_em(void* dbp, const mtb_em_map* maps, uint64_t n, uint64_t total_reads, mtb_em_read* reads_out,
           int32_t* sp_ids, double* sp_probs, uint32_t* sp_counts, uint64_t cap, uint64_t* n_sp, uint64_t* stats) {
    EmOut o;
    emReassign(*static_cast<Db*>(dbp), maps, n, total_reads, o);
    memcpy(reads_out, o.reads.data(), total_reads * sizeof(mtb_em_read));
    *n_sp = o.probs.size();
    stats[0] = o.queryCount;
    stats[1] = o.iterations;
    if (o.probs.size() > cap) return MTB_RETRY;
    uint64_t w = 0;
    for (auto& kv : o.probs) {
        sp_ids[w] = kv.first;
        sp_probs[w] = kv.second;
        sp_counts[w] = o.emTaxCounts[kv.first];
        w++;
    }
    return MTB_OK;
}

int orc_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_threads(int t) {
#ifdef _OPENMP
    omp_set_num_threads(t);
#else
    (void)t;
#endif
}

// Table dump used to pin the restated genetic code against the reference's GeneticCode.h.
void orc_genetic_tables(int32_t* nuc2aa512, int32_t* nuc2num512, uint8_t* atcg256, uint8_t* irct256) {
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++)
            for (int k = 0; k < 8; k++) {
                nuc2aa512[i * 64 + j * 8 + k] = kCode.nuc2aa[i][j][k];
                nuc2num512[i * 64 + j * 8 + k] = kCode.nuc2num[i][j][k];
            }
    memcpy(atcg256, kChars.atcg, 256);
    memcpy(irct256, kChars.iRCT, 256);
}

// The restated Hamming tables (orc_core.h: kHammingLookup, codonField) as the reference lays its
// own out (KmerMatcher.h:66-158): lookup64[q * 8 + t]; lut512[k * 64 + (q << 3 | t)] = field k's
// 2-bit value shifted to its place, as HAMMING_LUTk holds it.
void orc_hamming_tables(uint8_t* lookup64, uint16_t* lut512) {
    for (int q = 0; q < 8; q++)
        for (int t = 0; t < 8; t++) {
            lookup64[q * 8 + t] = kHammingLookup[q][t];
            for (int k = 0; k < 8; k++) lut512[k * 64 + (q << 3 | t)] = (uint16_t)(codonField(q, t, k) << (2 * k));
        }
}

// getHammingDistanceSum / getHammings / getHammings_reverse (KmerMatcher.h:348-416) as restated.
void orc_hamming(const uint64_t* a, const uint64_t* b, uint64_t n, uint8_t* sum, uint16_t* fwd, uint16_t* rev) {
    for (uint64_t i = 0; i < n; i++) {
        sum[i] = hammingSum(a[i], b[i]);
        fwd[i] = hammings(a[i], b[i]);
        rev[i] = hammingsReverse(a[i], b[i]);
    }
}

}  // extern "C"
