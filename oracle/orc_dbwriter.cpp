// ORACLE — test infrastructure only (see orc_core.h header).
// Reference DB writer restated from IndexCreator: extractTargetKmers (KmerExtractor.cpp:420-439),
// SORT_PARALLEL(compareTargetKmer) (IndexCreator.cpp:355-356, Kmer.h:77-87),
// filterKmers<DB_CREATION> (IndexCreator.h:475-617), areKmersDuplicate (:619-629),
// writeTargetFilesAndSplits / getDiffIdx (IndexCreator.cpp:811-886), writeDbParameters
// (:1245-1265). Used to make the synthetic fixture DBs of the parity tests.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <parallel/algorithm>

#include "orc_internal.h"

namespace orc {

struct TargetKmer {
    uint64_t value;
    TaxID taxId;
    TaxID speciesId;
};

static void getDiffIdx(uint64_t& lastKmer, uint64_t entry, std::vector<uint16_t>& out) {
    uint64_t kmerdiff = entry - lastKmer;
    uint16_t buffer[5];
    int idx = 3;
    buffer[4] = (uint16_t)(0x8000 | (kmerdiff & 0x7FFF));  // SET_END_FLAG(GET_15_BITS(diff))
    kmerdiff >>= 15U;
    while (kmerdiff) {
        buffer[idx] = (uint16_t)(kmerdiff & 0x7FFF);
        kmerdiff >>= 15U;
        idx--;
    }
    for (int i = idx + 1; i <= 4; i++) out.push_back(buffer[i]);
    lastKmer = entry;
}

// writeTargetFilesAndSplits (IndexCreator.cpp:811-865) over the unique (value, taxID) list: diffIdx,
// info and the AA-aligned split entries (MARKER = ~16777215, IndexCreator.cpp:31-37, AminoAcidPart
// IndexCreator.h:209-214)
static void writeTargetSplits(const uint64_t* values, const uint32_t* ids, size_t uniqKmerCnt, int splitNum, Db& db) {
    size_t sizeOfSplit = uniqKmerCnt / (size_t)(splitNum - 1);
    std::vector<size_t> offsetList(splitNum + 1);
    for (int os = 0; os < splitNum; os++) offsetList[os] = os * sizeOfSplit;
    offsetList[splitNum] = UINT64_MAX;
    db.split.assign(splitNum, DiffIdxSplit{0, 0, 0});
    int offsetListIdx = 1, splitListIdx = 1, splitCheck = 0;
    uint64_t AAofTempSplitOffset = UINT64_MAX, lastKmer = 0;
    const uint64_t AAMASK = ~(uint64_t)16777215;
    db.diffIdx.clear();
    db.info.clear();
    db.diffIdx.reserve(uniqKmerCnt * 3);
    db.info.reserve(uniqKmerCnt);
    for (size_t u = 0; u < uniqKmerCnt; u++) {
        db.info.push_back(ids[u]);
        getDiffIdx(lastKmer, values[u], db.diffIdx);
        if ((lastKmer & AAMASK) != AAofTempSplitOffset && splitCheck == 1) {
            db.split[splitListIdx++] = {lastKmer, (uint64_t)db.diffIdx.size(), (uint64_t)db.info.size()};
            splitCheck = 0;
        }
        if (db.info.size() == offsetList[offsetListIdx]) {
            AAofTempSplitOffset = lastKmer & AAMASK;
            splitCheck = 1;
            offsetListIdx++;
        }
    }
}

bool buildDb(const mtb_params& par, const Taxonomy& tax, const BuildInput& in, Db& db, std::string* err) {
    std::unique_ptr<Scanner> sc;
    if (par.kmer_format == 1) sc.reset(new OldMetamerScanner());
    else if (par.syncmer) sc.reset(new SyncmerScanner(par.smer_len));
    else sc.reset(new MetamerScanner());
    std::vector<TargetKmer> kmers;
    for (uint64_t b = 0; b < in.nBlocks; b++) {
        int g = in.blkGenome[b];
        TaxID taxId = in.genomeTaxId[g];
        TaxID sp = tax.getTaxIdAtRank(taxId, "species");
        const char* seq = in.seq + in.off[g];
        sc->init(seq, in.blkStart[b], in.blkEnd[b], in.blkStrand[b] > -1);
        for (ScanKmer k = sc->next(); k.value != UINT64_MAX; k = sc->next()) kmers.push_back({k.value, taxId, sp});
    }
    __gnu_parallel::sort(kmers.begin(), kmers.end(), [](const TargetKmer& a, const TargetKmer& b) {
        if (a.value != b.value) return a.value < b.value;
        if (a.speciesId != b.speciesId) return a.speciesId < b.speciesId;
        return a.taxId < b.taxId;
    });
    // filterKmers<DB_CREATION>: one entry per (value, species), taxID = LCA of the group.
    std::vector<size_t> uniq;
    std::vector<TaxID> taxIds;
    size_t n = kmers.size();
    size_t i = 0;
    while (i < n) {
        size_t j = i + 1;
        taxIds.clear();
        taxIds.push_back(kmers[i].taxId);
        while (j < n && kmers[j].speciesId == kmers[i].speciesId && kmers[j].value == kmers[i].value) {
            taxIds.push_back(kmers[j].taxId);
            j++;
        }
        kmers[i].taxId = tax.LCA(taxIds)->taxId;  // applied to every group, as the reference does
        uniq.push_back(i);
        i = j;
    }
    // writeTargetFilesAndSplits
    std::vector<uint64_t> uv(uniq.size());
    std::vector<uint32_t> ui(uniq.size());
    for (size_t u = 0; u < uniq.size(); u++) {
        uv[u] = kmers[uniq[u]].value;
        ui[u] = (uint32_t)kmers[uniq[u]].taxId;
    }
    writeTargetSplits(uv.data(), ui.data(), uniq.size(), in.splitNum, db);
    // taxID_list: the set of genome taxIDs (IndexCreator.cpp:329-333)
    std::vector<TaxID> ids(in.genomeTaxId, in.genomeTaxId + in.nGenomes);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    db.taxIdList = ids;
    (void)err;
    return true;
}

bool writeDbFiles(const Db& db, const mtb_params& par, const std::string& dir, std::string* err) {
    auto put = [&](const std::string& name, const void* p, size_t bytes) {
        FILE* f = fopen((dir + "/" + name).c_str(), "wb");
        if (!f) return false;
        bool ok = fwrite(p, 1, bytes, f) == bytes;
        fclose(f);
        return ok;
    };
    if (!put("diffIdx", db.diffIdx.data(), db.diffIdx.size() * 2) || !put("info", db.info.data(), db.info.size() * 4) ||
        !put("split", db.split.data(), db.split.size() * sizeof(DiffIdxSplit))) {
        *err = "cannot write DB files in " + dir;
        return false;
    }
    FILE* f = fopen((dir + "/taxID_list").c_str(), "w");
    if (!f) { *err = "cannot write taxID_list"; return false; }
    for (TaxID t : db.taxIdList) fprintf(f, "%d\n", t);
    fclose(f);
    f = fopen((dir + "/db.parameters").c_str(), "w");  // writeDbParameters
    if (!f) { *err = "cannot write db.parameters"; return false; }
    fprintf(f, "DB_name\t%s\n", "synthetic");
    fprintf(f, "Creation_date\t%s\n", "1970-01-01");
    fprintf(f, "Metabuli commit used to create the DB\t%s\n", "oracle");
    fprintf(f, "Reduced_alphabet\t%d\n", par.reduced_aa);
    fprintf(f, "Accession_level\t%d\n", par.accession_level);
    fprintf(f, "Mask_mode\t%d\n", 0);
    fprintf(f, "Mask_prob\t%f\n", 0.9);
    fprintf(f, "Skip_redundancy\t1\n");
    fprintf(f, "Syncmer\t%d\n", par.syncmer);
    if (par.syncmer == 1) fprintf(f, "Syncmer_len\t%d\n", par.smer_len);
    fprintf(f, "Kmer_format\t%d\n", par.kmer_format);
    fclose(f);
    return true;
}

}  // namespace orc

// Pin hook (test infrastructure: tests/test_ref_writer.py checks it against tests/golden/ref_writer.npz,
// which the reference's own writeTargetFilesAndSplits / getDiffIdx produced): the writer alone over a
// caller's sorted unique (value, taxID) list. diff_out holds at least 5 n words; *n_diff = words written.
extern "C" int orc_pin_write_db(const uint64_t* values, const uint32_t* ids, uint64_t n, int split_num,
                                uint16_t* diff_out, uint64_t* n_diff, uint32_t* info_out, uint64_t* split_out) {
    if (split_num < 2) return MTB_ERR_ARG;
    orc::Db db;
    orc::writeTargetSplits(values, ids, n, split_num, db);
    memcpy(diff_out, db.diffIdx.data(), db.diffIdx.size() * 2);
    *n_diff = db.diffIdx.size();
    memcpy(info_out, db.info.data(), db.info.size() * 4);
    for (int i = 0; i < split_num; i++) {
        split_out[3 * i] = db.split[i].ADkmer;
        split_out[3 * i + 1] = db.split[i].diffIdxOffset;
        split_out[3 * i + 2] = db.split[i].infoIdxOffset;
    }
    return MTB_OK;
}
