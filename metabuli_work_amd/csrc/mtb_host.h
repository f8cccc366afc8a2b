// Host-side state of a context: DB files read into memory and the taxonomy flattened into the
// arrays the device kernels read.
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/mtb_gpu.h"
#include "mtb_launch.h"

namespace mtb {

struct HostTaxonomy {
    int32_t maxTax = 0;
    int32_t eukaryota = 0;
    std::vector<int32_t> nodeOf;    // taxID -> node (D array of NcbiTaxonomy, merged IDs folded in)
    std::vector<int32_t> nodeTax;   // node -> taxID
    std::vector<int32_t> parent;    // node -> parent node
    std::vector<int32_t> depth;     // node -> depth below taxID 1
    std::vector<uint8_t> flags;     // bit0 under Eukaryota, bit1 rank "" or "accession"
    std::vector<int32_t> spParent;  // node -> parentTaxId of its species node (minSpScore branch)
    std::vector<std::string> rank;
    std::vector<std::string> name;
    std::vector<int32_t> internal2org;  // taxonomyDB with internal taxIDs; empty = IDs are original

    bool exists(int32_t t) const { return t >= 0 && t <= maxTax && nodeOf[t] >= 0; }
    // TaxonomyWrapper::getOriginalTaxID (TaxonomyWrapper.h:70-79)
    int32_t original(int32_t t) const {
        return internal2org.empty() || t < 0 || (size_t)t >= internal2org.size() ? t : internal2org[t];
    }
    int lcaNode(int i, int j) const;
    int32_t taxIdAtRank(int32_t taxId, const std::string& rank) const;  // TaxonomyWrapper.cpp:479-498
    static int rankIndex(const std::string& rank);
};

struct HostDb {
    std::vector<uint16_t> diffIdx;
    std::vector<uint32_t> info;
    // diffIdx / info as the open reads them: views of the vectors above or of the caller's arrays
    // (mtb_open_host), or, with the file names set, read straight into device memory (mtb_open:
    // the host never holds them)
    const uint16_t* diffP = nullptr;
    const uint32_t* infoP = nullptr;
    uint64_t nDiff = 0, nInfo = 0;
    std::string diffFile, infoFile;
    void use_vectors() {
        diffP = diffIdx.data();
        nDiff = diffIdx.size();
        infoP = info.data();
        nInfo = info.size();
    }
    std::vector<uint64_t> split;  // 3 words per DiffIdxSplit
    std::vector<int32_t> taxIdList;
    HostTaxonomy tax;
    std::vector<int32_t> speciesOf;  // dense taxId2speciesId (KmerMatcher::loadTaxIdList)
};

// The TSV writer's text per taxID, built once per context (mtb_tax_text): taxID t in [0, n) has
// its original ID's decimal digits at buf[idOff[t], idOff[t + 1]) and its rank name at
// buf[rankOff[t], rankOff[t + 1]) ("-" for an absent taxID, as mtb_taxon_rank).
struct TaxText {
    uint32_t n = 0;
    std::vector<uint32_t> idOff, rankOff;
    std::string buf;
};
const TaxText& tax_text(const mtb_ctx* c);
// Device bytes a context's grow-only batch buffers hold now (reused by its next batches).
uint64_t ctx_workspace_bytes(const mtb_ctx* c);
// Frees those buffers (a context holding more than its share of a device shared with others).
void ctx_release_workspace(mtb_ctx* c);
// Host-side state the file pipeline keeps in a context between runs (its pinned batch slots),
// destroyed with the context on its device.
std::shared_ptr<void>& ctx_pipeline_cache(mtb_ctx* c);
const mtb_params& ctx_params(const mtb_ctx* c);
// A batch this much smaller than the run's full batches (the ramp of mtb_start_classify): workspace
// growth steps allocate the full batch's size at once (clamped to [1, 32]; 1 = as needed)
void ctx_set_grow(mtb_ctx* c, double scale);
// After an MTB_MATCH_ONLY batch: the per-read match offsets (host copy, n_reads + 1) and device
// views of the matches (grouped by read), per-read counts and query lengths (range-partitioned run)
int ctx_match_view(mtb_ctx* c, std::vector<uint64_t>& mOff, const mtb_match** m, const uint32_t** counts,
                   const uint32_t** qlen);

void set_error(const std::string& msg);
HostTables make_tables();

bool build_taxonomy(const int32_t* taxid, const int32_t* parent, uint64_t n, const std::vector<std::string>& ranks,
                    const std::vector<std::string>& names, const int32_t* mergedOld, const int32_t* mergedNew,
                    uint64_t nMerged, HostTaxonomy& out);
bool load_dmp(const std::string& dir, HostTaxonomy& out);
constexpr int32_t kTaxonomyDbVersion = 2;  // NcbiTaxonomy::SERIALIZATION_VERSION (MMseqs2, unpinned)
int load_taxonomy_db(const std::string& path, HostTaxonomy& out);
bool build_species_map(HostDb& db);
// stream: diffIdx / info are left in their files (read_to_device at open) instead of host vectors
bool load_db_files(const std::string& dir, HostDb& db, bool stream = false);
// `bytes` of a file into device memory: parallel reads into pinned staging buffers, each uploaded
// as soon as it is full (the file read and the PCIe upload overlap); false + set_error on failure
// Pinned staging buffers and streams of the uploads below, reused across calls (the current device's)
struct StageLanes {
    static constexpr unsigned kLanes = 8;
    static constexpr uint64_t kChunk = 32ull << 20;
    struct Lane {
        hipStream_t st = nullptr;
        char* buf[2] = {nullptr, nullptr};
        hipEvent_t done[2] = {nullptr, nullptr};
    };
    int dev = 0;
    bool ok = true;
    Lane lane[kLanes];
    explicit StageLanes(int device);
    ~StageLanes();
    StageLanes(const StageLanes&) = delete;
    StageLanes& operator=(const StageLanes&) = delete;
};
bool read_to_device(const std::string& path, void* dst, uint64_t bytes, uint64_t fileOff = 0,
                    StageLanes* lanes = nullptr);
// the same from host memory (pageable: copied into the pinned buffers by the threads)
bool upload_to_device(const void* src, void* dst, uint64_t bytes, StageLanes* lanes = nullptr);
bool check_db(const HostDb& db);
bool partition_bounds(const uint64_t* split, uint64_t nSplit, uint64_t D, int parts, std::vector<uint64_t>& start,
                      std::vector<uint64_t>& entry);
bool slice_db_part(HostDb& db, int part, int parts);

}  // namespace mtb
