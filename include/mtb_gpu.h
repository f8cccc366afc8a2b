/*
 * mtb_gpu.h — C-ABI drop-in boundary for the MI355X-native Metabuli `classify` hot path.
 *
 * The reference has no FFI layer: its seam is four C++ member calls made by one host thread in
 * Classifier::startClassify (/root/reference/src/commons/Classifier.cpp:105-118):
 *
 *   KmerExtractor::extractQueryKmers  (KmerExtractor.h:77-83, KmerExtractor.cpp:52-81)
 *   KmerMatcher::matchKmers           (KmerMatcher.h:228-230, KmerMatcher.cpp:123-481)
 *   KmerMatcher::sortMatches          (KmerMatcher.h:244,     KmerMatcher.cpp:1071-1078)
 *   Classifier::assignTaxonomy        (Classifier.h:77-80,    Classifier.cpp:166-208)
 *
 * plus the state those calls read, built in the Classifier/KmerMatcher constructors
 * (Classifier.cpp:6-32, KmerMatcher.cpp:19-37,56-120, common.cpp:50-133).
 *
 * Every entry point here is plain C: pointers, sizes and POD structs, no C++ or torch types.
 * Status codes: 0 = ok, 1 = capacity retry (caller enlarges its buffer and calls again),
 * negative = fatal (the reference calls exit(1) in the same situations).
 * One mtb_ctx per device; a context is not thread-safe.
 */
#ifndef MTB_GPU_H
#define MTB_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTB_OK 0
#define MTB_RETRY 1
#define MTB_ERR_ARG (-1)
#define MTB_ERR_IO (-2)
#define MTB_ERR_HIP (-3)
#define MTB_ERR_DB (-4)        /* DB inconsistent with taxonomy: KmerMatcher.cpp:292-300 exits */
#define MTB_ERR_OOM (-5)
#define MTB_ERR_UNSUPPORTED (-6)
#define MTB_ERR_INTERNAL (-7)  /* a device-side consistency check failed */

/* Flags for mtb_classify_batch. */
#define MTB_INPUT_DEVICE 1u    /* seq/off pointers are device (HBM) pointers */
#define MTB_KEEP_STAGES 2u     /* keep sorted query k-mers and sorted matches for mtb_get_* */
#define MTB_MATCH_ONLY 4u      /* stop after the join: per-read match segments for mtb_copy_matches
                                  (range-partitioned DB); no results of its own */

/*
 * Parameters of the path. Mirrors the LocalParameters fields the path reads
 * (LocalParameters.h:165-190,222) with the classify workflow defaults (classify.cpp:10-37);
 * DB-driven overrides are applied by mtb_load_db_parameters (common.cpp:88-133).
 */
typedef struct mtb_params {
    int32_t seq_mode;         /* 1 single-end, 2 paired-end, 3 long reads       (--seq-mode)   */
    int32_t kmer_format;      /* 1 = base-21 AA, right-to-left; 2 = 5-bit AA    (Kmer_format)  */
    int32_t syncmer;          /* closed syncmer selection on/off                (Syncmer)      */
    int32_t smer_len;         /* s-mer length (default 5; DB key "S-mer_len")                  */
    int32_t reduced_aa;       /* must be 0: ReducedKmerMatcher is out of scope                 */
    int32_t skip_redundancy;  /* DB "Skip_redundancy": 0 => info & 0x7FFFFFFF                  */
    float min_score;          /* --min-score                                                   */
    float min_sp_score;       /* --min-sp-score                                                */
    int32_t min_cons_cnt;     /* --min-cons-cnt (4)                                            */
    int32_t min_cons_cnt_euk; /* --min-cons-cnt-euk (9)                                        */
    float tie_ratio;          /* --tie-ratio (0.95)                                            */
    int32_t accession_level;  /* 0, 1, or 2 (2 = DB has accessions but not requested)          */
    int32_t em;               /* --em: classified reads keep their best species (no lower-rank
                                 BFS, Taxonomer.cpp:193-201) and record EM mappings (mtb_em)    */
    int32_t threads;          /* host threads (oracle / host parsing only)                     */
    int32_t mask_mode;        /* --mask-residues 1: tantan low-complexity masking of the reads
                                 before extraction (KmerExtractor.cpp:328-335). PARITY UNPINNED:
                                 tantan and its scoring matrices are MMseqs2's, absent from the
                                 reference tree; restated from the published algorithm with
                                 +2/-3/-1 scores at uniform background            */
    int32_t db_part;          /* range-partitioned DB: this context holds part db_part of      */
    int32_t db_parts;         /* db_parts AA-aligned k-mer ranges (0 or 1 = the whole DB)      */
    float mask_prob;          /* --mask-prob (0.9): tantan's minMaskProb                       */
} mtb_params;

/* Query k-mer: 16 B, same layout as Kmer{uint64 value; QueryKmerInfo} (Kmer.h:11-31,45-46).
 * info bits: [0,32) pos, [32,61) seqID (1-based within the batch), [61,64) frame (0-2 fwd, 3-5 rev). */
typedef struct mtb_kmer {
    uint64_t value;
    uint64_t info;
} mtb_kmer;

/* Match: 24 B packed form of Match (Match.h:9-25; the reference's has a vptr and is 32 B). */
typedef struct mtb_match {
    uint64_t qinfo;             /* QueryKmerInfo bits, as mtb_kmer.info   */
    uint32_t target_id;         /* info[] & mask (taxID, internal)        */
    uint32_t species_id;        /* taxId2speciesId[target_id]             */
    uint32_t dna_encoding;      /* target value & 0xFFFFFF                */
    uint16_t right_end_hamming; /* 2 bits per codon                       */
    uint8_t hamming;            /* Hamming-distance sum                   */
    uint8_t pad;
} mtb_match;

/* Per-read classification result (the Query fields written by Taxonomer::chooseBestTaxon,
 * Taxonomer.cpp:130-202, and printed by Reporter::writeReadClassification, Reporter.cpp:38-83). */
typedef struct mtb_result {
    int32_t classification;   /* internal taxID; 0 = unclassified                            */
    float score;
    int32_t hamming_dist;
    uint32_t query_length;    /* queryLength + queryLength2 (getMaxCoveredLength of each mate) */
    uint32_t taxcnt_offset;   /* into the pooled mtb_taxcnt array of the batch               */
    uint32_t taxcnt_len;      /* entries, ascending taxID (std::map order)                   */
    uint8_t is_classified;
    uint8_t pad[7];
} mtb_result;                 /* 32 B */

typedef struct mtb_taxcnt {
    int32_t tax_id;
    uint32_t count;
} mtb_taxcnt;

typedef struct mtb_ctx mtb_ctx;

/* DB arrays held in host memory (the on-disk files of Appendix B, already read). */
typedef struct mtb_db_host {
    const uint16_t* diff_idx;   uint64_t n_diff_idx;   /* diffIdx  */
    const uint32_t* info;       uint64_t n_info;       /* info     */
    const uint64_t* split;      uint64_t n_split;      /* split: n_split DiffIdxSplit {ADkmer, diffIdxOffset, infoIdxOffset} */
    const int32_t* taxid_list;  uint64_t n_taxid_list; /* taxID_list */
    /* Taxonomy as nodes.dmp rows in file order (node index = row). rank/name are NUL-separated
     * string pools indexed by the offsets. merged.dmp pairs optional. */
    const int32_t* node_taxid;  const int32_t* node_parent; uint64_t n_nodes;
    const char* rank_pool;      const uint64_t* rank_off;
    const char* name_pool;      const uint64_t* name_off;   /* scientific names; may be NULL */
    const int32_t* merged_old;  const int32_t* merged_new;  uint64_t n_merged;
} mtb_db_host;

/* A decoded reference DB already resident in HBM (a DB built in place on the device, e.g. the
 * GTDB-scale synthetic DB of the bench, SURVEY §8(d) config 3, which is never written out).
 * records: a device array of n_kmers + 8 records of three uint32 {value low 32 bits, value high
 * 32 bits, taxID}, sorted by value: the diffIdx decoded (getNextTargetKmer, KmerMatcher.h:282-297)
 * next to its info entry. With rank_form = 1 and kmer_format 2 the AA part of each value is
 * already the base-21 rank of the 8 AA codes (the resident form). The context uses
 * the records in place (pads written, taxIDs masked, format-2 values converted to rank form) and
 * does not free them: they must outlive the context. */
typedef struct mtb_db_resident {
    void* records;
    uint64_t n_kmers;
    int32_t rank_form;
    int32_t reserved;
} mtb_db_resident;

/* ---- parameters ---------------------------------------------------------------------------- */
void mtb_default_params(mtb_params* par);                              /* classify.cpp:10-37   */
int mtb_load_db_parameters(const char* db_dir, mtb_params* par);       /* common.cpp:88-133    */

/* ---- context / DB residency ------------------------------------------------------------------ */
/* Replaces Classifier::Classifier + KmerMatcher::KmerMatcher/loadTaxIdList + loadTaxonomy
 * (Classifier.cpp:6-32, KmerMatcher.cpp:19-37,56-120, common.cpp:50-86): reads diffIdx, info,
 * split, taxID_list and taxonomy/{nodes,names,merged}.dmp and makes them resident in HBM. */
int mtb_open(const char* db_dir, const mtb_params* par, int device, mtb_ctx** out);
int mtb_open_host(const mtb_db_host* db, const mtb_params* par, int device, mtb_ctx** out);
/* Context over a resident DB; `taxonomy` supplies the taxonomy and taxID_list only (its diffIdx,
 * info and split pointers are not read). */
int mtb_open_resident(const mtb_db_resident* db, const mtb_db_host* taxonomy, const mtb_params* par, int device,
                      mtb_ctx** out);
void mtb_close(mtb_ctx* ctx);
const char* mtb_last_error(void);
int mtb_set_stream(mtb_ctx* ctx, void* hip_stream);   /* hipStream_t; NULL = library stream */
uint64_t mtb_db_kmers(const mtb_ctx* ctx);             /* number of reference k-mers          */
/* Device bytes the context's batch workspace holds now (grow-only buffers, reused by the next
 * batch), and a cap on them (0 = none; MTB_WORKSPACE_CAP=<bytes>[K|M|G] sets it at open): a batch
 * whose workspace would pass the cap, or the device's free memory, returns MTB_RETRY from
 * mtb_classify_batch with the workspace given back — the caller classifies it in smaller pieces,
 * as the reference re-searches a split after its match buffer ran out (Classifier.cpp:127-130,
 * KmerMatcher.cpp:474-476); mtb_start_classify* halve such a batch down to one read. */
uint64_t mtb_workspace_bytes(const mtb_ctx* ctx);
/* Seconds the context's open took, by phase: [0] reading and uploading diffIdx / info (files or
 * mtb_open_host's arrays, through pinned staging, chunk by chunk), [1] K3 decode of diffIdx into the
 * resident records, [2] AA-prefix directory, [3] probe lines, [4] run index, [5] taxonomy and species
 * map upload, [6] the whole open, [7] the records' allocation (part of [1]). */
int mtb_open_phases(const mtb_ctx* ctx, double* sec, int n);
int mtb_set_workspace_cap(mtb_ctx* ctx, uint64_t bytes);
/* Gives the context's batch workspace back to the device (the next batch regrows it), e.g. when a
 * server switches a context to another workload or frees HBM for another context; returns once
 * the memory can be allocated again (the runtime's release of tens of GB is paid here, not by the
 * next allocation of whatever runs next). */
int mtb_release_workspace(mtb_ctx* ctx);
int mtb_ctx_device(const mtb_ctx* ctx);                /* the HIP device the context runs on  */

/* ---- the hot path ------------------------------------------------------------------------- */
/* One QuerySplit worth of reads (Classifier.cpp:81-133): extract (K1) + sort (K2) + match
 * (K3/K4) + match sort (K5) + assign (K6). seq/off: concatenated bases of mate 1 and n_reads+1
 * byte offsets; seq2/off2 the same for mate 2 (NULL unless seq_mode == 2). With
 * MTB_INPUT_DEVICE the four pointers are device pointers. results: host array of n_reads, or
 * NULL to leave them on the device (mtb_device_results). */
int mtb_classify_batch(mtb_ctx* ctx, const char* seq, const uint64_t* off, const char* seq2,
                       const uint64_t* off2, uint32_t n_reads, uint32_t flags, mtb_result* results);
/* Pooled taxID:count lists of the last batch (ascending taxID per read). */
int mtb_get_taxcnt(mtb_ctx* ctx, mtb_taxcnt* out, uint64_t capacity, uint64_t* n_out);
/* Device pointers of the last batch's results (mtb_result[n_reads]) and pooled taxcnt. */
int mtb_device_results(mtb_ctx* ctx, void** results, void** taxcnt, uint64_t* n_taxcnt);
/* Counters the reference prints (Classifier.cpp:116, KmerMatcher.cpp:152): query_kmers = the
 * batch's non-blank query k-mers ("Query k-mer number": every window the scanners emitted, before
 * any test against the DB), matches = the matches found. */
int mtb_last_counts(const mtb_ctx* ctx, uint64_t* query_kmers, uint64_t* matches);
/* Work counts of the last batch: [0] reserved k-mer slots, [1] query k-mers, [2] query k-mers
 * with >= 1 match, [3] matches, [4] most matches of one read, [5] (read, species, frame) groups,
 * [6] groups of >= 2 matches, [7] (read, species) runs, [8] runs combined one per wave, [9] of those,
 * runs whose tied paths needed the std::sort emulation, [10] join path (1 sort-merge join, the
 * default; 0 probe join, MTB_JOIN=probe), [11] matches K6 read (live: their species has a frame
 * run of >= 2 matches; = [3] with MTB_KEEP_STAGES), [12] query k-mers whose DB run the unstaged
 * join found by a gallop over the DB (the run index covers probe lines of < 64K DB k-mers; queries
 * on longer lines fall back), [13] matches the direct join spilled past their read's stretch,
 * [14] query k-mers whose DB run held more than 48 k-mers (scanned a wave each, k_match_long),
 * [15] fused-filter reruns (the batch's present windows outgrew the output sized from earlier batches),
 * [16] DB records the DB-sweep join read (MTB_JOIN=sweep: the tiles that held queries; 0 otherwise),
 * [17] / [18] with MTB_DUP_STATS=1 (diagnostic pass after the sort): query k-mers whose AA rank /
 * whole value repeats an earlier query's in their 256-query K4 block (the reference's same-AA /
 * identical-query reuse, KmerMatcher.cpp:277-353; 0 otherwise), [19] K1 units per read when the
 * batch took uniform units (12 paired, 6 single-end: every frame one chunk, MTB_UNIFORM_UNITS; 0 otherwise).
 * Query k-mers = windows whose AA 8-mer the DB holds. Counts [5]..[9] are over the live matches. */
int mtb_last_stats(const mtb_ctx* ctx, uint64_t* out, int n);
/* Per-stage device time of the last batch in ms (HIP events on the launch stream):
 * [0] extract, [1] k-mer sort, [2] match, [3] match sort + assign, [4] total. */
int mtb_last_stage_ms(const mtb_ctx* ctx, float* ms, int n);
/* Device time of the main kernels of the last batch in ms, from event pairs recorded on the
 * launch stream tightly around each launch: [0] K1 extract, [1] K1F membership filter, [2] K2 radix
 * sort (sort-merge join only), [3] K4 join (probe join, or windows + select + stage), [4] K4
 * transpose into per-read segments, [5] K5 per-read match sort, [6] K6 assign. */
int mtb_last_kernel_ms(const mtb_ctx* ctx, float* ms, int n);
/* Copy the last batch's mtb_result[n_reads] to dst (device memory if dst_on_device). */
int mtb_copy_results(mtb_ctx* ctx, void* dst, int dst_on_device);
/* Copy the last batch's pooled taxID:count entries (mtb_taxcnt[*n_out], the lists mtb_result
 * offsets point into) to dst (device memory if dst_on_device); the multi-GPU gather (C1) moves them
 * with the records. */
int mtb_copy_taxcnt(mtb_ctx* ctx, void* dst, int dst_on_device, uint64_t* n_out);

/* ---- staged entry points (per-stage parity against the oracle) ----------------------------- */
/* Query k-mers of the last batch (blank slots dropped, and those whose AA 8-mer the DB does not
 * hold: they cannot match; mtb_last_stats[1] of them) in the order K4 consumed them: grouped by
 * the top 24 bits of the base-21 rank of their 8 AA codes (the index join needs locality, not
 * compareQueryKmer's total order); requires MTB_KEEP_STAGES. */
int mtb_get_query_kmers(mtb_ctx* ctx, mtb_kmer* out, uint64_t capacity, uint64_t* n_out);
/* Matches of the last batch in compareMatches order (KmerMatcher.cpp:1149-1166); requires
 * MTB_KEEP_STAGES. */
int mtb_get_matches(mtb_ctx* ctx, mtb_match* out, uint64_t capacity, uint64_t* n_out);
/* K5+K6 only, on caller-provided matches (any order): query_len[i] = queryLength+queryLength2
 * of read i (seqID i+1). Keeps every match (mtb_get_matches returns them in compareMatches order). */
int mtb_assign_matches(mtb_ctx* ctx, const mtb_match* matches, uint64_t n_matches,
                       const uint32_t* query_len, uint32_t n_reads, mtb_result* results);

/* K0M alone: SeqIterator::maskLowComplexityRegions (SeqIterator.cpp:154-175; tantan, restated:
 * parity unpinned) of n reads with the context's mask_prob, on the device. seq/off/out are host
 * arrays; out receives off[n] bytes: 'N' where masked (or not A/C/G/T/U), else the input letter. */
int mtb_mask_reads(mtb_ctx* ctx, const char* seq, const uint64_t* off, uint32_t n_reads, char* out);

/* bytes from src to dst, host or device memory either (hipMemcpyDefault: the runtime tells them
 * apart); for bindings that assemble device-resident results of split batches (classifier.py). */
int mtb_memcpy(void* dst, const void* src, uint64_t bytes);

/* compareDna's codon arithmetic alone (KmerMatcher.cpp:1117-1146 over KmerMatcher.h:66-158, 348-416),
 * on the device K4 runs on: for each (query, target) DNA part the Hamming sum (getHammingDistanceSum),
 * and the forward and reverse per-codon 2-bit words (getHammings / getHammings_reverse), from the
 * device functions the join emits matches with. Host arrays; MTB_ERR_INTERNAL if the join's
 * row-cached forms disagree with the plain forms on any pair. */
int mtb_hamming(int device, const uint64_t* query, const uint64_t* target, uint64_t n, uint8_t* sum, uint16_t* fwd,
                uint16_t* rev);

/* The path's dependency-free helper functions on the device, as the kernels call them (round 6;
 * pinned by tests/golden/ref_functions.json, which the reference's own function bodies computed):
 * fn selects one, every case i reads param[i], a[i], b[i] and writes out[i] (floats as their IEEE
 * bit pattern; MTB_PIN_TAXONOMER_SHAPE writes 6 values per case). n_out = cases written (values for
 * the decode). Host arrays. */
#define MTB_PIN_SCORE_INCREMENT 0     /* Taxonomer::calScoreIncrement(a, shift = param), Taxonomer.cpp:650-661 */
#define MTB_PIN_HAMMING_INCREMENT 1   /* calHammingDistIncrement(a, param), :663-669                            */
#define MTB_PIN_IS_CONSECUTIVE 2      /* isConsecutive(dna a, dna b, shift = param; 0 = no shift), :671-683     */
#define MTB_PIN_IS_CONSECUTIVE2 3     /* isConsecutive2(a, b, param), :686-699                                 */
#define MTB_PIN_MATCH_SCORE 4         /* Match::getScore of rightEndHamming a, Match.h:32-44                   */
#define MTB_PIN_RIGHT_PART_SCORE 5    /* Match::getRightPartScore(range = param), Match.h:46-57               */
#define MTB_PIN_LEFT_PART_SCORE 6     /* Match::getLeftPartScore(param), Match.h:59-70                        */
#define MTB_PIN_RIGHT_PART_HAMMING 7  /* Match::getRightPartHammingDist(param), Match.h:72-78                 */
#define MTB_PIN_LEFT_PART_HAMMING 8   /* Match::getLeftPartHammingDist(param), Match.h:80-86                  */
#define MTB_PIN_MAX_COVERED_LENGTH 9  /* LocalUtil::getMaxCoveredLength<int>(a), LocalUtil.h:50-59            */
#define MTB_PIN_QUERY_KMER_NUMBER 10  /* LocalUtil::getQueryKmerNumber<int>(a, spaceNum = param), :45-48       */
#define MTB_PIN_TAXONOMER_SHAPE 11    /* a = syncmer << 16 | smer_len, b = seq_mode: dnaShift, maxCodonShift,
                                       * denominator, bitsPerCodon, totalDnaBits, lastCodonMask (Taxonomer.cpp:34-58) */
#define MTB_PIN_DECODE_DIFF_IDX 12    /* a = n diffIdx words: every k-mer value (getNextTargetKmer,
                                       * KmerMatcher.h:282-297) through K3's decode (decode_diff_chunk)   */
int mtb_pin_eval(int device, int fn, const int64_t* param, const uint64_t* a, const uint64_t* b, uint64_t n,
                 int64_t* out, uint64_t* n_out);

/* K2 alone (round 6; SURVEY §8(b)'s staged mtb_sort): n (key, value) pairs sorted on key bits
 * [bit_lo, bit_hi) by the query sort's LSD radix passes, stable (equal keys keep their input order).
 * Host arrays; the tests check the stability directly (tests/test_radix.py). */
int mtb_sort_pairs(int device, const uint64_t* keys, const uint32_t* vals, uint64_t n, int bit_lo, int bit_hi,
                   uint64_t* keys_out, uint32_t* vals_out);

/* Diagnostics (round 5): the opened DB's run-length lines (the unstaged join's runs without a
 * run-index read) checked against its run index for every present AA rank within their reach:
 * out[0] ranks checked, out[1] those the codes resolve, out[2] mismatches (MTB_ERR_INTERNAL when
 * any). MTB_ERR_ARG when the context has no run-length lines (MTB_LINE_EXT=0) or no run index. */
int mtb_line_ext_check(mtb_ctx* ctx, uint64_t out[3]);

/* Diagnostics (round 6): the opened DB's link lines (K1F's one read per window pair: per AA 7-mer S
 * the 21 8-mers S·y and the 21 x·S) checked against its probe lines for every AA rank r — bit r % 21
 * of word r / 21 and bit 32 + r / 21^7 of word r % 21^7 must equal membership bit r: out[0] ranks
 * checked (21^8), out[1] present ranks, out[2] disagreeing bits (MTB_ERR_INTERNAL when any).
 * MTB_ERR_ARG when the context has no link lines (MTB_LINK_LINES=0, the probe or sweep join). */
int mtb_link_check(mtb_ctx* ctx, uint64_t out[3]);

/* ---- range-partitioned DB across GPUs ---------------------------- */
/* A DB larger than one GPU's HBM is cut at split entries (DiffIdxSplit, Kmer.h:111-119; written
 * AA-group aligned by IndexCreator.cpp:843-851, read by KmerMatcher.cpp:180-192,255-271) into
 * n_parts ranges of about equal k-mer count; a context opened with par->db_part/db_parts holds one
 * range. Every rank extracts the whole batch, its membership filter keeps the k-mers of its range
 * (an AA run never straddles two ranges), MTB_MATCH_ONLY stops after the join, the matches go
 * all-to-all to the rank owning their read, and mtb_assign_chunks scores them there.
 *
 * kmer_start[p] = first global k-mer index of part p (p = 0..n_parts; kmer_start[n_parts] = n_kmers)
 * and split_index[p] = the split entry it starts at. Host only (no device). MTB_ERR_DB when the
 * split table has fewer usable entries than parts. */
int mtb_partition_bounds(const uint64_t* split, uint64_t n_split, uint64_t n_kmers, int n_parts,
                         uint64_t* kmer_start, uint64_t* split_index);
/* After mtb_classify_batch(..., MTB_MATCH_ONLY): the batch's matches grouped by read (read order,
 * unsorted within a read), the per-read match counts and query lengths (queryLength +
 * queryLength2). Any pointer may be NULL; device pointers if dst_on_device. */
int mtb_copy_matches(mtb_ctx* ctx, mtb_match* matches, uint32_t* read_counts, uint32_t* query_len,
                     int dst_on_device);
/* K5 + K6 on n_chunks concatenated chunks of matches, chunk c holding the matches of reads
 * 0..n_reads-1 grouped by read with counts chunk_counts[c * n_reads + i] (the all-to-all receive
 * layout). With MTB_INPUT_DEVICE, matches / chunk_counts / query_len are device pointers; with
 * MTB_KEEP_STAGES, K5 keeps every match (mtb_get_matches), else it drops the dead ones.
 * results: host array or NULL (mtb_device_results / mtb_copy_results). */
int mtb_assign_chunks(mtb_ctx* ctx, const mtb_match* matches, uint64_t n_matches, const uint32_t* chunk_counts,
                      uint32_t n_chunks, const uint32_t* query_len, uint32_t n_reads, uint32_t flags,
                      mtb_result* results);

/* ---- reference-DB builder (IndexCreator analogue) ----------------------------- */
/* Genomes + gene blocks -> diffIdx / info / split / taxID_list in the reference's on-disk format
 * (IndexCreator.cpp:316-376,811-886, IndexCreator.h:475-629), built on the GPU. */
typedef struct mtb_build_input {
    const uint8_t* seq;          /* concatenated genomes (device pointer with MTB_INPUT_DEVICE)  */
    const uint64_t* off;         /* n_genomes+1 offsets (device pointer with MTB_INPUT_DEVICE)   */
    uint32_t n_genomes;
    const int32_t* genome_taxid; /* host */
    const int32_t* blk_genome;   /* host: gene blocks {genome, start, end, strand (+1/-1)}        */
    const int32_t* blk_start;
    const int32_t* blk_end;
    const int32_t* blk_strand;
    uint64_t n_blocks;
    int32_t split_num;           /* 4096 in the reference's build                               */
    uint32_t flags;
} mtb_build_input;

/* mtb_build_input.flags: MTB_INPUT_DEVICE (seq/off are device pointers) and */
#define MTB_BUILD_DEVICE_OUT 8u  /* keep the deduplicated DB on the device as resident-form values + info
                                    (dev_values / dev_info, n_info entries, capacity n_info + 8) instead
                                    of encoding diffIdx / split to the host */

typedef struct mtb_db_built {    /* malloc'd host arrays, release with mtb_free_built */
    uint16_t* diff_idx; uint64_t n_diff_idx;
    uint32_t* info;     uint64_t n_info;
    uint64_t* split;    uint64_t n_split;
    int32_t* taxid_list; uint64_t n_taxid_list;
    uint64_t* dev_values;        /* MTB_BUILD_DEVICE_OUT: device arrays (hipFree'd by mtb_free_built) */
    uint32_t* dev_info;
} mtb_db_built;

int mtb_build_db(const mtb_build_input* in, const mtb_db_host* taxonomy, const mtb_params* par, int device,
                 mtb_db_built* out);
void mtb_free_built(mtb_db_built* b);

/* ---- host I/O around the path ------------------------------------------ */
/* One batch of reads in the flat layout mtb_classify_batch takes; names are the header's first
 * token (kseq), concatenated, name i = names[name_off[i] .. name_off[i+1]). Buffers belong to the
 * reader and stay valid until its next call. */
typedef struct mtb_read_batch {
    uint32_t n_reads;
    const char* seq1;
    const uint64_t* off1;
    const char* seq2; /* NULL unless paired */
    const uint64_t* off2;
    const char* names;
    const uint64_t* name_off;
} mtb_read_batch;

typedef struct mtb_reader mtb_reader;
/* FASTA or FASTQ, plain or gzip; path2 NULL for single-end. Replaces QueryIndexer's indexing pass and
 * KmerExtractor::loadChunkOfReads (QueryIndexer.cpp:30-147, KmerExtractor.cpp:442-494). */
int mtb_reader_open(const char* path1, const char* path2, mtb_reader** out);
/* Up to max_reads reads (and about max_bases bases); n_reads == 0 at end of input. MTB_ERR_IO on
 * malformed input or mates with different read counts (QueryIndexer.cpp:121-124). */
int mtb_reader_next(mtb_reader* r, uint32_t max_reads, uint64_t max_bases, mtb_read_batch* batch);
void mtb_reader_close(mtb_reader* r);
/* Rank name of a taxID in the context's taxonomy ("-" if absent). */
const char* mtb_taxon_rank(const mtb_ctx* ctx, int32_t tax_id);
/* TaxonomyWrapper::getOriginalTaxID (TaxonomyWrapper.h:70-79): the taxID the user's taxonomy
 * names for an internal one (a taxonomyDB built with internal taxIDs); identity otherwise. Result
 * records and taxcnt entries hold internal taxIDs; the writers print original ones. */
int32_t mtb_original_taxid(const mtb_ctx* ctx, int32_t tax_id);
/* TaxonomyWrapper::taxLineage2 (TaxonomyWrapper.cpp:431-454): "d_Bacteria;p_...;s_..." ("-" if
 * the taxID is absent). The string lives as long as the context. */
const char* mtb_taxon_lineage(const mtb_ctx* ctx, int32_t tax_id);
/* Reporter::writeReadClassification (Reporter.cpp:38-83) for one batch: header line unless
 * append, one line per read; taxcnt as returned by mtb_get_taxcnt. flags: MTB_WRITE_LINEAGE adds
 * the lineage column (--lineage, par.printLineage). */
#define MTB_WRITE_LINEAGE 1u
int mtb_write_classifications(const mtb_ctx* ctx, const char* path, int append, const mtb_read_batch* batch,
                              const mtb_result* results, const mtb_taxcnt* taxcnt, uint32_t flags);
/* Reporter::writeReportFile's per-taxon report (Reporter.cpp:175-190, writeReport :217-244; clade
 * counts by NcbiTaxonomy::getCladeCounts / getParentToChildren semantics): tax_ids[i] / counts[i] =
 * reads classified to each taxID over the run (++taxCounts[classification], Classifier.cpp:201-203;
 * taxID 0 = unclassified), total_reads = all reads of the run. Writes the TSV
 * "#clade_proportion\tclade_count\ttaxon_count\trank\ttaxID\tname"; the Krona chart is not
 * written (its HTML prelude is MMseqs2 data absent from the reference). */
int mtb_write_report(const mtb_ctx* ctx, const char* path, uint64_t total_reads, const int32_t* tax_ids,
                     const uint32_t* counts, uint64_t n);

/* A second context over the same DB on the same device: its own stream and batch workspace, the
 * DB-derived device arrays (records, AA directory, probe lines, run index, species map, taxonomy)
 * shared, freed with the last context holding them (any close order). Two contexts on one GPU let
 * mtb_start_classify_multi keep two batches in flight: one batch's host round trips and result
 * copies overlap the other's kernels. */
int mtb_clone(const mtb_ctx* src, mtb_ctx** out);

/* ---- Classifier::startClassify over files ----------------------------------- */
/* Classifier.cpp:44-164 as a threaded native pipeline: per mate file a reader (BGZF blocks inflated
 * by a worker pool; gzip and plain files read ahead), a splitter cutting the bytes at record
 * boundaries and a pool of parse workers; an assembler filling pinned
 * batches of <= max_reads reads and <= max_bases bases (the reference's RAM-bounded QuerySplits,
 * QueryIndexer.cpp:62-67,132-137) and uploading each on a copy stream; mtb_classify_batch on the
 * calling thread; a writer emitting the per-read TSV (Reporter.cpp:38-83) while the next batch runs.
 * With report_tsv, the per-taxon report of the run (Classifier.cpp:149). */
typedef struct mtb_classify_opts {
    const char* query1;       /* FASTA/FASTQ, plain or gzip (BGZF inflates in parallel)        */
    const char* query2;       /* mate 2 (seq_mode 2), else NULL                                 */
    const char* out_tsv;      /* per-read classifications                                       */
    const char* report_tsv;   /* per-taxon report, or NULL                                      */
    uint32_t max_reads;       /* reads per batch (0: 4,000,000, bounded by max_bases; the first
                                 five batches ramp up from 1/32 of it so the GPU starts early)     */
    uint32_t write_flags;     /* MTB_WRITE_LINEAGE                                              */
    uint64_t max_bases;       /* bases per batch, both mates (0: from free HBM, < 2^30)         */
    int32_t threads;          /* host threads for inflating, per run (0: min(16, cores)); each
                                 mate also gets max(2, threads / 4) parse workers                 */
    int32_t reserved;
    /* --em outputs (context opened with em = 1; each NULL to skip): the reassigned reads
     * (Reporter::writeReclassifyResults), the EM abundance report and the reassignment report
     * (Reporter::writeReportFile with ReportType EM / EM_RECLASSIFY, Classifier.cpp:154-161) */
    const char* em_tsv;
    const char* em_report_tsv;
    const char* em_reclassify_report_tsv;
} mtb_classify_opts;
typedef struct mtb_classify_stats {
    uint64_t reads, bases, batches;
    double wall_s;            /* whole run                                                      */
    double gpu_s;             /* mtb_classify_batch calls                                       */
    double input_wait_s;      /* the GPU stage waiting for a parsed, uploaded batch             */
    double write_s;           /* TSV formatting and writing (overlapped with the GPU stage)     */
    /* host input stages, summed over the mates (and over the parse workers for parse_s)           */
    double source_s;          /* decompressed bytes from the file sources                       */
    double scan_s;            /* record-boundary scans (splitters)                              */
    double parse_s;           /* record parsing (parse workers)                                 */
    double fill_s;            /* pinned batch filling and upload issue (assembler)              */
    double first_batch_s;     /* run start until the first batch is uploaded                    */
    uint64_t split_batches;   /* batches classified in pieces (their workspace did not fit)     */
} mtb_classify_stats;
int mtb_start_classify(mtb_ctx* ctx, const mtb_classify_opts* opts, mtb_classify_stats* stats);
/* The same run over n_ctx contexts, one per GPU of the node (each holding the DB, or the same
 * device twice in tests): batch k runs on ctxs[k mod n_ctx] — the QuerySplit loop of
 * Classifier.cpp:81-133 spread over the GPUs — while one parser feeds them all and one writer emits
 * the batches in input order, so the TSV, the report and the --em outputs are byte-identical to a
 * one-context run. ctxs[0] supplies the taxonomy for the writers and runs --em. */
int mtb_start_classify_multi(mtb_ctx* const* ctxs, int n_ctx, const mtb_classify_opts* opts,
                             mtb_classify_stats* stats);

/* The same run over a DB larger than one GPU's HBM, range-partitioned:
 * ctxs[p] holds part db_part = p of db_parts = n_ctx (one context per GPU, opened with
 * mtb_params.db_part / db_parts). Every context matches each batch against its part
 * (MTB_MATCH_ONLY); the per-read match segments go to the owner of their reads (context p owns
 * the p-th 1/n of each batch's reads) by device-to-device copies (hipMemcpyPeerAsync over xGMI
 * between GPUs); each owner scores its reads (mtb_assign_chunks) and one writer emits the batch in
 * input order: the TSV and report are byte-identical to a one-context run over the whole DB. A
 * context out of HBM halves the batch for all of them (MTB_RETRY, as a whole batch does). This is
 * the reference's per-thread split seek over AA-aligned split entries (KmerMatcher.cpp:180-192,
 * 255-271; IndexCreator.cpp:843-851) spread over GPUs. --em is refused (db_parts > 1). */
int mtb_start_classify_partitioned(mtb_ctx* const* ctxs, int n_ctx, const mtb_classify_opts* opts,
                                   mtb_classify_stats* stats);

/* ---- --em: EM re-estimation of species abundances and read reassignment ------------------------
 * Replaces Reporter::writeMappings / Classifier::getTopSpecies (per batch) and Classifier::em +
 * reclassify (Classifier.cpp:209-386) after the last batch. */
typedef struct mtb_em_map {   /* MappingRes (common.h:24-28): 12 B */
    uint32_t query_id;        /* read index over the whole run                                   */
    int32_t species_id;       /* internal species taxID                                          */
    float score;              /* species score squared                                           */
} mtb_em_map;
typedef struct mtb_em_read {  /* Classification's taxId / score (common.h:83-93) of one read      */
    int32_t tax_id;           /* internal taxID of the reassignment, 0 = none                     */
    int32_t mapped;           /* 0 no mappings; 1 reassigned; 2 mappings with a zero sum (taxID 0,
                                 not counted in the reassignment report)                          */
    double score;             /* probability mass of the species the LCA was taken over           */
} mtb_em_read;
typedef struct mtb_em_stats {
    uint64_t query_count;     /* queries with a non-zero sum in the last iteration               */
    uint32_t iterations;      /* EM iterations run (<= 1000; stops at delta < 1e-6)             */
    uint32_t n_species;       /* top species (the abundance vector's support)                    */
    double delta;             /* last iteration's sum |p_new - p|                                */
} mtb_em_stats;
/* The last batch's mappings (context opened with em = 1): for each classified read, in read order,
 * its <= 10 best species by score (std::sort order: score descending, ties as libstdc++ leaves them)
 * with score^2, query_id = query_offset + the read's batch index. n_out = mappings of the batch;
 * returns MTB_RETRY (n_out set, nothing copied) when cap is too small. */
int mtb_get_em_mappings(mtb_ctx* ctx, uint32_t query_offset, mtb_em_map* out, uint64_t cap, uint64_t* n_out);
/* Classifier::em + reclassify over all mappings (query_id ascending, <= 10 per query): species
 * length factors 1 / log(DB k-mers of the species) (dbDir/sp2uniqKmerCnt when present, else
 * counted on the device and written there, as Classifier::countUniqueKmerPerSpecies does), the EM
 * iterations on the device in double precision (per-species sums in query order, fixed order: run
 * to run identical), then per query the reassignment. reads_out: total_reads entries. sp_ids /
 * sp_probs / sp_counts (cap entries, ascending species; n_sp = the top species): final abundances
 * and emTaxCounts (unsigned)(p * query_count). */
int mtb_em(mtb_ctx* ctx, const mtb_em_map* maps, uint64_t n_maps, uint64_t total_reads, mtb_em_read* reads_out,
           int32_t* sp_ids, double* sp_probs, uint32_t* sp_counts, uint64_t cap, uint64_t* n_sp, mtb_em_stats* stats);
/* Reporter::writeReclassifyResults (Reporter.cpp:417-458): the reassigned reads, names and query
 * lengths taken from the classification TSV written before (Classifier::loadOriginalResults,
 * Classifier.cpp:450-480). flags: MTB_WRITE_LINEAGE. */
int mtb_write_em_results(mtb_ctx* ctx, const char* path, const char* classification_tsv, const mtb_em_read* reads,
                         uint64_t n_reads, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* MTB_GPU_H */
