/*
 * abi_caller.c — a compiled C caller of include/mtb_gpu.h (the boundary a maintainer binds from the
 * reference's C++ host). Built by __graft_entry__.build() with gcc against
 * metabuli_work_amd/libmtbgpu.so; no ctypes, no torch.
 *
 *   abi_caller --layout
 *       prints every public struct's sizeof and field offsets as JSON (tests/test_abi.py compares
 *       them with the ctypes / numpy mirrors in metabuli_work_amd/_abi.py); no device call.
 *   abi_caller <db_dir> <seq_mode> <q1> [<q2>] <out.tsv> [<workspace_cap_bytes>]
 *       Classifier.cpp:6-32,81-133 in plain C: mtb_default_params, mtb_load_db_parameters, mtb_open,
 *       then per QuerySplit mtb_reader_next -> mtb_classify_batch -> mtb_get_taxcnt (halving a
 *       batch on MTB_RETRY, as Classifier.cpp:127-130 searches a split again; the workspace given
 *       back with mtb_release_workspace after every other split), and mtb_close. Writes
 *       one line per read: index, internal taxID (0 = unclassified), score bits (hex), hamming,
 *       query length, "taxID:count" list.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mtb_gpu.h"

_Static_assert(sizeof(mtb_kmer) == 16, "mtb_kmer is Kmer's 16 B (Kmer.h:45-46)");
_Static_assert(sizeof(mtb_match) == 24, "mtb_match is 24 B");
_Static_assert(sizeof(mtb_result) == 32, "mtb_result is 32 B");
_Static_assert(sizeof(mtb_taxcnt) == 8, "mtb_taxcnt is 8 B");
_Static_assert(sizeof(mtb_em_map) == 12, "mtb_em_map is MappingRes's 12 B (common.h:24-28)");
_Static_assert(offsetof(mtb_match, right_end_hamming) == 20 && offsetof(mtb_match, hamming) == 22,
               "mtb_match packing");
_Static_assert(offsetof(mtb_result, taxcnt_offset) == 16 && offsetof(mtb_result, is_classified) == 24,
               "mtb_result packing");

#define F(T, f) printf("%s\"%s\": %zu", first++ ? ", " : "", #f, offsetof(T, f))
#define S_BEGIN(T)                                                   \
    do {                                                             \
        int first = 0;                                               \
        printf("%s\"%s\": {\"size\": %zu, \"fields\": {", nst++ ? ", " : "", #T, sizeof(T));
#define S_END() \
    printf("}}"); \
    }           \
    while (0)

static void layout(void) {
    int nst = 0;
    printf("{");
    S_BEGIN(mtb_params);
    F(mtb_params, seq_mode); F(mtb_params, kmer_format); F(mtb_params, syncmer); F(mtb_params, smer_len);
    F(mtb_params, reduced_aa); F(mtb_params, skip_redundancy); F(mtb_params, min_score);
    F(mtb_params, min_sp_score); F(mtb_params, min_cons_cnt); F(mtb_params, min_cons_cnt_euk);
    F(mtb_params, tie_ratio); F(mtb_params, accession_level); F(mtb_params, em); F(mtb_params, threads);
    F(mtb_params, mask_mode); F(mtb_params, db_part); F(mtb_params, db_parts); F(mtb_params, mask_prob);
    S_END();
    S_BEGIN(mtb_kmer);
    F(mtb_kmer, value); F(mtb_kmer, info);
    S_END();
    S_BEGIN(mtb_match);
    F(mtb_match, qinfo); F(mtb_match, target_id); F(mtb_match, species_id); F(mtb_match, dna_encoding);
    F(mtb_match, right_end_hamming); F(mtb_match, hamming); F(mtb_match, pad);
    S_END();
    S_BEGIN(mtb_result);
    F(mtb_result, classification); F(mtb_result, score); F(mtb_result, hamming_dist); F(mtb_result, query_length);
    F(mtb_result, taxcnt_offset); F(mtb_result, taxcnt_len); F(mtb_result, is_classified); F(mtb_result, pad);
    S_END();
    S_BEGIN(mtb_taxcnt);
    F(mtb_taxcnt, tax_id); F(mtb_taxcnt, count);
    S_END();
    S_BEGIN(mtb_db_host);
    F(mtb_db_host, diff_idx); F(mtb_db_host, n_diff_idx); F(mtb_db_host, info); F(mtb_db_host, n_info);
    F(mtb_db_host, split); F(mtb_db_host, n_split); F(mtb_db_host, taxid_list); F(mtb_db_host, n_taxid_list);
    F(mtb_db_host, node_taxid); F(mtb_db_host, node_parent); F(mtb_db_host, n_nodes); F(mtb_db_host, rank_pool);
    F(mtb_db_host, rank_off); F(mtb_db_host, name_pool); F(mtb_db_host, name_off); F(mtb_db_host, merged_old);
    F(mtb_db_host, merged_new); F(mtb_db_host, n_merged);
    S_END();
    S_BEGIN(mtb_db_resident);
    F(mtb_db_resident, records); F(mtb_db_resident, n_kmers); F(mtb_db_resident, rank_form);
    F(mtb_db_resident, reserved);
    S_END();
    S_BEGIN(mtb_build_input);
    F(mtb_build_input, seq); F(mtb_build_input, off); F(mtb_build_input, n_genomes);
    F(mtb_build_input, genome_taxid); F(mtb_build_input, blk_genome); F(mtb_build_input, blk_start);
    F(mtb_build_input, blk_end); F(mtb_build_input, blk_strand); F(mtb_build_input, n_blocks);
    F(mtb_build_input, split_num); F(mtb_build_input, flags);
    S_END();
    S_BEGIN(mtb_db_built);
    F(mtb_db_built, diff_idx); F(mtb_db_built, n_diff_idx); F(mtb_db_built, info); F(mtb_db_built, n_info);
    F(mtb_db_built, split); F(mtb_db_built, n_split); F(mtb_db_built, taxid_list); F(mtb_db_built, n_taxid_list);
    F(mtb_db_built, dev_values); F(mtb_db_built, dev_info);
    S_END();
    S_BEGIN(mtb_read_batch);
    F(mtb_read_batch, n_reads); F(mtb_read_batch, seq1); F(mtb_read_batch, off1); F(mtb_read_batch, seq2);
    F(mtb_read_batch, off2); F(mtb_read_batch, names); F(mtb_read_batch, name_off);
    S_END();
    S_BEGIN(mtb_classify_opts);
    F(mtb_classify_opts, query1); F(mtb_classify_opts, query2); F(mtb_classify_opts, out_tsv);
    F(mtb_classify_opts, report_tsv); F(mtb_classify_opts, max_reads); F(mtb_classify_opts, write_flags);
    F(mtb_classify_opts, max_bases); F(mtb_classify_opts, threads); F(mtb_classify_opts, reserved);
    F(mtb_classify_opts, em_tsv); F(mtb_classify_opts, em_report_tsv); F(mtb_classify_opts, em_reclassify_report_tsv);
    S_END();
    S_BEGIN(mtb_classify_stats);
    F(mtb_classify_stats, reads); F(mtb_classify_stats, bases); F(mtb_classify_stats, batches);
    F(mtb_classify_stats, wall_s); F(mtb_classify_stats, gpu_s); F(mtb_classify_stats, input_wait_s);
    F(mtb_classify_stats, write_s); F(mtb_classify_stats, source_s); F(mtb_classify_stats, scan_s);
    F(mtb_classify_stats, parse_s); F(mtb_classify_stats, fill_s); F(mtb_classify_stats, first_batch_s);
    F(mtb_classify_stats, split_batches);
    S_END();
    S_BEGIN(mtb_em_map);
    F(mtb_em_map, query_id); F(mtb_em_map, species_id); F(mtb_em_map, score);
    S_END();
    S_BEGIN(mtb_em_read);
    F(mtb_em_read, tax_id); F(mtb_em_read, mapped); F(mtb_em_read, score);
    S_END();
    S_BEGIN(mtb_em_stats);
    F(mtb_em_stats, query_count); F(mtb_em_stats, iterations); F(mtb_em_stats, n_species); F(mtb_em_stats, delta);
    S_END();
    printf("}\n");
}

static int fail(const char* what, int rc) {
    fprintf(stderr, "abi_caller: %s failed (%d): %s\n", what, rc, mtb_last_error());
    return 1;
}

/* One QuerySplit, halved on MTB_RETRY (the reference's re-search of a split); lines to out. */
static int classify_range(mtb_ctx* ctx, const mtb_read_batch* b, uint32_t lo, uint32_t hi, uint64_t first, FILE* out) {
    const uint32_t n = hi - lo;
    mtb_result* res = (mtb_result*)calloc(n ? n : 1, sizeof(mtb_result));
    if (!res) return fail("calloc", MTB_ERR_OOM);
    int rc = mtb_classify_batch(ctx, b->seq1, b->off1 + lo, b->seq2, b->seq2 ? b->off2 + lo : NULL, n, 0, res);
    if (rc == MTB_RETRY && n > 1) {
        free(res);
        const uint32_t mid = lo + n / 2;
        int e = classify_range(ctx, b, lo, mid, first, out);
        return e ? e : classify_range(ctx, b, mid, hi, first, out);
    }
    if (rc != MTB_OK) {
        free(res);
        return fail("mtb_classify_batch", rc);
    }
    uint64_t nt = 0;
    mtb_get_taxcnt(ctx, NULL, 0, &nt);
    mtb_taxcnt* tc = (mtb_taxcnt*)calloc(nt ? nt : 1, sizeof(mtb_taxcnt));
    if (!tc || (rc = mtb_get_taxcnt(ctx, tc, nt, &nt)) != MTB_OK) {
        free(res);
        free(tc);
        return fail("mtb_get_taxcnt", rc);
    }
    for (uint32_t i = 0; i < n; i++) {
        const mtb_result* r = &res[i];
        uint32_t bits;
        memcpy(&bits, &r->score, 4);
        fprintf(out, "%llu\t%d\t%08x\t%d\t%u\t", (unsigned long long)(first + lo + i),
                r->is_classified ? r->classification : 0, bits, r->hamming_dist, r->query_length);
        for (uint32_t k = 0; k < r->taxcnt_len; k++)
            fprintf(out, "%d:%u ", tc[r->taxcnt_offset + k].tax_id, tc[r->taxcnt_offset + k].count);
        fputc('\n', out);
    }
    free(res);
    free(tc);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 2 && !strcmp(argv[1], "--layout")) {
        layout();
        return 0;
    }
    if (argc < 5) {
        fprintf(stderr, "usage: %s --layout | <db_dir> <seq_mode> <q1> [<q2>] <out.tsv> [<cap>]\n", argv[0]);
        return 2;
    }
    const int seqMode = atoi(argv[2]);
    const int paired = seqMode == 2;
    if (argc < 5 + paired) return 2;
    const char* q1 = argv[3];
    const char* q2 = paired ? argv[4] : NULL;
    const char* outPath = argv[4 + paired];
    const unsigned long long cap = argc > 5 + paired ? strtoull(argv[5 + paired], NULL, 10) : 0;

    mtb_params par;
    mtb_default_params(&par);  /* setClassifyDefaults (classify.cpp:10-37) */
    par.seq_mode = seqMode;
    mtb_load_db_parameters(argv[1], &par);  /* common.cpp:88-133 */
    mtb_ctx* ctx = NULL;
    int rc = mtb_open(argv[1], &par, 0, &ctx);
    if (rc != MTB_OK) return fail("mtb_open", rc);
    if (cap) mtb_set_workspace_cap(ctx, cap);
    mtb_reader* rd = NULL;
    if ((rc = mtb_reader_open(q1, q2, &rd)) != MTB_OK) return fail("mtb_reader_open", rc);
    FILE* out = fopen(outPath, "w");
    if (!out) return fail("fopen", MTB_ERR_IO);
    uint64_t first = 0;
    int err = 0;
    for (;;) {
        mtb_read_batch b;
        if ((rc = mtb_reader_next(rd, 1000, (uint64_t)1 << 40, &b)) != MTB_OK) {
            err = fail("mtb_reader_next", rc);
            break;
        }
        if (b.n_reads == 0) break;
        if ((err = classify_range(ctx, &b, 0, b.n_reads, first, out)) != 0) break;
        first += b.n_reads;
        /* every other split: the workspace goes back and the next split regrows it */
        if ((first / 1000) % 2 == 0 && (rc = mtb_release_workspace(ctx)) != MTB_OK) {
            err = fail("mtb_release_workspace", rc);
            break;
        }
    }
    uint64_t qk = 0, m = 0;
    mtb_last_counts(ctx, &qk, &m);
    fclose(out);
    mtb_reader_close(rd);
    mtb_close(ctx);
    if (!err) fprintf(stderr, "abi_caller: %llu reads classified\n", (unsigned long long)first);
    return err;
}
