// GPU reference-DB builder (the reference's IndexCreator, out of the classify path
// but needed to make GTDB-/RefSeq-scale synthetic DBs on the box). Produces the exact on-disk
// format of Appendix B:
//   extractTargetKmers (KmerExtractor.cpp:420-439) per gene block -> sort by (value, species)
//   (compareTargetKmer, Kmer.h:77-87) -> one entry per (value, species) with taxID = LCA of the
//   group (filterKmers<DB_CREATION>, IndexCreator.h:475-629) -> delta/varint diffIdx + info
//   (getDiffIdx, IndexCreator.cpp:868-886) -> split table (writeTargetFilesAndSplits, :811-861).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "mtb_host.h"
#include "mtb_launch.h"

namespace mtb {

struct BuildTabs {
    uint8_t base[256];
    int8_t aa[64];
    int8_t num[64];
};

// One thread per gene block: the block's scanner (same load orders as k_extract, with the
// block's strand); one slot per window; payload = species << 32 | taxID, or all-ones if blank.
__global__ void __launch_bounds__(256) k_target_extract(const uint8_t* __restrict__ seq, const uint64_t* __restrict__ off,
                                                        const int32_t* __restrict__ bg, const int32_t* __restrict__ bs,
                                                        const int32_t* __restrict__ be, const int32_t* __restrict__ bst,
                                                        const int32_t* __restrict__ gTax, const int32_t* __restrict__ gSp,
                                                        const uint64_t* __restrict__ slotOff, uint64_t nBlocks,
                                                        BuildTabs tabs, int kmerFormat, int syncmer, int smerLen,
                                                        uint64_t* __restrict__ keys, uint64_t* __restrict__ pay) {
    __shared__ uint8_t sBase[256];
    __shared__ int8_t sAA[64], sNum[64];
    sBase[threadIdx.x] = tabs.base[threadIdx.x];
    if (threadIdx.x < 64) { sAA[threadIdx.x] = tabs.aa[threadIdx.x]; sNum[threadIdx.x] = tabs.num[threadIdx.x]; }
    __syncthreads();
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nBlocks) return;
    const uint64_t slot0 = slotOff[b];
    const int W = (int)(slotOff[b + 1] - slot0);
    if (W <= 0) return;
    const int g = bg[b];
    const uint8_t* s = seq + off[g];
    const int s0 = bs[b], e0 = be[b];
    const int aaLen = (e0 - s0 + 1) / 3;
    const bool fwd = bst[b] > -1;
    const bool fromLeft = (kmerFormat == 2) ? fwd : !fwd;
    const bool comp = !fwd;
    const uint64_t payload = ((uint64_t)(uint32_t)gSp[g] << 32) | (uint32_t)gTax[g];
    const int nSm = 8 - smerLen + 1;
    const uint64_t smMask = (1ull << (5 * smerLen)) - 1;
    uint64_t aaAcc = 0, dnaAcc = 0, smAcc = 0;
    uint64_t sm0 = 0, sm1 = 0, sm2 = 0, sm3 = 0, sm4 = 0, sm5 = 0, sm6 = 0, sm7 = 0;
    int run = 0;
    for (int j = 0; j < aaLen; j++) {
        int c0 = fromLeft ? s0 + 3 * j : e0 - 3 * j;
        uint32_t b1, b2, b3;
        if (fromLeft) {
            uint32_t x = sBase[s[c0]], y = sBase[s[c0 + 1]], z = sBase[s[c0 + 2]];
            if (comp) { b1 = z; b2 = y; b3 = x; } else { b1 = x; b2 = y; b3 = z; }
        } else {
            uint32_t x = sBase[s[c0]], y = sBase[s[c0 - 1]], z = sBase[s[c0 - 2]];
            if (comp) { b1 = x; b2 = y; b3 = z; } else { b1 = z; b2 = y; b3 = x; }
        }
        int aa = -1, num = 0;
        if ((b1 | b2 | b3) < 4u) {
            if (comp) { b1 ^= 2u; b2 ^= 2u; b3 ^= 2u; }
            int idx = (int)(b1 << 4 | b2 << 2 | b3);
            aa = sAA[idx];
            num = sNum[idx];
        }
        if (aa < 0) run = 0;
        else {
            run++;
            aaAcc = (aaAcc << 5) | (uint64_t)aa;
            dnaAcc = (dnaAcc << 3) | (uint64_t)num;
            smAcc = ((smAcc << 5) | (uint64_t)aa) & smMask;
        }
        if (syncmer) { sm7 = sm6; sm6 = sm5; sm5 = sm4; sm4 = sm3; sm3 = sm2; sm2 = sm1; sm1 = sm0; sm0 = smAcc; }
        if (j < 7) continue;
        const int p = j - 7;
        bool ok = run >= 8;
        if (ok && syncmer) {
            const uint64_t sv[8] = {sm0, sm1, sm2, sm3, sm4, sm5, sm6, sm7};
            int bestK = -1;
            uint64_t best = ~0ull;
#pragma unroll
            for (int k = 7; k >= 0; k--)
                if (k <= nSm - 1 && sv[k] < best) { best = sv[k]; bestK = k; }
            ok = (bestK == nSm - 1) || (bestK == 0);
        }
        uint64_t key = kSentinel, pl = kSentinel;
        if (ok) {
            uint64_t aaPart;
            if (kmerFormat == 2) aaPart = aaAcc & ((1ull << 40) - 1);
            else {
                aaPart = 0;
#pragma unroll
                for (int k = 7; k >= 0; k--) aaPart = aaPart * 21 + ((aaAcc >> (5 * k)) & 31u);
            }
            key = (aaPart << 24) | (dnaAcc & 0xFFFFFFull);
            pl = payload;
        }
        keys[slot0 + p] = key;
        pay[slot0 + p] = pl;
    }
}

__global__ void k_block_windows(const int32_t* __restrict__ bs, const int32_t* __restrict__ be, uint64_t n,
                                uint64_t* __restrict__ w) {
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n) {
        int aaLen = (be[b] - bs[b] + 1) / 3;
        w[b] = aaLen >= 8 ? (uint64_t)(aaLen - 7) : 0;
    }
}

struct TaxLca {
    const int32_t *nodeOf, *nodeTax, *parent, *depth;
    int32_t maxTax;
    __device__ bool exists(int32_t t) const { return t >= 0 && t <= maxTax && nodeOf[t] >= 0; }
    __device__ int lca_node(int i, int j) const {
        if (i == 0 || j == 0) return 0;
        while (i != j) {
            int di = depth[i], dj = depth[j];
            if (di >= dj) i = parent[i];
            if (dj >= di) j = parent[j];
        }
        return i;
    }
};

// Group heads of equal (value, species) and the group's taxID = NcbiTaxonomy::LCA(vector).
__global__ void k_group_heads(const uint64_t* __restrict__ v, const uint64_t* __restrict__ pay, uint64_t n,
                              uint32_t* __restrict__ head) {
    MTB_GRID_STRIDE(i, n) head[i] = (i == 0 || v[i] != v[i - 1] || (pay[i] >> 32) != (pay[i - 1] >> 32)) ? 1u : 0u;
}

__global__ void k_group_reduce(const uint64_t* __restrict__ v, const uint64_t* __restrict__ pay, uint64_t n,
                               const uint32_t* __restrict__ head, const uint64_t* __restrict__ uidx, TaxLca tax,
                               uint64_t* __restrict__ uval, uint32_t* __restrict__ uinfo) {
    MTB_GRID_STRIDE(i, n) {
        if (!head[i]) continue;
        const uint32_t sp = (uint32_t)(pay[i] >> 32);
        int red = -1;
        for (uint64_t j = i; j < n && v[j] == v[i] && (uint32_t)(pay[j] >> 32) == sp; j++) {
            int32_t t = (int32_t)(uint32_t)pay[j];
            if (!tax.exists(t)) continue;
            int nd = tax.nodeOf[t];
            red = red < 0 ? nd : tax.lca_node(red, nd);
        }
        const uint64_t u = uidx[i];
        uval[u] = v[i];
        uinfo[u] = red >= 0 ? (uint32_t)tax.nodeTax[red] : (uint32_t)pay[i];
    }
}

__device__ __forceinline__ uint32_t diff_words(uint64_t d) {
    uint32_t w = 1;
    d >>= 15;
    while (d) { w++; d >>= 15; }
    return w;
}

__global__ void k_count_words(const uint64_t* __restrict__ uval, uint64_t U, uint32_t* __restrict__ words) {
    MTB_GRID_STRIDE(u, U) words[u] = diff_words(uval[u] - (u ? uval[u - 1] : 0ull));
}

__global__ void k_write_words(const uint64_t* __restrict__ uval, uint64_t U, const uint64_t* __restrict__ woff,
                              uint16_t* __restrict__ diff) {
    MTB_GRID_STRIDE(u, U) {
        uint64_t d = uval[u] - (u ? uval[u - 1] : 0ull);
        uint64_t o = woff[u], e = woff[u + 1];
        // getDiffIdx: last group carries the 0x8000 end flag, groups big-endian
        diff[e - 1] = (uint16_t)(0x8000u | (uint32_t)(d & 0x7FFFu));
        d >>= 15;
        for (uint64_t k = e - 1; k > o; k--) {
            diff[k - 1] = (uint16_t)(d & 0x7FFFu);
            d >>= 15;
        }
    }
}

__global__ void k_split_ends(const uint64_t* __restrict__ uval, uint64_t U, uint64_t sizeOfSplit, int splitNum,
                             uint64_t* __restrict__ gend) {
    int k = blockIdx.x * blockDim.x + threadIdx.x + 1;  // boundaries 1 .. splitNum-1
    if (k >= splitNum) return;
    uint64_t cnt = (uint64_t)k * sizeOfSplit;  // writeCnt that hits offsetList[k]
    if (sizeOfSplit == 0 || cnt == 0 || cnt > U) { gend[k - 1] = U; return; }
    uint64_t i = cnt - 1;
    uint64_t key = (uval[i] & kAAMask) + (1ull << 24);
    uint64_t lo = i + 1, hi = U;
    while (lo < hi) {
        uint64_t mid = lo + ((hi - lo) >> 1);
        if (uval[mid] < key) lo = mid + 1; else hi = mid;
    }
    gend[k - 1] = lo;  // first later k-mer with a different AA part
}

}  // namespace mtb

using namespace mtb;

#define HIP_B(x)                                                                                \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #x);            \
            goto fail;                                                                          \
        }                                                                                       \
    } while (0)

extern "C" {

void mtb_free_built(mtb_db_built* b) {
    if (!b) return;
    free(b->diff_idx);
    free(b->info);
    free(b->split);
    free(b->taxid_list);
    if (b->dev_values) hipFree(b->dev_values);
    if (b->dev_info) hipFree(b->dev_info);
    memset(b, 0, sizeof(*b));
}

int mtb_build_db(const mtb_build_input* in, const mtb_db_host* taxo, const mtb_params* par, int device,
                 mtb_db_built* out) {
    if (!in || !taxo || !par || !out) { set_error("null argument"); return MTB_ERR_ARG; }
    memset(out, 0, sizeof(*out));
    HostTaxonomy T;
    {
        std::vector<std::string> ranks(taxo->n_nodes), names(taxo->n_nodes);
        for (uint64_t i = 0; i < taxo->n_nodes; i++) {
            ranks[i] = taxo->rank_pool + taxo->rank_off[i];
            if (taxo->name_pool) names[i] = taxo->name_pool + taxo->name_off[i];
        }
        if (!build_taxonomy(taxo->node_taxid, taxo->node_parent, taxo->n_nodes, ranks, names, taxo->merged_old,
                            taxo->merged_new, taxo->n_merged, T))
            return MTB_ERR_DB;
    }
    std::vector<int32_t> gSp(in->n_genomes);
    for (uint32_t g = 0; g < in->n_genomes; g++) gSp[g] = T.taxIdAtRank(in->genome_taxid[g], "species");
    HostTables tabs = make_tables();
    BuildTabs bt;
    memcpy(bt.base, tabs.base, 256);
    memcpy(bt.aa, tabs.aa, 64);
    memcpy(bt.num, tabs.num, 64);

    hipStream_t s = nullptr;
    const uint64_t nb = in->n_blocks;
    uint8_t* dSeq = nullptr;
    uint64_t *dOff = nullptr, *dW = nullptr, *dSlot = nullptr, *kA = nullptr, *pA = nullptr, *kB = nullptr, *pB = nullptr;
    int32_t *dBg = nullptr, *dBs = nullptr, *dBe = nullptr, *dBst = nullptr, *dTax = nullptr, *dSp = nullptr;
    int32_t *tNodeOf = nullptr, *tNodeTax = nullptr, *tParent = nullptr, *tDepth = nullptr;
    uint32_t *counts = nullptr, *head = nullptr, *words = nullptr, *uinfo = nullptr;
    uint64_t *offs = nullptr, *uidx = nullptr, *uval = nullptr, *woff = nullptr, *gend = nullptr;
    uint16_t* dDiff = nullptr;
    void* scanTmp = nullptr;
    uint64_t R = 0, kept = 0, U = 0, NW = 0;
    bool inB1 = false, inB2 = false;
    uint64_t *sk, *sp_;
    int rc = MTB_ERR_HIP;
    std::vector<uint64_t> ge;
    std::vector<uint64_t> splitHost;
    int spBits = 1;
    uint64_t sizeOfSplit = 0;

    HIP_B(hipSetDevice(device));
    HIP_B(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (in->flags & MTB_INPUT_DEVICE) {
        dSeq = (uint8_t*)in->seq;
        dOff = (uint64_t*)in->off;
    } else {
        uint64_t bytes = in->off[in->n_genomes];
        HIP_B(hipMalloc(&dSeq, bytes + 1));
        HIP_B(hipMalloc(&dOff, sizeof(uint64_t) * (in->n_genomes + 1)));
        HIP_B(hipMemcpyAsync(dSeq, in->seq, bytes, hipMemcpyHostToDevice, s));
        HIP_B(hipMemcpyAsync(dOff, in->off, sizeof(uint64_t) * (in->n_genomes + 1), hipMemcpyHostToDevice, s));
    }
    HIP_B(hipMalloc(&dBg, 4 * nb + 4));
    HIP_B(hipMalloc(&dBs, 4 * nb + 4));
    HIP_B(hipMalloc(&dBe, 4 * nb + 4));
    HIP_B(hipMalloc(&dBst, 4 * nb + 4));
    HIP_B(hipMalloc(&dTax, 4 * in->n_genomes + 4));
    HIP_B(hipMalloc(&dSp, 4 * in->n_genomes + 4));
    HIP_B(hipMemcpyAsync(dBg, in->blk_genome, 4 * nb, hipMemcpyHostToDevice, s));
    HIP_B(hipMemcpyAsync(dBs, in->blk_start, 4 * nb, hipMemcpyHostToDevice, s));
    HIP_B(hipMemcpyAsync(dBe, in->blk_end, 4 * nb, hipMemcpyHostToDevice, s));
    HIP_B(hipMemcpyAsync(dBst, in->blk_strand, 4 * nb, hipMemcpyHostToDevice, s));
    HIP_B(hipMemcpyAsync(dTax, in->genome_taxid, 4 * in->n_genomes, hipMemcpyHostToDevice, s));
    HIP_B(hipMemcpyAsync(dSp, gSp.data(), 4 * in->n_genomes, hipMemcpyHostToDevice, s));
    // windows per block -> slots
    HIP_B(hipMalloc(&dW, 8 * (nb + 1)));
    HIP_B(hipMalloc(&dSlot, 8 * (nb + 1)));
    HIP_B(hipMalloc(&scanTmp, 8 * scan_tmp_elems(nb + 1)));
    if (nb) k_block_windows<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(dBs, dBe, nb, dW);
    exclusive_scan_u64(dW, nb, dSlot, scanTmp, s);
    HIP_B(hipMemcpyAsync(&R, dSlot + nb, 8, hipMemcpyDeviceToHost, s));
    HIP_B(hipStreamSynchronize(s));
    HIP_B(hipMalloc(&kA, 8 * (R + 1)));
    HIP_B(hipMalloc(&pA, 8 * (R + 1)));
    HIP_B(hipMalloc(&kB, 8 * (R + 1)));
    HIP_B(hipMalloc(&pB, 8 * (R + 1)));
    if (nb)
        k_target_extract<<<(unsigned)((nb + 255) / 256), 256, 0, s>>>(dSeq, dOff, dBg, dBs, dBe, dBst, dTax, dSp, dSlot,
                                                                      nb, bt, par->kmer_format, par->syncmer,
                                                                      par->smer_len, kA, pA);
    // sort by (value, species): species digits first (payload bits 32..), then the value
    while ((1ll << spBits) <= (long long)T.maxTax) spBits++;
    HIP_B(hipFree(scanTmp));
    scanTmp = nullptr;
    HIP_B(hipMalloc(&counts, 4 * radix_counts_elems(R + 1)));
    HIP_B(hipMalloc(&offs, 8 * (radix_counts_elems(R + 1) + 1)));
    HIP_B(hipMalloc(&scanTmp, 8 * scan_tmp_elems(radix_counts_elems(R + 1) + R + 2)));
    kept = radix_sort_pairs(pA, kA, pB, kB, R, 32, 32 + ((spBits + 7) / 8) * 8, true, false, counts, offs, scanTmp, &inB1, s);
    {
        uint64_t* k1 = inB1 ? kB : kA;
        uint64_t* p1 = inB1 ? pB : pA;
        uint64_t* k2 = inB1 ? kA : kB;
        uint64_t* p2 = inB1 ? pA : pB;
        radix_sort_pairs(k1, p1, k2, p2, kept, 0, 64, false, false, counts, offs, scanTmp, &inB2, s);
        sk = inB2 ? k2 : k1;
        sp_ = inB2 ? p2 : p1;
    }
    // dedup per (value, species) with the LCA of the group's taxIDs
    {
        std::vector<int32_t>* arrs[4] = {&T.nodeOf, &T.nodeTax, &T.parent, &T.depth};
        int32_t** dst[4] = {&tNodeOf, &tNodeTax, &tParent, &tDepth};
        for (int a = 0; a < 4; a++) {
            HIP_B(hipMalloc(dst[a], 4 * arrs[a]->size() + 4));
            HIP_B(hipMemcpyAsync(*dst[a], arrs[a]->data(), 4 * arrs[a]->size(), hipMemcpyHostToDevice, s));
        }
    }
    HIP_B(hipMalloc(&head, 4 * (kept + 1)));
    HIP_B(hipMalloc(&uidx, 8 * (kept + 1)));
    if (kept) k_group_heads<<<stride_grid(kept), 256, 0, s>>>(sk, sp_, kept, head);
    exclusive_scan_u32(head, kept, uidx, scanTmp, s);
    HIP_B(hipMemcpyAsync(&U, uidx + kept, 8, hipMemcpyDeviceToHost, s));
    HIP_B(hipStreamSynchronize(s));
    HIP_B(hipMalloc(&uval, 8 * (U + kDbPad)));
    HIP_B(hipMalloc(&uinfo, 4 * (U + kDbPad)));
    if (kept)
        k_group_reduce<<<stride_grid(kept), 256, 0, s>>>(
            sk, sp_, kept, head, uidx, TaxLca{tNodeOf, tNodeTax, tParent, tDepth, T.maxTax}, uval, uinfo);
    if (in->flags & MTB_BUILD_DEVICE_OUT) {  // resident form for mtb_open_resident; no diffIdx / split
        if (par->kmer_format == 2) launch_to_rank_form(uval, U, s);
        HIP_B(hipStreamSynchronize(s));
        out->dev_values = uval;
        out->dev_info = uinfo;
        out->n_info = U;
        uval = nullptr;
        uinfo = nullptr;
        goto taxids;
    }
    // diffIdx words
    HIP_B(hipMalloc(&words, 4 * (U + 1)));
    HIP_B(hipMalloc(&woff, 8 * (U + 1)));
    if (U) k_count_words<<<stride_grid(U), 256, 0, s>>>(uval, U, words);
    exclusive_scan_u32(words, U, woff, scanTmp, s);
    HIP_B(hipMemcpyAsync(&NW, woff + U, 8, hipMemcpyDeviceToHost, s));
    HIP_B(hipStreamSynchronize(s));
    HIP_B(hipMalloc(&dDiff, 2 * (NW + 1)));
    if (U) k_write_words<<<stride_grid(U), 256, 0, s>>>(uval, U, woff, dDiff);
    // split table: the distinct first-AA-change indices after every uniqKmerCnt/(splitNum-1) k-mers
    sizeOfSplit = in->split_num > 1 ? U / (uint64_t)(in->split_num - 1) : 0;
    HIP_B(hipMalloc(&gend, 8 * (size_t)std::max(1, in->split_num)));
    if (in->split_num > 1)
        k_split_ends<<<(in->split_num + 255) / 256, 256, 0, s>>>(uval, U, sizeOfSplit, in->split_num, gend);
    ge.assign((size_t)std::max(0, in->split_num - 1), U);
    if (!ge.empty()) HIP_B(hipMemcpyAsync(ge.data(), gend, 8 * ge.size(), hipMemcpyDeviceToHost, s));
    out->n_diff_idx = NW;
    out->n_info = U;
    out->diff_idx = (uint16_t*)malloc(2 * NW + 2);
    out->info = (uint32_t*)malloc(4 * U + 4);
    HIP_B(hipMemcpyAsync(out->diff_idx, dDiff, 2 * NW, hipMemcpyDeviceToHost, s));
    HIP_B(hipMemcpyAsync(out->info, uinfo, 4 * U, hipMemcpyDeviceToHost, s));
    HIP_B(hipStreamSynchronize(s));
    {
        out->n_split = (uint64_t)std::max(1, in->split_num);
        out->split = (uint64_t*)calloc(3 * out->n_split, sizeof(uint64_t));
        uint64_t idx = 1, last = ~0ull;
        for (uint64_t g : ge) {
            if (g >= U || g == last) continue;
            last = g;
            uint64_t val = 0, wo = 0;
            HIP_B(hipMemcpy(&val, uval + g, 8, hipMemcpyDeviceToHost));
            HIP_B(hipMemcpy(&wo, woff + g + 1, 8, hipMemcpyDeviceToHost));
            out->split[3 * idx + 0] = val;
            out->split[3 * idx + 1] = wo;
            out->split[3 * idx + 2] = g + 1;
            idx++;
        }
    }
taxids:
    {
        std::vector<int32_t> ids(in->genome_taxid, in->genome_taxid + in->n_genomes);
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        out->n_taxid_list = ids.size();
        out->taxid_list = (int32_t*)malloc(4 * ids.size() + 4);
        memcpy(out->taxid_list, ids.data(), 4 * ids.size());
    }
    rc = MTB_OK;
fail:
    void* frees[] = {dW, dSlot, kA, pA, kB, pB, dBg, dBs, dBe, dBst, dTax, dSp, tNodeOf, tNodeTax, tParent, tDepth,
                     counts, head, words, uinfo, offs, uidx, uval, woff, gend, dDiff, scanTmp};
    if (s) hipStreamSynchronize(s);
    for (void* p : frees)
        if (p) hipFree(p);
    if (!(in->flags & MTB_INPUT_DEVICE)) {
        if (dSeq) hipFree(dSeq);
        if (dOff) hipFree(dOff);
    }
    if (s) hipStreamDestroy(s);
    if (rc != MTB_OK) mtb_free_built(out);
    return rc;
}

}  // extern "C"
