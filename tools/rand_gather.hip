// Random-line ceiling of the HBM on this GPU (context for K1F / K4, which make one random 64/128-B
// line read per probe): every thread issues kPer independent 4-B loads at pseudo-random 64-B-aligned
// offsets of a buffer of `gb` GB (no index array: offsets from a hash of the thread id), sums them
// into one word per thread. Prints lines/s for buffer sizes like the probe lines (5.4 GB) and the
// resident DB (144 GB).
//   hipcc -O3 --offload-arch=gfx950 -o tools/_rand_gather tools/rand_gather.hip
//   tools/_rand_gather 5.4 144
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kPer = 16;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ void __launch_bounds__(256) k_gather(const uint32_t* __restrict__ buf, uint64_t nLines, uint64_t seed,
                                                uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) v[j] = buf[(mix(t * kPer + j + seed) % nLines) * 16];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) s += v[j];
    out[t] = s;
}

// Non-temporal loads (argument "n<gb>"): the same random 4-B loads with the nontemporal hint, to see
// whether a miss then fetches less than the L2's 128-B line (request-size counters, time).
__global__ void __launch_bounds__(256) k_gather_nt(const uint32_t* __restrict__ buf, uint64_t nLines, uint64_t seed,
                                                   uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) v[j] = __builtin_nontemporal_load(&buf[(mix(t * kPer + j + seed) % nLines) * 16]);
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) s += v[j];
    out[t] = s;
}

// Scoped loads (argument "c<gb>": system scope, "a<gb>": agent scope): relaxed atomic loads, i.e. plain
// loads carrying the scope's cache bits — do they still fetch whole 128-B lines?
template <int kScope>
__global__ void __launch_bounds__(256) k_gather_scoped(const uint32_t* __restrict__ buf, uint64_t nLines, uint64_t seed,
                                                       uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++)
        v[j] = __hip_atomic_load(&buf[(mix(t * kPer + j + seed) % nLines) * 16], __ATOMIC_RELAXED, kScope);
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) s += v[j];
    out[t] = s;
}

// Streaming reads (argument "s<gb>"): 16 B per lane, coalesced, the calibrated case of the guide.
__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ buf, uint64_t n16, uint32_t* __restrict__ out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t s = 0;
    for (uint64_t i = t; i < n16; i += stride) {
        const uint4 v = buf[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[t] = s;
}

// The store side (argument "w<gb>"): kPer independent 16-B stores per thread at pseudo-random 64-B-aligned
// offsets, the pattern of K4's scattered 16-B match writes (WRITE_SIZE calibration).
__global__ void __launch_bounds__(256) k_scatter(uint4* __restrict__ buf, uint64_t nLines, uint64_t seed) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int j = 0; j < kPer; j++) buf[(mix(t * kPer + j + seed) % nLines) * 4] = make_uint4((uint32_t)t, j, 0, 0);
}

int main(int argc, char** argv) {
    for (int a = 1; a < argc; a++) {
        const char mode = (argv[a][0] >= 'a' && argv[a][0] <= 'z') ? argv[a][0] : 'l';
        const bool store = mode == 'w';
        const double gb = atof(argv[a] + (mode != 'l' ? 1 : 0));
        const uint64_t bytes = (uint64_t)(gb * 1e9) & ~63ull;
        const uint64_t nLines = bytes / 64;
        uint32_t *buf = nullptr, *out = nullptr;
        // "u<gb>" / "f<gb>": the buffer uncached / fine-grained (plain random loads)
        const unsigned flags = mode == 'u' ? hipDeviceMallocUncached : mode == 'f' ? hipDeviceMallocFinegrained : 0;
        const hipError_t ae = flags ? hipExtMallocWithFlags((void**)&buf, bytes, flags) : hipMalloc(&buf, bytes);
        if (ae != hipSuccess) { printf("{\"kind\": \"%c\", \"alloc_failed_gb\": %.1f}\n", mode, gb); continue; }
        hipMemset(buf, 1, bytes);
        const uint64_t threads = 1ull << 25;  // 537M loads per launch
        hipMalloc(&out, threads * 4);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        const int reps = 5;
        if (mode == 'c' || mode == 'a') {
            auto run = [&](uint64_t seed) {
                if (mode == 'c')
                    k_gather_scoped<__HIP_MEMORY_SCOPE_SYSTEM><<<(unsigned)(threads / 256), 256>>>(buf, nLines, seed, out);
                else
                    k_gather_scoped<__HIP_MEMORY_SCOPE_AGENT><<<(unsigned)(threads / 256), 256>>>(buf, nLines, seed, out);
            };
            run(1);
            hipEventRecord(e0);
            for (int r = 0; r < reps; r++) run(7 + r);
        } else if (mode == 'n') {
            k_gather_nt<<<(unsigned)(threads / 256), 256>>>(buf, nLines, 1, out);  // warm-up
            hipEventRecord(e0);
            for (int r = 0; r < reps; r++) k_gather_nt<<<(unsigned)(threads / 256), 256>>>(buf, nLines, 7 + r, out);
        } else if (mode == 's') {
            k_stream<<<(unsigned)(threads / 256), 256>>>(reinterpret_cast<const uint4*>(buf), bytes / 16, out);
            hipEventRecord(e0);
            for (int r = 0; r < reps; r++) k_stream<<<(unsigned)(threads / 256), 256>>>(reinterpret_cast<const uint4*>(buf), bytes / 16, out);
        } else if (store) {
            k_scatter<<<(unsigned)(threads / 256), 256>>>(reinterpret_cast<uint4*>(buf), nLines, 1);  // warm-up
            hipEventRecord(e0);
            for (int r = 0; r < reps; r++) k_scatter<<<(unsigned)(threads / 256), 256>>>(reinterpret_cast<uint4*>(buf), nLines, 7 + r);
        } else {
            k_gather<<<(unsigned)(threads / 256), 256>>>(buf, nLines, 1, out);  // warm-up
            hipEventRecord(e0);
            for (int r = 0; r < reps; r++) k_gather<<<(unsigned)(threads / 256), 256>>>(buf, nLines, 7 + r, out);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double loads = (double)threads * kPer * reps;
        printf("{\"kind\": \"%s\", \"buffer_gb\": %.1f, \"random_loads\": %.0f, \"ms\": %.3f, \"glines_per_s\": %.2f, "
               "\"tb_per_s_at_64B\": %.2f, \"tb_per_s_at_128B\": %.2f}\n",
               mode == 'w' ? "store16" : mode == 'n' ? "load4_nt" : mode == 's' ? "stream16" : mode == 'c' ? "load4_sys"
               : mode == 'a' ? "load4_agent" : mode == 'u' ? "load4_uncached" : mode == 'f' ? "load4_finegrained" : "load4", gb,
               mode == 's' ? (double)bytes / 16 * reps : loads, ms, loads / (ms * 1e-3) / 1e9, loads * 64 / (ms * 1e-3) / 1e12,
               loads * 128 / (ms * 1e-3) / 1e12);
        hipFree(buf);
        hipFree(out);
    }
    return 0;
}
