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

int main(int argc, char** argv) {
    for (int a = 1; a < argc; a++) {
        const double gb = atof(argv[a]);
        const uint64_t bytes = (uint64_t)(gb * 1e9) & ~63ull;
        const uint64_t nLines = bytes / 64;
        uint32_t *buf = nullptr, *out = nullptr;
        if (hipMalloc(&buf, bytes) != hipSuccess) { printf("alloc %.1f GB failed\n", gb); return 1; }
        hipMemset(buf, 1, bytes);
        const uint64_t threads = 1ull << 25;  // 537M loads per launch
        hipMalloc(&out, threads * 4);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        k_gather<<<(unsigned)(threads / 256), 256>>>(buf, nLines, 1, out);  // warm-up
        hipEventRecord(e0);
        const int reps = 5;
        for (int r = 0; r < reps; r++) k_gather<<<(unsigned)(threads / 256), 256>>>(buf, nLines, 7 + r, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double loads = (double)threads * kPer * reps;
        printf("{\"buffer_gb\": %.1f, \"random_loads\": %.0f, \"ms\": %.3f, \"glines_per_s\": %.2f, "
               "\"tb_per_s_at_64B\": %.2f, \"tb_per_s_at_128B\": %.2f}\n",
               gb, loads, ms, loads / (ms * 1e-3) / 1e9, loads * 64 / (ms * 1e-3) / 1e12,
               loads * 128 / (ms * 1e-3) / 1e12);
        hipFree(buf);
        hipFree(out);
    }
    return 0;
}
