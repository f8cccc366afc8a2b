// Check of mtb::xor_lane (DPP / permlane cross-lane moves) against __shfl_xor on the device:
// random 32-bit values, every J, several waves. Prints "xor_lane ok" or the first mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#include "../metabuli_work_amd/csrc/mtb_device.h"

__global__ void k_check(const uint32_t* in, uint32_t* bad) {
    const int lane = threadIdx.x & 63;
    const uint32_t v = in[blockIdx.x * blockDim.x + threadIdx.x];
    const uint64_t w = (uint64_t)v * 0x9E3779B97F4A7C15ull;
    for (int j = 1; j < 64; j <<= 1) {
        const uint32_t a = mtb::xor_lane32(v, j, lane), b = (uint32_t)__shfl_xor((int)v, j, 64);
        const uint64_t c = mtb::xor_lane64(w, j, lane), d = __shfl_xor(w, j, 64);
        if (a != b || c != d) atomicMax(bad, (uint32_t)(j << 16 | (blockIdx.x * blockDim.x + threadIdx.x)) + 1u);
    }
}

int main() {
    const int n = 256 * 64;
    std::vector<uint32_t> h(n);
    uint32_t x = 12345;
    for (auto& v : h) v = (x = x * 1664525u + 1013904223u);
    uint32_t *din, *dbad, bad = 0;
    if (hipMalloc(&din, n * 4) != hipSuccess || hipMalloc(&dbad, 4) != hipSuccess) return 2;
    hipMemcpy(din, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 4);
    k_check<<<n / 256, 256>>>(din, dbad);
    hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    if (bad) printf("xor_lane MISMATCH: j %u thread %u\n", (bad - 1) >> 16, (bad - 1) & 0xFFFF);
    else printf("xor_lane ok\n");
    return bad ? 1 : 0;
}
