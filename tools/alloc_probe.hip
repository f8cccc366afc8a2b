// Times large hipMalloc calls on a fresh process (is the cost the allocation itself, e.g. the
// driver clearing VRAM, or waiting for an earlier free?): 144 GB at once, freed, again, then 16 x 9 GB.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    void* p = nullptr;
    hipFree(0);
    size_t gb = 1ull << 30;
    double t = now();
    hipError_t e = hipMalloc(&p, 144 * gb);
    printf("fresh 144 GB: %s %.3f s\n", hipGetErrorString(e), now() - t);
    t = now();
    hipFree(p);
    printf("free: %.3f s\n", now() - t);
    t = now();
    e = hipMalloc(&p, 144 * gb);
    printf("again 144 GB: %s %.3f s\n", hipGetErrorString(e), now() - t);
    hipFree(p);
    std::this_thread::sleep_for(std::chrono::seconds(6));
    t = now();
    e = hipMalloc(&p, 144 * gb);
    printf("144 GB after free + 6 s idle: %s %.3f s\n", hipGetErrorString(e), now() - t);
    hipFree(p);
    void* q[16];
    t = now();
    for (int i = 0; i < 16; i++) hipMalloc(&q[i], 9 * gb);
    printf("16 x 9 GB: %.3f s\n", now() - t);
    t = now();
    hipMemset(q[0], 0, 9 * gb);
    hipDeviceSynchronize();
    printf("memset 9 GB: %.3f s\n", now() - t);
    for (int i = 0; i < 16; i++) hipFree(q[i]);
    return 0;
}
