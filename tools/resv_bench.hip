// Microbenchmark for k_proc's reservation phase: on the
// configs[3] shape, 256 workgroups of 1024 lanes each reserve slots in K = 300
// buckets of a 3169-bucket ring, every workgroup in the same K buckets (the
// near future all partitions send to).  Per launch, µs:
//   0 base     the wbase row stores only (no atomic)
//   1 add      a returning 32-bit atomicAdd on the bucket counter, its result
//              stored into the row (the reservation)
//   2 add+min  1, then a 64-bit atomicMin on the bucket's minimum (what
//              reserve_buckets does)
//   3 min      the 64-bit atomicMin alone
//   4 add+rmw  1, then the minimum kept per (workgroup, bucket) in a row of its
//              own: a plain load, min, store (no atomic)
// Build: hipcc --offload-arch=gfx950 -O3 tools/resv_bench.hip -o tools/resv_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            return 1;                                                       \
        }                                                                   \
    } while (0)

constexpr uint32_t NB = 3169, T = 1024, WG = 256, K = 300;

template <int MODE>
__global__ __launch_bounds__(T) void k_resv(uint32_t* bk, unsigned long long* bmin, uint32_t* wbase,
                                            uint32_t* pmin, uint32_t round) {
    const uint32_t p = blockIdx.x, j = threadIdx.x;
    if (j >= K) return;
    const uint32_t b = (round * 7 + j) % NB;
    const uint32_t c = 1 + ((p * 31 + j) & 7);
    const uint64_t t = (uint64_t)round * 1000000 + ((p * 977 + j * 131) & 0xFFFFF);
    uint32_t base = 0;
    if (MODE == 1 || MODE == 2 || MODE == 4) base = atomicAdd(&bk[b], c);
    wbase[(size_t)p * NB + b] = base + c;
    if (MODE == 2 || MODE == 3) atomicMin(&bmin[b], (unsigned long long)t);
    if (MODE == 4) {
        uint32_t* q = &pmin[(size_t)p * NB + b];
        const uint32_t x = *q, y = (uint32_t)(t & 0xFFFFFFFF);
        *q = y < x ? y : x;
    }
}

template <int MODE>
int run(const char* name, uint32_t* bk, unsigned long long* bmin, uint32_t* wbase, uint32_t* pmin) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (uint32_t r = 0; r < 20; ++r) hipLaunchKernelGGL(k_resv<MODE>, dim3(WG), dim3(T), 0, 0, bk, bmin, wbase, pmin, r);
    CK(hipDeviceSynchronize());
    const int n = 200;
    float tot = 0;
    for (int r = 0; r < n; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_resv<MODE>, dim3(WG), dim3(T), 0, 0, bk, bmin, wbase, pmin, (uint32_t)(r + 20));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
    }
    printf("%-8s %7.2f us per launch\n", name, tot * 1e3 / n);
    return 0;
}

int main() {
    uint32_t *bk, *wbase, *pmin;
    unsigned long long* bmin;
    CK(hipMalloc(&bk, NB * 4));
    CK(hipMalloc(&bmin, NB * 8));
    CK(hipMalloc(&wbase, (size_t)WG * NB * 4));
    CK(hipMalloc(&pmin, (size_t)WG * NB * 4));
    CK(hipMemset(bk, 0, NB * 4));
    CK(hipMemset(bmin, 0xFF, NB * 8));
    CK(hipMemset(pmin, 0xFF, (size_t)WG * NB * 4));
    for (int rep = 0; rep < 2; ++rep) {
        if (run<0>("base", bk, bmin, wbase, pmin) || run<1>("add", bk, bmin, wbase, pmin) ||
            run<2>("add+min", bk, bmin, wbase, pmin) || run<3>("min", bk, bmin, wbase, pmin) ||
            run<4>("add+rmw", bk, bmin, wbase, pmin))
            return 1;
    }
    return 0;
}
