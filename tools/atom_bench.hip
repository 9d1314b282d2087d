// Microbenchmark for a calendar design question: can k_proc
// append every new event straight into a (bucket, partition) cell of the
// calendar with one returning device-scope atomic per event?  Times, on the
// configs[3] shape (256 workgroups x 1024 lanes, ~1.5 events per lane,
// 3169 x 256 cells), per launch:
//   store   : each event's 16-B record to a random cell slot (no atomic)
//   atomic  : a returning atomicAdd on the event's cell counter, then the store
//             at the slot it returned
//   agg     : the same counters, one atomic per (workgroup, cell) after an LDS
//             count (most cells get one event per workgroup, so this measures
//             the LDS pass's cost on top of the same atomics)
// Build: hipcc --offload-arch=gfx950 -O3 tools/atom_bench.hip -o tools/atom_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr uint32_t NB = 3169, NP = 256, CAP = 4096;  // cells, slots per cell
constexpr uint32_t T = 1024, WG = 256, EV = 1540;    // events per workgroup

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// the event's cell: a bucket within ~100 of the front, a uniform partition
__device__ __forceinline__ uint32_t cell_of(uint32_t e, uint32_t round) {
    const uint32_t h = mix(e * 2654435761u + round);
    const uint32_t b = (round + 1 + (h >> 8) % 100) % NB, p = h & (NP - 1);
    return b * NP + p;
}

template <int MODE>
__global__ __launch_bounds__(T) void k_app(uint32_t* cnt, uint4* pool, uint32_t round) {
    __shared__ uint32_t s_cnt[4096];
    __shared__ uint32_t s_key[4096];
    const uint32_t tid = threadIdx.x;
    uint32_t c[2];
    bool v[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const uint32_t i = tid + q * T;
        v[q] = i < EV;
        c[q] = cell_of(blockIdx.x * EV + i, round);
    }
    if (MODE == 0) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (v[q]) {
                const uint32_t slot = mix(c[q] + tid) & (CAP - 1);
                pool[(size_t)c[q] * CAP + slot] = make_uint4(c[q], tid, round, 1);
            }
    } else if (MODE == 1) {
        uint32_t s[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) s[q] = v[q] ? atomicAdd(&cnt[c[q]], 1u) : 0u;
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (v[q]) pool[(size_t)c[q] * CAP + (s[q] & (CAP - 1))] = make_uint4(c[q], tid, round, 1);
    } else {
        // LDS open-addressing table of the workgroup's cells, one global atomic per cell
        for (uint32_t i = tid; i < 4096; i += T) {
            s_key[i] = 0xFFFFFFFFu;
            s_cnt[i] = 0;
        }
        __syncthreads();
        uint32_t pos[2], rank[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            pos[q] = 0;
            rank[q] = 0;
            if (!v[q]) continue;
            uint32_t h = mix(c[q]) & 4095;
            for (;;) {
                const uint32_t old = atomicCAS(&s_key[h], 0xFFFFFFFFu, c[q]);
                if (old == 0xFFFFFFFFu || old == c[q]) break;
                h = (h + 1) & 4095;
            }
            pos[q] = h;
            rank[q] = atomicAdd(&s_cnt[h], 1u);
        }
        __syncthreads();
        for (uint32_t i = tid; i < 4096; i += T) {
            const uint32_t k = s_key[i];
            if (k != 0xFFFFFFFFu) s_cnt[i] = atomicAdd(&cnt[k], s_cnt[i]);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 2; ++q)
            if (v[q]) {
                const uint32_t slot = s_cnt[pos[q]] + rank[q];
                pool[(size_t)c[q] * CAP + (slot & (CAP - 1))] = make_uint4(c[q], tid, round, 1);
            }
    }
}

int main() {
    uint32_t* cnt;
    uint4* pool;
    CK(hipMalloc(&cnt, (size_t)NB * NP * 4));
    CK(hipMalloc(&pool, (size_t)NB * NP * CAP * sizeof(uint4)));
    CK(hipMemset(cnt, 0, (size_t)NB * NP * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[3] = {"store", "atomic", "agg"};
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            const int N = 200;
            for (int w = 0; w < 20; ++w) {
                if (mode == 0) hipLaunchKernelGGL(k_app<0>, dim3(WG), dim3(T), 0, 0, cnt, pool, (uint32_t)w);
                if (mode == 1) hipLaunchKernelGGL(k_app<1>, dim3(WG), dim3(T), 0, 0, cnt, pool, (uint32_t)w);
                if (mode == 2) hipLaunchKernelGGL(k_app<2>, dim3(WG), dim3(T), 0, 0, cnt, pool, (uint32_t)w);
            }
            CK(hipEventRecord(a));
            for (int r = 0; r < N; ++r) {
                if (mode == 0) hipLaunchKernelGGL(k_app<0>, dim3(WG), dim3(T), 0, 0, cnt, pool, (uint32_t)r);
                if (mode == 1) hipLaunchKernelGGL(k_app<1>, dim3(WG), dim3(T), 0, 0, cnt, pool, (uint32_t)r);
                if (mode == 2) hipLaunchKernelGGL(k_app<2>, dim3(WG), dim3(T), 0, 0, cnt, pool, (uint32_t)r);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%-7s %.2f us per launch (%u events)\n", names[mode], ms * 1e3 / N, WG * EV);
        }
    }
    CK(hipFree(cnt));
    CK(hipFree(pool));
    return 0;
}
