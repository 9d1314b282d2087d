// Microbenchmark for a k_scatter design question: does the gather role's
// scatter of due events into their host partitions finish sooner when the
// workgroup first groups its records by partition in LDS and then stores each
// partition's run with consecutive lanes (coalesced), instead of every lane
// storing its own record at its own slot (one cache line per lane)?
// Shape of configs[3]'s gather: 128 workgroups x 512 lanes, 3072 records each
// (three 1024-event chunks), 256 partitions, one reservation per (workgroup,
// partition) by a returning atomic, as in gather_role.
//   direct : slot = base[p] + LDS rank; each lane stores its records
//   noatomic: direct, the reservation replaced by a fixed base (no global atomic)
//   nostore: direct without the stores (loads, LDS work, reservations only)
//   lines  : runs padded to whole 128-B lines, staged, one line per 8 lanes
//   staged1: the same staging without the padding (one pass, no halves)
//   odd / engine / engodd / odd8: direct with partition strides of 8192 + 64,
//            126976 (configs[3]'s CAPP), 126976 + 72, 8192 + 8 records
//   contig : each workgroup's records stored lane-consecutively into its own region
//   staged : records into LDS grouped by partition (local scan), then lane i
//            stores staged record i (two halves of 1536 to fit the LDS)
// Build: hipcc --offload-arch=gfx950 -O3 tools/scatter_bench.hip -o tools/scatter_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr uint32_t T = 512, WG = 128, NREC = 3072, P = 256, CAPP = 8192, GR = NREC / T;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(T) void k_sc(const uint4* src, uint4* part, uint32_t* pcnt, uint32_t round,
                                          uint32_t stride = CAPP) {
    __shared__ uint32_t s_cnt[P], s_cur[P], s_loc[P];
    __shared__ uint4 s_rec[NREC / 2];
    __shared__ uint32_t s_idx[NREC / 2];
    __shared__ uint32_t s_sum[T / 64];
    const uint32_t tid = threadIdx.x;
    uint4 r[GR];
    uint32_t pp[GR];
#pragma unroll
    for (uint32_t q = 0; q < GR; ++q) {
        r[q] = src[(size_t)blockIdx.x * NREC + tid + q * T];
        pp[q] = mix(r[q].x + round) & (P - 1);
    }
    for (uint32_t p = tid; p < P; p += T) {
        s_cnt[p] = 0;
        s_cur[p] = 0;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < GR; ++q) atomicAdd(&s_cnt[pp[q]], 1u);
    __syncthreads();
    // one reservation per partition (the slots wrap inside the partition's region)
    for (uint32_t p = tid; p < P; p += T) {
        const uint32_t c = s_cnt[p];
        s_loc[p] = c;
        if (c) s_cnt[p] = MODE == 2 ? blockIdx.x * 24u : atomicAdd(&pcnt[p], c);
    }
    __syncthreads();
    if (MODE == 6) {  // contiguous: the workgroup's records to its own region, lane-consecutive
#pragma unroll
        for (uint32_t q = 0; q < GR; ++q) {
            const uint32_t p = pp[q], slot = (s_cnt[p] + atomicAdd(&s_cur[p], 1u)) & (CAPP - 1);
            r[q].w ^= slot;
            part[(size_t)blockIdx.x * NREC + tid + q * T] = r[q];
        }
    } else if (MODE == 0 || MODE == 2 || MODE == 3) {
        uint32_t acc = 0;
#pragma unroll
        for (uint32_t q = 0; q < GR; ++q) {
            const uint32_t p = pp[q], slot = (s_cnt[p] + atomicAdd(&s_cur[p], 1u)) & (CAPP - 1);
            if (MODE == 3) acc += slot ^ r[q].y;
            else part[(size_t)p * stride + slot] = r[q];
        }
        if (MODE == 3 && acc == 0x12345678u) part[tid] = r[0];
    } else {
        // two halves: q < GR/2, then the rest; per half, local counts, a scan,
        // records grouped by partition in LDS, then lane i stores record i
        for (uint32_t h = 0; h < 2; ++h) {
            for (uint32_t p = tid; p < P; p += T) s_loc[p] = 0;
            __syncthreads();
#pragma unroll
            for (uint32_t q = h * GR / 2; q < (h + 1) * GR / 2; ++q) atomicAdd(&s_loc[pp[q]], 1u);
            __syncthreads();
            // exclusive scan of s_loc (P <= T: one entry per lane)
            const uint32_t c = tid < P ? s_loc[tid] : 0u;
            uint32_t x = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if ((tid & 63) >= (uint32_t)o) x += y;
            }
            if ((tid & 63) == 63) s_sum[tid >> 6] = x;
            __syncthreads();
            uint32_t pre = 0;
            for (uint32_t w = 0; w < (tid >> 6); ++w) pre += s_sum[w];
            if (tid < P) s_loc[tid] = pre + x - c;
            __syncthreads();
#pragma unroll
            for (uint32_t q = h * GR / 2; q < (h + 1) * GR / 2; ++q) {
                const uint32_t p = pp[q];
                const uint32_t rk = atomicAdd(&s_cur[p], 1u);
                const uint32_t slot = (s_cnt[p] + rk) & (CAPP - 1);
                const uint32_t l = atomicAdd(&s_loc[p], 1u);
                s_rec[l] = r[q];
                s_idx[l] = p * CAPP + slot;
            }
            __syncthreads();
            for (uint32_t i = tid; i < NREC / 2; i += T) part[s_idx[i]] = s_rec[i];
            __syncthreads();
        }
    }
}

// MODE 4: every (workgroup, partition) run padded to whole 128-B lines (8
// records), staged in LDS, lane i storing staged record i: every line written
// whole by one store instruction.  MODE 5: the same staging, no padding.
template <int MODE>
__global__ __launch_bounds__(T) void k_sc2(const uint4* src, uint4* part, uint32_t* pcnt, uint32_t round) {
    constexpr uint32_t SMAX = NREC + P * 7;
    __shared__ uint32_t s_cnt[P], s_loc[P], s_base[P];
    __shared__ uint4 s_rec[SMAX];
    __shared__ uint32_t s_sum[T / 64], s_tot;
    const uint32_t tid = threadIdx.x;
    uint4 r[GR];
    uint32_t pp[GR];
#pragma unroll
    for (uint32_t q = 0; q < GR; ++q) {
        r[q] = src[(size_t)blockIdx.x * NREC + tid + q * T];
        pp[q] = mix(r[q].x + round) & (P - 1);
    }
    for (uint32_t p = tid; p < P; p += T) s_cnt[p] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < GR; ++q) atomicAdd(&s_cnt[pp[q]], 1u);
    __syncthreads();
    const uint32_t c = tid < P ? s_cnt[tid] : 0u;
    const uint32_t cp = MODE == 4 ? (c + 7) & ~7u : c;
    if (tid < P && cp) s_base[tid] = atomicAdd(&pcnt[tid], cp);
    uint32_t x = cp;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((tid & 63) >= (uint32_t)o) x += y;
    }
    if ((tid & 63) == 63) s_sum[tid >> 6] = x;
    __syncthreads();
    uint32_t pre = 0;
    for (uint32_t w = 0; w < (tid >> 6); ++w) pre += s_sum[w];
    if (tid == T - 1) s_tot = pre + x;
    if (tid < P) s_loc[tid] = pre + x - cp;
    // pads: the run's tail entries past its count
    if (tid < P)
        for (uint32_t k = c; k < cp; ++k) s_rec[pre + x - cp + k] = make_uint4(0xFFFFFFFFu, 0, 0, 0);
    __syncthreads();
    uint32_t l[GR];
#pragma unroll
    for (uint32_t q = 0; q < GR; ++q) l[q] = atomicAdd(&s_loc[pp[q]], 1u);
#pragma unroll
    for (uint32_t q = 0; q < GR; ++q) s_rec[l[q]] = r[q];
    __syncthreads();
    // s_loc[p] is now the run's end (start + count): find each staged entry's run by its partition
    const uint32_t tot = s_tot;
    for (uint32_t i = tid; i < tot; i += T) {
        // binary search: the last partition whose run starts at or before i
        uint32_t lo = 0, hi = P - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            const uint32_t st = s_loc[mid] - s_cnt[mid];  // run start (count, not padded, consumed)
            if (st <= i) lo = mid; else hi = mid - 1;
        }
        (void)lo;
        const uint32_t p = lo, start = s_loc[p] - s_cnt[p];
        const uint32_t slot = (s_base[p] + (i - start)) & (CAPP - 1);
        part[(size_t)p * CAPP + slot] = s_rec[i];
    }
}

int main() {
    uint4 *src, *part;
    uint32_t* pcnt;
    CK(hipMalloc(&src, (size_t)WG * NREC * 16));
    CK(hipMalloc(&part, (size_t)P * 126976 * 16));
    CK(hipMalloc(&pcnt, P * 4));
    CK(hipMemset(src, 0, (size_t)WG * NREC * 16));
    CK(hipMemset(pcnt, 0, P * 4));
    hipLaunchKernelGGL(k_sc<0>, dim3(1), dim3(1), 0, 0, src, part, pcnt, 0u);  // warm the code object
    uint32_t* h = (uint32_t*)malloc((size_t)WG * NREC * 16);
    for (size_t i = 0; i < (size_t)WG * NREC * 4; ++i) h[i] = (uint32_t)(i * 2654435761u);
    CK(hipMemcpy(src, h, (size_t)WG * NREC * 16, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto launch = [&](int mode, int w) {
        if (mode == 0) hipLaunchKernelGGL(k_sc<0>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w);
        if (mode == 1) hipLaunchKernelGGL(k_sc<1>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w);
        if (mode == 2) hipLaunchKernelGGL(k_sc<2>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w);
        if (mode == 3) hipLaunchKernelGGL(k_sc<3>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w);
        if (mode == 7) hipLaunchKernelGGL(k_sc<0>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w, CAPP + 64);
        if (mode == 8) hipLaunchKernelGGL(k_sc<0>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w, 126976u);
        if (mode == 9) hipLaunchKernelGGL(k_sc<0>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w, 126976u + 72);
        if (mode == 10) hipLaunchKernelGGL(k_sc<0>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w, 8192u + 8);
        if (mode == 6) hipLaunchKernelGGL(k_sc<6>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w);
        if (mode == 4) hipLaunchKernelGGL(k_sc2<4>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w);
        if (mode == 5) hipLaunchKernelGGL(k_sc2<5>, dim3(WG), dim3(T), 0, 0, src, part, pcnt, (uint32_t)w);
    };
    const char* names[11] = {"direct", "staged", "noatomic", "nostore", "lines", "staged1", "contig", "odd", "engine", "engodd", "odd8"};
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 11; ++mode) {
            const int N = 200;
            for (int w = 0; w < 20; ++w) {
                launch(mode, w);
            }
            CK(hipEventRecord(a));
            for (int i = 0; i < N; ++i) {
                launch(mode, i);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%-7s %.2f us per launch (%u records)\n", names[mode], ms * 1e3 / N, WG * NREC);
        }
    CK(hipFree(src));
    CK(hipFree(part));
    CK(hipFree(pcnt));
    free(h);
    return 0;
}
