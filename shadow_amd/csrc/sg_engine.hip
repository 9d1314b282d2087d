// sg_engine.hip — MI355X (gfx950) device engine of libshadowgpu.
//
// One conservative round of Shadow's host-family scheduler on HBM-resident
// per-host queues (contract: include/shadowgpu.h; design: DESIGN.md):
//
//   k_process  one lane per host. Pops every queued event with time < barrier in
//              event_compare order (core/work/event.c:110-153) — self events it
//              creates inside the window included (host_single.c:237-267) — and
//              runs the PHOLD body: destination draw (test_phold.c:160-178),
//              reliability draw + ceil delay (worker.c:243-304), srcHostEventID
//              (event.c:38), endTime drop (scheduler.c:343), barrier bump
//              (host_single.c:180-184). New events are staged per workgroup.
//   k_pack     (multi-shard) moves staged events owned by other shards into the
//              per-peer outbox for the RCCL all-to-all.
//   k_insert   delivers staged / received events into destination queues and
//              maintains each host's and each 256-host block's minimum time.
//   k_reduce   MIN next event time (host_single.c:273-305, scheduler.c:393-398)
//              and the minimum discovered latency (topology.c:1374-1385).
//   k_window   master_slaveFinishedCurrentRound (master.c:450-480).
//
// Queue layout: slot-major SoA, slot j of local host h at [j * L + h], so lanes
// of a wave (consecutive hosts) read consecutive addresses.  Compiled with
// -ffp-contract=off: the only FP is the FP64 destination rule, which must round
// exactly as the reference does.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "shadowgpu.h"

extern "C" void sg_set_error(const char* fmt, ...);

namespace {

constexpr int BLOCK = 256;
constexpr int MAXG = 64;  // max shards
constexpr uint64_t SIMTIME_MAX = UINT64_MAX - 1;

enum Ctr {
    C_POPS = 0, C_BOOTS, C_SENDS, C_NULL, C_DROPREL, C_DROPEND, C_BUMPED, C_SAME,
    C_ACTIVE, C_EMIT, NCTR
};
constexpr int NPART = NCTR + 1;  // + jmin

struct RoundState {
    uint64_t S, E, done, rounds;
    uint64_t min_jump, next_min_jump, jmin;
    uint64_t overflow;
    uint64_t trace_len;
    uint64_t ctr[NCTR];
    uint64_t last_min;
};

struct Dev {
    // configuration
    uint32_t N, V, L, lo, CAP, load, dst_rule, window_rule, G, g, nblocks, bcap;
    uint64_t end_time, bootstrap_end, fixed_jump, runahead_min, trace_cap, xcap;
    uint32_t bounds[MAXG + 1];
    // tables
    const uint32_t* vertex;   // [N]
    const int32_t* wthresh;   // [N]
    const uint64_t* delay;    // [V*V]
    const int32_t* keep;      // [V*V]
    const uint32_t* jump;     // [V*V]
    // per local host
    uint64_t* bag_time;       // [CAP*L]
    uint64_t* bag_seq;        // [CAP*L]
    uint32_t* bag_src;        // [CAP*L]
    uint32_t* bag_cnt;        // [L]
    uint64_t* hmin;           // [L]
    uint32_t* rng;            // [L]
    uint64_t* evc;            // [L]
    uint64_t* pops;           // [L]
    uint64_t* digest;         // [L]
    // per 256-host block
    uint64_t* blockmin;       // [nblocks]
    uint64_t* part;           // [nblocks][NPART]
    uint32_t* blockcnt;       // [nblocks] staged events
    uint32_t* peercnt;        // [nblocks][G]
    uint32_t* peeroff;        // [nblocks][G]
    // staging (per block region of bcap events)
    uint64_t* st_time;
    uint64_t* st_seq;
    uint32_t* st_dst;
    uint32_t* st_src;
    // trace
    sg_trace_rec* trace;
    RoundState* rs;
    uint64_t* red3;           // local reduce output {min, jmin, ~overflow}
};

__device__ __forceinline__ int32_t dev_rand_r(uint32_t& state) {
    // glibc rand_r, utility/random.c:32-37
    uint32_t next = state;
    uint32_t result;
    next = next * 1103515245u + 12345u;
    result = (next >> 16) % 2048u;
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (next >> 16) % 1024u;
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (next >> 16) % 1024u;
    state = next;
    return (int32_t)result;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t z) {
    z ^= z >> 33;
    z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33;
    z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}

// Per-host trace digest term (order-sensitive through pos); same as the oracle.
__device__ __forceinline__ uint64_t digest_mix(uint64_t pos, uint64_t t, uint32_t src, uint64_t seq) {
    uint64_t z = fmix64(pos + 0x9E3779B97F4A7C15ULL);
    z = fmix64(z ^ t);
    z = fmix64(z ^ (uint64_t)src);
    return fmix64(z ^ seq);
}

// Destination draw. Returns N when no host is selected (test_phold.c:176-177).
__device__ __forceinline__ uint32_t choose_dst(const Dev& d, int32_t x) {
    const uint32_t N = d.N;
    if (d.dst_rule == SG_DST_UNIFORM_FLOOR) {
        double r = (double)x / 2147483647.0;
        double f = floor(r * (double)N);
        uint32_t dd = (uint32_t)f;
        return dd >= N ? N - 1 : dd;
    }
    // first i with x <= wthresh[i] (non-decreasing): guess from the uniform
    // position, walk a few steps, bisect the rest.
    const int32_t* w = d.wthresh;
    if (x > w[N - 1]) return N;
    uint32_t g = (uint32_t)(((uint64_t)(uint32_t)x * N) >> 31);
    if (g >= N) g = N - 1;
    if (x <= w[g]) {
        for (int k = 0; k < 8; ++k) {
            if (g == 0 || x > w[g - 1]) return g;
            --g;
        }
        uint32_t lo = 0, hi = g;  // answer in [lo, hi]
        while (lo < hi) {
            uint32_t mid = lo + (hi - lo) / 2;
            if (x <= w[mid]) hi = mid; else lo = mid + 1;
        }
        return lo;
    }
    for (int k = 0; k < 8; ++k) {
        ++g;
        if (x <= w[g]) return g;
    }
    uint32_t lo = g + 1, hi = N - 1;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (x <= w[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}

__device__ __forceinline__ uint32_t owner_of(const Dev& d, uint32_t h) {
    uint32_t p = 0;
    while (p + 1 < d.G && h >= d.bounds[p + 1]) ++p;
    return p;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

__global__ void k_boot(Dev d) {
    const uint32_t lh = blockIdx.x * BLOCK + threadIdx.x;
    if (lh < d.L) {
        const uint32_t h = d.lo + lh;
        // worker_bootHosts: self event at t=0 carrying id 0 (event.c:38)
        d.bag_time[lh] = 0;
        d.bag_seq[lh] = 0;
        d.bag_src[lh] = h;
        d.bag_cnt[lh] = 1;
        d.hmin[lh] = 0;
        d.evc[lh] = 1;
        d.pops[lh] = 0;
        d.digest[lh] = 0;
    }
    if (threadIdx.x == 0) d.blockmin[blockIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        RoundState* rs = d.rs;
        rs->S = 0;  // slave.c:431
        rs->E = 1;
        rs->done = 0;
        rs->rounds = 0;
        rs->min_jump = 0;
        rs->next_min_jump = d.window_rule == SG_WINDOW_FIXED ? d.fixed_jump : 0;
        rs->jmin = UINT64_MAX;
        rs->overflow = 0;
        rs->trace_len = 0;
        for (int i = 0; i < NCTR; ++i) rs->ctr[i] = 0;
        rs->last_min = 0;
    }
}

__global__ __launch_bounds__(BLOCK) void k_process(Dev d) {
    __shared__ uint32_t s_emit;
    __shared__ uint32_t s_peer[MAXG];
    __shared__ uint64_t s_red[BLOCK / 64][NPART + 1];
    const RoundState* rs = d.rs;
    if (rs->done) return;
    const uint64_t E = rs->E;
    const uint32_t lh = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t L = d.L;
    if (threadIdx.x == 0) s_emit = 0;
    if (threadIdx.x < MAXG) s_peer[threadIdx.x] = 0;
    __syncthreads();

    uint64_t ctr[NCTR];
#pragma unroll
    for (int i = 0; i < NCTR; ++i) ctr[i] = 0;
    uint64_t jmin = UINT64_MAX;
    uint64_t newmin = SIMTIME_MAX;
    bool overflow = false;

    if (lh < L) {
        const uint64_t hm = d.hmin[lh];
        newmin = hm;
        if (hm < E) {
            const uint32_t h = d.lo + lh;
            const uint32_t vh = d.vertex[h];
            uint32_t cnt = d.bag_cnt[lh];
            uint32_t rng = d.rng[lh];
            uint64_t ev = d.evc[lh];
            uint64_t pops = d.pops[lh];
            uint64_t dig = d.digest[lh];
            ctr[C_ACTIVE] = 1;
            const uint64_t base_bstride = L;
            for (;;) {
                // select the event_compare-minimum queued event before the barrier
                int best = -1;
                uint64_t bt = 0, bq = 0;
                uint32_t bs = 0;
                uint64_t rest_min = SIMTIME_MAX;
                for (uint32_t j = 0; j < cnt; ++j) {
                    const size_t k = (size_t)j * base_bstride + lh;
                    const uint64_t t = d.bag_time[k];
                    if (t < E) {
                        if (best < 0 || t <= bt) {
                            const uint32_t s = d.bag_src[k];
                            const uint64_t q = d.bag_seq[k];
                            if (best < 0 || t < bt || s < bs || (s == bs && q < bq)) {
                                best = (int)j;
                                bt = t;
                                bs = s;
                                bq = q;
                            }
                        }
                    } else if (t < rest_min) {
                        rest_min = t;
                    }
                }
                if (best < 0) {
                    newmin = rest_min;
                    break;
                }
                // remove: last slot fills the hole
                --cnt;
                if ((uint32_t)best != cnt) {
                    const size_t kb = (size_t)best * base_bstride + lh;
                    const size_t kl = (size_t)cnt * base_bstride + lh;
                    d.bag_time[kb] = d.bag_time[kl];
                    d.bag_seq[kb] = d.bag_seq[kl];
                    d.bag_src[kb] = d.bag_src[kl];
                }
                // execute the event (worker.c:165-176)
                dig += digest_mix(pops, bt, bs, bq);
                if (d.trace) {
                    const uint64_t ts = atomicAdd((unsigned long long*)&d.rs->trace_len, 1ULL);
                    if (ts < d.trace_cap) {
                        sg_trace_rec r;
                        r.time = bt;
                        r.seq = bq;
                        r.host = h;
                        r.src = bs;
                        r.pos = pops;
                        d.trace[ts] = r;
                    } else {
                        overflow = true;
                    }
                }
                ++pops;
                ++ctr[C_POPS];
                const bool boot = (bs == h && bq == 0);
                ctr[C_BOOTS] += boot;
                const uint32_t nsend = boot ? d.load : 1u;
                for (uint32_t m = 0; m < nsend; ++m) {
                    const int32_t x = dev_rand_r(rng);
                    const uint32_t dst = choose_dst(d, x);
                    if (dst >= d.N) {
                        ++ctr[C_NULL];
                        continue;
                    }
                    ++ctr[C_SENDS];
                    const size_t pair = (size_t)vh * d.V + d.vertex[dst];
                    const uint64_t jm = d.jump[pair];
                    jmin = jm < jmin ? jm : jmin;
                    const int32_t c = dev_rand_r(rng);
                    if (!(bt < d.bootstrap_end || c <= d.keep[pair])) {
                        ++ctr[C_DROPREL];
                        continue;
                    }
                    uint64_t tn = bt + d.delay[pair];
                    const uint64_t sq = ev++;
                    if (tn >= d.end_time) {  // scheduler.c:343-346
                        ++ctr[C_DROPEND];
                        continue;
                    }
                    if (dst == h && tn < E) {
                        // self event inside the window: popped later this round
                        ++ctr[C_SAME];
                        if (cnt >= d.CAP) {
                            overflow = true;
                            continue;
                        }
                        const size_t kn = (size_t)cnt * base_bstride + lh;
                        d.bag_time[kn] = tn;
                        d.bag_seq[kn] = sq;
                        d.bag_src[kn] = h;
                        ++cnt;
                        continue;
                    }
                    if (dst != h && tn < E) {  // host_single.c:180-184
                        tn = E;
                        ++ctr[C_BUMPED];
                    }
                    const uint32_t slot = atomicAdd(&s_emit, 1u);
                    if (slot >= d.bcap) {
                        overflow = true;
                        continue;
                    }
                    const size_t so = (size_t)blockIdx.x * d.bcap + slot;
                    d.st_time[so] = tn;
                    d.st_seq[so] = sq;
                    d.st_dst[so] = dst;
                    d.st_src[so] = h;
                    if (d.G > 1) atomicAdd(&s_peer[owner_of(d, dst)], 1u);
                    ++ctr[C_EMIT];
                }
            }
            d.bag_cnt[lh] = cnt;
            d.rng[lh] = rng;
            d.evc[lh] = ev;
            d.pops[lh] = pops;
            d.digest[lh] = dig;
            d.hmin[lh] = newmin;
        }
    }

    // block reductions: min next time, discovery min, counters
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t m = wave_min(newmin);
    uint64_t jm = wave_min(jmin);
    uint64_t vals[NCTR];
#pragma unroll
    for (int i = 0; i < NCTR; ++i) vals[i] = wave_sum(ctr[i]);
    if (lane == 0) {
        s_red[wid][0] = m;
        s_red[wid][1] = jm;
#pragma unroll
        for (int i = 0; i < NCTR; ++i) s_red[wid][2 + i] = vals[i];
    }
    if (overflow) atomicOr((unsigned long long*)&d.rs->overflow, 1ULL);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t bm = s_red[0][0], bj = s_red[0][1];
        uint64_t acc[NCTR];
        for (int i = 0; i < NCTR; ++i) acc[i] = s_red[0][2 + i];
        for (int w = 1; w < BLOCK / 64; ++w) {
            bm = s_red[w][0] < bm ? s_red[w][0] : bm;
            bj = s_red[w][1] < bj ? s_red[w][1] : bj;
            for (int i = 0; i < NCTR; ++i) acc[i] += s_red[w][2 + i];
        }
        d.blockmin[blockIdx.x] = bm;
        uint64_t* p = d.part + (size_t)blockIdx.x * NPART;
        for (int i = 0; i < NCTR; ++i) p[i] = acc[i];
        p[NCTR] = bj;
        const uint32_t ne = s_emit < d.bcap ? s_emit : d.bcap;
        d.blockcnt[blockIdx.x] = ne;
    }
    if (d.G > 1 && threadIdx.x < d.G) d.peercnt[(size_t)blockIdx.x * d.G + threadIdx.x] = s_peer[threadIdx.x];
}

// Multi-shard: exclusive prefix of per-block peer counts (one workgroup).
__global__ void k_peer_scan(Dev d, int64_t* send_counts) {
    if (d.rs->done) return;
    __shared__ uint64_t s_tot[MAXG];
    const uint32_t p = threadIdx.x;
    if (p < d.G) {
        uint64_t run = 0;
        for (uint32_t b = 0; b < d.nblocks; ++b) {
            const size_t k = (size_t)b * d.G + p;
            d.peeroff[k] = (uint32_t)run;
            run += d.peercnt[k];
        }
        s_tot[p] = run;
        send_counts[p] = p == d.g ? 0 : (int64_t)(run < d.xcap ? run : d.xcap);
        if (p != d.g && run > d.xcap) atomicOr((unsigned long long*)&d.rs->overflow, 2ULL);
    }
}

// Multi-shard: staged events for other shards → outbox triples.
__global__ __launch_bounds__(BLOCK) void k_pack(Dev d, int64_t* send) {
    if (d.rs->done) return;
    __shared__ uint32_t s_slot[MAXG];
    if (threadIdx.x < MAXG) s_slot[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t b = blockIdx.x;
    const uint32_t n = d.blockcnt[b];
    for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
        const size_t so = (size_t)b * d.bcap + i;
        const uint32_t dst = d.st_dst[so];
        const uint32_t p = owner_of(d, dst);
        if (p == d.g) continue;
        const uint64_t slot = (uint64_t)d.peeroff[(size_t)b * d.G + p] + atomicAdd(&s_slot[p], 1u);
        if (slot >= d.xcap) continue;  // flagged by k_peer_scan
        int64_t* o = send + ((size_t)p * d.xcap + slot) * 3;
        o[0] = (int64_t)d.st_time[so];
        o[1] = (int64_t)d.st_seq[so];
        o[2] = (int64_t)(((uint64_t)dst << 32) | d.st_src[so]);
    }
}

__device__ __forceinline__ void deliver(const Dev& d, uint64_t t, uint64_t seq, uint32_t dst, uint32_t src) {
    const uint32_t dl = dst - d.lo;
    const uint32_t slot = atomicAdd(&d.bag_cnt[dl], 1u);
    if (slot >= d.CAP) {
        atomicOr((unsigned long long*)&d.rs->overflow, 4ULL);
        return;
    }
    const size_t k = (size_t)slot * d.L + dl;
    d.bag_time[k] = t;
    d.bag_seq[k] = seq;
    d.bag_src[k] = src;
    atomicMin((unsigned long long*)&d.hmin[dl], (unsigned long long)t);
    atomicMin((unsigned long long*)&d.blockmin[dl / BLOCK], (unsigned long long)t);
}

// Staged events of this shard's own hosts → destination queues.
__global__ __launch_bounds__(BLOCK) void k_insert(Dev d) {
    if (d.rs->done) return;
    const uint32_t b = blockIdx.x;
    const uint32_t n = d.blockcnt[b];
    for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
        const size_t so = (size_t)b * d.bcap + i;
        const uint32_t dst = d.st_dst[so];
        if (dst - d.lo >= d.L) continue;  // another shard's host
        deliver(d, d.st_time[so], d.st_seq[so], dst, d.st_src[so]);
    }
}

// Received triples → destination queues.
__global__ __launch_bounds__(BLOCK) void k_insert_recv(Dev d, const int64_t* recv, uint64_t n) {
    if (d.rs->done) return;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const int64_t* r = recv + i * 3;
        const uint64_t w = (uint64_t)r[2];
        const uint32_t dst = (uint32_t)(w >> 32);
        if (dst - d.lo >= d.L) {
            atomicOr((unsigned long long*)&d.rs->overflow, 8ULL);
            continue;
        }
        deliver(d, (uint64_t)r[0], (uint64_t)r[1], dst, (uint32_t)(w & 0xffffffffu));
    }
}

// Local MIN next time / discovery min / counters (one workgroup of 1024).
__global__ __launch_bounds__(1024) void k_reduce(Dev d, uint64_t* out3) {
    if (d.rs->done) return;
    __shared__ uint64_t s_m[16], s_j[16], s_c[16][NCTR];
    uint64_t m = SIMTIME_MAX, j = UINT64_MAX, c[NCTR];
    for (int i = 0; i < NCTR; ++i) c[i] = 0;
    for (uint32_t b = threadIdx.x; b < d.nblocks; b += 1024) {
        const uint64_t bm = d.blockmin[b];
        m = bm < m ? bm : m;
        const uint64_t* p = d.part + (size_t)b * NPART;
        for (int i = 0; i < NCTR; ++i) c[i] += p[i];
        j = p[NCTR] < j ? p[NCTR] : j;
    }
    m = wave_min(m);
    j = wave_min(j);
    for (int i = 0; i < NCTR; ++i) c[i] = wave_sum(c[i]);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        s_m[wid] = m;
        s_j[wid] = j;
        for (int i = 0; i < NCTR; ++i) s_c[wid][i] = c[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) {
            m = s_m[w] < m ? s_m[w] : m;
            j = s_j[w] < j ? s_j[w] : j;
        }
        m = s_m[0] < m ? s_m[0] : m;
        j = s_j[0] < j ? s_j[0] : j;
        RoundState* rs = d.rs;
        for (int i = 0; i < NCTR; ++i) {
            uint64_t t = 0;
            for (int w = 0; w < 16; ++w) t += s_c[w][i];
            rs->ctr[i] += t;
        }
        j = rs->jmin < j ? rs->jmin : j;
        rs->jmin = j;
        out3[0] = m;
        out3[1] = j;
        out3[2] = ~rs->overflow;
    }
}

// master_slaveFinishedCurrentRound (master.c:450-480) on the reduced triple.
__global__ void k_window(Dev d, const uint64_t* in3) {
    RoundState* rs = d.rs;
    if (rs->done) return;
    const uint64_t minNext = in3[0], jmin = in3[1];
    rs->overflow |= ~in3[2];
    rs->rounds += 1;
    rs->last_min = minNext;
    uint64_t jump;
    if (d.window_rule == SG_WINDOW_FIXED) {
        jump = d.fixed_jump;
    } else {
        if (jmin != UINT64_MAX) rs->next_min_jump = jmin * SG_ONE_MS;  // master.c:153
        rs->min_jump = rs->next_min_jump;                            // master.c:459
        jump = rs->min_jump > 0 ? rs->min_jump : 10 * SG_ONE_MS;     // master.c:137
        if (d.runahead_min > 0 && jump < d.runahead_min) jump = d.runahead_min;
    }
    const uint64_t start = minNext;
    uint64_t end = minNext + jump;
    if (end > d.end_time) end = d.end_time;
    rs->S = start;
    rs->E = end;
    rs->done = start < end ? 0 : 1;
}

__global__ void k_pending(Dev d, unsigned long long* out) {
    uint64_t s = 0;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < d.L; i += gridDim.x * BLOCK) s += d.bag_cnt[i];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)s);
}

}  // namespace

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
struct sg_engine {
    sg_phold_params p;
    Dev d;
    int device;
    hipStream_t stream;
    bool own_stream;
    bool booted;
    std::vector<void*> allocs;
    RoundState* h_rs;  // pinned
    bool timing;
    struct Pair { hipEvent_t a, b; int cls; };
    std::vector<Pair> pending_ev;
    std::vector<hipEvent_t> free_ev;
    double ms[3];
    uint64_t launches[3];
};

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t _e = (x);                                                           \
        if (_e != hipSuccess) {                                                        \
            sg_set_error("%s failed: %s (%s:%d)", #x, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                    \
            return SG_ERR_HIP;                                                         \
        }                                                                              \
    } while (0)

template <typename T>
static int dalloc(sg_engine* e, T** p, size_t n) {
    void* ptr = nullptr;
    if (n == 0) n = 1;
    hipError_t err = hipMalloc(&ptr, n * sizeof(T));
    if (err != hipSuccess) {
        sg_set_error("hipMalloc(%zu bytes) failed: %s", n * sizeof(T), hipGetErrorString(err));
        return SG_ERR_NOMEM;
    }
    e->allocs.push_back(ptr);
    *p = (T*)ptr;
    return SG_OK;
}

static hipEvent_t get_event(sg_engine* e) {
    if (!e->free_ev.empty()) {
        hipEvent_t ev = e->free_ev.back();
        e->free_ev.pop_back();
        return ev;
    }
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return nullptr;
    return ev;
}

template <typename F>
static int timed_launch(sg_engine* e, int cls, F&& launch) {
    hipEvent_t a = nullptr, b = nullptr;
    if (e->timing) {
        a = get_event(e);
        b = get_event(e);
        if (a && b) HIPCHK(hipEventRecord(a, e->stream));
    }
    launch();
    HIPCHK(hipGetLastError());
    if (e->timing && a && b) {
        HIPCHK(hipEventRecord(b, e->stream));
        e->pending_ev.push_back({a, b, cls});
    }
    e->launches[cls]++;
    return SG_OK;
}

static void harvest_timing(sg_engine* e) {
    for (auto& pr : e->pending_ev) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pr.a, pr.b) == hipSuccess) e->ms[pr.cls] += ms;
        e->free_ev.push_back(pr.a);
        e->free_ev.push_back(pr.b);
    }
    e->pending_ev.clear();
}

extern "C" {

int sg_engine_create(const sg_phold_params* params, const sg_phold_tables* t, int device,
                     void* hip_stream, sg_engine** out) {
    if (!params || !t || !out) {
        sg_set_error("sg_engine_create: NULL argument");
        return SG_ERR_INVAL;
    }
    *out = nullptr;
    const sg_phold_params& p = *params;
    const uint32_t G = p.shard_count ? p.shard_count : 1;
    if (p.n_hosts == 0 || p.n_vertices == 0 || G > MAXG || p.shard_index >= G || G > p.n_hosts ||
        !t->host_vertex || !t->host_rng || !t->delay_ns || !t->keep_max || !t->jump_ms ||
        (p.dst_rule == SG_DST_WEIGHTS && !t->weight_thresh) || p.dst_rule > 1 || p.window_rule > 1 ||
        p.load == 0) {
        sg_set_error("sg_engine_create: invalid parameters");
        return SG_ERR_INVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || device < 0 || device >= ndev) {
        sg_set_error("sg_engine_create: no HIP device %d (count %d)", device, ndev);
        return SG_ERR_NODEV;
    }
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        sg_set_error("sg_engine_create: device %d is %s, need gfx950", device, prop.gcnArchName);
        return SG_ERR_NODEV;
    }
    HIPCHK(hipSetDevice(device));

    sg_engine* e = new sg_engine();
    e->p = p;
    e->device = device;
    e->timing = false;
    for (int i = 0; i < 3; ++i) {
        e->ms[i] = 0;
        e->launches[i] = 0;
    }
    Dev& d = e->d;
    memset(&d, 0, sizeof d);
    d.N = p.n_hosts;
    d.V = p.n_vertices;
    d.G = G;
    d.g = p.shard_index;
    for (uint32_t i = 0; i <= G; ++i) d.bounds[i] = (uint32_t)(((uint64_t)i * p.n_hosts) / G);
    d.lo = d.bounds[d.g];
    d.L = d.bounds[d.g + 1] - d.lo;
    d.CAP = p.queue_cap ? p.queue_cap : 64;
    if (d.CAP < p.load) d.CAP = p.load;  // a boot event may queue `load` self events
    d.load = p.load;
    d.dst_rule = p.dst_rule;
    d.window_rule = p.window_rule;
    d.end_time = p.end_time;
    d.bootstrap_end = p.bootstrap_end;
    d.fixed_jump = p.fixed_jump;
    d.runahead_min = p.runahead_min;
    d.trace_cap = p.trace_capacity;
    d.xcap = p.exchange_cap ? p.exchange_cap : 1;
    d.nblocks = (d.L + BLOCK - 1) / BLOCK;
    const uint32_t per_host = d.CAP > d.load ? d.CAP : d.load;
    d.bcap = BLOCK * per_host;
    if (d.L == 0) {
        delete e;
        sg_set_error("sg_engine_create: shard has no hosts");
        return SG_ERR_INVAL;
    }

    int rc = SG_OK;
    const size_t N = d.N, VV = (size_t)d.V * d.V, L = d.L, S = (size_t)d.CAP * L;
    const size_t NB = d.nblocks, ST = (size_t)NB * d.bcap;
#define ALLOC(ptr, n)                                  \
    do {                                               \
        if ((rc = dalloc(e, &(ptr), (n))) != SG_OK) {  \
            sg_engine_destroy(e);                      \
            return rc;                                 \
        }                                              \
    } while (0)
    uint32_t* vtx;
    int32_t* wt;
    uint64_t* dl;
    int32_t* kp;
    uint32_t* jp;
    ALLOC(vtx, N);
    ALLOC(wt, N);
    ALLOC(dl, VV);
    ALLOC(kp, VV);
    ALLOC(jp, VV);
    d.vertex = vtx;
    d.wthresh = wt;
    d.delay = dl;
    d.keep = kp;
    d.jump = jp;
    ALLOC(d.bag_time, S);
    ALLOC(d.bag_seq, S);
    ALLOC(d.bag_src, S);
    ALLOC(d.bag_cnt, L);
    ALLOC(d.hmin, L);
    ALLOC(d.rng, L);
    ALLOC(d.evc, L);
    ALLOC(d.pops, L);
    ALLOC(d.digest, L);
    ALLOC(d.blockmin, NB);
    ALLOC(d.part, NB * NPART);
    ALLOC(d.blockcnt, NB);
    ALLOC(d.peercnt, NB * G);
    ALLOC(d.peeroff, NB * G);
    ALLOC(d.st_time, ST);
    ALLOC(d.st_seq, ST);
    ALLOC(d.st_dst, ST);
    ALLOC(d.st_src, ST);
    ALLOC(d.rs, 1);
    ALLOC(d.red3, 4);
    if (d.trace_cap) ALLOC(d.trace, d.trace_cap);
#undef ALLOC

    if (hip_stream) {
        e->stream = (hipStream_t)hip_stream;
        e->own_stream = false;
    } else {
        if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
            sg_engine_destroy(e);
            sg_set_error("hipStreamCreate failed");
            return SG_ERR_HIP;
        }
        e->own_stream = true;
    }
    if (hipHostMalloc((void**)&e->h_rs, sizeof(RoundState), hipHostMallocDefault) != hipSuccess) {
        e->h_rs = nullptr;
        sg_engine_destroy(e);
        sg_set_error("hipHostMalloc failed");
        return SG_ERR_NOMEM;
    }
    hipError_t err = hipSuccess;
    err = err != hipSuccess ? err : hipMemcpy(vtx, t->host_vertex, N * 4, hipMemcpyHostToDevice);
    if (t->weight_thresh) err = err != hipSuccess ? err : hipMemcpy(wt, t->weight_thresh, N * 4, hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(dl, t->delay_ns, VV * 8, hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(kp, t->keep_max, VV * 4, hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(jp, t->jump_ms, VV * 4, hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(d.rng, t->host_rng + d.lo, L * 4, hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemset(d.rs, 0, sizeof(RoundState));
    if (err != hipSuccess) {
        sg_set_error("table upload failed: %s", hipGetErrorString(err));
        sg_engine_destroy(e);
        return SG_ERR_HIP;
    }
    e->booted = false;
    *out = e;
    return SG_OK;
}

int sg_engine_destroy(sg_engine* e) {
    if (!e) return SG_OK;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (void* p : e->allocs) (void)hipFree(p);
    for (auto& pr : e->pending_ev) {
        (void)hipEventDestroy(pr.a);
        (void)hipEventDestroy(pr.b);
    }
    for (auto ev : e->free_ev) (void)hipEventDestroy(ev);
    if (e->h_rs) (void)hipHostFree(e->h_rs);
    if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return SG_OK;
}

void* sg_engine_stream(sg_engine* e) { return e ? (void*)e->stream : nullptr; }

int sg_engine_host_range(sg_engine* e, uint32_t* first_host, uint32_t* n_local) {
    if (!e) return SG_ERR_INVAL;
    if (first_host) *first_host = e->d.lo;
    if (n_local) *n_local = e->d.L;
    return SG_OK;
}

int sg_engine_boot(sg_engine* e) {
    if (!e) return SG_ERR_INVAL;
    if (e->booted) {
        sg_set_error("sg_engine_boot: already booted");
        return SG_ERR_STATE;
    }
    HIPCHK(hipSetDevice(e->device));
    Dev d = e->d;
    hipLaunchKernelGGL(k_boot, dim3(d.nblocks), dim3(BLOCK), 0, e->stream, d);
    HIPCHK(hipGetLastError());
    e->booted = true;
    return SG_OK;
}

static int enqueue_process(sg_engine* e) {
    const Dev& d = e->d;
    return timed_launch(e, 0, [&] {
        hipLaunchKernelGGL(k_process, dim3(d.nblocks), dim3(BLOCK), 0, e->stream, d);
    });
}

static int enqueue_local_insert(sg_engine* e) {
    const Dev& d = e->d;
    return timed_launch(e, 1, [&] {
        hipLaunchKernelGGL(k_insert, dim3(d.nblocks), dim3(BLOCK), 0, e->stream, d);
    });
}

int sg_engine_enqueue_round(sg_engine* e) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_enqueue_round: engine not booted");
        return SG_ERR_STATE;
    }
    if (e->d.G != 1) {
        sg_set_error("sg_engine_enqueue_round: sharded engine, use the step API");
        return SG_ERR_STATE;
    }
    int rc;
    if ((rc = enqueue_process(e))) return rc;
    if ((rc = enqueue_local_insert(e))) return rc;
    const Dev& d = e->d;
    return timed_launch(e, 2, [&] {
        hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, e->stream, d, d.red3);
        hipLaunchKernelGGL(k_window, dim3(1), dim3(1), 0, e->stream, d, (const uint64_t*)d.red3);
    });
}

int sg_engine_sync(sg_engine* e) {
    if (!e) return SG_ERR_INVAL;
    HIPCHK(hipStreamSynchronize(e->stream));
    if (e->timing) harvest_timing(e);
    return SG_OK;
}

static int read_rs(sg_engine* e) {
    HIPCHK(hipMemcpyAsync(e->h_rs, e->d.rs, sizeof(RoundState), hipMemcpyDeviceToHost, e->stream));
    return sg_engine_sync(e);
}

int sg_engine_run(sg_engine* e, uint64_t max_rounds, uint32_t batch) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_run: engine not booted");
        return SG_ERR_STATE;
    }
    if (batch == 0) batch = 16;
    int rc = read_rs(e);
    if (rc) return rc;
    uint64_t done_rounds = 0;
    while (done_rounds < max_rounds && !e->h_rs->done) {
        uint64_t n = max_rounds - done_rounds;
        if (n > batch) n = batch;
        for (uint64_t i = 0; i < n; ++i)
            if ((rc = sg_engine_enqueue_round(e))) return rc;
        done_rounds += n;
        if ((rc = read_rs(e))) return rc;
        if (e->h_rs->overflow) {
            sg_set_error("sg_engine_run: device queue overflow (flags 0x%llx); raise queue_cap",
                         (unsigned long long)e->h_rs->overflow);
            return SG_ERR_OVERFLOW;
        }
    }
    return SG_OK;
}

int sg_engine_stats(sg_engine* e, sg_round_stats* out) {
    if (!e || !out) return SG_ERR_INVAL;
    unsigned long long* dp = (unsigned long long*)e->d.red3 + 3;
    HIPCHK(hipMemsetAsync(dp, 0, 8, e->stream));
    hipLaunchKernelGGL(k_pending, dim3(256), dim3(BLOCK), 0, e->stream, e->d, dp);
    HIPCHK(hipGetLastError());
    uint64_t pend = 0;
    HIPCHK(hipMemcpyAsync(&pend, dp, 8, hipMemcpyDeviceToHost, e->stream));
    int rc = read_rs(e);
    if (rc) return rc;
    const RoundState& r = *e->h_rs;
    memset(out, 0, sizeof *out);
    out->rounds = r.rounds;
    out->pops = r.ctr[C_POPS];
    out->boots = r.ctr[C_BOOTS];
    out->sends = r.ctr[C_SENDS];
    out->null_dst = r.ctr[C_NULL];
    out->drop_reliability = r.ctr[C_DROPREL];
    out->drop_endtime = r.ctr[C_DROPEND];
    out->bumped = r.ctr[C_BUMPED];
    out->same_round = r.ctr[C_SAME];
    out->overflow = r.overflow;
    out->window_start = r.S;
    out->window_end = r.E;
    out->done = r.done;
    out->min_jump = r.min_jump;
    out->next_min_jump = r.next_min_jump;
    out->jmin_ms = r.jmin;
    out->pending = pend;
    out->trace_len = r.trace_len;
    return SG_OK;
}

int sg_engine_active_hosts(sg_engine* e, uint64_t* active, uint64_t* emitted) {
    if (!e) return SG_ERR_INVAL;
    int rc = read_rs(e);
    if (rc) return rc;
    if (active) *active = e->h_rs->ctr[C_ACTIVE];
    if (emitted) *emitted = e->h_rs->ctr[C_EMIT];
    return SG_OK;
}

int sg_engine_host_state(sg_engine* e, uint64_t* digest, uint64_t* pops, uint32_t* rng,
                         uint64_t* event_counter) {
    if (!e) return SG_ERR_INVAL;
    const size_t L = e->d.L;
    if (digest) HIPCHK(hipMemcpyAsync(digest, e->d.digest, L * 8, hipMemcpyDeviceToHost, e->stream));
    if (pops) HIPCHK(hipMemcpyAsync(pops, e->d.pops, L * 8, hipMemcpyDeviceToHost, e->stream));
    if (rng) HIPCHK(hipMemcpyAsync(rng, e->d.rng, L * 4, hipMemcpyDeviceToHost, e->stream));
    if (event_counter) HIPCHK(hipMemcpyAsync(event_counter, e->d.evc, L * 8, hipMemcpyDeviceToHost, e->stream));
    return sg_engine_sync(e);
}

int sg_engine_trace(sg_engine* e, sg_trace_rec* out, uint64_t capacity, uint64_t* n_out) {
    if (!e) return SG_ERR_INVAL;
    int rc = read_rs(e);
    if (rc) return rc;
    uint64_t n = e->h_rs->trace_len;
    if (n > e->d.trace_cap) n = e->d.trace_cap;
    if (n_out) *n_out = n;
    if (out && capacity) {
        uint64_t m = n < capacity ? n : capacity;
        if (m) HIPCHK(hipMemcpy(out, e->d.trace, m * sizeof(sg_trace_rec), hipMemcpyDeviceToHost));
    }
    return SG_OK;
}

int sg_engine_step_process(sg_engine* e, int64_t* send, int64_t* send_counts) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_step_process: engine not booted");
        return SG_ERR_STATE;
    }
    int rc;
    if ((rc = enqueue_process(e))) return rc;
    const Dev& d = e->d;
    if (d.G > 1) {
        if (!send || !send_counts) {
            sg_set_error("sg_engine_step_process: sharded engine needs send buffers");
            return SG_ERR_INVAL;
        }
        hipLaunchKernelGGL(k_peer_scan, dim3(1), dim3(MAXG), 0, e->stream, d, send_counts);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_pack, dim3(d.nblocks), dim3(BLOCK), 0, e->stream, d, send);
        HIPCHK(hipGetLastError());
    }
    return SG_OK;
}

int sg_engine_step_insert(sg_engine* e, const int64_t* recv, uint64_t n_recv) {
    if (!e || !e->booted) return SG_ERR_STATE;
    int rc;
    if ((rc = enqueue_local_insert(e))) return rc;
    if (n_recv) {
        const Dev& d = e->d;
        uint32_t grid = (uint32_t)((n_recv + BLOCK - 1) / BLOCK);
        if (grid > 2048) grid = 2048;
        hipLaunchKernelGGL(k_insert_recv, dim3(grid), dim3(BLOCK), 0, e->stream, d, recv, n_recv);
        HIPCHK(hipGetLastError());
    }
    return SG_OK;
}

int sg_engine_step_reduce(sg_engine* e, uint64_t* out3) {
    if (!e || !out3) return SG_ERR_INVAL;
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, e->stream, e->d, out3);
    HIPCHK(hipGetLastError());
    return SG_OK;
}

int sg_engine_step_window(sg_engine* e, const uint64_t* in3) {
    if (!e || !in3) return SG_ERR_INVAL;
    hipLaunchKernelGGL(k_window, dim3(1), dim3(1), 0, e->stream, e->d, in3);
    HIPCHK(hipGetLastError());
    return SG_OK;
}

int sg_engine_set_timing(sg_engine* e, int enabled) {
    if (!e) return SG_ERR_INVAL;
    e->timing = enabled != 0;
    for (int i = 0; i < 3; ++i) {
        e->ms[i] = 0;
        e->launches[i] = 0;
    }
    return SG_OK;
}

int sg_engine_kernel_times(sg_engine* e, double* ms3, uint64_t* launches) {
    if (!e) return SG_ERR_INVAL;
    int rc = sg_engine_sync(e);
    if (rc) return rc;
    for (int i = 0; i < 3; ++i) {
        if (ms3) ms3[i] = e->ms[i];
        if (launches) launches[i] = e->launches[i];
    }
    return SG_OK;
}

}  // extern "C"
