// sg_policy_dev.hip — device half of the `gpu` SchedulerPolicy (Mode P).
//
// The queued events of every host live in one HBM calendar: a ring of RB time
// buckets of width 2^shift ns (bucket b holds times [b << shift, (b + 1) << shift),
// ring slot b mod RB), each an array of 32-B records spread over fixed-size
// chunks of a shared pool (a per-bucket chunk table, a stack of free chunks).
// Events beyond the ring's horizon, or beyond a bucket's capacity, go to a flat
// "far" list, which is read only when it holds a due event.  So an extraction
// reads the due buckets and nothing else: its cost follows the events of the
// round, not the events queued (host_single.c:210-271 pops every event before
// the barrier, per host in event_compare order).
//
//   insert   k_cins1   slots reserved per (workgroup, bucket) through an LDS
//                      hash (one global atomic per distinct bucket), far
//                      records appended
//            k_cneed   chunks the new slots need; the host grows the pool if
//                      the free stack is short (the one sync of an insert)
//            k_calloc  chunks popped from the free stack into the tables
//            k_cins2   records stored, bucket minima
//   extract  k_xplan   one work item per due chunk (and far piece)
//            k_hist / k_mscan / k_part   level 1 of a two-level host sort:
//                      due records partitioned by host block (4096 hosts)
//                      through per-unit LDS histograms and one scan, no global
//                      atomics; extracted records of the straddling bucket and
//                      the far list tombstoned
//            k_local   level 2, one workgroup per host block: LDS counting
//                      sort by host, the block's run offsets off[]
//            k_xrank   each record ranked in its host's run in event_compare
//                      order (event.c:110-153); runs longer than XR_SHORT
//                      are listed for k_xlong (LDS bitonic sort per run)
//                      (and, on the side, spent buckets reset, their chunks
//                      freed, the straddling bucket's and far list's minima set)
//   MIN      k_cmin    over the RB bucket minima and the far minimum
//                      (host_single.c:273-305)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "sg_policy_dev.h"

extern "C" void sg_set_error(const char* fmt, ...);

namespace {

constexpr int BLOCK = 256;
constexpr uint64_t SIMTIME_MAX = UINT64_MAX - 1;
constexpr uint64_t TOMB = UINT64_MAX;  // an extracted record left in place
constexpr uint32_t CH = 1024;          // records per chunk (32 KB)
constexpr uint32_t RB = 16384;         // ring buckets
constexpr uint32_t FAR = 0xFFFFFFFFu;  // rslot: the record went to the far list
constexpr uint32_t FARBIT = 0x80000000u;
constexpr uint32_t IPW = 4 * BLOCK;    // records per workgroup in k_cins1 / k_cins2
constexpr uint32_t HT = 2048;          // k_cins1 LDS hash entries (load <= 1/2)
constexpr uint32_t XG = 2048;          // grid of the item-driven extraction kernels
constexpr uint32_t PIECE = BLOCK;      // records per workgroup step of an item
constexpr uint32_t PPI = CH / PIECE;   // pieces per item
constexpr uint32_t HB = 12;            // host block = dst >> HB (level 1 of the host sort)
constexpr uint32_t HPB = 1u << HB;     // hosts per block
constexpr uint32_t MAXP2 = 4096;       // host blocks: up to 16M hosts
constexpr uint32_t UI = 4;             // items per level-1 unit (4096 records)
constexpr uint32_t XU = 512;           // grid of the level-1 kernels

struct Scal {
    uint32_t ftop;                 // chunks on the free stack
    uint32_t need;                 // chunks the pending insert needs
    uint32_t nitems;               // work items of the current plan
    uint32_t farscan;              // the plan includes the far list
    unsigned long long nfar;       // far records, tombstones included
    unsigned long long farmin;     // earliest live far time
    unsigned long long farlive;    // live far records
    unsigned long long total;      // records of the current extraction
    unsigned long long smin;       // earliest remaining time of the last due bucket
    unsigned long long fmin;       // earliest remaining far time (scan)
    unsigned long long flive;      // remaining far records (scan)
    unsigned long long pmin[RB / 1024];  // k_cmin's partial minima
    unsigned long long nall;       // k_call's count
    uint32_t nlong;                // runs longer than XR_SHORT (k_xrank lists them for k_xlong)
    uint32_t pad_;
};

// One cache line per bucket: the insert's atomics on neighbouring buckets do
// not queue behind each other.
struct BH {
    uint32_t cnt;      // slots reserved (beyond cap: those went far)
    uint32_t chk;      // chunks attached
    uint64_t min;      // earliest stored time (SIMTIME_MAX: none)
    uint32_t pad[12];
};

struct Cal {
    uint32_t n;        // hosts
    uint32_t shift;    // bucket = time >> shift
    uint32_t nchb;     // chunk-table entries per bucket
    uint32_t cap;      // records per bucket = nchb * CH
    sgp_rec* pool;     // nchunks * CH records
    uint32_t* btab;    // [RB][nchb] chunk ids
    BH* bh;            // [RB]
    uint32_t* fst;     // free chunk stack
    sgp_rec* far;      // far list
    uint4* items;      // plan: {chunk id | FARBIT piece, records, ring slot, last-bucket flag}
    Scal* sc;
};

__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ bool key_less(uint64_t t, uint32_t s, uint64_t q, uint64_t bt, uint32_t bs,
                                         uint64_t bq) {
    // bitwise, not short-circuit (see sg_engine.hip key_less)
    return (t < bt) | ((t == bt) & ((s < bs) | ((s == bs) & (q < bq))));
}

__global__ void k_cinit(Cal c, uint32_t nchunks) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < RB) {
        c.bh[i].cnt = 0;
        c.bh[i].chk = 0;
        c.bh[i].min = SIMTIME_MAX;
    }
    if (i < nchunks) c.fst[i] = i;
}

// Free-stack entries [at, at + k) = chunk ids first.. (a grown pool's new chunks)
__global__ void k_fpush(uint32_t* fst, uint32_t at, uint32_t first, uint32_t k) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < k) fst[at + i] = first + i;
}

// Slots for up to IPW staged records per workgroup: an LDS hash groups them by
// bucket so each distinct bucket costs one global atomic.  Records outside the
// ring [cur, cur + RB) or past their bucket's capacity are appended to the far
// list (the host sized it for every record of this insert).
__global__ __launch_bounds__(BLOCK) void k_cins1(Cal c, uint64_t cur, const sgp_rec* in, uint64_t n,
                                                 uint32_t* rslot) {
    __shared__ unsigned long long s_key[HT];  // bucket + 1, 0 = empty
    __shared__ uint32_t s_cnt[HT];
    __shared__ uint32_t s_base[HT];
    __shared__ unsigned long long s_min[HT];
    __shared__ uint32_t s_nfar;
    __shared__ unsigned long long s_fbase, s_fmin;
    for (uint32_t e = threadIdx.x; e < HT; e += BLOCK) {
        s_key[e] = 0;
        s_cnt[e] = 0;
        s_min[e] = SIMTIME_MAX;
    }
    if (threadIdx.x == 0) {
        s_nfar = 0;
        s_fmin = SIMTIME_MAX;
    }
    __syncthreads();
    const uint64_t i0 = (uint64_t)blockIdx.x * IPW;
    uint32_t ent[4], loc[4];
    uint64_t tim[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = i0 + q * BLOCK + threadIdx.x;
        ent[q] = FAR;
        tim[q] = 0;
        if (i >= n) continue;
        const uint64_t t = in[i].time;
        tim[q] = t;
        const uint64_t b = t >> c.shift;
        if (b < cur || b >= cur + RB) continue;
        uint32_t h = (uint32_t)((b * 0x9E3779B97F4A7C15ull) >> 53) & (HT - 1);
        for (;;) {
            const unsigned long long old = atomicCAS(&s_key[h], 0ull, (unsigned long long)(b + 1));
            if (old == 0 || old == b + 1) break;
            h = (h + 1) & (HT - 1);
        }
        ent[q] = h;
        loc[q] = atomicAdd(&s_cnt[h], 1u);
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < HT; e += BLOCK)
        if (s_key[e]) s_base[e] = atomicAdd(&c.bh[(uint32_t)(s_key[e] - 1) & (RB - 1)].cnt, s_cnt[e]);
    __syncthreads();
    uint32_t fl[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = i0 + q * BLOCK + threadIdx.x;
        fl[q] = 0;
        if (i >= n) continue;
        uint32_t slot = ent[q] == FAR ? FAR : s_base[ent[q]] + loc[q];
        if (slot != FAR && slot >= c.cap) slot = FAR;
        rslot[i] = slot;
        if (slot == FAR) {
            fl[q] = atomicAdd(&s_nfar, 1u) + 1;
            atomicMin(&s_fmin, (unsigned long long)tim[q]);
        } else {
            atomicMin(&s_min[ent[q]], (unsigned long long)tim[q]);  // stored in the bucket
        }
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < HT; e += BLOCK)
        if (s_key[e] && s_min[e] != SIMTIME_MAX)
            atomicMin((unsigned long long*)&c.bh[(uint32_t)(s_key[e] - 1) & (RB - 1)].min, s_min[e]);
    if (threadIdx.x == 0 && s_nfar) {
        s_fbase = atomicAdd(&c.sc->nfar, (unsigned long long)s_nfar);
        atomicAdd(&c.sc->farlive, (unsigned long long)s_nfar);
        atomicMin(&c.sc->farmin, s_fmin);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (!fl[q]) continue;
        const uint64_t i = i0 + q * BLOCK + threadIdx.x;
        c.far[s_fbase + fl[q] - 1] = in[i];
    }
}

__device__ __forceinline__ uint32_t chunks_for(uint32_t cnt, uint32_t cap) {
    const uint32_t m = cnt < cap ? cnt : cap;
    return (m + CH - 1) / CH;
}

__global__ void k_cneed(Cal c) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t k = 0;
    if (s < RB) k = chunks_for(c.bh[s].cnt, c.cap) - c.bh[s].chk;
    k = wave_sum(k);
    if ((threadIdx.x & 63) == 0 && k) atomicAdd(&c.sc->need, (uint32_t)k);
}

__global__ void k_calloc(Cal c) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= RB) return;
    const uint32_t have = c.bh[s].chk, want = chunks_for(c.bh[s].cnt, c.cap);
    if (want <= have) return;
    const uint32_t k = want - have;
    const uint32_t top = atomicSub(&c.sc->ftop, k);  // the host made sure top >= k
    for (uint32_t j = 0; j < k; ++j) c.btab[(size_t)s * c.nchb + have + j] = c.fst[top - k + j];
    c.bh[s].chk = want;
}

// Store the bucket records (their minima were taken in k_cins1).
__global__ __launch_bounds__(BLOCK) void k_cins2(Cal c, const sgp_rec* in, uint64_t n, const uint32_t* rslot) {
    const uint64_t i0 = (uint64_t)blockIdx.x * IPW;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = i0 + q * BLOCK + threadIdx.x;
        const uint32_t slot = i < n ? rslot[i] : FAR;
        if (slot == FAR) continue;
        const sgp_rec r = in[i];
        const uint32_t s = (uint32_t)(r.time >> c.shift) & (RB - 1);
        const uint32_t ch = c.btab[(size_t)s * c.nchb + slot / CH];
        c.pool[(size_t)ch * CH + slot % CH] = r;
    }
}

// Work items for the due buckets [cur, cur + nbk) (ring order) and, when it
// holds a due event (or `all`), the far list.  One workgroup: a scan of the
// buckets' chunk counts, then the items written in parallel (each finds its
// bucket by binary search over the prefix).
__global__ __launch_bounds__(1024) void k_xplan(Cal c, uint64_t cur, uint32_t nbk, uint64_t barrier, int all) {
    __shared__ uint32_t s_sum[1024];
    __shared__ uint32_t s_pre[RB + 1];
    constexpr uint32_t PER = RB / 1024;
    const uint32_t t = threadIdx.x;
    uint32_t nch[PER], tot = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t k = t * PER + j;
        nch[j] = k < nbk ? chunks_for(c.bh[(uint32_t)(cur + k) & (RB - 1)].cnt, c.cap) : 0;
        tot += nch[j];
    }
    s_sum[t] = tot;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint32_t u = t >= o ? s_sum[t - o] : 0;
        __syncthreads();
        s_sum[t] += u;
        __syncthreads();
    }
    uint32_t at = s_sum[t] - tot;
    const uint32_t nbucket_items = s_sum[1023];
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        s_pre[t * PER + j] = at;
        at += nch[j];
    }
    __syncthreads();
    const uint32_t nb = nbk ? nbk : 1;
    for (uint32_t q = t; q < nbucket_items; q += 1024) {
        uint32_t lo = 0, hi = nb - 1;  // last k with s_pre[k] <= q
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_pre[mid] <= q) lo = mid; else hi = mid - 1;
        }
        const uint32_t s = (uint32_t)(cur + lo) & (RB - 1), x = q - s_pre[lo];
        const uint32_t m = c.bh[s].cnt < c.cap ? c.bh[s].cnt : c.cap;
        c.items[q] = make_uint4(c.btab[(size_t)s * c.nchb + x], m - x * CH < CH ? m - x * CH : CH, s, lo + 1 == nbk);
    }
    const unsigned long long nfar = c.sc->nfar;
    const bool farscan = nfar && (all || c.sc->farmin < barrier);
    const uint32_t nfi = farscan ? (uint32_t)((nfar + CH - 1) / CH) : 0;
    for (uint32_t q = t; q < nfi; q += 1024)
        c.items[nbucket_items + q] =
            make_uint4(FARBIT | q, q + 1 < nfi ? CH : (uint32_t)(nfar - (uint64_t)q * CH), RB, 0);
    if (t == 0) {
        c.sc->nitems = nbucket_items + nfi;
        c.sc->farscan = farscan;
        c.sc->smin = SIMTIME_MAX;
        c.sc->fmin = SIMTIME_MAX;
        c.sc->flive = 0;
    }
}

__device__ __forceinline__ const sgp_rec* item_base(const Cal& c, uint4 it) {
    return it.x & FARBIT ? c.far + (size_t)(it.x & ~FARBIT) * CH : c.pool + (size_t)it.x * CH;
}

// Exclusive scan across a 1024-thread workgroup (16 waves); *total = the sum.
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t k = 0; k < 16; ++k) {
        before += k < w ? s_w[k] : 0;
        all += s_w[k];
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

// Level 1 of the host sort: per unit of UI items (UI * CH records), due events
// per host block (HB bits: dst >> HB) into a block-major count matrix
// mat[d * nu + u]; the times that stay give the straddling bucket's and the
// far list's new minima.
__global__ __launch_bounds__(1024) void k_hist(Cal c, uint64_t barrier, uint32_t P2, uint32_t* mat) {
    __shared__ uint32_t s_h[MAXP2];
    const uint32_t t = threadIdx.x, ni = c.sc->nitems, nu = (ni + UI - 1) / UI;
    uint64_t smin = SIMTIME_MAX, fmin = SIMTIME_MAX, flive = 0;
    for (uint32_t u = blockIdx.x; u < nu; u += gridDim.x) {
        for (uint32_t d = t; d < P2; d += 1024) s_h[d] = 0;
        uint64_t tm[UI];
        uint32_t dst[UI];
        bool far[UI];
#pragma unroll
        for (uint32_t k = 0; k < UI; ++k) {  // every load first, then the bins
            const uint32_t j = u * UI + k;
            const uint4 it = j < ni ? c.items[j] : make_uint4(0, 0, 0, 0);
            far[k] = it.x & FARBIT;
            tm[k] = TOMB;
            dst[k] = 0;
            if (t < it.y) {
                const sgp_rec* r = item_base(c, it) + t;
                tm[k] = r->time;
                dst[k] = r->dst;
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < UI; ++k) {
            if (tm[k] < barrier) {
                atomicAdd(&s_h[dst[k] >> HB], 1u);
            } else if (tm[k] != TOMB) {
                if (far[k]) {
                    fmin = tm[k] < fmin ? tm[k] : fmin;
                    ++flive;
                } else {
                    smin = tm[k] < smin ? tm[k] : smin;
                }
            }
        }
        __syncthreads();
        for (uint32_t d = t; d < P2; d += 1024) mat[d * nu + u] = s_h[d];
        __syncthreads();
    }
    smin = wave_min(smin);
    fmin = wave_min(fmin);
    flive = wave_sum(flive);
    if ((t & 63) == 0) {
        if (smin != SIMTIME_MAX) atomicMin(&c.sc->smin, (unsigned long long)smin);
        if (fmin != SIMTIME_MAX) atomicMin(&c.sc->fmin, (unsigned long long)fmin);
        if (flive) atomicAdd(&c.sc->flive, (unsigned long long)flive);
    }
}

// The count matrix scanned in place (it is block-major, so in (block, unit)
// order): mat[d * nu + u] becomes where unit u's events of host block d start;
// pbase[d] = host block d's start.  One workgroup; tiles of 16K entries are
// staged through LDS so global loads and stores stay coalesced.
__global__ __launch_bounds__(1024) void k_mscan(uint32_t* mat, uint32_t P2, const Cal c, uint32_t* pbase) {
    constexpr uint32_t V = 16, TILE = 1024 * V;
    __shared__ uint32_t s_buf[TILE];
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x;
    const uint32_t nu = (c.sc->nitems + UI - 1) / UI;
    const uint32_t E = nu * P2;
    uint32_t carry = 0;
    for (uint32_t x0 = 0; x0 < E; x0 += TILE) {
#pragma unroll
        for (uint32_t k = 0; k < V; ++k) {
            const uint32_t x = x0 + k * 1024 + t;
            s_buf[k * 1024 + t] = x < E ? mat[x] : 0;
        }
        __syncthreads();
        uint32_t v[V], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < V; ++k) {
            v[k] = s_buf[t * V + k];
            sum += v[k];
        }
        uint32_t tot;
        uint32_t at = carry + block_excl(sum, s_w, &tot);  // (its barriers order the reads above)
#pragma unroll
        for (uint32_t k = 0; k < V; ++k) {
            s_buf[t * V + k] = at;
            at += v[k];
        }
        carry += tot;
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < V; ++k) {
            const uint32_t x = x0 + k * 1024 + t;
            if (x < E) {
                mat[x] = s_buf[k * 1024 + t];
                if (x % nu == 0) pbase[x / nu] = s_buf[k * 1024 + t];
            }
        }
        __syncthreads();
    }
    if (nu == 0)
        for (uint32_t d = t; d < P2; d += 1024) pbase[d] = 0;
    if (t == 0) {
        pbase[P2] = carry;
        c.sc->total = carry;
    }
}

// Level 1 scatter: each unit's due events to their host block's range;
// extracted records that stay in place (last due bucket, far list) tombstoned.
__global__ __launch_bounds__(1024) void k_part(Cal c, uint64_t barrier, uint32_t P2, const uint32_t* mat,
                                               sgp_rec* tmp) {
    __shared__ uint32_t s_c[MAXP2];
    const uint32_t t = threadIdx.x, ni = c.sc->nitems, nu = (ni + UI - 1) / UI;
    for (uint32_t u = blockIdx.x; u < nu; u += gridDim.x) {
        for (uint32_t d = t; d < P2; d += 1024) s_c[d] = mat[d * nu + u];
        sgp_rec e[UI];
#pragma unroll
        for (uint32_t k = 0; k < UI; ++k) {
            const uint32_t j = u * UI + k;
            const uint4 it = j < ni ? c.items[j] : make_uint4(0, 0, 0, 0);
            e[k] = item_base(c, it)[t < it.y ? t : 0];  // unconditional load
            if (t >= it.y) e[k].time = TOMB;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < UI; ++k) {
            if (e[k].time >= barrier) continue;
            tmp[atomicAdd(&s_c[e[k].dst >> HB], 1u)] = e[k];
            const uint4 it = c.items[u * UI + k];  // (uniform: reloaded rather than kept)
            if ((it.x & FARBIT) || it.w)  // records that stay must be told apart
                const_cast<sgp_rec*>(item_base(c, it))[t].time = TOMB;
        }
        __syncthreads();
    }
}

// Spent buckets back to the free stack (workgroup p takes due buckets p,
// p + P2, ...); the straddling bucket and the far list get their new minima.
__device__ __forceinline__ void finish_buckets(const Cal& c, uint64_t cur, uint32_t nbk, uint32_t p, uint32_t P2,
                                               uint32_t* s_at) {
    if (p == 0 && threadIdx.x == 0 && c.sc->farscan) {
        c.sc->farmin = c.sc->fmin;
        c.sc->farlive = c.sc->flive;
    }
    const uint64_t smin = c.sc->smin;
    for (uint32_t k = p; k < nbk; k += P2) {
        const uint32_t s = (uint32_t)(cur + k) & (RB - 1);
        if (k + 1 == nbk && smin != SIMTIME_MAX) {  // events remain in the last due bucket
            if (threadIdx.x == 0) c.bh[s].min = smin;
            continue;
        }
        const uint32_t m = c.bh[s].chk;
        __syncthreads();
        if (threadIdx.x == 0) {
            *s_at = m ? atomicAdd(&c.sc->ftop, m) : 0;
            c.bh[s].cnt = 0;
            c.bh[s].chk = 0;
            c.bh[s].min = SIMTIME_MAX;
        }
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < m; j += 1024) c.fst[*s_at + j] = c.btab[(size_t)s * c.nchb + j];
    }
}

// Level 2, one workgroup per host block: an LDS counting sort by host writes
// the block's run offsets off[] and its events in host order; the spent
// buckets are released on the side.
__global__ __launch_bounds__(1024) void k_local(Cal c, uint64_t cur, uint32_t nbk, uint32_t n, uint32_t P2,
                                                const uint32_t* pbase, const sgp_rec* tmp, sgp_rec* tmp2,
                                                uint32_t* off) {
    __shared__ uint32_t s_c[HPB];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_at;
    const uint32_t t = threadIdx.x, p = blockIdx.x, h0 = p << HB;
    finish_buckets(c, cur, nbk, p, P2, &s_at);
    const uint32_t pb = pbase[p], pe = pbase[p + 1];
    const uint32_t nh = n - h0 < HPB ? n - h0 : HPB;
    for (uint32_t j = t; j < HPB; j += 1024) s_c[j] = 0;
    __syncthreads();
    for (uint32_t i = pb + t; i < pe; i += 1024) atomicAdd(&s_c[tmp[i].dst - h0], 1u);
    __syncthreads();
    constexpr uint32_t PT = HPB / 1024;
    uint32_t v[PT], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
        v[k] = s_c[t * PT + k];
        sum += v[k];
    }
    uint32_t tot;
    uint32_t at = pb + block_excl(sum, s_w, &tot);
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
        if (t * PT + k < nh) off[h0 + t * PT + k] = at;
        s_c[t * PT + k] = at;  // the scatter cursor
        at += v[k];
    }
    if (p + 1 == P2 && t == 0) off[n] = pe;
    __syncthreads();
    for (uint32_t i = pb + t; i < pe; i += 1024) {
        const sgp_rec e = tmp[i];
        tmp2[atomicAdd(&s_c[e.dst - h0], 1u)] = e;
    }
}

// Each extracted event ranked inside its host's run in event_compare order
// (event.c:110-153; the keys are unique, srcHostEventID being unique per source).
// A short run (most hosts: one or a few events) is ranked by one lane per event
// scanning the run; a longer one (an incast) is listed for k_xlong, which sorts
// it in LDS, so no lane scans more than XR_SHORT records.
constexpr uint32_t XR_SHORT = 32;    // longest run ranked by scanning
constexpr uint32_t XL_SORT = 2048;   // longest run k_xlong sorts in LDS (bitonic)
constexpr uint32_t XL_T = 1024;      // k_xlong workgroup
constexpr uint32_t XL_G = 256;       // k_xlong grid (workgroups loop over the list)
__global__ __launch_bounds__(BLOCK) void k_xrank(const sgp_rec* tmp2, const uint32_t* off,
                                                 const unsigned long long* total, sgp_rec* out, Scal* sc,
                                                 uint32_t* longl) {
    const uint64_t T = *total;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < T; i += (uint64_t)gridDim.x * BLOCK) {
        const sgp_rec e = tmp2[i];
        const uint32_t s = off[e.dst], f = off[e.dst + 1];
        if (f - s > XR_SHORT) {
            if (i == s) longl[atomicAdd(&sc->nlong, 1u)] = e.dst;  // the run's first record lists it
            continue;
        }
        uint32_t rank = 0;
        for (uint32_t j = s; j < f; ++j)
            rank += key_less(tmp2[j].time, tmp2[j].src_id, tmp2[j].seq, e.time, e.src_id, e.seq);
        out[s + rank] = e;
    }
}

// The long runs k_xrank listed, one workgroup per run: up to XL_SORT records
// bitonic-sorted in LDS by event_compare key (a padding key above every real
// one); beyond that (a host receiving thousands of events in one round) each
// record's rank counted against the run in LDS tiles of XL_SORT.
__global__ __launch_bounds__(XL_T) void k_xlong(const sgp_rec* tmp2, const uint32_t* off, const Scal* sc,
                                                const uint32_t* longl, sgp_rec* out) {
    __shared__ uint64_t s_t[XL_SORT], s_q[XL_SORT];
    __shared__ uint32_t s_s[XL_SORT];
    __shared__ uint16_t s_i[XL_SORT];
    const uint32_t tid = threadIdx.x, nl = sc->nlong;
    for (uint32_t j = blockIdx.x; j < nl; j += gridDim.x) {  // uniform per workgroup
        const uint32_t h = longl[j], s = off[h], k = off[h + 1] - s;
        __syncthreads();  // the previous run's LDS reads are done
        if (k <= XL_SORT) {
            uint32_t P = 64;
            while (P < k) P <<= 1;
            for (uint32_t i = tid; i < P; i += XL_T) {
                const bool v = i < k;
                const sgp_rec e = tmp2[s + (v ? i : 0)];
                s_t[i] = v ? e.time : UINT64_MAX;
                s_s[i] = v ? e.src_id : UINT32_MAX;
                s_q[i] = v ? e.seq : UINT64_MAX;
                s_i[i] = (uint16_t)i;
            }
            __syncthreads();
            for (uint32_t size = 2; size <= P; size <<= 1) {
                for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                    for (uint32_t i = tid; i < P / 2; i += XL_T) {
                        const uint32_t lo = 2 * stride * (i / stride) + (i % stride), hi = lo + stride;
                        const bool up = (lo & size) == 0;
                        const bool lt = key_less(s_t[hi], s_s[hi], s_q[hi], s_t[lo], s_s[lo], s_q[lo]);
                        if (lt == up) {
                            const uint64_t t = s_t[lo], q = s_q[lo];
                            const uint32_t a = s_s[lo];
                            const uint16_t x = s_i[lo];
                            s_t[lo] = s_t[hi];
                            s_q[lo] = s_q[hi];
                            s_s[lo] = s_s[hi];
                            s_i[lo] = s_i[hi];
                            s_t[hi] = t;
                            s_q[hi] = q;
                            s_s[hi] = a;
                            s_i[hi] = x;
                        }
                    }
                    __syncthreads();
                }
            }
            for (uint32_t i = tid; i < k; i += XL_T) out[s + i] = tmp2[s + s_i[i]];
            continue;
        }
        for (uint32_t b = 0; b < k; b += XL_T) {  // every record's rank, tile by tile
            const bool v = b + tid < k;
            const sgp_rec e = tmp2[s + (v ? b + tid : 0)];
            uint32_t rank = 0;
            for (uint32_t t0 = 0; t0 < k; t0 += XL_SORT) {
                const uint32_t m = k - t0 < XL_SORT ? k - t0 : XL_SORT;
                __syncthreads();
                for (uint32_t i = tid; i < m; i += XL_T) {
                    const sgp_rec r = tmp2[s + t0 + i];
                    s_t[i] = r.time;
                    s_s[i] = r.src_id;
                    s_q[i] = r.seq;
                }
                __syncthreads();
                for (uint32_t i = 0; i < m; ++i) rank += key_less(s_t[i], s_s[i], s_q[i], e.time, e.src_id, e.seq);
            }
            if (v) out[s + rank] = e;
        }
    }
}

// MIN over the bucket minima: RB / 1024 workgroups, one partial each (the host
// takes the minimum of the partials and the far list's).
__global__ __launch_bounds__(1024) void k_cmin(Cal c) {
    __shared__ uint64_t s_m[16];
    const uint64_t x = c.bh[blockIdx.x * 1024 + threadIdx.x].min;
    const uint64_t m = wave_min(x);
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t r = SIMTIME_MAX;
        for (int i = 0; i < 16; ++i) r = s_m[i] < r ? s_m[i] : r;
        c.sc->pmin[blockIdx.x] = r;
    }
}

__global__ __launch_bounds__(BLOCK) void k_call(Cal c, sgp_rec* out, uint64_t cap) {
    const uint32_t np = c.sc->nitems * PPI;
    for (uint32_t j = blockIdx.x; j < np; j += gridDim.x) {  // uniform per workgroup
        const uint4 it = c.items[j / PPI];
        const sgp_rec* r = item_base(c, it);
        const uint32_t i = (j % PPI) * PIECE + threadIdx.x;
        sgp_rec e{};
        e.time = TOMB;
        if (i < it.y) e = r[i];
        const bool live = e.time != TOMB;
        const uint64_t m = __ballot(live);
        unsigned long long base = 0;
        const int lane = threadIdx.x & 63;
        if (lane == 0 && m) base = atomicAdd(&c.sc->nall, (unsigned long long)__popcll(m));
        base = __shfl(base, 0, 64);
        const unsigned long long p = base + __popcll(m & ((1ull << lane) - 1));
        if (live && p < cap) out[p] = e;
    }
}

// Far list without its tombstones, into `to` (order does not matter: runs are
// ranked by key).
__global__ void k_fcompact(const sgp_rec* from, uint64_t n, sgp_rec* to, unsigned long long* count) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const sgp_rec e = from[i];
        if (e.time != TOMB) to[atomicAdd(count, 1ull)] = e;
    }
}

uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, nullptr, 10) : dflt;
}

}  // namespace

// Kernel classes of the per-kernel profile (sg_policy_kernel_profile).
enum KCls { KC_CINS1, KC_CNEED, KC_CALLOC, KC_CINS2, KC_CMIN, KC_XPLAN, KC_HIST, KC_MSCAN, KC_PART, KC_LOCAL,
            KC_XRANK, KC_XLONG, KC_N };
const char* const KC_NAMES[KC_N] = {"k_cins1", "k_cneed", "k_calloc", "k_cins2", "k_cmin", "k_xplan",
                                    "k_hist", "k_mscan", "k_part", "k_local", "k_xrank", "k_xlong"};

struct sgp_dev {
    int device;
    hipStream_t s;
    // per-kernel profile: dispatch-packet timestamps of every launch
    // (hipExtLaunchKernelGGL), harvested at the next synchronisation
    bool kprof = false;
    uint32_t kskip = 0;  // extractions still to skip
    double kms[KC_N] = {}, kbytes[KC_N] = {};
    uint64_t kn[KC_N] = {};
    struct KEv { hipEvent_t a, b; int cls; };
    std::vector<KEv> kpend;
    std::vector<hipEvent_t> kfree;
    Cal c;
    Scal* h_sc;          // pinned mirror of the device scalars
    uint64_t cur;        // lowest bucket that may hold a live event
    uint32_t nchunks;    // pool chunks
    uint64_t farcap;     // far list capacity (records)
    sgp_rec* far2;       // compaction target
    uint64_t items_cap;
    sgp_rec* d_in;       // staged records
    uint32_t* d_rslot;
    uint64_t in_cap;
    sgp_rec* d_tmp;      // extracted, by host block
    sgp_rec* d_tmp2;     // extracted, by host
    sgp_rec* d_out;      // extracted runs, ranked
    uint64_t out_cap;
    uint32_t* d_off;     // [N + 1] host-ordered run offsets
    uint32_t* d_long;    // [N] hosts whose run k_xlong ranks
    uint32_t P2;         // host blocks
    uint32_t* d_mat;     // [units][P2] level-1 counts, then bases
    uint32_t* d_pbase;   // [P2 + 1] host block starts
    sgp_rec* h_runs;     // pinned
    uint32_t* h_off;
    uint64_t queued;     // events in HBM
    uint64_t far_compact;  // far records before a tombstone-heavy list is compacted
};

#define PCHK(x)                                                                         \
    do {                                                                                \
        hipError_t _e = (x);                                                            \
        if (_e != hipSuccess) {                                                         \
            sg_set_error("%s: %s (%s:%d)", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
            return 3;                                                                   \
        }                                                                               \
    } while (0)

static int dmalloc(void** p, size_t bytes) {
    if (hipMalloc(p, bytes ? bytes : 8) != hipSuccess) {
        *p = nullptr;
        sg_set_error("sgp: hipMalloc of %zu bytes failed", bytes);
        return 2;
    }
    return 0;
}

// items: every chunk of the pool plus every far piece, once
static int fit_items(sgp_dev* d) {
    const uint64_t need = (uint64_t)d->nchunks + (d->farcap + CH - 1) / CH + 1;
    if (need <= d->items_cap) return 0;
    if (d->c.items) (void)hipFree(d->c.items);
    int rc = dmalloc((void**)&d->c.items, need * sizeof(uint4));
    if (rc) return rc;
    d->items_cap = need;
    const uint64_t units = (need + UI - 1) / UI;
    if (d->d_mat) (void)hipFree(d->d_mat);
    d->d_mat = nullptr;
    if ((rc = dmalloc((void**)&d->d_mat, units * d->P2 * 4))) return rc;
    return 0;
}

static int grow_far(sgp_dev* d, uint64_t n) {
    if (n <= d->farcap) return 0;
    uint64_t c = d->farcap ? d->farcap : 4096;
    while (c < n) c *= 2;
    sgp_rec *a = nullptr, *b = nullptr;
    int rc = dmalloc((void**)&a, c * sizeof(sgp_rec));
    if (!rc) rc = dmalloc((void**)&b, c * sizeof(sgp_rec));
    if (rc) {
        if (a) (void)hipFree(a);
        return rc;
    }
    if (d->h_sc->nfar) PCHK(hipMemcpyAsync(a, d->c.far, d->h_sc->nfar * sizeof(sgp_rec), hipMemcpyDeviceToDevice, d->s));
    PCHK(hipStreamSynchronize(d->s));
    if (d->c.far) (void)hipFree(d->c.far);
    if (d->far2) (void)hipFree(d->far2);
    d->c.far = a;
    d->far2 = b;
    d->farcap = c;
    return fit_items(d);
}

// Pool of at least `want` chunks; live chunks keep their ids.
static int grow_pool(sgp_dev* d, uint32_t want) {
    if (want <= d->nchunks) return 0;
    uint64_t nc = (uint64_t)d->nchunks * 2;
    if (nc < want) nc = want;
    if (nc > 0x7FFFFFFFull) {
        sg_set_error("sgp: chunk pool over 2^31 chunks");
        return 2;
    }
    sgp_rec* pool = nullptr;
    uint32_t* fst = nullptr;
    int rc = dmalloc((void**)&pool, nc * CH * sizeof(sgp_rec));
    if (!rc) rc = dmalloc((void**)&fst, nc * 4);
    if (rc) {
        if (pool) (void)hipFree(pool);
        return rc;
    }
    const uint32_t top = d->h_sc->ftop, add = (uint32_t)nc - d->nchunks;
    PCHK(hipMemcpyAsync(pool, d->c.pool, (size_t)d->nchunks * CH * sizeof(sgp_rec), hipMemcpyDeviceToDevice, d->s));
    if (top) PCHK(hipMemcpyAsync(fst, d->c.fst, (size_t)top * 4, hipMemcpyDeviceToDevice, d->s));
    hipLaunchKernelGGL(k_fpush, dim3((add + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, d->s, fst, top, d->nchunks, add);
    PCHK(hipGetLastError());
    const uint32_t ntop = top + add;
    PCHK(hipMemcpyAsync(&d->c.sc->ftop, &ntop, 4, hipMemcpyHostToDevice, d->s));
    PCHK(hipStreamSynchronize(d->s));
    (void)hipFree(d->c.pool);
    (void)hipFree(d->c.fst);
    d->c.pool = pool;
    d->c.fst = fst;
    d->nchunks = (uint32_t)nc;
    d->h_sc->ftop = ntop;
    return fit_items(d);
}

static int grow_in(sgp_dev* d, uint64_t n) {
    if (n <= d->in_cap) return 0;
    uint64_t c = d->in_cap ? d->in_cap : 4096;
    while (c < n) c *= 2;
    if (d->d_in) (void)hipFree(d->d_in);
    if (d->d_rslot) (void)hipFree(d->d_rslot);
    d->d_in = nullptr;
    d->d_rslot = nullptr;
    int rc = dmalloc((void**)&d->d_in, c * sizeof(sgp_rec));
    if (!rc) rc = dmalloc((void**)&d->d_rslot, c * 4);
    if (rc) return rc;
    d->in_cap = c;
    return 0;
}

static int grow_out(sgp_dev* d, uint64_t n) {
    if (n <= d->out_cap) return 0;
    uint64_t c = d->out_cap ? d->out_cap : 4096;
    while (c < n) c *= 2;
    if (d->d_out) (void)hipFree(d->d_out);
    if (d->d_tmp) (void)hipFree(d->d_tmp);
    if (d->d_tmp2) (void)hipFree(d->d_tmp2);
    if (d->h_runs) (void)hipHostFree(d->h_runs);
    d->d_out = nullptr;
    d->d_tmp = nullptr;
    d->d_tmp2 = nullptr;
    d->h_runs = nullptr;
    int rc = dmalloc((void**)&d->d_out, c * sizeof(sgp_rec));
    if (!rc) rc = dmalloc((void**)&d->d_tmp, c * sizeof(sgp_rec));
    if (!rc) rc = dmalloc((void**)&d->d_tmp2, c * sizeof(sgp_rec));
    if (rc) return rc;
    PCHK(hipHostMalloc((void**)&d->h_runs, c * sizeof(sgp_rec), hipHostMallocDefault));
    d->out_cap = c;
    return 0;
}

static hipEvent_t kev(sgp_dev* d) {
    if (!d->kfree.empty()) {
        hipEvent_t e = d->kfree.back();
        d->kfree.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
static bool counting(const sgp_dev* d) { return d->kprof && d->kskip == 0; }
// One launch of class cls on the policy's stream; profiled, it carries its
// dispatch packet's own timestamps and adds `bytes` to the class.
template <typename K, typename... A>
static void klaunch(sgp_dev* d, int cls, double bytes, K kernel, dim3 g, dim3 b, A... args) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (counting(d)) {
        e0 = kev(d);
        e1 = kev(d);
    }
    if (e0 && e1) {
        hipExtLaunchKernelGGL(kernel, g, b, 0, d->s, e0, e1, 0, args...);
        d->kpend.push_back({e0, e1, cls});
    } else {
        hipLaunchKernelGGL(kernel, g, b, 0, d->s, args...);
    }
    if (counting(d)) {
        d->kn[cls]++;
        d->kbytes[cls] += bytes;
    }
}
static void kharvest(sgp_dev* d) {  // after a stream synchronisation
    for (auto& e : d->kpend) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) d->kms[e.cls] += ms;
        d->kfree.push_back(e.a);
        d->kfree.push_back(e.b);
    }
    d->kpend.clear();
}

static int read_scal(sgp_dev* d) {
    PCHK(hipMemcpyAsync(d->h_sc, d->c.sc, sizeof(Scal), hipMemcpyDeviceToHost, d->s));
    PCHK(hipStreamSynchronize(d->s));
    kharvest(d);
    return 0;
}

extern "C" {

int sgp_dev_create(int device, uint32_t n_hosts, uint32_t cap, sgp_dev** out) {
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        sg_set_error("sgp_dev_create: no HIP device %d", device);
        return 6;
    }
    hipDeviceProp_t prop;
    PCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        sg_set_error("sgp_dev_create: device is %s, need gfx950", prop.gcnArchName);
        return 6;
    }
    PCHK(hipSetDevice(device));
    if (n_hosts == 0) n_hosts = 1;
    if (n_hosts > MAXP2 * HPB) {
        sg_set_error("sgp_dev_create: %u hosts, at most %u", n_hosts, MAXP2 * HPB);
        return 1;
    }
    if (cap == 0) cap = 16;
    sgp_dev* d = new sgp_dev();  // value-initialised: pointers and counters zero
    d->device = device;
    Cal& c = d->c;
    c.n = n_hosts;
    // bucket width 2^shift ns (default 2^18 = 262 us: a 1 ms round reads ~5
    // buckets, the ring reaches 4.3 s ahead); chunk-table entries per bucket
    c.shift = env_u32("SG_PBUCKET_SHIFT", 18);
    c.nchb = env_u32("SG_PBUCKET_CHUNKS", 1024);
    if (c.shift > 40) c.shift = 40;
    if (c.nchb == 0) c.nchb = 1;
    if (c.nchb > (1u << 20)) c.nchb = 1u << 20;
    c.cap = c.nchb * CH;
    d->far_compact = env_u32("SG_PFAR_COMPACT", 65536);
    const uint64_t nch = ((uint64_t)n_hosts * cap + CH - 1) / CH + 1;
    d->nchunks = nch > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)nch;
    int rc = 0;
    if (!rc) rc = dmalloc((void**)&c.pool, (size_t)d->nchunks * CH * sizeof(sgp_rec));
    if (!rc) rc = dmalloc((void**)&c.fst, (size_t)d->nchunks * 4);
    if (!rc) rc = dmalloc((void**)&c.btab, (size_t)RB * c.nchb * 4);
    if (!rc) rc = dmalloc((void**)&c.bh, RB * sizeof(BH));
    if (!rc) rc = dmalloc((void**)&c.sc, sizeof(Scal));
    if (!rc) rc = dmalloc((void**)&d->d_off, ((size_t)n_hosts + 1) * 4);
    if (!rc) rc = dmalloc((void**)&d->d_long, (size_t)n_hosts * 4);
    d->P2 = (n_hosts + HPB - 1) / HPB;
    if (!rc) rc = dmalloc((void**)&d->d_pbase, ((size_t)d->P2 + 1) * 4);
    if (!rc && (hipHostMalloc((void**)&d->h_off, ((size_t)n_hosts + 1) * 4, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&d->h_sc, sizeof(Scal), hipHostMallocDefault) != hipSuccess ||
                hipStreamCreateWithFlags(&d->s, hipStreamNonBlocking) != hipSuccess)) {
        sg_set_error("sgp_dev_create: allocation failed");
        rc = 2;
    }
    Scal init{};
    init.ftop = d->nchunks;
    init.farmin = SIMTIME_MAX;
    if (!rc) *d->h_sc = init;
    if (!rc) rc = grow_far(d, 4096);
    if (!rc) rc = fit_items(d);
    if (rc) {
        sgp_dev_destroy(d);
        return rc;
    }
    uint32_t g = (RB > d->nchunks ? RB : d->nchunks);
    hipLaunchKernelGGL(k_cinit, dim3((g + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, d->s, c, d->nchunks);
    if (hipMemcpyAsync(c.sc, &init, sizeof init, hipMemcpyHostToDevice, d->s) != hipSuccess ||
        hipStreamSynchronize(d->s) != hipSuccess) {
        sgp_dev_destroy(d);
        sg_set_error("sgp_dev_create: init failed");
        return 3;
    }
    *out = d;
    return 0;
}

int sgp_dev_destroy(sgp_dev* d) {
    if (!d) return 0;
    if (d->s) (void)hipStreamSynchronize(d->s);
    void* dp[] = {d->c.pool, d->c.fst, d->c.btab, d->c.bh, d->c.sc, d->c.far,
                  d->far2, d->c.items, d->d_in, d->d_rslot, d->d_tmp, d->d_tmp2, d->d_out, d->d_off, d->d_mat, d->d_pbase,
                  d->d_long};
    for (void* p : dp)
        if (p) (void)hipFree(p);
    if (d->h_runs) (void)hipHostFree(d->h_runs);
    if (d->h_off) (void)hipHostFree(d->h_off);
    if (d->h_sc) (void)hipHostFree(d->h_sc);
    for (auto& e : d->kpend) {
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    for (hipEvent_t e : d->kfree) (void)hipEventDestroy(e);
    if (d->s) (void)hipStreamDestroy(d->s);
    delete d;
    return 0;
}

void* sgp_host_alloc(uint64_t bytes) {
    void* p = nullptr;
    return hipHostMalloc(&p, bytes ? bytes : 8, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

void sgp_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int sgp_dev_insert(sgp_dev* d, const sgp_rec* recs, uint64_t n) {
    return sgp_dev_insert_segs(d, &recs, &n, 1);
}

int sgp_dev_insert_segs(sgp_dev* d, const sgp_rec* const* segs, const uint64_t* lens, uint32_t nseg) {
    uint64_t n = 0;
    for (uint32_t i = 0; i < nseg; ++i) n += lens[i];
    if (n == 0) return 0;
    PCHK(hipSetDevice(d->device));
    int rc = grow_in(d, n);
    if (rc) return rc;
    // h_sc is current: every call that changes the device scalars ends in read_scal
    Scal* h = d->h_sc;
    // a far list mostly of tombstones is compacted first
    if (h->nfar > d->far_compact && h->nfar - h->farlive > h->farlive) {
        PCHK(hipMemsetAsync(&d->c.sc->nfar, 0, 8, d->s));
        hipLaunchKernelGGL(k_fcompact, dim3(1024), dim3(BLOCK), 0, d->s, d->c.far, (uint64_t)h->nfar, d->far2,
                           &d->c.sc->nfar);
        PCHK(hipGetLastError());
        sgp_rec* t = d->c.far;
        d->c.far = d->far2;
        d->far2 = t;
        h->nfar = h->farlive;
    }
    if ((rc = grow_far(d, h->nfar + n))) return rc;
    uint64_t o = 0;
    for (uint32_t i = 0; i < nseg; ++i) {
        if (lens[i])
            PCHK(hipMemcpyAsync(d->d_in + o, segs[i], lens[i] * sizeof(sgp_rec), hipMemcpyHostToDevice, d->s));
        o += lens[i];
    }
    const uint32_t grid = (uint32_t)((n + IPW - 1) / IPW);
    PCHK(hipMemsetAsync(&d->c.sc->need, 0, 4, d->s));
    // algorithmic bytes: k_cins1 reads each time and writes its
    // slot (12 B); k_cneed / k_calloc read a bucket's counts (8 B) and
    // k_calloc moves each new chunk id (8 B); k_cins2 reads the slot, the
    // record and its chunk id and writes the record (72 B)
    klaunch(d, KC_CINS1, 12.0 * n, k_cins1, dim3(grid), dim3(BLOCK), d->c, d->cur, (const sgp_rec*)d->d_in, n,
            d->d_rslot);
    klaunch(d, KC_CNEED, 8.0 * RB, k_cneed, dim3(RB / BLOCK), dim3(BLOCK), d->c);
    PCHK(hipGetLastError());
    if ((rc = read_scal(d))) return rc;
    if (h->need > h->ftop && (rc = grow_pool(d, d->nchunks + (h->need - h->ftop)))) return rc;
    klaunch(d, KC_CALLOC, 8.0 * RB + 8.0 * h->need, k_calloc, dim3(RB / BLOCK), dim3(BLOCK), d->c);
    klaunch(d, KC_CINS2, 72.0 * n, k_cins2, dim3(grid), dim3(BLOCK), d->c, (const sgp_rec*)d->d_in, n,
            (const uint32_t*)d->d_rslot);
    PCHK(hipGetLastError());
    h->ftop -= h->need;
    d->queued += n;
    return 0;
}

int sgp_dev_min(sgp_dev* d, uint64_t* min_out) {
    PCHK(hipSetDevice(d->device));
    klaunch(d, KC_CMIN, 8.0 * RB, k_cmin, dim3(RB / 1024), dim3(1024), d->c);  // each bucket's minimum
    PCHK(hipGetLastError());
    int rc = read_scal(d);
    if (rc) return rc;
    const Scal* h = d->h_sc;
    uint64_t m = h->farlive ? (uint64_t)h->farmin : SIMTIME_MAX;
    for (uint32_t i = 0; i < RB / 1024; ++i) m = h->pmin[i] < m ? h->pmin[i] : m;
    *min_out = m;
    return 0;
}

int sgp_dev_extract(sgp_dev* d, uint64_t barrier, const sgp_rec** runs, const uint32_t** off,
                    uint64_t* total) {
    PCHK(hipSetDevice(d->device));
    int rc = grow_out(d, d->queued ? d->queued : 1);
    if (rc) return rc;
    const uint32_t n = d->c.n, P2 = d->P2;
    uint32_t nbk = 0;  // due buckets [cur, cur + nbk)
    if (barrier > 0) {
        const uint64_t last = (barrier - 1) >> d->c.shift;
        if (last >= d->cur) nbk = last - d->cur + 1 < RB ? (uint32_t)(last - d->cur + 1) : RB;
    }
    // sizes known only at the end (items, extracted records): the bytes of
    // these launches are added below
    const bool cnt = counting(d);
    klaunch(d, KC_XPLAN, 0, k_xplan, dim3(1), dim3(1024), d->c, d->cur, nbk, barrier, 0);
    klaunch(d, KC_HIST, 0, k_hist, dim3(XU), dim3(1024), d->c, barrier, P2, d->d_mat);
    klaunch(d, KC_MSCAN, 0, k_mscan, dim3(1), dim3(1024), d->d_mat, P2, (const Cal)d->c, d->d_pbase);
    klaunch(d, KC_PART, 0, k_part, dim3(XU), dim3(1024), d->c, barrier, P2, (const uint32_t*)d->d_mat, d->d_tmp);
    klaunch(d, KC_LOCAL, 0, k_local, dim3(P2), dim3(1024), d->c, d->cur, nbk, n, P2, (const uint32_t*)d->d_pbase,
            (const sgp_rec*)d->d_tmp, d->d_tmp2, d->d_off);
    PCHK(hipMemsetAsync(&d->c.sc->nlong, 0, 4, d->s));
    klaunch(d, KC_XRANK, 0, k_xrank, dim3(XG), dim3(BLOCK), (const sgp_rec*)d->d_tmp2, (const uint32_t*)d->d_off,
            (const unsigned long long*)&d->c.sc->total, d->d_out, d->c.sc, d->d_long);
    klaunch(d, KC_XLONG, 0, k_xlong, dim3(XL_G), dim3(XL_T), (const sgp_rec*)d->d_tmp2, (const uint32_t*)d->d_off,
            (const Scal*)d->c.sc, (const uint32_t*)d->d_long, d->d_out);
    PCHK(hipGetLastError());
    PCHK(hipMemcpyAsync(d->h_off, d->d_off, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost, d->s));
    if ((rc = read_scal(d))) return rc;
    const uint64_t t = d->h_sc->total;
    if (cnt) {
        // algorithmic bytes, t extracted records of 32 B:
        // k_xplan reads the due buckets' counts and writes a 16-B item with
        // its chunk id per due chunk; the level-1 sort reads each due time and
        // host (12 B) and writes / scans / reads the count matrix (4 B per
        // entry), k_part moves each record (64 B); k_local reads each host,
        // moves each record (68 B) and writes off[] (4 B per host); k_xrank
        // reads each record and its run bounds and writes it (72 B); k_xlong
        // (incast runs only) is not counted
        const double nu = (double)((d->h_sc->nitems + UI - 1) / UI), mat = 4.0 * nu * P2;
        d->kbytes[KC_XPLAN] += 8.0 * nbk + 20.0 * d->h_sc->nitems;
        d->kbytes[KC_HIST] += 12.0 * t + mat;
        d->kbytes[KC_MSCAN] += 2.0 * mat;
        d->kbytes[KC_PART] += 64.0 * t + mat;
        d->kbytes[KC_LOCAL] += 68.0 * t + 4.0 * n;
        d->kbytes[KC_XRANK] += 72.0 * t;
    }
    if (d->kskip) --d->kskip;
    if (t) PCHK(hipMemcpy(d->h_runs, d->d_out, t * sizeof(sgp_rec), hipMemcpyDeviceToHost));
    if (barrier > 0 && (barrier >> d->c.shift) > d->cur) d->cur = barrier >> d->c.shift;
    d->queued -= t;
    *runs = d->h_runs;
    *off = d->h_off;
    *total = t;
    return 0;
}

int sgp_dev_kprof(sgp_dev* d, int enable, uint32_t skip_rounds) {
    PCHK(hipStreamSynchronize(d->s));
    kharvest(d);
    d->kprof = enable != 0;
    d->kskip = skip_rounds;
    for (int i = 0; i < KC_N; ++i) {
        d->kms[i] = d->kbytes[i] = 0;
        d->kn[i] = 0;
    }
    return 0;
}

int sgp_dev_kstats(sgp_dev* d, const char** names, uint64_t* launches, double* ms, double* bytes, uint32_t cap,
                   uint32_t* n_out) {
    PCHK(hipStreamSynchronize(d->s));
    kharvest(d);
    for (uint32_t i = 0; i < (uint32_t)KC_N && i < cap; ++i) {
        names[i] = KC_NAMES[i];
        launches[i] = d->kn[i];
        ms[i] = d->kms[i];
        bytes[i] = d->kbytes[i];
    }
    *n_out = KC_N;
    return 0;
}

int sgp_dev_all(sgp_dev* d, sgp_rec* out, uint64_t capacity, uint64_t* n_out) {
    PCHK(hipSetDevice(d->device));
    int rc = grow_out(d, d->queued ? d->queued : 1);
    if (rc) return rc;
    PCHK(hipMemsetAsync(&d->c.sc->nall, 0, 8, d->s));
    hipLaunchKernelGGL(k_xplan, dim3(1), dim3(1024), 0, d->s, d->c, d->cur, RB, (uint64_t)0, 1);
    hipLaunchKernelGGL(k_call, dim3(XG), dim3(BLOCK), 0, d->s, d->c, d->d_out, d->out_cap);
    PCHK(hipGetLastError());
    if ((rc = read_scal(d))) return rc;
    const uint64_t t = d->h_sc->nall;
    const uint64_t m = t < capacity ? t : capacity;
    if (out && m) PCHK(hipMemcpy(out, d->d_out, m * sizeof(sgp_rec), hipMemcpyDeviceToHost));
    *n_out = t;
    return 0;
}

}  // extern "C"
