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
//              per-peer outbox; k_fill copies up to exchange_cap of them per peer
//              into the fixed-size blocks of the RCCL all-to-all, behind a header
//              that also carries this shard's MIN terms (so no all-reduce).
//   k_insert   delivers staged / received events into destination queues and
//              keeps each host's earliest queued time.
//   k_reduce   MIN next event time (host_single.c:273-305, scheduler.c:393-398),
//              the minimum discovered latency (topology.c:1374-1385) and, for a
//              single shard, the next window (master.c:450-480).
//
// HBM layout:
//   queue slot   16 B {time, key}, key = src << 40 | srcHostEventID: with the
//                destination implied by the queue, event_compare is the
//                lexicographic order of (time, key)
//   queues       host-major, slot j of local host h at [h * CAP + j]: a round
//                reads only the queues of hosts with an event before the barrier
//   per pair     16 B {ceil delay ns, keep threshold, truncated ms}: one random
//                access per send
//   per host     8 B {weight threshold, vertex} (read-only, all N hosts) and
//                32 B {rand_r state, event counter, pops, digest} (local hosts)
// Compiled with -ffp-contract=off: the only FP is the FP64 floor destination
// rule, which must round exactly as the reference does.
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
constexpr int SRC_SHIFT = 40;
constexpr uint64_t SEQ_MASK = (1ULL << SRC_SHIFT) - 1;
// exchange block = HDR header rows + exchange_cap event rows, 3 x int64 per row
constexpr int HDR = 2;
enum Hdr { H_N = 0, H_MORE, H_MIN, H_JMIN, H_OVF, H_ROUND };

enum Ctr {
    C_POPS = 0, C_BOOTS, C_SENDS, C_NULL, C_DROPREL, C_DROPEND, C_BUMPED, C_SAME,
    C_ACTIVE, C_EMIT, NCTR
};
enum Mins { M_JMIN = 0, M_EMIN, M_RMIN, NMIN };

struct Slot {
    uint64_t t;   // event time
    uint64_t k;   // src << 40 | srcHostEventID
};
struct HostInfo {
    int32_t wt;       // PHOLD weight threshold (test_phold.c:160-178)
    uint32_t vertex;  // attachment vertex
};
struct PairRec {
    uint64_t delay;   // ceil(latency_ms * 1e6)   (worker.c:275-277)
    int32_t keep;     // max rand_r value kept     (worker.c:268-273)
    uint32_t jump;    // (uint64)latency_ms        (master.c:153)
};
struct HostState {
    uint32_t rng;     // host Random (host.c:176)
    uint32_t pad;
    uint64_t evc;     // eventIDCounter (host.c:397-400)
    uint64_t pops;
    uint64_t digest;
};

struct RoundState {
    uint64_t S, E, done, rounds;
    uint64_t min_jump, next_min_jump, jmin;
    uint64_t overflow;
    uint64_t trace_len;
    uint64_t ctr[NCTR];
    uint64_t last_min;
    // multi-shard step protocol
    uint64_t phase;      // 0: process step, 1: drain step (outbox leftovers only)
    uint64_t loc_min;    // this shard's MIN next time of the round being exchanged
    uint64_t loc_jmin;   // this shard's cumulative min discovered latency (ms)
    uint64_t steps;      // exchange steps executed
    uint64_t peak_peer;  // largest per-peer outbox of a process step (since reset)
};

struct Dev {
    uint32_t N, V, L, lo, CAP, load, dst_rule, window_rule, G, g, nblocks, bcap;
    uint64_t end_time, bootstrap_end, fixed_jump, runahead_min, trace_cap, xcap, xrows;
    uint32_t bounds[MAXG + 1];
    const HostInfo* hinfo;    // [N]
    const PairRec* pairs;     // [V*V]
    Slot* bag;                // [L][CAP]
    uint32_t* bag_cnt;        // [L]
    uint64_t* hmin;           // [L]
    HostState* hs;            // [L]
    uint64_t* pmin;           // [NMIN][nblocks], this round
    uint64_t* pcum;           // [NCTR][nblocks], cumulative
    uint32_t* blockcnt;       // [nblocks] staged events
    uint32_t* peercnt;        // [nblocks][G]
    uint32_t* peeroff;        // [nblocks][G]
    int64_t* outq;            // [nblocks * bcap][3] per-peer outbox, peer p at peer_base[p]
    uint64_t* peer_base;      // [G]
    uint64_t* outn;           // [G] events in peer p's outbox this round
    uint64_t* sent;           // [G] of which already sent
    Slot* st;                 // staging, bcap per block
    uint32_t* st_dst;
    sg_trace_rec* trace;
    uint64_t* wlog;           // [wlog_cap][2] executed windows {start, end}
    uint64_t wlog_cap;
    RoundState* rs;
    uint64_t* red3;           // single-shard reduce output
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

// Destination draw; returns N when no host is selected (test_phold.c:176-177)
// and the chosen host's info record.
__device__ __forceinline__ uint32_t choose_dst(const Dev& d, int32_t x, HostInfo& info) {
    const uint32_t N = d.N;
    const HostInfo* w = d.hinfo;
    if (d.dst_rule == SG_DST_UNIFORM_FLOOR) {
        double r = (double)x / 2147483647.0;
        double f = floor(r * (double)N);
        uint32_t dd = (uint32_t)f;
        dd = dd >= N ? N - 1 : dd;
        info = w[dd];
        return dd;
    }
    // first i with x <= wt[i] (non-decreasing): guess from the uniform
    // position, walk a few steps, bisect the rest.
    uint32_t g = (uint32_t)(((uint64_t)(uint32_t)x * N) >> 31);
    if (g >= N) g = N - 1;
    HostInfo cur = w[g];
    if (x <= cur.wt) {
        for (int k = 0; k < 8; ++k) {
            if (g == 0) break;
            const HostInfo prev = w[g - 1];
            if (x > prev.wt) break;
            --g;
            cur = prev;
        }
        if (g > 0 && x <= w[g - 1].wt) {
            uint32_t lo = 0, hi = g - 1;  // answer in [lo, hi]
            while (lo < hi) {
                const uint32_t mid = lo + (hi - lo) / 2;
                if (x <= w[mid].wt) hi = mid; else lo = mid + 1;
            }
            g = lo;
            cur = w[g];
        }
        info = cur;
        return g;
    }
    if (x > w[N - 1].wt) return N;
    for (int k = 0; k < 8; ++k) {
        ++g;
        cur = w[g];
        if (x <= cur.wt) {
            info = cur;
            return g;
        }
    }
    uint32_t lo = g + 1, hi = N - 1;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (x <= w[mid].wt) hi = mid; else lo = mid + 1;
    }
    info = w[lo];
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

// event_compare with equal dst (event.c:122-148) on (time, src<<40|seq).
// Bitwise, not short-circuit, and the running minimum is updated through one
// select mask: ROCm 7.2 mis-compiled the branchy form inside the selection
// loop (the winning slot index was not updated on a time tie).
__device__ __forceinline__ bool key_less(uint64_t t, uint64_t k, uint64_t bt, uint64_t bk) {
    return (t < bt) | ((t == bt) & (k < bk));
}
struct Best {
    uint64_t t, k;
    uint32_t slot;
};
__device__ __forceinline__ void best_take(Best& b, uint64_t t, uint64_t k, uint32_t slot) {
    const bool take = key_less(t, k, b.t, b.k);
    b.t = take ? t : b.t;
    b.k = take ? k : b.k;
    b.slot = take ? slot : b.slot;
}

__global__ void k_boot(Dev d) {
    const uint32_t lh = blockIdx.x * BLOCK + threadIdx.x;
    if (lh < d.L) {
        const uint32_t h = d.lo + lh;
        // worker_bootHosts: self event at t=0 carrying id 0 (event.c:38)
        d.bag[(size_t)lh * d.CAP] = Slot{0, (uint64_t)h << SRC_SHIFT};
        d.bag_cnt[lh] = 1;
        d.hmin[lh] = 0;
        HostState s = d.hs[lh];
        s.evc = 1;
        s.pops = 0;
        s.digest = 0;
        d.hs[lh] = s;
    }
    if (threadIdx.x < NCTR) d.pcum[(size_t)threadIdx.x * d.nblocks + blockIdx.x] = 0;
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
        rs->phase = 0;
        rs->loc_min = SIMTIME_MAX;
        rs->loc_jmin = UINT64_MAX;
        rs->steps = 0;
        rs->peak_peer = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x < d.G && d.outn) {
        d.outn[threadIdx.x] = 0;
        d.sent[threadIdx.x] = 0;
        d.peer_base[threadIdx.x] = 0;
    }
}

struct Acc {
    uint64_t ctr[NCTR];
    uint64_t jmin;   // min truncated latency of attempted sends
    uint64_t emin;   // min time of staged (emitted) events
    bool overflow;
};

struct HostCtx {
    uint32_t h, vh;
    HostState s;
};

// Execute one popped event (worker.c:165-176 + the PHOLD body + worker_sendPacket).
// Self events that fall inside the window go back to the host's own queue
// through `append` (they are popped later this round); everything else is
// staged in the workgroup's region for k_insert / k_pack.
template <class Append>
__device__ __forceinline__ void execute_event(const Dev& d, uint64_t E, HostCtx& c, Acc& a, uint64_t bt,
                                              uint64_t bk, uint32_t* s_emit, uint32_t* s_peer,
                                              Append append) {
    const uint32_t bsrc = (uint32_t)(bk >> SRC_SHIFT);
    const uint64_t bseq = bk & SEQ_MASK;
    c.s.digest += digest_mix(c.s.pops, bt, bsrc, bseq);
    if (d.trace) {
        const uint64_t ts = atomicAdd((unsigned long long*)&d.rs->trace_len, 1ULL);
        if (ts < d.trace_cap) {
            sg_trace_rec r;
            r.time = bt;
            r.seq = bseq;
            r.host = c.h;
            r.src = bsrc;
            r.pos = c.s.pops;
            d.trace[ts] = r;
        } else {
            a.overflow = true;
        }
    }
    ++c.s.pops;
    ++a.ctr[C_POPS];
    const bool boot = (bsrc == c.h && bseq == 0);
    a.ctr[C_BOOTS] += boot;
    const uint32_t nsend = boot ? d.load : 1u;  // test_phold.c:234-239 / 310-312
    for (uint32_t m = 0; m < nsend; ++m) {
        const int32_t x = dev_rand_r(c.s.rng);
        HostInfo di;
        const uint32_t dst = choose_dst(d, x, di);
        if (dst >= d.N) {
            ++a.ctr[C_NULL];
            continue;
        }
        ++a.ctr[C_SENDS];
        const PairRec pr = d.pairs[(size_t)c.vh * d.V + di.vertex];
        a.jmin = pr.jump < a.jmin ? pr.jump : a.jmin;  // path discovery (topology.c:1374-1385)
        const int32_t ch = dev_rand_r(c.s.rng);          // worker.c:268-269
        if (!(bt < d.bootstrap_end || ch <= pr.keep)) {
            ++a.ctr[C_DROPREL];
            continue;
        }
        uint64_t tn = bt + pr.delay;        // worker.c:275-277
        const uint64_t sq = c.s.evc++;      // event.c:38
        if (tn >= d.end_time) {             // scheduler.c:343-346
            ++a.ctr[C_DROPEND];
            continue;
        }
        const uint64_t key = ((uint64_t)c.h << SRC_SHIFT) | sq;
        if (dst == c.h && tn < E) {
            ++a.ctr[C_SAME];
            if (!append(tn, key)) a.overflow = true;
            continue;
        }
        if (dst != c.h && tn < E) {  // host_single.c:180-184
            tn = E;
            ++a.ctr[C_BUMPED];
        }
        const uint32_t slot = atomicAdd(s_emit, 1u);
        if (slot >= d.bcap) {
            a.overflow = true;
            continue;
        }
        const size_t so = (size_t)blockIdx.x * d.bcap + slot;
        d.st[so] = Slot{tn, key};
        d.st_dst[so] = dst;
        if (d.G > 1) atomicAdd(&s_peer[owner_of(d, dst)], 1u);
        a.emin = tn < a.emin ? tn : a.emin;
        ++a.ctr[C_EMIT];
    }
}

// One lane per host.  MASKED (queue_cap <= 64): the queue is read once with
// independent 16-B loads, the minimum event before the barrier and the last
// slot are kept from that scan, further due slots are tracked in a 64-bit
// mask.  Otherwise every pop rescans the queue.
template <bool MASKED>
__global__ __launch_bounds__(BLOCK) void k_process(Dev d) {
    __shared__ uint32_t s_emit;
    __shared__ uint32_t s_peer[MAXG];
    __shared__ uint64_t s_red[BLOCK / 64][NCTR + NMIN];
    const RoundState* rs = d.rs;
    if (rs->done | rs->phase) return;
    const uint64_t E = rs->E;
    const uint32_t lh = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t L = d.L;
    if (threadIdx.x == 0) s_emit = 0;
    if (threadIdx.x < MAXG) s_peer[threadIdx.x] = 0;
    __syncthreads();

    Acc a;
#pragma unroll
    for (int i = 0; i < NCTR; ++i) a.ctr[i] = 0;
    a.jmin = UINT64_MAX;
    a.emin = SIMTIME_MAX;
    a.overflow = false;
    uint64_t newmin = SIMTIME_MAX;

    if (lh < L) {
        const uint64_t hm = d.hmin[lh];
        newmin = hm;
        if (hm < E) {
            HostCtx c;
            c.h = d.lo + lh;
            c.s = d.hs[lh];
            c.vh = d.hinfo[c.h].vertex;
            uint32_t cnt = d.bag_cnt[lh];
            // k_insert counts deliveries past capacity (flagged as overflow and
            // reported at the next sync); never read beyond the queue
            cnt = cnt < d.CAP ? cnt : d.CAP;
            a.ctr[C_ACTIVE] = 1;
            Slot* bag = d.bag + (size_t)lh * d.CAP;  // this host's queue, contiguous
            if (MASKED) {
                uint64_t due = 0, rest_min = SIMTIME_MAX;
                Best b{UINT64_MAX, 0, 0};
                Slot lastslot{0, 0};
                for (uint32_t base = 0; base < cnt; base += 8) {
                    Slot s[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) s[i] = bag[base + i];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint32_t j = base + i;
                        const bool live = j < cnt;
                        const bool isdue = live & (s[i].t < E);
                        due |= (uint64_t)isdue << j;
                        const uint64_t rt = (live & !isdue) ? s[i].t : SIMTIME_MAX;
                        rest_min = rt < rest_min ? rt : rest_min;
                        best_take(b, isdue ? s[i].t : UINT64_MAX, s[i].k, j);
                        const bool is_last = j + 1 == cnt;
                        lastslot.t = is_last ? s[i].t : lastslot.t;
                        lastslot.k = is_last ? s[i].k : lastslot.k;
                    }
                }
                // slots after the barrier only move (never leave) while popping
                newmin = rest_min;
                bool fresh = true;  // b / lastslot still describe the scanned queue
                auto append = [&](uint64_t tn, uint64_t key) -> bool {
                    if (cnt >= d.CAP) return false;
                    bag[cnt] = Slot{tn, key};
                    due |= 1ULL << cnt;
                    ++cnt;
                    return true;
                };
                while (due) {
                    if (!fresh) {
                        b = Best{UINT64_MAX, 0, 0};
                        uint64_t m = due;
                        while (m) {
                            const uint32_t j = (uint32_t)__builtin_ctzll(m);
                            m &= m - 1;
                            const Slot s = bag[j];
                            best_take(b, s.t, s.k, j);
                        }
                    }
                    const uint32_t best = b.slot;
                    const uint64_t bt = b.t, bk = b.k;
                    // remove `best`: the last slot fills the hole
                    const uint32_t last = cnt - 1;
                    due &= ~(1ULL << best);
                    if (best != last) {
                        const Slot ls = fresh ? lastslot : bag[last];
                        bag[best] = ls;
                        const uint64_t lastbit = (due >> last) & 1ULL;
                        due &= ~(1ULL << last);
                        due |= lastbit << best;
                    }
                    cnt = last;
                    fresh = false;
                    execute_event(d, E, c, a, bt, bk, &s_emit, s_peer, append);
                }
            } else {
                auto append = [&](uint64_t tn, uint64_t key) -> bool {
                    if (cnt >= d.CAP) return false;
                    bag[cnt] = Slot{tn, key};
                    ++cnt;
                    return true;
                };
                for (;;) {
                    Best b{UINT64_MAX, 0, UINT32_MAX};
                    uint64_t rest_min = SIMTIME_MAX;
                    for (uint32_t j = 0; j < cnt; ++j) {
                        const Slot s = bag[j];
                        if (s.t < E) {
                            best_take(b, s.t, s.k, j);
                        } else if (s.t < rest_min) {
                            rest_min = s.t;
                        }
                    }
                    if (b.slot == UINT32_MAX) {
                        newmin = rest_min;
                        break;
                    }
                    --cnt;
                    if (b.slot != cnt) bag[b.slot] = bag[cnt];
                    execute_event(d, E, c, a, b.t, b.k, &s_emit, s_peer, append);
                }
            }
            d.bag_cnt[lh] = cnt;
            d.hs[lh] = c.s;
            d.hmin[lh] = newmin;
        }
    }

    // workgroup partials: cumulative counters and this round's three minima
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t v[NCTR + NMIN];
#pragma unroll
    for (int i = 0; i < NCTR; ++i) v[i] = wave_sum(a.ctr[i]);
    v[NCTR + M_JMIN] = wave_min(a.jmin);
    v[NCTR + M_EMIN] = wave_min(a.emin);
    v[NCTR + M_RMIN] = wave_min(newmin);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NCTR + NMIN; ++i) s_red[wid][i] = v[i];
    }
    if (a.overflow) atomicOr((unsigned long long*)&d.rs->overflow, 1ULL);
    __syncthreads();
    if (threadIdx.x < NCTR + NMIN) {
        const int i = threadIdx.x;
        uint64_t r = s_red[0][i];
        for (int w = 1; w < BLOCK / 64; ++w) {
            const uint64_t x = s_red[w][i];
            r = i < NCTR ? r + x : (x < r ? x : r);
        }
        if (i < NCTR) d.pcum[(size_t)i * d.nblocks + blockIdx.x] += r;
        else d.pmin[(size_t)(i - NCTR) * d.nblocks + blockIdx.x] = r;
    }
    if (threadIdx.x == 0) d.blockcnt[blockIdx.x] = s_emit < d.bcap ? s_emit : d.bcap;
    if (d.G > 1 && threadIdx.x < d.G) d.peercnt[(size_t)blockIdx.x * d.G + threadIdx.x] = s_peer[threadIdx.x];
}

// Inclusive scan across one workgroup of 1024 (16 waves).
__device__ __forceinline__ uint64_t block_incl_scan(uint64_t v, uint64_t* s_w) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    uint64_t add = 0;
    for (int w = 0; w < wid; ++w) add += s_w[w];
    __syncthreads();
    return v + add;
}

// Multi-shard, process steps: per-(block, peer) offsets of the staged events
// and each peer's outbox region.  One workgroup of 1024.
__global__ __launch_bounds__(1024) void k_peer_scan(Dev d) {
    RoundState* rs = d.rs;
    if (rs->done | rs->phase) return;
    __shared__ uint64_t s_w[16];
    __shared__ uint64_t s_tot[MAXG];
    const uint32_t NB = d.nblocks, G = d.G;
    const uint32_t chunk = (NB + 1023) / 1024;
    const uint32_t b0 = threadIdx.x * chunk;
    const uint32_t b1 = b0 + chunk < NB ? b0 + chunk : NB;
    for (uint32_t p = 0; p < G; ++p) {
        uint64_t sum = 0;
        for (uint32_t b = b0; b < b1; ++b) sum += d.peercnt[(size_t)b * G + p];
        const uint64_t incl = block_incl_scan(sum, s_w);
        uint64_t run = incl - sum;
        for (uint32_t b = b0; b < b1; ++b) {
            const size_t k = (size_t)b * G + p;
            d.peeroff[k] = (uint32_t)run;
            run += d.peercnt[k];
        }
        if (threadIdx.x == 1023) s_tot[p] = incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint64_t base = 0, peak = rs->peak_peer;
        for (uint32_t p = 0; p < G; ++p) {
            const uint64_t n = p == d.g ? 0 : s_tot[p];
            d.peer_base[p] = base;
            d.outn[p] = n;
            d.sent[p] = 0;
            base += n;
            peak = n > peak ? n : peak;
        }
        rs->peak_peer = peak;
    }
}

// Multi-shard, process steps: staged events owned by other shards → outbox
// triples {time, key, dst}, grouped by owner.
__global__ __launch_bounds__(BLOCK) void k_pack(Dev d) {
    if (d.rs->done | d.rs->phase) return;
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
        const uint64_t slot = d.peer_base[p] + d.peeroff[(size_t)b * d.G + p] + atomicAdd(&s_slot[p], 1u);
        const Slot s = d.st[so];
        int64_t* o = d.outq + slot * 3;
        o[0] = (int64_t)s.t;
        o[1] = (int64_t)s.k;
        o[2] = (int64_t)dst;
    }
}

// Every step: up to xcap outbox events per peer into the peer's exchange
// block, behind the header {n, sender has more, MIN next, min jump, overflow,
// round}.  Grid (chunks, G).
__global__ __launch_bounds__(BLOCK) void k_fill(Dev d, int64_t* send) {
    const RoundState* rs = d.rs;
    if (rs->done) return;
    const uint32_t p = blockIdx.y;
    const uint64_t left = d.outn[p] - d.sent[p];
    const uint64_t n = left < d.xcap ? left : d.xcap;
    int64_t* blk = send + (size_t)p * d.xrows * 3;
    const int64_t* src = d.outq + (d.peer_base[p] + d.sent[p]) * 3;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n * 3;
         i += (uint64_t)gridDim.x * BLOCK)
        blk[HDR * 3 + i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        uint64_t more = 0;
        for (uint32_t q = 0; q < d.G; ++q) more |= (d.outn[q] - d.sent[q] > d.xcap) ? 1u : 0u;
        blk[H_N] = (int64_t)n;
        blk[H_MORE] = (int64_t)more;
        blk[H_MIN] = (int64_t)rs->loc_min;
        blk[H_JMIN] = (int64_t)rs->loc_jmin;
        blk[H_OVF] = (int64_t)rs->overflow;
        blk[H_ROUND] = (int64_t)rs->rounds;
    }
}

__device__ __forceinline__ void deliver(const Dev& d, const Slot s, uint32_t dst) {
    const uint32_t dl = dst - d.lo;
    const uint32_t slot = atomicAdd(&d.bag_cnt[dl], 1u);
    if (slot >= d.CAP) {
        atomicOr((unsigned long long*)&d.rs->overflow, 4ULL);
        return;
    }
    d.bag[(size_t)dl * d.CAP + slot] = s;
    // the earliest-time word only decreases here: skip the atomic when it is
    // already at or below this event
    if (s.t < __hip_atomic_load(&d.hmin[dl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin((unsigned long long*)&d.hmin[dl], (unsigned long long)s.t);
}

// Staged events of this shard's own hosts → destination queues.
__global__ __launch_bounds__(BLOCK) void k_insert(Dev d) {
    if (d.rs->done | d.rs->phase) return;
    const uint32_t b = blockIdx.x;
    const uint32_t n = d.blockcnt[b];
    for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
        const size_t so = (size_t)b * d.bcap + i;
        const uint32_t dst = d.st_dst[so];
        if (dst - d.lo >= d.L) continue;  // another shard's host
        deliver(d, d.st[so], dst);
    }
}

// Received exchange blocks → destination queues.  Grid (chunks, G).
__global__ __launch_bounds__(BLOCK) void k_insert_recv(Dev d, const int64_t* recv) {
    if (d.rs->done) return;
    const uint32_t p = blockIdx.y;
    if (p == d.g) return;
    const int64_t* blk = recv + (size_t)p * d.xrows * 3;
    const uint64_t n = (uint64_t)blk[H_N];
    if (n > d.xcap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long*)&d.rs->overflow, 8ULL);
        return;
    }
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const int64_t* r = blk + (HDR + i) * 3;
        const uint32_t dst = (uint32_t)r[2];
        if (dst - d.lo >= d.L) {
            atomicOr((unsigned long long*)&d.rs->overflow, 8ULL);
            continue;
        }
        deliver(d, Slot{(uint64_t)r[0], (uint64_t)r[1]}, dst);
    }
}

// master_slaveFinishedCurrentRound (master.c:450-480) on a reduced triple.
__device__ void apply_window(const Dev& d, uint64_t minNext, uint64_t jmin, uint64_t not_overflow) {
    RoundState* rs = d.rs;
    rs->overflow |= ~not_overflow;
    if (d.wlog && rs->rounds < d.wlog_cap) {  // the window just executed
        d.wlog[2 * rs->rounds] = rs->S;
        d.wlog[2 * rs->rounds + 1] = rs->E;
    }
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
    uint64_t end = minNext + jump;  // unsigned wrap as in the reference
    if (end > d.end_time) end = d.end_time;
    rs->S = start;
    rs->E = end;
    rs->done = start < end ? 0 : 1;
}

// Local MIN next time (remaining ∪ staged) and discovery min; with apply != 0
// (single shard) also the next window.  One workgroup of 1024.
__global__ __launch_bounds__(1024) void k_reduce(Dev d, uint64_t* out3, int apply) {
    if (d.rs->done | d.rs->phase) return;
    __shared__ uint64_t s_v[16][NMIN];
    uint64_t v[NMIN];
#pragma unroll
    for (int i = 0; i < NMIN; ++i) v[i] = UINT64_MAX;
    const size_t NB = d.nblocks;
    for (uint32_t b = threadIdx.x; b < NB; b += 1024) {
#pragma unroll
        for (int i = 0; i < NMIN; ++i) {
            const uint64_t x = d.pmin[(size_t)i * NB + b];
            v[i] = x < v[i] ? x : v[i];
        }
    }
#pragma unroll
    for (int i = 0; i < NMIN; ++i) v[i] = wave_min(v[i]);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NMIN; ++i) s_v[wid][i] = v[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t r[NMIN];
        for (int i = 0; i < NMIN; ++i) {
            r[i] = s_v[0][i];
            for (int w = 1; w < 16; ++w) r[i] = s_v[w][i] < r[i] ? s_v[w][i] : r[i];
        }
        RoundState* rs = d.rs;
        const uint64_t j = rs->jmin < r[M_JMIN] ? rs->jmin : r[M_JMIN];
        rs->jmin = j;
        const uint64_t m = r[M_EMIN] < r[M_RMIN] ? r[M_EMIN] : r[M_RMIN];
        rs->loc_min = m;
        rs->loc_jmin = j;
        if (out3) {
            out3[0] = m;
            out3[1] = j;
            out3[2] = ~rs->overflow;
        }
        if (apply) apply_window(d, m, j, ~rs->overflow);
    }
}

// Multi-shard step end: the window from the G received headers (every shard
// sees the same headers, so every shard takes the same decision).  A sender
// with outbox leftovers makes the next step a drain step: same window, no
// processing, more exchange.
__global__ void k_window(Dev d, const int64_t* recv) {
    RoundState* rs = d.rs;
    if (rs->done) return;
    uint64_t m = UINT64_MAX, j = UINT64_MAX, ovf = 0, more = 0;
    for (uint32_t p = 0; p < d.G; ++p) {
        const int64_t* blk = recv + (size_t)p * d.xrows * 3;
        more |= (uint64_t)blk[H_MORE];
        const uint64_t bm = (uint64_t)blk[H_MIN], bj = (uint64_t)blk[H_JMIN];
        m = bm < m ? bm : m;
        j = bj < j ? bj : j;
        ovf |= (uint64_t)blk[H_OVF];
        if ((uint64_t)blk[H_ROUND] != rs->rounds) ovf |= 16;  // shards out of step
    }
    for (uint32_t q = 0; q < d.G; ++q) {
        const uint64_t left = d.outn[q] - d.sent[q];
        d.sent[q] += left < d.xcap ? left : d.xcap;
    }
    rs->steps += 1;
    if (more) {
        rs->phase = 1;
        rs->overflow |= ovf;
        return;
    }
    rs->phase = 0;
    apply_window(d, m, j, ~ovf);
}

// Cumulative counters (stats on demand) and pending events.
__global__ __launch_bounds__(1024) void k_stats(Dev d, unsigned long long* pending) {
    __shared__ uint64_t s_c[16][NCTR + 1];
    uint64_t c[NCTR + 1];
    for (int i = 0; i <= NCTR; ++i) c[i] = 0;
    for (uint32_t b = threadIdx.x; b < d.nblocks; b += 1024)
        for (int i = 0; i < NCTR; ++i) c[i] += d.pcum[(size_t)i * d.nblocks + b];
    for (uint32_t h = threadIdx.x; h < d.L; h += 1024) {
        const uint32_t n = d.bag_cnt[h];
        c[NCTR] += n < d.CAP ? n : d.CAP;
    }
    for (int i = 0; i <= NCTR; ++i) c[i] = wave_sum(c[i]);
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i <= NCTR; ++i) s_c[threadIdx.x >> 6][i] = c[i];
    __syncthreads();
    if (threadIdx.x <= NCTR) {
        uint64_t t = 0;
        for (int w = 0; w < 16; ++w) t += s_c[w][threadIdx.x];
        if (threadIdx.x < NCTR) d.rs->ctr[threadIdx.x] = t;
        else *pending = t;
    }
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
    if (p.n_hosts == 0 || p.n_hosts > (1u << (64 - SRC_SHIFT)) || p.n_vertices == 0 || G > MAXG ||
        p.shard_index >= G || G > p.n_hosts || !t->host_vertex || !t->host_rng || !t->delay_ns ||
        !t->keep_max || !t->jump_ms || (p.dst_rule == SG_DST_WEIGHTS && !t->weight_thresh) ||
        p.dst_rule > 1 || p.window_rule > 1 || p.load == 0) {
        sg_set_error("sg_engine_create: invalid parameters (n_hosts must be in [1, 2^24])");
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
    d.CAP = (d.CAP + 7u) & ~7u;           // the masked scan reads slots in groups of 8
    d.load = p.load;
    d.dst_rule = p.dst_rule;
    d.window_rule = p.window_rule;
    d.end_time = p.end_time;
    d.bootstrap_end = p.bootstrap_end;
    d.fixed_jump = p.fixed_jump;
    d.runahead_min = p.runahead_min;
    d.trace_cap = p.trace_capacity;
    d.xcap = p.exchange_cap ? p.exchange_cap : 4096;
    d.xrows = HDR + d.xcap;
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
    HostInfo* hinfo;
    PairRec* pairs;
    ALLOC(hinfo, N);
    ALLOC(pairs, VV);
    d.hinfo = hinfo;
    d.pairs = pairs;
    ALLOC(d.bag, S);
    ALLOC(d.bag_cnt, L);
    ALLOC(d.hmin, L);
    ALLOC(d.hs, L);
    ALLOC(d.pmin, NB * NMIN);
    ALLOC(d.pcum, NB * NCTR);
    ALLOC(d.blockcnt, NB);
    ALLOC(d.peercnt, NB * G);
    ALLOC(d.peeroff, NB * G);
    if (G > 1) {
        ALLOC(d.outq, ST * 3);
        ALLOC(d.peer_base, G);
        ALLOC(d.outn, G);
        ALLOC(d.sent, G);
    }
    ALLOC(d.st, ST);
    ALLOC(d.st_dst, ST);
    ALLOC(d.rs, 1);
    ALLOC(d.red3, 4);
    if (d.trace_cap) ALLOC(d.trace, d.trace_cap);
    d.wlog_cap = d.trace_cap ? 1u << 20 : 0;
    if (d.wlog_cap) ALLOC(d.wlog, 2 * d.wlog_cap);
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
    // pack the tables on the host
    std::vector<HostInfo> hi(N);
    for (size_t i = 0; i < N; ++i) {
        hi[i].vertex = t->host_vertex[i];
        hi[i].wt = t->weight_thresh ? t->weight_thresh[i] : 0;
        if (hi[i].vertex >= d.V) {
            sg_engine_destroy(e);
            sg_set_error("sg_engine_create: host %zu attached to vertex %u >= %u", i, hi[i].vertex, d.V);
            return SG_ERR_INVAL;
        }
    }
    std::vector<PairRec> pr(VV);
    for (size_t i = 0; i < VV; ++i) pr[i] = PairRec{t->delay_ns[i], t->keep_max[i], t->jump_ms[i]};
    std::vector<HostState> hs(L);
    for (size_t i = 0; i < L; ++i) hs[i] = HostState{t->host_rng[d.lo + i], 0, 0, 0, 0};
    hipError_t err = hipSuccess;
    err = err != hipSuccess ? err : hipMemcpy(hinfo, hi.data(), N * sizeof(HostInfo), hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(pairs, pr.data(), VV * sizeof(PairRec), hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(d.hs, hs.data(), L * sizeof(HostState), hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemset(d.rs, 0, sizeof(RoundState));
    err = err != hipSuccess ? err : hipMemset(d.pcum, 0, NB * NCTR * 8);
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
        if (d.CAP <= 64)
            hipLaunchKernelGGL(k_process<true>, dim3(d.nblocks), dim3(BLOCK), 0, e->stream, d);
        else
            hipLaunchKernelGGL(k_process<false>, dim3(d.nblocks), dim3(BLOCK), 0, e->stream, d);
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
        hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, e->stream, d, d.red3, 1);
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
    hipLaunchKernelGGL(k_stats, dim3(1), dim3(1024), 0, e->stream, e->d, dp);
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
    out->exchange_steps = r.steps;
    out->phase = r.phase;
    return SG_OK;
}

int sg_engine_active_hosts(sg_engine* e, uint64_t* active, uint64_t* emitted) {
    if (!e) return SG_ERR_INVAL;
    sg_round_stats s;
    int rc = sg_engine_stats(e, &s);
    if (rc) return rc;
    if (active) *active = e->h_rs->ctr[C_ACTIVE];
    if (emitted) *emitted = e->h_rs->ctr[C_EMIT];
    return SG_OK;
}

int sg_engine_host_state(sg_engine* e, uint64_t* digest, uint64_t* pops, uint32_t* rng,
                         uint64_t* event_counter) {
    if (!e) return SG_ERR_INVAL;
    const size_t L = e->d.L;
    std::vector<HostState> hs(L);
    HIPCHK(hipMemcpyAsync(hs.data(), e->d.hs, L * sizeof(HostState), hipMemcpyDeviceToHost, e->stream));
    int rc = sg_engine_sync(e);
    if (rc) return rc;
    for (size_t i = 0; i < L; ++i) {
        if (digest) digest[i] = hs[i].digest;
        if (pops) pops[i] = hs[i].pops;
        if (rng) rng[i] = hs[i].rng;
        if (event_counter) event_counter[i] = hs[i].evc;
    }
    return SG_OK;
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

int sg_engine_windows(sg_engine* e, uint64_t* out_pairs, uint64_t capacity, uint64_t* n_out) {
    if (!e) return SG_ERR_INVAL;
    int rc = read_rs(e);
    if (rc) return rc;
    uint64_t n = e->h_rs->rounds < e->d.wlog_cap ? e->h_rs->rounds : e->d.wlog_cap;
    if (n_out) *n_out = n;
    if (out_pairs && capacity && n) {
        const uint64_t m = n < capacity ? n : capacity;
        HIPCHK(hipMemcpy(out_pairs, e->d.wlog, m * 16, hipMemcpyDeviceToHost));
    }
    return SG_OK;
}

static int need_sharded(sg_engine* e, const char* fn) {
    if (!e || !e->booted) {
        sg_set_error("%s: engine not booted", fn);
        return SG_ERR_STATE;
    }
    if (e->d.G < 2) {
        sg_set_error("%s: single-shard engine, use sg_engine_run / enqueue_round", fn);
        return SG_ERR_STATE;
    }
    return SG_OK;
}

static uint32_t fill_chunks(const Dev& d) {
    uint64_t c = (d.xcap * 3 + BLOCK * 4 - 1) / (BLOCK * 4);
    return (uint32_t)(c < 1 ? 1 : c > 256 ? 256 : c);
}

int sg_engine_exchange_rows(sg_engine* e, uint64_t* rows) {
    if (!e || !rows) return SG_ERR_INVAL;
    *rows = e->d.xrows;
    return SG_OK;
}

int sg_engine_set_exchange_cap(sg_engine* e, uint64_t exchange_cap) {
    if (!e || exchange_cap == 0) {
        sg_set_error("sg_engine_set_exchange_cap: exchange_cap must be > 0");
        return SG_ERR_INVAL;
    }
    e->d.xcap = exchange_cap;
    e->d.xrows = HDR + exchange_cap;
    return SG_OK;
}

int sg_engine_exchange_peak(sg_engine* e, uint64_t* peak, int reset) {
    if (!e) return SG_ERR_INVAL;
    int rc = read_rs(e);
    if (rc) return rc;
    if (peak) *peak = e->h_rs->peak_peer;
    if (reset) HIPCHK(hipMemsetAsync(&e->d.rs->peak_peer, 0, 8, e->stream));
    return SG_OK;
}

int sg_engine_step_send(sg_engine* e, int64_t* send) {
    int rc = need_sharded(e, "sg_engine_step_send");
    if (rc) return rc;
    if (!send) {
        sg_set_error("sg_engine_step_send: NULL send buffer");
        return SG_ERR_INVAL;
    }
    if ((rc = enqueue_process(e))) return rc;
    const Dev& d = e->d;
    return timed_launch(e, 2, [&] {
        hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, e->stream, d, (uint64_t*)nullptr, 0);
        hipLaunchKernelGGL(k_peer_scan, dim3(1), dim3(1024), 0, e->stream, d);
        hipLaunchKernelGGL(k_pack, dim3(d.nblocks), dim3(BLOCK), 0, e->stream, d);
        hipLaunchKernelGGL(k_fill, dim3(fill_chunks(d), d.G), dim3(BLOCK), 0, e->stream, d, send);
    });
}

int sg_engine_step_recv(sg_engine* e, const int64_t* recv) {
    int rc = need_sharded(e, "sg_engine_step_recv");
    if (rc) return rc;
    if (!recv) {
        sg_set_error("sg_engine_step_recv: NULL receive buffer");
        return SG_ERR_INVAL;
    }
    if ((rc = enqueue_local_insert(e))) return rc;
    const Dev& d = e->d;
    if ((rc = timed_launch(e, 1, [&] {
             hipLaunchKernelGGL(k_insert_recv, dim3(fill_chunks(d), d.G), dim3(BLOCK), 0, e->stream, d,
                                recv);
         })))
        return rc;
    return timed_launch(e, 2, [&] {
        hipLaunchKernelGGL(k_window, dim3(1), dim3(1), 0, e->stream, d, recv);
    });
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
