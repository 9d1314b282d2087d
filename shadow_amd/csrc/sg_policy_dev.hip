// sg_policy_dev.hip — device half of the `gpu` SchedulerPolicy (Mode P).
//
// Per-host event queues live in HBM (slot-major SoA, as in sg_engine.hip) and
// carry an opaque 64-bit handle (the Shadow Event*) next to the event_compare
// key (time, src host id, srcHostEventID; the destination is the queue).
//   k_pins      staged events → destination queues; overflowing records are
//               listed so the host can grow the queues and re-deliver them
//   extraction  three passes over the hosts whose earliest event is before
//               the barrier (every other host is one 8-byte read):
//     k_pcount    due events per host, block sums
//     k_pscan     exclusive scan of the block sums (one workgroup)
//     k_pwrite    per host: its due events' slots gathered in registers,
//                 ranked among themselves in event_compare order
//                 (event.c:110-153), written as one contiguous run at the
//                 host-ordered offset; the rest compacted in place
//     The runs are in host order, so off[h + 1] - off[h] is host h's count:
//     one N + 1 offset array crosses PCIe, no count array.
//   k_pmin      MIN over the hosts' earliest times (host_single.c:273-305)
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "sg_policy_dev.h"

extern "C" void sg_set_error(const char* fmt, ...);

namespace {

constexpr int BLOCK = 256;
constexpr uint64_t SIMTIME_MAX = UINT64_MAX - 1;

struct Q {
    uint32_t n, cap;
    uint64_t* time;
    uint64_t* seq;
    uint64_t* handle;
    uint32_t* src;
    uint32_t* cnt;
    uint64_t* hmin;
};

__global__ void k_pinit(Q q) {
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    if (h < q.n) {
        q.cnt[h] = 0;
        q.hmin[h] = SIMTIME_MAX;
    }
}

__global__ void k_pins(Q q, const sgp_rec* r, uint64_t n, uint32_t* fail, uint32_t* nfail) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const sgp_rec e = r[i];
        const uint32_t slot = atomicAdd(&q.cnt[e.dst], 1u);
        if (slot >= q.cap) {
            fail[atomicAdd(nfail, 1u)] = (uint32_t)i;
            continue;
        }
        const size_t k = (size_t)slot * q.n + e.dst;
        q.time[k] = e.time;
        q.seq[k] = e.seq;
        q.handle[k] = e.handle;
        q.src[k] = e.src_id;
        atomicMin((unsigned long long*)&q.hmin[e.dst], (unsigned long long)e.time);
    }
}

__global__ void k_pclamp(Q q, uint32_t oldcap) {
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    if (h < q.n && q.cnt[h] > oldcap) q.cnt[h] = oldcap;
}

__global__ void k_pcopy(Q to, Q from) {
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    if (h >= from.n) return;
    const uint32_t c = from.cnt[h];
    for (uint32_t j = 0; j < c; ++j) {
        const size_t a = (size_t)j * from.n + h, b = (size_t)j * to.n + h;
        to.time[b] = from.time[a];
        to.seq[b] = from.seq[a];
        to.handle[b] = from.handle[a];
        to.src[b] = from.src[a];
    }
    to.cnt[h] = c;
    to.hmin[h] = from.hmin[h];
}

__device__ __forceinline__ bool key_less(uint64_t t, uint32_t s, uint64_t q, uint64_t bt, uint32_t bs,
                                         uint64_t bq) {
    // bitwise, not short-circuit (see sg_engine.hip key_less)
    return (t < bt) | ((t == bt) & ((s < bs) | ((s == bs) & (q < bq))));
}

// Due events of host h (time < barrier) and the earliest time after it.
__global__ __launch_bounds__(BLOCK) void k_pcount(Q q, uint64_t barrier, uint32_t* kcnt, uint32_t* bsum) {
    __shared__ uint32_t s_w[BLOCK / 64];
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t k = 0;
    if (h < q.n && q.hmin[h] < barrier) {
        const uint32_t c = q.cnt[h];
        for (uint32_t j = 0; j < c; ++j) k += q.time[(size_t)j * q.n + h] < barrier;
    }
    if (h < q.n) kcnt[h] = k;
    uint32_t w = k;
    for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < BLOCK / 64; ++i) t += s_w[i];
        bsum[blockIdx.x] = t;
    }
}

// Exclusive scan of nb block sums in place (one workgroup of 1024), total out.
__global__ __launch_bounds__(1024) void k_pscan(uint32_t* bsum, uint32_t nb, unsigned long long* total) {
    __shared__ uint32_t s[1024];
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < nb ? bsum[i] : 0;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const uint32_t u = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
            __syncthreads();
            s[threadIdx.x] += u;
            __syncthreads();
        }
        if (i < nb) bsum[i] = carry + s[threadIdx.x] - v;
        carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

constexpr uint32_t KREG = 8;  // due events a lane ranks in registers; more take the slow path

__global__ __launch_bounds__(BLOCK) void k_pwrite(Q q, uint64_t barrier, const uint32_t* kcnt,
                                                  const uint32_t* boff, sgp_rec* out, uint32_t* off) {
    __shared__ uint32_t s[BLOCK];
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    const size_t N = q.n;
    const uint32_t k = h < q.n ? kcnt[h] : 0;
    s[threadIdx.x] = k;
    __syncthreads();
    for (int o = 1; o < BLOCK; o <<= 1) {
        const uint32_t u = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
        __syncthreads();
        s[threadIdx.x] += u;
        __syncthreads();
    }
    const uint32_t base = boff[blockIdx.x] + s[threadIdx.x] - k;
    if (h < q.n) off[h] = base;
    if (h + 1 == q.n) off[q.n] = base + k;
    if (k == 0) return;
    const uint32_t c = q.cnt[h];
    // the due slots, in registers (the host's times are read once)
    uint32_t idx[KREG] = {};
    uint64_t tt[KREG] = {};
    uint32_t nd = 0;
    uint64_t rest = SIMTIME_MAX;
    for (uint32_t j = 0; j < c; ++j) {
        const uint64_t t = q.time[(size_t)j * N + h];
        if (t < barrier) {
#pragma unroll
            for (uint32_t a = 0; a < KREG; ++a) {  // selects, so the arrays stay in registers
                const bool w = a == nd;
                idx[a] = w ? j : idx[a];
                tt[a] = w ? t : tt[a];
            }
            ++nd;
        } else if (t < rest) {
            rest = t;
        }
    }
    if (nd <= KREG) {
        uint32_t ss[KREG];
        uint64_t sq[KREG];
#pragma unroll
        for (uint32_t a = 0; a < KREG; ++a) {
            if (a >= nd) break;
            const size_t ka = (size_t)idx[a] * N + h;
            ss[a] = q.src[ka];
            sq[a] = q.seq[ka];
        }
#pragma unroll
        for (uint32_t a = 0; a < KREG; ++a) {
            if (a >= nd) break;
            uint32_t rank = 0;
#pragma unroll
            for (uint32_t b = 0; b < KREG; ++b) {
                if (b >= nd) break;
                rank += key_less(tt[b], ss[b], sq[b], tt[a], ss[a], sq[a]);
            }
            sgp_rec r;
            r.time = tt[a];
            r.seq = sq[a];
            r.handle = q.handle[(size_t)idx[a] * N + h];
            r.src_id = ss[a];
            r.dst = h;
            out[base + rank] = r;
        }
    } else {
        // many due events at one host: rank each among the due ones from memory
        for (uint32_t i = 0; i < c; ++i) {
            const size_t ki = (size_t)i * N + h;
            const uint64_t ti = q.time[ki];
            if (ti >= barrier) continue;
            const uint32_t si = q.src[ki];
            const uint64_t qi = q.seq[ki];
            uint32_t rank = 0;
            for (uint32_t j = 0; j < c; ++j) {
                const size_t kj = (size_t)j * N + h;
                const uint64_t tj = q.time[kj];
                if (tj < barrier && key_less(tj, q.src[kj], q.seq[kj], ti, si, qi)) ++rank;
            }
            sgp_rec r;
            r.time = ti;
            r.seq = qi;
            r.handle = q.handle[ki];
            r.src_id = si;
            r.dst = h;
            out[base + rank] = r;
        }
    }
    // compact the events after the barrier to the front
    uint32_t w = 0;
    for (uint32_t j = 0; j < c; ++j) {
        const size_t kj = (size_t)j * N + h;
        const uint64_t t = q.time[kj];
        if (t < barrier) continue;
        if (w != j) {
            const size_t kw = (size_t)w * N + h;
            q.time[kw] = t;
            q.seq[kw] = q.seq[kj];
            q.handle[kw] = q.handle[kj];
            q.src[kw] = q.src[kj];
        }
        ++w;
    }
    q.cnt[h] = w;
    q.hmin[h] = rest;
}

__global__ void k_pmin(Q q, unsigned long long* out) {
    uint64_t m = SIMTIME_MAX;
    for (uint32_t h = blockIdx.x * BLOCK + threadIdx.x; h < q.n; h += gridDim.x * BLOCK) {
        const uint64_t x = q.hmin[h];
        m = x < m ? x : m;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(m, o, 64);
        m = w < m ? w : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMin(out, (unsigned long long)m);
}

__global__ void k_pall(Q q, sgp_rec* out, uint64_t cap, unsigned long long* n) {
    const uint32_t h = blockIdx.x * BLOCK + threadIdx.x;
    if (h >= q.n) return;
    const uint32_t c = q.cnt[h];
    for (uint32_t j = 0; j < c; ++j) {
        const size_t k = (size_t)j * q.n + h;
        const unsigned long long i = atomicAdd(n, 1ULL);
        if (i < cap) {
            sgp_rec r;
            r.time = q.time[k];
            r.seq = q.seq[k];
            r.handle = q.handle[k];
            r.src_id = q.src[k];
            r.dst = h;
            out[i] = r;
        }
    }
}

}  // namespace

struct sgp_dev {
    int device;
    hipStream_t s;
    Q q;
    std::vector<void*> qallocs;
    sgp_rec* d_in;      // staged records
    uint64_t in_cap;
    uint32_t* d_fail;
    uint32_t* d_nfail;
    sgp_rec* d_out;     // extracted runs
    uint64_t out_cap;
    uint32_t* d_off;     // [N + 1] host-ordered run offsets
    uint32_t* d_cnt;     // [N] due events per host
    uint32_t* d_bsum;    // [N / BLOCK] block sums, scanned in place
    unsigned long long* d_scalar;
    sgp_rec* h_runs;    // pinned
    uint64_t h_runs_cap;
    uint32_t* h_off;
    uint64_t queued;    // events in HBM
};

#define PCHK(x)                                                                         \
    do {                                                                                \
        hipError_t _e = (x);                                                            \
        if (_e != hipSuccess) {                                                         \
            sg_set_error("%s: %s (%s:%d)", #x, hipGetErrorString(_e), __FILE__, __LINE__); \
            return 3;                                                                   \
        }                                                                               \
    } while (0)

static int alloc_q(sgp_dev* d, Q* q, uint32_t n, uint32_t cap, std::vector<void*>& keep) {
    const size_t S = (size_t)n * cap;
    q->n = n;
    q->cap = cap;
    void* p[6] = {};
    size_t sz[6] = {S * 8, S * 8, S * 8, S * 4, (size_t)n * 4, (size_t)n * 8};
    for (int i = 0; i < 6; ++i) {
        if (hipMalloc(&p[i], sz[i] ? sz[i] : 8) != hipSuccess) {
            for (int j = 0; j < i; ++j) (void)hipFree(p[j]);
            sg_set_error("sgp: hipMalloc of %zu bytes failed", sz[i]);
            return 2;
        }
        keep.push_back(p[i]);
    }
    q->time = (uint64_t*)p[0];
    q->seq = (uint64_t*)p[1];
    q->handle = (uint64_t*)p[2];
    q->src = (uint32_t*)p[3];
    q->cnt = (uint32_t*)p[4];
    q->hmin = (uint64_t*)p[5];
    (void)d;
    return 0;
}

static int grow_in(sgp_dev* d, uint64_t n) {
    if (n <= d->in_cap) return 0;
    uint64_t c = d->in_cap ? d->in_cap : 4096;
    while (c < n) c *= 2;
    if (d->d_in) (void)hipFree(d->d_in);
    if (d->d_fail) (void)hipFree(d->d_fail);
    d->d_in = nullptr;
    d->d_fail = nullptr;
    PCHK(hipMalloc(&d->d_in, c * sizeof(sgp_rec)));
    PCHK(hipMalloc(&d->d_fail, c * sizeof(uint32_t)));
    d->in_cap = c;
    return 0;
}

static int grow_out(sgp_dev* d, uint64_t n) {
    if (n <= d->out_cap) return 0;
    uint64_t c = d->out_cap ? d->out_cap : 4096;
    while (c < n) c *= 2;
    if (d->d_out) (void)hipFree(d->d_out);
    if (d->h_runs) (void)hipHostFree(d->h_runs);
    d->d_out = nullptr;
    d->h_runs = nullptr;
    PCHK(hipMalloc(&d->d_out, c * sizeof(sgp_rec)));
    PCHK(hipHostMalloc((void**)&d->h_runs, c * sizeof(sgp_rec), hipHostMallocDefault));
    d->out_cap = c;
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
    sgp_dev* d = new sgp_dev();  // value-initialised: pointers and counters zero
    d->device = device;
    if (n_hosts == 0) n_hosts = 1;
    if (cap == 0) cap = 64;
    int rc = alloc_q(d, &d->q, n_hosts, cap, d->qallocs);
    if (rc) {
        sgp_dev_destroy(d);
        return rc;
    }
    if (hipStreamCreateWithFlags(&d->s, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d->d_off, ((size_t)n_hosts + 1) * 4) != hipSuccess ||
        hipMalloc(&d->d_cnt, (size_t)n_hosts * 4) != hipSuccess ||
        hipMalloc(&d->d_bsum, ((size_t)n_hosts + BLOCK - 1) / BLOCK * 4) != hipSuccess ||
        hipMalloc(&d->d_nfail, 4) != hipSuccess || hipMalloc(&d->d_scalar, 16) != hipSuccess ||
        hipHostMalloc((void**)&d->h_off, ((size_t)n_hosts + 1) * 4, hipHostMallocDefault) != hipSuccess) {
        sg_set_error("sgp_dev_create: allocation failed");
        sgp_dev_destroy(d);
        return 2;
    }
    hipLaunchKernelGGL(k_pinit, dim3((n_hosts + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, d->s, d->q);
    if (hipStreamSynchronize(d->s) != hipSuccess) {
        sgp_dev_destroy(d);
        sg_set_error("sgp_dev_create: init kernel failed");
        return 3;
    }
    *out = d;
    return 0;
}

int sgp_dev_destroy(sgp_dev* d) {
    if (!d) return 0;
    if (d->s) (void)hipStreamSynchronize(d->s);
    for (void* p : d->qallocs) (void)hipFree(p);
    void* dp[] = {d->d_in, d->d_fail, d->d_out, d->d_off, d->d_cnt, d->d_bsum, d->d_nfail, d->d_scalar};
    for (void* p : dp)
        if (p) (void)hipFree(p);
    if (d->h_runs) (void)hipHostFree(d->h_runs);
    if (d->h_off) (void)hipHostFree(d->h_off);
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
    uint64_t o = 0;
    for (uint32_t i = 0; i < nseg; ++i) {
        if (lens[i])
            PCHK(hipMemcpyAsync(d->d_in + o, segs[i], lens[i] * sizeof(sgp_rec), hipMemcpyHostToDevice, d->s));
        o += lens[i];
    }
    const sgp_rec* src = d->d_in;
    uint64_t m = n;
    for (int attempt = 0; attempt < 32; ++attempt) {
        PCHK(hipMemsetAsync(d->d_nfail, 0, 4, d->s));
        uint32_t grid = (uint32_t)((m + BLOCK - 1) / BLOCK);
        if (grid > 4096) grid = 4096;
        // attempt > 0 re-delivers the records that overflowed (gathered into d_out)
        hipLaunchKernelGGL(k_pins, dim3(grid), dim3(BLOCK), 0, d->s, d->q, src, m, d->d_fail, d->d_nfail);
        PCHK(hipGetLastError());
        uint32_t nfail = 0;
        PCHK(hipMemcpyAsync(&nfail, d->d_nfail, 4, hipMemcpyDeviceToHost, d->s));
        PCHK(hipStreamSynchronize(d->s));
        if (nfail == 0) break;
        // grow every queue x2, keep the delivered events, re-deliver the rest
        const uint32_t oldcap = d->q.cap;
        hipLaunchKernelGGL(k_pclamp, dim3((d->q.n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, d->s, d->q, oldcap);
        Q nq;
        std::vector<void*> nk;
        if ((rc = alloc_q(d, &nq, d->q.n, oldcap * 2, nk))) return rc;
        hipLaunchKernelGGL(k_pcopy, dim3((d->q.n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, d->s, nq, d->q);
        PCHK(hipGetLastError());
        std::vector<uint32_t> fidx(nfail);
        std::vector<sgp_rec> all(m);
        PCHK(hipMemcpyAsync(fidx.data(), d->d_fail, nfail * 4ull, hipMemcpyDeviceToHost, d->s));
        PCHK(hipMemcpyAsync(all.data(), src, m * sizeof(sgp_rec), hipMemcpyDeviceToHost, d->s));
        PCHK(hipStreamSynchronize(d->s));
        for (void* p : d->qallocs) (void)hipFree(p);
        d->qallocs = nk;
        d->q = nq;
        std::vector<sgp_rec> redo(nfail);
        for (uint32_t i = 0; i < nfail; ++i) redo[i] = all[fidx[i]];
        if ((rc = grow_out(d, nfail))) return rc;
        PCHK(hipMemcpy(d->d_out, redo.data(), nfail * sizeof(sgp_rec), hipMemcpyHostToDevice));
        src = d->d_out;
        m = nfail;
    }
    d->queued += n;
    return 0;
}

int sgp_dev_min(sgp_dev* d, uint64_t* min_out) {
    PCHK(hipSetDevice(d->device));
    const unsigned long long init = SIMTIME_MAX;
    PCHK(hipMemcpyAsync(d->d_scalar, &init, 8, hipMemcpyHostToDevice, d->s));
    uint32_t grid = (d->q.n + BLOCK - 1) / BLOCK;
    if (grid > 1024) grid = 1024;
    hipLaunchKernelGGL(k_pmin, dim3(grid), dim3(BLOCK), 0, d->s, d->q, d->d_scalar);
    PCHK(hipGetLastError());
    unsigned long long m = 0;
    PCHK(hipMemcpyAsync(&m, d->d_scalar, 8, hipMemcpyDeviceToHost, d->s));
    PCHK(hipStreamSynchronize(d->s));
    *min_out = m;
    return 0;
}

int sgp_dev_extract(sgp_dev* d, uint64_t barrier, const sgp_rec** runs, const uint32_t** off,
                    uint64_t* total) {
    PCHK(hipSetDevice(d->device));
    int rc = grow_out(d, d->queued ? d->queued : 1);
    if (rc) return rc;
    const uint32_t n = d->q.n, nb = (n + BLOCK - 1) / BLOCK;
    hipLaunchKernelGGL(k_pcount, dim3(nb), dim3(BLOCK), 0, d->s, d->q, barrier, d->d_cnt, d->d_bsum);
    hipLaunchKernelGGL(k_pscan, dim3(1), dim3(1024), 0, d->s, d->d_bsum, nb, d->d_scalar);
    hipLaunchKernelGGL(k_pwrite, dim3(nb), dim3(BLOCK), 0, d->s, d->q, barrier, d->d_cnt, d->d_bsum,
                       d->d_out, d->d_off);
    PCHK(hipGetLastError());
    unsigned long long t = 0;
    PCHK(hipMemcpyAsync(&t, d->d_scalar, 8, hipMemcpyDeviceToHost, d->s));
    PCHK(hipMemcpyAsync(d->h_off, d->d_off, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost, d->s));
    PCHK(hipStreamSynchronize(d->s));
    if (t) PCHK(hipMemcpy(d->h_runs, d->d_out, t * sizeof(sgp_rec), hipMemcpyDeviceToHost));
    d->queued -= t;
    *runs = d->h_runs;
    *off = d->h_off;
    *total = t;
    return 0;
}

int sgp_dev_all(sgp_dev* d, sgp_rec* out, uint64_t capacity, uint64_t* n_out) {
    PCHK(hipSetDevice(d->device));
    int rc = grow_out(d, d->queued ? d->queued : 1);
    if (rc) return rc;
    PCHK(hipMemsetAsync(d->d_scalar, 0, 8, d->s));
    hipLaunchKernelGGL(k_pall, dim3((d->q.n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, d->s, d->q, d->d_out,
                       d->out_cap, d->d_scalar);
    PCHK(hipGetLastError());
    unsigned long long t = 0;
    PCHK(hipMemcpyAsync(&t, d->d_scalar, 8, hipMemcpyDeviceToHost, d->s));
    PCHK(hipStreamSynchronize(d->s));
    const uint64_t m = t < capacity ? t : capacity;
    if (out && m) PCHK(hipMemcpy(out, d->d_out, m * sizeof(sgp_rec), hipMemcpyDeviceToHost));
    *n_out = t;
    return 0;
}

}  // extern "C"
