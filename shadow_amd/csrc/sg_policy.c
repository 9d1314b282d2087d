/*
 * sg_policy.c — host half of the `gpu` SchedulerPolicy (include/shadowgpu.h §3).
 *
 * Semantics follow scheduler_policy_host_single.c (the host-family policies
 * whose per-host pop sequences are independent of the worker count):
 *   push     barrier bump for inter-host events (host_single.c:180-184); self
 *            events before the barrier stay on the CPU in a per-host heap because
 *            they must be popped in this same round; everything else is staged
 *            in the pushing thread's arena (no lock) for the end-of-round flush.
 *   pop      per thread, hosts in assignment order (host_single.c:222-267): the
 *            host's device-extracted run merged with its CPU heap, in
 *            event_compare order (event.c:110-153), while time < barrier.
 *   next     every worker arrives (after scheduler.c:386's execute barrier); the
 *            last one delivers all staged events to HBM and reduces the MIN
 *            (host_single.c:273-305, scheduler.c:393-398).
 *   prepare  the first pop with a new barrier extracts, on the device, every
 *            queued event before it, sorted per host.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "sg_policy_dev.h"
#include "shadowgpu.h"

void sg_set_error(const char* fmt, ...);

/* ---------------------------------------------------------------- heap --- */
typedef struct sheap {      /* same-round self events of one host: src = dst */
    sgp_rec* a;
    uint32_t n, cap;
} sheap;

static int rec_less(const sgp_rec* a, const sgp_rec* b) { /* event_compare, equal dst */
    if (a->time != b->time) return a->time < b->time;
    if (a->src_id != b->src_id) return a->src_id < b->src_id;
    return a->seq < b->seq;
}

static int sheap_push(sheap* h, const sgp_rec* r) {
    if (h->n == h->cap) {
        uint32_t nc = h->cap ? 2 * h->cap : 8;
        sgp_rec* na = (sgp_rec*)realloc(h->a, (size_t)nc * sizeof *na);
        if (!na) return -1;
        h->a = na;
        h->cap = nc;
    }
    uint32_t i = h->n;
    h->a[i] = *r;
    /* the owner's pop reads n without the lock (sg_policy_pop): an atomic
     * store keeps that read well-defined whoever pushes */
    __atomic_store_n(&h->n, i + 1, __ATOMIC_RELEASE);
    while (i) {
        uint32_t p = (i - 1) / 2;
        if (!rec_less(&h->a[i], &h->a[p])) break;
        sgp_rec t = h->a[i];
        h->a[i] = h->a[p];
        h->a[p] = t;
        i = p;
    }
    return 0;
}

static void sheap_pop(sheap* h) {
    const uint32_t n = h->n - 1;
    __atomic_store_n(&h->n, n, __ATOMIC_RELEASE);
    h->a[0] = h->a[n];
    uint32_t i = 0;
    for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && rec_less(&h->a[c + 1], &h->a[c])) c++;
        if (!rec_less(&h->a[c], &h->a[i])) break;
        sgp_rec t = h->a[i];
        h->a[i] = h->a[c];
        h->a[c] = t;
        i = c;
    }
}

/* ---------------------------------------------------------------- state -- */
/* Per host: what other threads may touch.  The owner's pop position lives in
 * its thread_rt (pos / gen, by the host's place in the thread's list), so the
 * pops of different workers never write a shared cache line (hosts of
 * different workers sit side by side in this array: the assignment is a
 * shuffle, scheduler.c:437-531). */
typedef struct host_rt {
    sheap selfq;              /* same-round self events (owner pushes and pops) */
    uint32_t id;              /* GQuark */
    uint32_t thread;          /* owning thread slot */
    uint32_t lpos;            /* place in the owner's host list */
    int in_self_list;
    pthread_mutex_t lock;     /* selfq, for a push from another thread */
} host_rt;

/* Per worker, one 128-B aligned slot each: a worker's pushes (arena) and pops
 * (cursor, positions) write only its own lines. */
typedef struct __attribute__((aligned(128))) thread_rt {
    uint64_t token;
    uint32_t* hosts;
    uint32_t* pos;            /* [n] next event of the host's extracted run ... */
    uint32_t* gen;            /* [n] ... valid while equal to sg_policy.run_gen */
    uint32_t n, cap, cursor;
    sg_simtime cur_barrier;
    sgp_rec* arena;
    uint64_t na, ca;
} thread_rt;

/* The calling thread's slot of the last policy it used (pop / push are called
 * per event; a linear search over the workers would read every slot). */
static _Atomic uint64_t g_policy_uid;
static __thread uint64_t tl_uid;
static __thread uint64_t tl_token;
static __thread void* tl_slot;

struct sg_policy {
    sg_simtime prepared;      /* barrier the current runs were extracted for (read per pop) */
    uint64_t uid;             /* this policy's id for the per-thread slot cache */
    sg_policy_params prm;
    sgp_dev* dev;
    host_rt* hosts;
    uint32_t n_hosts;
    uint64_t* map;            /* open addressing: id << 32 | (index + 1), one load per probe */
    uint32_t map_cap;
    thread_rt* threads;
    uint32_t n_threads;
    pthread_mutex_t foreign_lock; /* pushes from threads that own no host */
    sgp_rec* foreign;
    uint64_t nf, cf;
    /* round state */
    pthread_mutex_t m;
    pthread_cond_t cv;
    int preparing;
    uint32_t arrivals;
    uint64_t gen;
    sg_simtime next_min;
    int error;
    const sgp_rec* runs;
    const uint32_t* run_off;  /* [n + 1] per host index, host-ordered runs of the last extract */
    uint32_t run_gen;         /* bumped per extract: host run_pos values reset lazily */
    uint32_t* self_list;      /* hosts whose CPU heap may hold events */
    uint32_t n_self;
    pthread_mutex_t self_lock;
    /* SG_POLICY_PROF=1: seconds in the serial sections, printed at destroy */
    int prof;
    int pinned;               /* worker arenas in pinned memory (SG_POLICY_PINNED=1; measured
                               * no faster than pageable ones, so off by default) */
    /* flush scratch, kept across rounds (no allocation per round) */
    sgp_rec* ex;
    uint64_t ex_cap;
    const sgp_rec** segs;
    uint64_t* lens;
    double t_gather, t_insert, t_min, t_extract, t_runs;
};

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

static int64_t host_index(const sg_policy* p, uint32_t id) {
    uint32_t mask = p->map_cap - 1, i = hash32(id) & mask;
    for (;;) {
        const uint64_t e = p->map[i];
        if (e == 0) return -1;
        if ((uint32_t)(e >> 32) == id) return (int64_t)(uint32_t)e - 1;
        i = (i + 1) & mask;
    }
}

static thread_rt* thread_lookup(sg_policy* p, uint64_t token) {
    for (uint32_t i = 0; i < p->n_threads; i++)
        if (p->threads[i].token == token) return &p->threads[i];
    return NULL;
}

/* Workers are registered by add_host before any push / pop, so a slot found
 * (or not) stays valid for the policy's life. */
static thread_rt* thread_of(sg_policy* p, uint64_t token) {
    if (tl_uid == p->uid && tl_token == token) return (thread_rt*)tl_slot;
    thread_rt* t = thread_lookup(p, token);
    tl_uid = p->uid;
    tl_token = token;
    tl_slot = t;
    return t;
}

int sg_policy_create(const sg_policy_params* prm, sg_policy** out) {
    if (!prm || !out || prm->n_threads == 0 || prm->max_hosts == 0) {
        sg_set_error("sg_policy_create: bad parameters");
        return SG_ERR_INVAL;
    }
    *out = NULL;
    sg_policy* p = (sg_policy*)calloc(1, sizeof *p);
    if (!p) return SG_ERR_NOMEM;
    p->prm = *prm;
    p->uid = __atomic_add_fetch(&g_policy_uid, 1, __ATOMIC_RELAXED);
    p->hosts = (host_rt*)calloc(prm->max_hosts, sizeof(host_rt));
    p->map_cap = 16;
    while (p->map_cap < 2 * prm->max_hosts) p->map_cap <<= 1;
    p->map = (uint64_t*)calloc(p->map_cap, 8);
    const size_t tbytes = (prm->n_threads + 1) * sizeof(thread_rt);
    p->threads = (thread_rt*)aligned_alloc(128, tbytes);
    if (p->threads) memset(p->threads, 0, tbytes);
    p->self_list = (uint32_t*)malloc((size_t)prm->max_hosts * 4);
    p->segs = (const sgp_rec**)malloc((prm->n_threads + 1) * sizeof *p->segs);
    p->lens = (uint64_t*)malloc((prm->n_threads + 1) * sizeof *p->lens);
    if (!p->hosts || !p->map || !p->threads || !p->self_list || !p->segs || !p->lens) {
        sg_policy_destroy(p);
        return SG_ERR_NOMEM;
    }
    int rc = sgp_dev_create(prm->device, prm->max_hosts, prm->queue_cap, &p->dev);
    if (rc) {
        sg_policy_destroy(p);
        return rc;
    }
    pthread_mutex_init(&p->m, NULL);
    pthread_cond_init(&p->cv, NULL);
    pthread_mutex_init(&p->foreign_lock, NULL);
    pthread_mutex_init(&p->self_lock, NULL);
    p->prepared = SG_SIMTIME_INVALID;
    const char* pe = getenv("SG_POLICY_PROF");
    p->prof = pe && *pe == '1';
    const char* pp = getenv("SG_POLICY_PINNED");
    p->pinned = pp && *pp == '1';
    *out = p;
    return SG_OK;
}

int sg_policy_kernel_profile(sg_policy* p, int enable, uint32_t skip_rounds) {
    if (!p || !p->dev) return SG_ERR_INVAL;
    return sgp_dev_kprof(p->dev, enable, skip_rounds) ? SG_ERR_HIP : SG_OK;
}

int sg_policy_kernel_stats(sg_policy* p, sg_kernel_stat* out, uint32_t cap, uint32_t* n_out) {
    if (!p || !p->dev || (cap && !out)) return SG_ERR_INVAL;
    enum { MAXK = 32 };
    const char* names[MAXK];
    uint64_t n[MAXK];
    double ms[MAXK], by[MAXK];
    uint32_t k = 0;
    if (sgp_dev_kstats(p->dev, names, n, ms, by, MAXK, &k)) return SG_ERR_HIP;
    for (uint32_t i = 0; i < k && i < cap; i++) {
        memset(&out[i], 0, sizeof out[i]);
        snprintf(out[i].name, sizeof out[i].name, "%s", names[i]);
        out[i].launches = n[i];
        out[i].ms = ms[i];
        out[i].alg_bytes = by[i];
    }
    if (n_out) *n_out = k;
    return SG_OK;
}

int sg_policy_destroy(sg_policy* p) {
    if (!p) return SG_OK;
    if (p->prof)
        fprintf(stderr, "sg_policy serial sections (s): flush gather %.3f insert %.3f min %.3f; "
                "prepare extract %.3f runs %.3f\n", p->t_gather, p->t_insert, p->t_min, p->t_extract,
                p->t_runs);
    if (p->dev) sgp_dev_destroy(p->dev);
    if (p->hosts)
        for (uint32_t i = 0; i < p->n_hosts; i++) {
            free(p->hosts[i].selfq.a);
            pthread_mutex_destroy(&p->hosts[i].lock);
        }
    if (p->threads)
        for (uint32_t i = 0; i < p->n_threads; i++) {
            free(p->threads[i].hosts);
            free(p->threads[i].pos);
            free(p->threads[i].gen);
            if (p->pinned) sgp_host_free(p->threads[i].arena);
            else free(p->threads[i].arena);
        }
    free(p->hosts);
    free(p->map);
    free(p->threads);
    free(p->foreign);
    free(p->self_list);
    free(p->ex);
    free(p->segs);
    free(p->lens);
    free(p);
    return SG_OK;
}

int sg_policy_add_host(sg_policy* p, uint32_t host_id, uint64_t token) {
    if (!p || p->n_hosts >= p->prm.max_hosts || host_index(p, host_id) >= 0) {
        sg_set_error("sg_policy_add_host: capacity exceeded or duplicate host %u", host_id);
        return SG_ERR_INVAL;
    }
    thread_rt* t = thread_lookup(p, token);
    if (!t) {
        if (p->n_threads >= p->prm.n_threads) {
            sg_set_error("sg_policy_add_host: more than %u worker threads", p->prm.n_threads);
            return SG_ERR_INVAL;
        }
        t = &p->threads[p->n_threads++];
        t->token = token;
    }
    if (t->n == t->cap) {
        uint32_t nc = t->cap ? 2 * t->cap : 64;
        uint32_t* nh = (uint32_t*)realloc(t->hosts, (size_t)nc * 4);
        if (nh) t->hosts = nh;
        uint32_t* np = (uint32_t*)realloc(t->pos, (size_t)nc * 4);
        if (np) t->pos = np;
        uint32_t* ng = (uint32_t*)realloc(t->gen, (size_t)nc * 4);
        if (ng) t->gen = ng;
        if (!nh || !np || !ng) return SG_ERR_NOMEM;
        t->cap = nc;
    }
    uint32_t idx = p->n_hosts++;
    host_rt* h = &p->hosts[idx];
    memset(h, 0, sizeof *h);
    h->id = host_id;
    h->thread = (uint32_t)(t - p->threads);
    h->lpos = t->n;
    pthread_mutex_init(&h->lock, NULL);
    t->pos[t->n] = 0;
    t->gen[t->n] = 0;
    t->hosts[t->n++] = idx;
    uint32_t mask = p->map_cap - 1, i = hash32(host_id) & mask;
    while (p->map[i]) i = (i + 1) & mask;
    p->map[i] = ((uint64_t)host_id << 32) | (idx + 1);
    return SG_OK;
}

int sg_policy_thread_hosts(sg_policy* p, uint64_t token, uint32_t* ids, uint32_t cap, uint32_t* n) {
    thread_rt* t = thread_lookup(p, token);
    uint32_t c = t ? t->n : 0;
    for (uint32_t i = 0; i < c && i < cap; i++) ids[i] = p->hosts[t->hosts[i]].id;
    if (n) *n = c;
    return SG_OK;
}

static int arena_push(sgp_rec** a, uint64_t* n, uint64_t* c, const sgp_rec* r) {
    if (*n == *c) {
        uint64_t nc = *c ? 2 * *c : 1024;
        sgp_rec* na = (sgp_rec*)realloc(*a, nc * sizeof(sgp_rec));
        if (!na) return -1;
        *a = na;
        *c = nc;
    }
    (*a)[(*n)++] = *r;
    return 0;
}

/* A worker's arena lives in pinned memory: the flush DMAs it in place. */
static int arena_push_pinned(sgp_rec** a, uint64_t* n, uint64_t* c, const sgp_rec* r) {
    if (*n == *c) {
        uint64_t nc = *c ? 2 * *c : 65536;
        sgp_rec* na = (sgp_rec*)sgp_host_alloc(nc * sizeof(sgp_rec));
        if (!na) return -1;
        if (*n) memcpy(na, *a, *n * sizeof(sgp_rec));
        sgp_host_free(*a);
        *a = na;
        *c = nc;
    }
    (*a)[(*n)++] = *r;
    return 0;
}

int sg_policy_push(sg_policy* p, uint64_t token, uint64_t handle, sg_simtime time, uint32_t src_id,
                   uint32_t dst_id, uint64_t src_event_id, sg_simtime barrier, sg_simtime* time_out) {
    int64_t di = host_index(p, dst_id);
    if (di < 0 || handle == 0) {
        sg_set_error("sg_policy_push: unknown destination host %u or null handle", dst_id);
        return SG_ERR_INVAL;
    }
    if (src_id != dst_id && time < barrier) time = barrier; /* host_single.c:180-184 */
    if (time_out) *time_out = time;
    sgp_rec r = {time, src_event_id, handle, src_id, (uint32_t)di};
    if (src_id == dst_id && time < barrier) {
        host_rt* h = &p->hosts[di];
        pthread_mutex_lock(&h->lock);
        int rc = sheap_push(&h->selfq, &r);
        int add = !h->in_self_list;
        h->in_self_list = 1;
        pthread_mutex_unlock(&h->lock);
        if (add) {
            pthread_mutex_lock(&p->self_lock);
            p->self_list[p->n_self++] = (uint32_t)di;
            pthread_mutex_unlock(&p->self_lock);
        }
        return rc ? SG_ERR_NOMEM : SG_OK;
    }
    thread_rt* t = thread_of(p, token);
    int rc;
    if (t) {
        rc = p->pinned ? arena_push_pinned(&t->arena, &t->na, &t->ca, &r)
                       : arena_push(&t->arena, &t->na, &t->ca, &r);
    } else {
        pthread_mutex_lock(&p->foreign_lock);
        rc = arena_push(&p->foreign, &p->nf, &p->cf, &r);
        pthread_mutex_unlock(&p->foreign_lock);
    }
    return rc ? SG_ERR_NOMEM : SG_OK;
}

/* This round's run of host idx: its length, and its position (the owner's
 * pos[] entry) reset on first use. */
static uint32_t run_len(const sg_policy* p, uint32_t idx) {
    return p->run_off ? p->run_off[idx + 1] - p->run_off[idx] : 0;
}
static uint32_t* run_pos(sg_policy* p, thread_rt* t, uint32_t lpos) {
    if (t->gen[lpos] != p->run_gen) {
        t->gen[lpos] = p->run_gen;
        t->pos[lpos] = 0;
    }
    return &t->pos[lpos];
}

/* Extract the runs for `barrier` once; other threads wait for the leader. */
static int prepare(sg_policy* p, sg_simtime barrier) {
    pthread_mutex_lock(&p->m);
    while (p->prepared != barrier && p->preparing) pthread_cond_wait(&p->cv, &p->m);
    if (p->prepared != barrier && !p->error) {
        p->preparing = 1;
        pthread_mutex_unlock(&p->m);
        const sgp_rec* runs;
        const uint32_t* off;
        uint64_t total;
        double t0 = p->prof ? now_s() : 0;
        int rc = sgp_dev_extract(p->dev, barrier, &runs, &off, &total);
        double t1 = p->prof ? now_s() : 0;
        if (rc == 0) {  /* no per-host pass: pop reads off / cnt and resets run_pos lazily */
            p->runs = runs;
            p->run_off = off;
            p->run_gen++;
        }
        if (p->prof) {
            p->t_extract += t1 - t0;
            p->t_runs += now_s() - t1;
        }
        pthread_mutex_lock(&p->m);
        if (rc) p->error = rc;
        p->prepared = barrier;
        p->preparing = 0;
        pthread_cond_broadcast(&p->cv);
    }
    int err = p->error;
    pthread_mutex_unlock(&p->m);
    return err;
}

int sg_policy_pop(sg_policy* p, uint64_t token, sg_simtime barrier, uint64_t* handle_out) {
    *handle_out = 0;
    if (__atomic_load_n(&p->prepared, __ATOMIC_ACQUIRE) != barrier) {
        int rc = prepare(p, barrier);
        if (rc) return rc;
    }
    thread_rt* t = thread_of(p, token);
    if (!t) return SG_OK; /* this thread was assigned no host */
    if (barrier > t->cur_barrier) { /* host_single.c:222-235: all hosts unprocessed again */
        t->cur_barrier = barrier;
        t->cursor = 0;
    }
    while (t->cursor < t->n) {
        const uint32_t c = t->cursor;
        const uint32_t idx = t->hosts[c];
        host_rt* h = &p->hosts[idx];
        const uint32_t len = run_len(p, idx);
        uint32_t* rp = run_pos(p, t, c);  /* only this thread pops its hosts */
        /* self events are pushed by the thread executing the host, its owner
         * (worker.c:218-234), so the heap needs the lock only when it is not
         * empty (a push from elsewhere takes it too) */
        if (__atomic_load_n(&h->selfq.n, __ATOMIC_ACQUIRE) == 0) {
            if (*rp < len) {
                *handle_out = p->runs[p->run_off[idx] + (*rp)++].handle;
                return SG_OK;
            }
            t->cursor++; /* nothing left this round */
            continue;
        }
        pthread_mutex_lock(&h->lock);
        const sgp_rec* a = *rp < len ? &p->runs[p->run_off[idx] + *rp] : NULL;
        const sgp_rec* b = (h->selfq.n && h->selfq.a[0].time < barrier) ? &h->selfq.a[0] : NULL;
        uint64_t handle = 0;
        if (a && (!b || rec_less(a, b))) {
            handle = a->handle;
            (*rp)++;
        } else if (b) {
            handle = b->handle;
            sheap_pop(&h->selfq);
        }
        pthread_mutex_unlock(&h->lock);
        if (handle) {
            *handle_out = handle;
            return SG_OK;
        }
        t->cursor++; /* host done for this round (host_single.c:266) */
    }
    return SG_OK;
}

/* Last arriver: deliver every staged event (and left-over CPU heap entries) to
 * HBM, then reduce the MIN. */
static int flush(sg_policy* p) {
    double t0 = p->prof ? now_s() : 0;
    /* the workers' pinned arenas go to the device in place; foreign pushes
     * and left-over CPU heap entries (few) are gathered into one more segment */
    uint64_t extra = p->nf;
    for (uint32_t k = 0; k < p->n_self; k++) extra += p->hosts[p->self_list[k]].selfq.n;
    if (extra > p->ex_cap) {  /* grows rarely: foreign pushes and left-over self events are few */
        uint64_t nc = p->ex_cap ? 2 * p->ex_cap : 1024;
        while (nc < extra) nc *= 2;
        sgp_rec* nx = (sgp_rec*)realloc(p->ex, nc * sizeof(sgp_rec));
        if (!nx) return SG_ERR_NOMEM;
        p->ex = nx;
        p->ex_cap = nc;
    }
    sgp_rec* ex = p->ex;
    const sgp_rec** segs = p->segs;
    uint64_t* lens = p->lens;
    for (uint32_t i = 0; i < p->n_threads; i++) {
        segs[i] = p->threads[i].arena;
        lens[i] = p->threads[i].na;
    }
    uint64_t n = 0;
    if (p->nf) memcpy(ex, p->foreign, p->nf * sizeof(sgp_rec));
    n += p->nf;
    p->nf = 0;
    for (uint32_t k = 0; k < p->n_self; k++) {
        host_rt* h = &p->hosts[p->self_list[k]];
        memcpy(ex + n, h->selfq.a, h->selfq.n * sizeof(sgp_rec));
        n += h->selfq.n;
        __atomic_store_n(&h->selfq.n, 0, __ATOMIC_RELEASE);
        h->in_self_list = 0;
    }
    p->n_self = 0;
    segs[p->n_threads] = ex;
    lens[p->n_threads] = n;
    double t1 = p->prof ? now_s() : 0;
    int rc = sgp_dev_insert_segs(p->dev, segs, lens, p->n_threads + 1);  /* synchronises */
    for (uint32_t i = 0; i < p->n_threads; i++) p->threads[i].na = 0;   /* arenas reusable */
    if (rc) return rc;
    double t2 = p->prof ? now_s() : 0;
    rc = sgp_dev_min(p->dev, &p->next_min);
    if (p->prof) {
        double t3 = now_s();
        p->t_gather += t1 - t0;
        p->t_insert += t2 - t1;
        p->t_min += t3 - t2;
    }
    return rc;
}

int sg_policy_next_time(sg_policy* p, uint64_t token, sg_simtime* next_out) {
    (void)token;
    pthread_mutex_lock(&p->m);
    uint64_t my_gen = p->gen;
    if (++p->arrivals == p->prm.n_threads) {
        int rc = flush(p);
        if (rc) p->error = rc;
        p->arrivals = 0;
        p->gen++;
        p->prepared = SG_SIMTIME_INVALID; /* queues changed: runs must be re-extracted */
        pthread_cond_broadcast(&p->cv);
    } else {
        while (p->gen == my_gen) pthread_cond_wait(&p->cv, &p->m);
    }
    int err = p->error;
    *next_out = p->next_min;
    pthread_mutex_unlock(&p->m);
    return err;
}

int sg_policy_remaining(sg_policy* p, uint64_t* handles, uint64_t cap, uint64_t* n_out) {
    uint64_t n = 0;
    for (uint32_t i = 0; i < p->n_threads; i++)
        for (uint64_t k = 0; k < p->threads[i].na; k++, n++)
            if (n < cap) handles[n] = p->threads[i].arena[k].handle;
    for (uint64_t k = 0; k < p->nf; k++, n++)
        if (n < cap) handles[n] = p->foreign[k].handle;
    for (uint32_t i = 0; i < p->n_hosts; i++) {
        host_rt* h = &p->hosts[i];
        for (uint32_t k = 0; k < h->selfq.n; k++, n++)
            if (n < cap) handles[n] = h->selfq.a[k].handle;
        const uint32_t rp = *run_pos(p, &p->threads[h->thread], h->lpos);
        for (uint32_t k = rp; k < run_len(p, i); k++, n++)
            if (n < cap) handles[n] = p->runs[p->run_off[i] + k].handle;
    }
    uint64_t nd = 0;
    sgp_rec* tmp = NULL;
    int rc = sgp_dev_all(p->dev, NULL, 0, &nd);
    if (rc) return rc;
    if (nd) {
        tmp = (sgp_rec*)malloc(nd * sizeof(sgp_rec));
        if (!tmp) return SG_ERR_NOMEM;
        rc = sgp_dev_all(p->dev, tmp, nd, &nd);
        for (uint64_t k = 0; k < nd; k++, n++)
            if (n < cap) handles[n] = tmp[k].handle;
        free(tmp);
    }
    if (n_out) *n_out = n;
    return rc;
}
