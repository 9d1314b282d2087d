/*
 * host_steal.c — TEST INFRASTRUCTURE / CPU BASELINE, not product code.
 *
 * C restatement of the reference's CPU policies behind the SchedulerPolicy-
 * shaped vtable of include/shadowgpu.h (sg_sched_policy_ops), so the same
 * round driver (sg_sched_run_phold) can run them next to the `gpu` policy:
 *
 *   host_steal   core/scheduler/scheduler_policy_host_steal.c:132-456
 *                per-host mutex + binary heap (priority_queue.c:115-175),
 *                per-thread unprocessed/processed host lists + runningHost,
 *                push locks the pushing thread's lock then the queue
 *                (host_steal.c:254-271), pop steals with ordered lock pairs
 *                (host_steal.c:366-416), migration on a stolen pop
 *                (host_steal.c:172-196, 303)
 *   host_single  scheduler_policy_host_single.c:120-305 (steal = 0)
 *
 * Used (a) to cross-check the gpu policy under real worker threads and
 * (b) as bench.py's timed CPU baseline ("port" of host_steal, all cores).
 * Built twice (oracle/Makefile): liborc.so with plain binary heaps of event
 * pointers (a lower bound on the reference's cost), and libhsglib.so with
 * -DHS_GLIB_PQ, whose per-host queue is priority_queue.c's heap with its
 * GLib hash-table position map (the reference's cost).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../include/shadowgpu.h"

#ifndef HS_GLIB_PQ
typedef struct hq {            /* HostStealQueueData */
    pthread_mutex_t lock;
    sg_hevent** a;
    uint32_t n, cap;
    sg_simtime last;
} hq;
#else
/* The faithful heap (bench.py's cpu_baseline "faithful" variant, built as
 * libhsglib.so): priority_queue.c:17-175 restated with GLib itself.  The heap
 * holds element pointers and a GHashTable maps every element to its heap slot;
 * each swap re-inserts both elements (priority_queue.c:78-85), a push looks
 * the element up first (:126), a pop removes it (:165) and the array starts at
 * 100 slots, doubles when full and halves below a quarter, refreshing the
 * whole map when realloc moves it (:115-124, :166-173).  The compare runs
 * through a function pointer, as GCompareDataFunc does. */
#include <glib.h>
typedef struct hq {
    pthread_mutex_t lock;
    gpointer* heap;
    GHashTable* map;
    gsize n, cap;
    GCompareDataFunc cmp;
    sg_simtime last;
} hq;
#endif

typedef struct dq {            /* GQueue of host indices */
    uint32_t* a;
    uint32_t head, n, cap;
} dq;

typedef struct td {            /* HostStealThreadData */
    uint64_t token;
    dq unproc, proc;
    int64_t running;           /* runningHost or -1 */
    sg_simtime barrier;
    uint32_t tnumber;
    pthread_mutex_t lock;
} td;

typedef struct pol {
    int steal;
    uint32_t nh;
    hq* q;
    uint32_t* owner;           /* hostToThreadMap */
    td* t;
    uint32_t nt, maxt;
    pthread_rwlock_t lock;
} pol;

static int ev_less(const sg_hevent* a, const sg_hevent* b) { /* event.c:110-153 */
    if (a->time != b->time) return a->time < b->time;
    if (a->dst != b->dst) return a->dst < b->dst;
    if (a->src != b->src) return a->src < b->src;
    return a->seq < b->seq;
}

#ifndef HS_GLIB_PQ
static void hq_init(hq* q) { pthread_mutex_init(&q->lock, NULL); }
static uint32_t hq_len(const hq* q) { return q->n; }
static sg_hevent* hq_top(const hq* q) { return q->a[0]; }
static sg_hevent* hq_at(const hq* q, uint32_t i) { return q->a[i]; }
static void hq_free(hq* q) { free(q->a); }

static void hq_push(hq* q, sg_hevent* e) {
    if (q->n == q->cap) {
        q->cap = q->cap ? 2 * q->cap : 16;
        q->a = (sg_hevent**)realloc(q->a, q->cap * sizeof(sg_hevent*));
    }
    uint32_t i = q->n++;
    q->a[i] = e;
    while (i) {
        uint32_t p = (i - 1) / 2;
        if (!ev_less(q->a[i], q->a[p])) break;
        sg_hevent* t = q->a[i];
        q->a[i] = q->a[p];
        q->a[p] = t;
        i = p;
    }
}

static sg_hevent* hq_pop(hq* q) {
    sg_hevent* top = q->a[0];
    q->a[0] = q->a[--q->n];
    uint32_t i = 0;
    for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= q->n) break;
        if (c + 1 < q->n && ev_less(q->a[c + 1], q->a[c])) c++;
        if (!ev_less(q->a[c], q->a[i])) break;
        sg_hevent* t = q->a[i];
        q->a[i] = q->a[c];
        q->a[c] = t;
        i = c;
    }
    return top;
}
#else
enum { PQ_FIRST = 100 };  /* priority_queue.c:15 */
static gint ev_cmp(gconstpointer a, gconstpointer b, gpointer unused) {  /* event_compare as a GCompareDataFunc */
    (void)unused;
    return ev_less((const sg_hevent*)a, (const sg_hevent*)b) ? -1 : ev_less((const sg_hevent*)b, (const sg_hevent*)a);
}
static void hq_init(hq* q) {
    pthread_mutex_init(&q->lock, NULL);
    q->heap = g_new(gpointer, PQ_FIRST);
    q->map = g_hash_table_new(NULL, NULL);
    q->cap = PQ_FIRST;
    q->n = 0;
    q->cmp = ev_cmp;
}
static uint32_t hq_len(const hq* q) { return (uint32_t)q->n; }
static sg_hevent* hq_top(const hq* q) { return (sg_hevent*)q->heap[0]; }
static sg_hevent* hq_at(const hq* q, uint32_t i) { return (sg_hevent*)q->heap[i]; }
static void hq_free(hq* q) {
    g_hash_table_destroy(q->map);
    g_free(q->heap);
}
static void pq_remap(hq* q) {  /* every element's slot again after the array moved */
    g_hash_table_remove_all(q->map);
    for (gsize i = 0; i < q->n; i++) g_hash_table_insert(q->map, q->heap[i], q->heap + i);
}
static void pq_swap(hq* q, gsize i, gsize j) {
    gpointer x = q->heap[i], y = q->heap[j];
    q->heap[i] = y;
    q->heap[j] = x;
    g_hash_table_insert(q->map, x, q->heap + j);
    g_hash_table_insert(q->map, y, q->heap + i);
}
static int pq_below(hq* q, gsize i, gsize j) { return q->cmp(q->heap[i], q->heap[j], NULL) < 0; }
static gsize pq_up(hq* q, gsize i) {
    for (; i > 0 && pq_below(q, i, (i - 1) / 2); i = (i - 1) / 2) pq_swap(q, i, (i - 1) / 2);
    return i;
}
static gsize pq_down(hq* q, gsize i) {
    for (gsize c; (c = 2 * i + 1) < q->n; i = c) {
        if (c + 1 < q->n && pq_below(q, c + 1, c)) c++;
        if (!pq_below(q, c, i)) break;
        pq_swap(q, i, c);
    }
    return i;
}
static void pq_resize(hq* q, gsize cap) {
    gpointer* old = q->heap;
    q->cap = cap;
    q->heap = g_renew(gpointer, q->heap, q->cap);
    if (q->heap != old) pq_remap(q);
}
static void hq_push(hq* q, sg_hevent* e) {
    if (q->n >= q->cap) pq_resize(q, 2 * q->cap);
    gpointer* at = (gpointer*)g_hash_table_lookup(q->map, e);
    if (at) {  /* already queued: only re-placed (never the case for fresh events) */
        pq_up(q, pq_down(q, (gsize)(at - q->heap)));
        return;
    }
    q->heap[q->n] = e;
    g_hash_table_insert(q->map, e, q->heap + q->n);
    q->n++;
    pq_up(q, q->n - 1);
}
static sg_hevent* hq_pop(hq* q) {
    gpointer top = q->heap[0];
    pq_swap(q, 0, q->n - 1);
    g_hash_table_remove(q->map, top);
    q->n--;
    pq_down(q, 0);
    if (q->cap > PQ_FIRST && q->n * 4 < q->cap) pq_resize(q, q->cap / 2);
    return (sg_hevent*)top;
}
#endif

static void dq_init(dq* d, uint32_t cap) {
    d->a = (uint32_t*)malloc((cap ? cap : 1) * 4);
    d->cap = cap ? cap : 1;
    d->head = d->n = 0;
}
static void dq_push(dq* d, uint32_t v) { d->a[(d->head + d->n++) % d->cap] = v; }
static uint32_t dq_pop(dq* d) {
    uint32_t v = d->a[d->head];
    d->head = (d->head + 1) % d->cap;
    d->n--;
    return v;
}

static td* tdata(pol* p, uint64_t token) {
    pthread_rwlock_rdlock(&p->lock);
    td* r = NULL;
    for (uint32_t i = 0; i < p->nt; i++)
        if (p->t[i].token == token) {
            r = &p->t[i];
            break;
        }
    pthread_rwlock_unlock(&p->lock);
    return r;
}

/* addHost (host_steal.c:132-167) */
static void p_add_host(void* data, uint32_t host, uint64_t token) {
    pol* p = (pol*)data;
    td* t = tdata(p, token);
    pthread_rwlock_wrlock(&p->lock);
    if (!t) {
        t = &p->t[p->nt];
        t->token = token;
        t->tnumber = p->nt++;
        t->running = -1;
        dq_init(&t->unproc, p->nh);
        dq_init(&t->proc, p->nh);
        pthread_mutex_init(&t->lock, NULL);
    }
    p->owner[host] = t->tnumber;
    pthread_rwlock_unlock(&p->lock);
    if ((int64_t)host != t->running) dq_push(&t->unproc, host);
}

/* getAssignedHosts (host_steal.c:202-223) */
static uint32_t p_hosts(void* data, uint64_t token, uint32_t* out, uint32_t cap) {
    pol* p = (pol*)data;
    td* t = tdata(p, token);
    if (!t) return 0;
    uint32_t n = 0;
    for (uint32_t i = 0; i < t->proc.n && n < cap; i++) out[n++] = t->proc.a[(t->proc.head + i) % t->proc.cap];
    for (uint32_t i = 0; i < t->unproc.n && n < cap; i++)
        out[n++] = t->unproc.a[(t->unproc.head + i) % t->unproc.cap];
    return n;
}

/* push (host_steal.c:225-272; host_single.c:167-208) */
static void p_push(void* data, sg_hevent* e, uint32_t src, uint32_t dst, sg_simtime barrier) {
    pol* p = (pol*)data;
    if (src != dst && e->time < barrier) e->time = barrier;
    td* t = p->steal ? tdata(p, (uint64_t)pthread_self()) : NULL;
    hq* q = &p->q[dst];
    if (t) pthread_mutex_lock(&t->lock);
    pthread_mutex_lock(&q->lock);
    hq_push(q, e);
    pthread_mutex_unlock(&q->lock);
    if (t) pthread_mutex_unlock(&t->lock);
}

/* popFromThread (host_steal.c:274-323) */
static sg_hevent* pop_from(pol* p, td* t, dq* assigned, sg_simtime barrier) {
    while (assigned->n || t->running >= 0) {
        if (t->running < 0) t->running = dq_pop(assigned);
        uint32_t h = (uint32_t)t->running;
        hq* q = &p->q[h];
        pthread_mutex_lock(&q->lock);
        sg_hevent* e = NULL;
        if (hq_len(q) && hq_top(q)->time < barrier) {
            q->last = hq_top(q)->time;
            e = hq_pop(q);
            /* migrate iff the host was stolen (host_steal.c:172-196, 303): the
             * owner is read under the reader lock, written only on a change */
            pthread_rwlock_rdlock(&p->lock);
            const uint32_t old = p->owner[h];
            pthread_rwlock_unlock(&p->lock);
            if (old != t->tnumber) {
                pthread_rwlock_wrlock(&p->lock);
                p->owner[h] = t->tnumber;
                pthread_rwlock_unlock(&p->lock);
            }
        } else {
            dq_push(&t->proc, h);
            t->running = -1;
        }
        pthread_mutex_unlock(&q->lock);
        if (e) return e;
    }
    return NULL;
}

/* pop (host_steal.c:325-418); without stealing it is host_single.c:210-271 */
static sg_hevent* p_pop(void* data, sg_simtime barrier) {
    pol* p = (pol*)data;
    td* t = tdata(p, (uint64_t)pthread_self());
    if (!t) return NULL;
    pthread_mutex_lock(&t->lock);
    if (barrier > t->barrier) {
        t->barrier = barrier;
        while (t->proc.n) dq_push(&t->unproc, dq_pop(&t->proc));
    }
    sg_hevent* e = pop_from(p, t, &t->unproc, barrier);
    pthread_mutex_unlock(&t->lock);
    if (e || !p->steal) return e;
    uint32_t n = p->nt;
    for (uint32_t i = 1; i < n; i++) {
        td* s = &p->t[(i + t->tnumber) % n];
        if (s->unproc.n == 0) continue; /* unlocked peek, as the reference */
        if (t->tnumber < s->tnumber) {
            pthread_mutex_lock(&t->lock);
            pthread_mutex_lock(&s->lock);
        } else {
            pthread_mutex_lock(&s->lock);
            pthread_mutex_lock(&t->lock);
        }
        e = pop_from(p, t, &s->unproc, barrier);
        if (t->tnumber < s->tnumber) {
            pthread_mutex_unlock(&s->lock);
            pthread_mutex_unlock(&t->lock);
        } else {
            pthread_mutex_unlock(&t->lock);
            pthread_mutex_unlock(&s->lock);
        }
        if (e) break;
    }
    return e;
}

/* getNextTime (host_steal.c:420-456) */
static sg_simtime p_next(void* data) {
    pol* p = (pol*)data;
    td* t = tdata(p, (uint64_t)pthread_self());
    sg_simtime m = SG_SIMTIME_MAX;
    if (!t) return m;
    dq* lists[2] = {&t->unproc, &t->proc};
    for (int l = 0; l < 2; l++)
        for (uint32_t i = 0; i < lists[l]->n; i++) {
            hq* q = &p->q[lists[l]->a[(lists[l]->head + i) % lists[l]->cap]];
            pthread_mutex_lock(&q->lock);
            if (hq_len(q) && hq_top(q)->time < m) m = hq_top(q)->time;
            pthread_mutex_unlock(&q->lock);
        }
    return m;
}

static void p_free(void* data) {
    pol* p = (pol*)data;
    for (uint32_t h = 0; h < p->nh; h++) {
        for (uint32_t i = 0; i < hq_len(&p->q[h]); i++) free(hq_at(&p->q[h], i));
        hq_free(&p->q[h]);
        pthread_mutex_destroy(&p->q[h].lock);
    }
    for (uint32_t i = 0; i < p->nt; i++) {
        free(p->t[i].unproc.a);
        free(p->t[i].proc.a);
        pthread_mutex_destroy(&p->t[i].lock);
    }
    free(p->q);
    free(p->t);
    free(p->owner);
    pthread_rwlock_destroy(&p->lock);
    free(p);
}

int orc_policy_ops_cpu(int steal, uint32_t n_threads, uint32_t n_hosts, sg_sched_policy_ops* out) {
    pol* p = (pol*)calloc(1, sizeof *p);
    if (!p) return -1;
    p->steal = steal;
    p->nh = n_hosts;
    p->q = (hq*)calloc(n_hosts, sizeof(hq));
    p->owner = (uint32_t*)calloc(n_hosts, 4);
    p->maxt = n_threads;
    p->t = (td*)calloc(n_threads, sizeof(td));
    if (!p->q || !p->owner || !p->t) return -1;
    for (uint32_t h = 0; h < n_hosts; h++) hq_init(&p->q[h]);
    pthread_rwlock_init(&p->lock, NULL);
    out->data = p;
    out->add_host = p_add_host;
    out->get_assigned_hosts = p_hosts;
    out->push = p_push;
    out->pop = p_pop;
    out->get_next_time = p_next;
    out->free = p_free;
    return 0;
}
