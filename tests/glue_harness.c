/*
 * glue_harness.c — CPU test of integration/scheduler_policy_gpu.c's own logic
 * (ownership of the getAssignedHosts queues, the worker count it passes to the
 * library, the srcHostEventID relabelling, teardown), built with
 * -fsanitize=address by tests/test_integration_glue.py against the unmodified
 * reference headers.
 *
 * Test doubles only: the handful of Shadow functions the glue calls (host_getID,
 * event_getTime/setTime/unref, logger_*, worker_getOptions,
 * options_getNWorkerThreads) and an in-memory stand-in for libshadowgpu's
 * sg_policy_* (include/shadowgpu.h §3) that pops by (time, dst, src, seq) like
 * event_compare (event.c:110-153) and flushes on the n_threads-th getNextTime
 * arrival of a round, as sg_policy.c does.  Nothing of the reference is
 * compiled here.  The same glue linked to the real libshadowgpu.so runs PHOLD
 * on the GPU through tests/glue_phold.c (tests/test_gpu_glue.py).
 */
#include <glib.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include "main/core/scheduler/scheduler_policy.h"
#include "main/core/support/options.h"
#include "main/core/work/event.h"
#include "main/core/worker.h"
#include "main/host/host.h"
#include "shadowgpu.h"
#include "support/logger/logger.h"

SchedulerPolicy* schedulerpolicygpu_new(void);

/* ---------------------------------------------------------------- Shadow */
struct _Host { GQuark id; };
struct _Event { SimulationTime time; Host* src; Host* dst; int refs; int order; guint64 id; };
#ifdef HARNESS_EXACT_ID
guint64 event_getSrcHostEventID(Event* e) { return e->id; }
#endif

GQuark host_getID(Host* host) { return host->id; }
SimulationTime event_getTime(Event* e) { return e->time; }
void event_setTime(Event* e, SimulationTime t) { e->time = t; }
static int g_unrefs;
void event_unref(Event* e) { if (--e->refs == 0) { g_unrefs++; free(e); } }
Logger* logger_getDefault() { return NULL; }
/* slave.c:196 → scheduler_new(nWorkers): the scheduler's worker count */
static guint g_n_workers;
static int g_options_token;
Options* worker_getOptions() { return (Options*)&g_options_token; }
guint options_getNWorkerThreads(Options* o) { return o == (Options*)&g_options_token ? g_n_workers : 0; }
static int g_errors;
void logger_log(Logger* l, LogLevel lv, const gchar* f, const gchar* fn, const gint ln,
                const gchar* fmt, ...) {
    va_list ap; va_start(ap, fmt); vfprintf(stderr, fmt, ap); va_end(ap);
    fputc('\n', stderr); g_errors++;
}

/* ------------------------------------------------ sg_policy_* test double */
#define MAXH 16
#define MAXE 256
struct sg_policy {
    uint32_t n_threads, n_hosts, ids[MAXH];
    uint64_t thr[MAXH];
    struct { uint64_t h; sg_simtime t; uint32_t src, dst; uint64_t seq; int live; } ev[MAXE];
    int n_ev;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    uint32_t arrivals;
    uint64_t gen, flushes;
    sg_simtime next_min;
};
static uint32_t g_created_threads;
static uint64_t g_flushes;
const char* sg_last_error(void) { return "test double"; }
int sg_policy_create(const sg_policy_params* prm, sg_policy** out) {
    sg_policy* p = calloc(1, sizeof *p);
    p->n_threads = prm->n_threads;
    g_created_threads = prm->n_threads;
    pthread_mutex_init(&p->mu, NULL);
    pthread_cond_init(&p->cv, NULL);
    *out = p;
    return SG_OK;
}
int sg_policy_destroy(sg_policy* p) {
    g_flushes = p->flushes;
    pthread_mutex_destroy(&p->mu);
    pthread_cond_destroy(&p->cv);
    free(p);
    return SG_OK;
}
int sg_policy_add_host(sg_policy* p, uint32_t id, uint64_t thr) {
    if (p->n_hosts == MAXH) return SG_ERR_INVAL;
    p->ids[p->n_hosts] = id; p->thr[p->n_hosts++] = thr;
    return SG_OK;
}
int sg_policy_thread_hosts(sg_policy* p, uint64_t thr, uint32_t* out, uint32_t cap, uint32_t* n) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < p->n_hosts; i++)
        if (p->thr[i] == thr) { if (k < cap) out[k] = p->ids[i]; k++; }
    *n = k;
    return SG_OK;
}
static uint64_t owner(sg_policy* p, uint32_t id) {
    for (uint32_t i = 0; i < p->n_hosts; i++) if (p->ids[i] == id) return p->thr[i];
    return 0;
}
int sg_policy_push(sg_policy* p, uint64_t thr, uint64_t h, sg_simtime t, uint32_t src, uint32_t dst,
                   uint64_t seq, sg_simtime barrier, sg_simtime* t_out) {
    if (src != dst && t < barrier) t = barrier;   /* host_single.c:180-184 */
    pthread_mutex_lock(&p->mu);
    int i = p->n_ev++;
    p->ev[i].h = h; p->ev[i].t = t; p->ev[i].src = src; p->ev[i].dst = dst;
    p->ev[i].seq = seq; p->ev[i].live = 1;
    pthread_mutex_unlock(&p->mu);
    *t_out = t;
    return SG_OK;
}
int sg_policy_pop(sg_policy* p, uint64_t thr, sg_simtime barrier, uint64_t* out) {
    pthread_mutex_lock(&p->mu);
    int best = -1;
    for (int i = 0; i < p->n_ev; i++) {
        if (!p->ev[i].live || p->ev[i].t >= barrier || owner(p, p->ev[i].dst) != thr) continue;
        if (best < 0) { best = i; continue; }
#define LT(a, b) (p->ev[a].t != p->ev[b].t ? p->ev[a].t < p->ev[b].t : \
                  p->ev[a].dst != p->ev[b].dst ? p->ev[a].dst < p->ev[b].dst : \
                  p->ev[a].src != p->ev[b].src ? p->ev[a].src < p->ev[b].src : p->ev[a].seq < p->ev[b].seq)
        if (LT(i, best)) best = i;
    }
    *out = 0;
    if (best >= 0) { p->ev[best].live = 0; *out = p->ev[best].h; }
    pthread_mutex_unlock(&p->mu);
    return SG_OK;
}
/* sg_policy.c's arrival count: the n_threads-th arrival of a round flushes and
 * releases the others, so a wrong worker count either flushes twice a round or
 * never releases (the harness's alarm then fails the run). */
int sg_policy_next_time(sg_policy* p, uint64_t thr, sg_simtime* t) {
    pthread_mutex_lock(&p->mu);
    uint64_t my = p->gen;
    if (++p->arrivals == p->n_threads) {   /* the flush: MIN over what is queued now */
        p->next_min = SG_SIMTIME_MAX;
        for (int i = 0; i < p->n_ev; i++)
            if (p->ev[i].live && p->ev[i].t < p->next_min) p->next_min = p->ev[i].t;
        p->arrivals = 0;
        p->gen++;
        p->flushes++;
        pthread_cond_broadcast(&p->cv);
    } else {
        while (p->gen == my) pthread_cond_wait(&p->cv, &p->mu);
    }
    *t = p->next_min;
    pthread_mutex_unlock(&p->mu);
    return SG_OK;
}
int sg_policy_remaining(sg_policy* p, uint64_t* hs, uint64_t cap, uint64_t* n) {
    uint64_t k = 0;
    for (int i = 0; i < p->n_ev; i++) if (p->ev[i].live) { if (k < cap) hs[k] = p->ev[i].h; k++; }
    *n = k;
    return SG_OK;
}

/* ---------------------------------------------------------------- driver */
static SchedulerPolicy* g_pol;
static Host g_hosts[4] = {{11}, {12}, {13}, {14}};
static pthread_barrier_t g_bar;
static int g_fail, g_order[5] = {-1, -1, -1, -1, -1}, g_w0_got;
static sg_simtime g_next[3];
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); g_fail = 1; } } while (0)

static Event* mk(SimulationTime t, int src, int dst, int order) {
    Event* e = calloc(1, sizeof *e);
    e->time = t; e->src = &g_hosts[src]; e->dst = &g_hosts[dst]; e->refs = 1; e->order = order;
    e->id = 100 + (guint64)order;   /* srcHostEventID: creation order on the source */
    return e;
}

/* Scenario 1: two workers with two hosts each. */
static void* worker(void* arg) {
    int w = (int)(intptr_t)arg;
    pthread_barrier_wait(&g_bar);            /* 1: hosts registered */
    /* boot and shutdown both ask (scheduler.c:78-113): the first queue must be
     * freed exactly once (by the hash table when the second replaces it) */
    GQueue* q1 = g_pol->getAssignedHosts(g_pol);
    CHECK(g_queue_get_length(q1) == 2);
    GQueue* q2 = g_pol->getAssignedHosts(g_pol);
    CHECK(g_queue_get_length(q2) == 2);
    CHECK(g_queue_peek_head(q2) == &g_hosts[2 * w]);
    pthread_barrier_wait(&g_bar);            /* 2: assigned */
    pthread_barrier_wait(&g_bar);            /* 3: events pushed */
    g_next[w] = g_pol->getNextTime(g_pol);   /* every worker arrives (scheduler.c:393-394) */
    for (int i = 0; i < 5; i++) {
        Event* x = g_pol->pop(g_pol, 10);
        if (!x) break;
        if (w == 1) g_order[i] = x->order; else g_w0_got++;
        event_unref(x);
    }
    return NULL;
}

static void scenario_two_workers(void) {
    g_n_workers = 2;
    g_pol = schedulerpolicygpu_new();
    CHECK(g_pol->referenceCount == 1);
    pthread_barrier_init(&g_bar, NULL, 3);
    pthread_t thr[2];
    for (int w = 0; w < 2; w++) pthread_create(&thr[w], NULL, worker, (void*)(intptr_t)w);
    /* hosts 0,1 -> worker 0; 2,3 -> worker 1 (scheduler.c:488-531) */
    for (int h = 0; h < 4; h++) g_pol->addHost(g_pol, &g_hosts[h], thr[h / 2]);
    pthread_barrier_wait(&g_bar);            /* 1 */
    pthread_barrier_wait(&g_bar);            /* 2 */
    CHECK(g_created_threads == 2);           /* the scheduler's nWorkers */
    /* srcHostEventID relabelling: host 0 sends three events to host 2 at the
     * same time; they must pop in creation order.  Host 3's event at that time
     * pops after them (src order), host 1's at t = 99 stays queued. */
    Event* e[5] = {mk(5, 0, 2, 0), mk(5, 0, 2, 1), mk(5, 3, 2, 3), mk(5, 0, 2, 2), mk(99, 1, 2, 4)};
    for (int i = 0; i < 5; i++) g_pol->push(g_pol, e[i], e[i]->src, e[i]->dst, 1);
    pthread_barrier_wait(&g_bar);            /* 3 */
    for (int w = 0; w < 2; w++) pthread_join(thr[w], NULL);
    CHECK(g_next[0] == 5 && g_next[1] == 5);
    CHECK(g_w0_got == 0);
    for (int i = 0; i < 4; i++) CHECK(g_order[i] == i);
    CHECK(g_order[4] == -1);
    CHECK(g_unrefs == 4);
    g_pol->free(g_pol);                      /* unrefs the queued event through remaining() */
    CHECK(g_unrefs == 5);
    pthread_barrier_destroy(&g_bar);
}

/* Scenario 2: three workers, two hosts: the third worker is assigned
 * nothing but still pops and calls getNextTime every round, so the library must
 * be sized for three arrivals.  Sized from the hosts' threads (two) it would
 * flush on the second arrival and leave the third waiting for a generation that
 * never comes; the alarm below turns that hang into a failure. */
#define S2_ROUNDS 3
static pthread_barrier_t g_start;
static void* worker3(void* arg) {
    int w = (int)(intptr_t)arg;
    pthread_barrier_wait(&g_start);          /* hosts registered (startBarrier, scheduler.c:583) */
    GQueue* q = g_pol->getAssignedHosts(g_pol);
    CHECK(g_queue_get_length(q) == (w < 2 ? 1u : 0u));
    pthread_barrier_wait(&g_bar);            /* prepareRoundBarrier (scheduler.c:589) */
    for (int r = 0; r < S2_ROUNDS; r++) {
        SimulationTime barrier = 10 * (SimulationTime)(r + 1);
        if (w < 2) {                         /* each host sends itself one event per round */
            Event* x = mk(barrier + 1, w, w, r);
            g_pol->push(g_pol, x, x->src, x->dst, barrier);
        }
        Event* x;
        while ((x = g_pol->pop(g_pol, barrier)) != NULL) event_unref(x);
        pthread_barrier_wait(&g_bar);        /* executeEventsBarrier (scheduler.c:386) */
        g_next[w] = g_pol->getNextTime(g_pol);
        pthread_barrier_wait(&g_bar);        /* collectInfoBarrier (scheduler.c:405) */
    }
    return NULL;
}

static void scenario_idle_worker(void) {
    g_n_workers = 3;
    g_unrefs = 0;
    g_pol = schedulerpolicygpu_new();
    pthread_barrier_init(&g_bar, NULL, 3);
    pthread_barrier_init(&g_start, NULL, 4);
    pthread_t thr[3];
    for (int w = 0; w < 3; w++) pthread_create(&thr[w], NULL, worker3, (void*)(intptr_t)w);
    for (int h = 0; h < 2; h++) g_pol->addHost(g_pol, &g_hosts[h], thr[h]);  /* round-robin */
    pthread_barrier_wait(&g_start);
    for (int w = 0; w < 3; w++) pthread_join(thr[w], NULL);
    CHECK(g_created_threads == 3);
    for (int w = 0; w < 3; w++) CHECK(g_next[w] == 10 * S2_ROUNDS + 1);
    g_pol->free(g_pol);
    CHECK(g_unrefs == 2 * S2_ROUNDS);        /* the last round's two events, by free */
    CHECK(g_flushes == S2_ROUNDS);           /* one flush per round */
    pthread_barrier_destroy(&g_bar);
    pthread_barrier_destroy(&g_start);
}

int main(void) {
    alarm(30);                               /* a lost arrival hangs: SIGALRM fails the run */
    scenario_two_workers();
    scenario_idle_worker();
    CHECK(g_errors == 0);
    if (!g_fail) printf("glue harness ok\n");
    return g_fail;
}
