/*
 * glue_phold.c — integration/scheduler_policy_gpu.c, the Shadow-side file a
 * maintainer drops into src/main/core/scheduler/, linked to the REAL
 * libshadowgpu.so and driven through its SchedulerPolicy vtable
 * (scheduler_policy.h:31-58) by the Shadow-style round driver of
 * libshadowgpu (sg_sched_run_phold: scheduler.c:339-414, 617-650 and
 * worker.c:149-216 restated, with the PHOLD body on the CPU workers).
 *
 * Built by shadow_amd/build.py (build_glue) into integration/_bin/ wherever the
 * reference headers and conda GLib are present, as two variants:
 * libsgglue_relabel.so (per-source srcHostEventID relabelling, the glue's
 * default) and libsgglue_exact.so (-DSHADOW_HAS_EVENT_SRCID: the maintainer's
 * one-line getter).  tests/test_gpu_glue.py loads them with
 * ctypes and compares per-host digests / pops / rng / event counters with the
 * oracle.
 *
 * What this file supplies is test doubles for the Shadow objects the glue
 * touches — Host (host_getID), Event (event_getTime / setTime / unref and the
 * getter), worker_getOptions / options_getNWorkerThreads and the logger — plus
 * the adapter from the driver's sg_sched_policy_ops to the SchedulerPolicy the
 * glue builds.  Every sg_policy_* call is the library's own.
 */
#include <glib.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "main/core/scheduler/scheduler_policy.h"
#include "main/core/support/options.h"
#include "main/core/work/event.h"
#include "main/core/worker.h"
#include "main/host/host.h"
#include "shadowgpu.h"
#include "support/logger/logger.h"

SchedulerPolicy* schedulerpolicygpu_new(void);

/* ------------------------------------------------------ Shadow doubles -- */
struct _Host { GQuark id; guint32 index; };
/* The driver's record is the event's payload; the wrapper is the Event* the
 * policy holds (and unrefs at free). */
struct _Event { sg_hevent* h; };

static gint64 g_live;      /* Event wrappers alive */
static gint64 g_unref_free;/* wrappers released by the glue's free (remaining()) */
static int g_in_free;
static int g_errors;
static guint g_n_workers;
static int g_options_token;

GQuark host_getID(Host* host) { return host->id; }
SimulationTime event_getTime(Event* e) { return e->h->time; }
void event_setTime(Event* e, SimulationTime t) { e->h->time = t; }
#ifdef SHADOW_HAS_EVENT_SRCID
guint64 event_getSrcHostEventID(Event* e) { return e->h->seq; }
#endif
void event_unref(Event* e) {  /* the last reference: the event and its payload go */
    free(e->h);
    free(e);
    __atomic_sub_fetch(&g_live, 1, __ATOMIC_RELAXED);
    if (g_in_free) g_unref_free++;
}
Options* worker_getOptions() { return (Options*)&g_options_token; }
guint options_getNWorkerThreads(Options* o) { return o == (Options*)&g_options_token ? g_n_workers : 0; }
Logger* logger_getDefault() { return NULL; }
void logger_log(Logger* l, LogLevel lv, const gchar* f, const gchar* fn, const gint ln, const gchar* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fputc('\n', stderr);
    __atomic_add_fetch(&g_errors, 1, __ATOMIC_RELAXED);
}

/* --------------------------------------- driver ops → SchedulerPolicy -- */
typedef struct adapt {
    SchedulerPolicy* pol;
    Host* hosts;
} adapt;

/* scheduler.c:488-531: addHost on the main thread, before the workers start */
static void a_add_host(void* data, uint32_t host, uint64_t token) {
    adapt* a = data;
    a->pol->addHost(a->pol, &a->hosts[host], (pthread_t)token);
}
/* scheduler.c:78-88: the calling worker's hosts, for worker_bootHosts */
static uint32_t a_hosts(void* data, uint64_t token, uint32_t* out, uint32_t cap) {
    adapt* a = data;
    (void)token;  /* the glue identifies the worker by pthread_self() */
    GQueue* q = a->pol->getAssignedHosts(a->pol);
    uint32_t n = 0;
    for (GList* l = q ? q->head : NULL; l && n < cap; l = l->next) out[n++] = ((Host*)l->data)->index;
    return n;
}
/* scheduler_push (scheduler.c:339-357) after its endTime drop, which the driver
 * applies: the policy takes the reference */
static void a_push(void* data, sg_hevent* e, uint32_t src, uint32_t dst, sg_simtime barrier) {
    adapt* a = data;
    Event* ev = malloc(sizeof *ev);
    ev->h = e;
    __atomic_add_fetch(&g_live, 1, __ATOMIC_RELAXED);
    a->pol->push(a->pol, ev, &a->hosts[src], &a->hosts[dst], barrier);
}
/* scheduler_pop (scheduler.c:369-378): the worker executes the payload and
 * unrefs the event (worker.c:170-171); the driver frees the payload */
static sg_hevent* a_pop(void* data, sg_simtime barrier) {
    adapt* a = data;
    Event* ev = a->pol->pop(a->pol, barrier);
    if (!ev) return NULL;
    sg_hevent* h = ev->h;
    free(ev);
    __atomic_sub_fetch(&g_live, 1, __ATOMIC_RELAXED);
    return h;
}
static sg_simtime a_next(void* data) {
    adapt* a = data;
    return a->pol->getNextTime(a->pol);
}
static void a_free(void* data) { (void)data; }  /* glue_run_phold frees the policy */

typedef struct glue_report {
    int64_t live_after_free;   /* Event references the policy leaked (must be 0) */
    int64_t unref_at_free;     /* events the glue's free unref'd (queued at the end) */
    int64_t errors;            /* logger error() calls (SGCHK failures) */
    int64_t exact_ids;         /* 1 when built with SHADOW_HAS_EVENT_SRCID */
} glue_report;

/* Run PHOLD with n_workers worker threads through schedulerpolicygpu_new()'s
 * vtable; the policy is freed at the end (scheduler.c:276), which unrefs every
 * event still queued.  Not reentrant (the doubles are process globals). */
int glue_run_phold(const sg_phold_params* P, const sg_phold_tables* T, uint32_t n_workers,
                   uint32_t scheduler_seed, uint64_t max_rounds, sg_sched_result* res, uint64_t* digest,
                   uint64_t* pops, uint32_t* rng, uint64_t* event_counter, glue_report* rep) {
    g_live = 0;
    g_unref_free = 0;
    g_errors = 0;
    g_in_free = 0;
    g_n_workers = n_workers;
    adapt a;
    a.hosts = calloc(P->n_hosts ? P->n_hosts : 1, sizeof(Host));
    if (!a.hosts) return SG_ERR_NOMEM;
    /* GQuarks are positive and increase with registration order in a Shadow
     * run; a sparse mapping shows the glue relies on neither density nor value */
    for (uint32_t i = 0; i < P->n_hosts; i++) {
        a.hosts[i].id = 5 + 3 * i;
        a.hosts[i].index = i;
    }
    a.pol = schedulerpolicygpu_new();
    sg_sched_policy_ops ops = {&a, a_add_host, a_hosts, a_push, a_pop, a_next, a_free};
    int rc = sg_sched_run_phold(P, T, n_workers, scheduler_seed, &ops, max_rounds, res, digest, pops, rng,
                                event_counter);
    g_in_free = 1;
    a.pol->free(a.pol);
    g_in_free = 0;
    free(a.hosts);
    if (rep) {
        rep->live_after_free = g_live;
        rep->unref_at_free = g_unref_free;
        rep->errors = g_errors;
#ifdef SHADOW_HAS_EVENT_SRCID
        rep->exact_ids = 1;
#else
        rep->exact_ids = 0;
#endif
    }
    return rc;
}
