/*
 * scheduler_policy_gpu.c — the Shadow-side glue of the `gpu` SchedulerPolicy.
 *
 * Drop into src/main/core/scheduler/ next to scheduler_policy_host_single.c and
 * register it as INTEGRATION.md §2 lists (enum value, scheduler.c case, slave.c
 * policy string, options.c help, CMake source list).  It maps Host* / Event* onto
 * the opaque ids and handles of include/shadowgpu.h §3; the library never
 * dereferences a Shadow pointer.  The vtable it fills is
 * core/scheduler/scheduler_policy.h:31-51.
 *
 * tests/test_integration_glue.py compiles this file -fsyntax-only against the
 * unmodified reference headers (and conda GLib) whenever /root/reference is
 * present.  Two additions the maintainer makes are therefore declared here:
 *   - the enum value SP_PARALLEL_GPU (scheduler_policy.h:12-29): define
 *     SHADOW_HAS_SP_PARALLEL_GPU once it is in the enum;
 *   - event_getSrcHost / event_getSrcHostEventID, two
 *     one-line getters added to core/work/event.{h,c}.
 */
#include <glib.h>
#include <pthread.h>

#include "main/core/scheduler/scheduler_policy.h"
#include "main/core/work/event.h"
#include "main/host/host.h"
#include "main/utility/utility.h"
#include "shadowgpu.h"
#include "support/logger/logger.h"

#ifdef SHADOW_HAS_SP_PARALLEL_GPU
#define SG_POLICY_TYPE SP_PARALLEL_GPU
#else /* the value the new enumerator takes after SP_PARALLEL_THREAD_PERHOST */
#define SG_POLICY_TYPE ((SchedulerPolicyType)(SP_PARALLEL_THREAD_PERHOST + 1))
#endif

/* added to core/work/event.{h,c} */
gpointer event_getSrcHost(Event* event);
guint64 event_getSrcHostEventID(Event* event);

SchedulerPolicy* schedulerpolicygpu_new(guint nWorkers);

typedef struct { GQuark id; pthread_t thread; } PendingHost;

typedef struct {
    guint nWorkers;
    GArray* pending;            /* addHost calls, replayed once the host count is known */
    GHashTable* idToHost;       /* GQuark -> Host* */
    GHashTable* threadToHosts;  /* pthread_t -> GQueue* (getAssignedHosts result) */
    GMutex lock;
    GOnce once;
    sg_policy* p;
} GpuPolicyData;

#define SGCHK(x) do { int _rc = (x); if (_rc != SG_OK) error("gpu policy: %s", sg_last_error()); } while (0)

/* addHost runs single-threaded from scheduler_start (scheduler.c:488-531); the
 * device policy is created at the first call after it, when every host is known. */
static gpointer _gpu_create(gpointer arg) {
    GpuPolicyData* d = arg;
    sg_policy_params prm = {.n_threads = d->nWorkers, .max_hosts = d->pending->len,
                            .queue_cap = 0, .device = 0};
    SGCHK(sg_policy_create(&prm, &d->p));
    for (guint i = 0; i < d->pending->len; i++) {
        PendingHost* ph = &g_array_index(d->pending, PendingHost, i);
        SGCHK(sg_policy_add_host(d->p, ph->id, (uint64_t)ph->thread));
    }
    return d->p;
}
static sg_policy* _gpu(SchedulerPolicy* policy) {
    GpuPolicyData* d = policy->data;
    return g_once(&d->once, _gpu_create, d);
}

static void _gpu_addHost(SchedulerPolicy* policy, Host* host, pthread_t thread) {
    GpuPolicyData* d = policy->data;
    PendingHost ph = {host_getID(host), thread};
    g_array_append_val(d->pending, ph);
    g_hash_table_insert(d->idToHost, GUINT_TO_POINTER(ph.id), host);
}

static GQueue* _gpu_getAssignedHosts(SchedulerPolicy* policy) {   /* host_single.c:146-165 */
    GpuPolicyData* d = policy->data;
    sg_policy* p = _gpu(policy);
    pthread_t self = pthread_self();
    guint32 n = 0;
    SGCHK(sg_policy_thread_hosts(p, (uint64_t)self, NULL, 0, &n));
    guint32* ids = g_new(guint32, n ? n : 1);
    SGCHK(sg_policy_thread_hosts(p, (uint64_t)self, ids, n, &n));
    GQueue* q = g_queue_new();
    for (guint32 i = 0; i < n; i++)
        g_queue_push_tail(q, g_hash_table_lookup(d->idToHost, GUINT_TO_POINTER(ids[i])));
    g_free(ids);
    g_mutex_lock(&d->lock);
    GQueue* old = g_hash_table_lookup(d->threadToHosts, GUINT_TO_POINTER(self));
    g_hash_table_insert(d->threadToHosts, GUINT_TO_POINTER(self), q);
    g_mutex_unlock(&d->lock);
    if (old) g_queue_free(old);
    return q;
}

/* push takes the caller's reference (scheduler.c:354); the bumped time is written
 * back into the event as host_single.c:181 does. */
static void _gpu_push(SchedulerPolicy* policy, Event* event, Host* srcHost, Host* dstHost,
                      SimulationTime barrier) {
    SimulationTime t = 0;
    SGCHK(sg_policy_push(_gpu(policy), (uint64_t)pthread_self(), (uint64_t)(uintptr_t)event,
                         event_getTime(event), host_getID(srcHost), host_getID(dstHost),
                         event_getSrcHostEventID(event), barrier, &t));
    event_setTime(event, t);
}

/* pop returns one owned reference or NULL (scheduler.c:369-409). */
static Event* _gpu_pop(SchedulerPolicy* policy, SimulationTime barrier) {
    uint64_t h = 0;
    SGCHK(sg_policy_pop(_gpu(policy), (uint64_t)pthread_self(), barrier, &h));
    return (Event*)(uintptr_t)h;
}

/* Every worker calls this once per round after the execute barrier
 * (scheduler.c:386-398); the last arrival flushes the round to HBM. */
static SimulationTime _gpu_getNextTime(SchedulerPolicy* policy) {
    SimulationTime t = SIMTIME_MAX;
    SGCHK(sg_policy_next_time(_gpu(policy), (uint64_t)pthread_self(), &t));
    return t;
}

static void _gpu_free(SchedulerPolicy* policy) {                      /* scheduler.c:276 */
    GpuPolicyData* d = policy->data;
    if (d->p) {
        uint64_t n = 0;
        SGCHK(sg_policy_remaining(d->p, NULL, 0, &n));
        uint64_t* hs = g_new(uint64_t, n ? n : 1);
        SGCHK(sg_policy_remaining(d->p, hs, n, &n));
        for (uint64_t i = 0; i < n; i++) event_unref((Event*)(uintptr_t)hs[i]); /* host_single.c:104 */
        g_free(hs);
        sg_policy_destroy(d->p);
    }
    g_array_free(d->pending, TRUE);
    g_hash_table_destroy(d->idToHost);
    g_hash_table_destroy(d->threadToHosts);
    g_mutex_clear(&d->lock);
    g_free(d);
    MAGIC_CLEAR(policy);
    g_free(policy);
}

SchedulerPolicy* schedulerpolicygpu_new(guint nWorkers) {
    GpuPolicyData* d = g_new0(GpuPolicyData, 1);
    d->nWorkers = nWorkers;
    d->pending = g_array_new(FALSE, FALSE, sizeof(PendingHost));
    d->idToHost = g_hash_table_new(g_direct_hash, g_direct_equal);
    d->threadToHosts = g_hash_table_new_full(g_direct_hash, g_direct_equal, NULL,
                                             (GDestroyNotify)g_queue_free);
    g_mutex_init(&d->lock);
    d->once = (GOnce)G_ONCE_INIT;

    SchedulerPolicy* policy = g_new0(SchedulerPolicy, 1);
    MAGIC_INIT(policy);
    policy->type = SG_POLICY_TYPE;
    policy->data = d;
    policy->referenceCount = 1;
    policy->addHost = _gpu_addHost;
    policy->getAssignedHosts = _gpu_getAssignedHosts;
    policy->push = _gpu_push;
    policy->pop = _gpu_pop;
    policy->getNextTime = _gpu_getNextTime;
    policy->free = _gpu_free;
    return policy;
}
