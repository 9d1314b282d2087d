/*
 * scheduler_policy_gpu.c — the Shadow-side glue of the `gpu` SchedulerPolicy.
 *
 * Drop into src/main/core/scheduler/ next to scheduler_policy_host_single.c and
 * register it as INTEGRATION.md §2 lists (enum value, scheduler.c case, slave.c
 * policy string, options.c help, CMake source list).  It maps Host* / Event* onto
 * the opaque ids and handles of include/shadowgpu.h §3; the library never
 * dereferences a Shadow pointer.  The vtable it fills is
 * core/scheduler/scheduler_policy.h:31-51, and the constructor has the same
 * `(void)` shape as its siblings at scheduler_policy.h:53-58.
 *
 * No other reference file needs an edit beyond the registration lines:
 *   - the enum value SP_PARALLEL_GPU (scheduler_policy.h:12-29): define
 *     SHADOW_HAS_SP_PARALLEL_GPU once it is in the enum;
 *   - srcHostEventID.  Event is opaque outside event.c and event.h has no getter
 *     for it.  event_compare (event.c:110-153) uses it only to order events of
 *     the same (src, dst) pair at equal times.  Every event is pushed right after
 *     event_new_ on the thread executing its source host (worker.c:229-230,
 *     297-300), so one source's pushes arrive in creation order, minus the
 *     events scheduler_push drops at endTime (scheduler.c:343-346).  A per-source
 *     push counter is therefore a monotone relabelling of srcHostEventID and
 *     gives the same pop order.  A maintainer who adds the one-line getter
 *     event_getSrcHostEventID to event.{h,c} defines
 *     SHADOW_HAS_EVENT_SRCID and the exact value is passed instead.
 *
 * tests/test_integration_glue.py compiles this file against the unmodified
 * reference headers (and conda GLib) whenever /root/reference is present, and
 * runs it under AddressSanitizer through tests/glue_harness.c (test doubles).
 * tests/glue_phold.c links it to the real libshadowgpu.so, and
 * tests/test_gpu_glue.py runs PHOLD through its vtable on the GPU against the
 * oracle.
 */
#include <glib.h>
#include <pthread.h>

#include "main/core/scheduler/scheduler_policy.h"
#include "main/core/support/options.h"
#include "main/core/work/event.h"
#include "main/core/worker.h"
#include "main/host/host.h"
#include "main/utility/utility.h"
#include "shadowgpu.h"
#include "support/logger/logger.h"

#ifdef SHADOW_HAS_SP_PARALLEL_GPU
#define SG_POLICY_TYPE SP_PARALLEL_GPU
#else /* the value the new enumerator takes after SP_PARALLEL_THREAD_PERHOST */
#define SG_POLICY_TYPE ((SchedulerPolicyType)(SP_PARALLEL_THREAD_PERHOST + 1))
#endif

#ifdef SHADOW_HAS_EVENT_SRCID
guint64 event_getSrcHostEventID(Event* event); /* INTEGRATION.md §3 */
#endif

SchedulerPolicy* schedulerpolicygpu_new(void);

typedef struct { GQuark id; pthread_t thread; } PendingHost;

typedef struct {
    GArray* pending;            /* addHost calls, replayed once every host is known */
    GHashTable* idToHost;       /* GQuark -> Host* */
    GHashTable* idToIndex;      /* GQuark -> registration index + 1 (read-only after create) */
    guint64* pushCount;         /* per source host: pushes so far (srcHostEventID order) */
    GHashTable* threadToHosts;  /* pthread_t -> GQueue* (getAssignedHosts result; owns it) */
    GMutex lock;
    GOnce once;
    sg_policy* p;
} GpuPolicyData;

#define SGCHK(x) do { int _rc = (x); if (_rc != SG_OK) error("gpu policy: %s", sg_last_error()); } while (0)

/* addHost runs single-threaded from scheduler_start (scheduler.c:488-531); the
 * device policy is created at the first call after it, when every host is known.
 * That first call comes from a worker thread (getAssignedHosts at boot,
 * scheduler.c:572-589), so worker_getOptions() is valid there.  The worker count
 * is the scheduler's nWorkers (slave.c:196 passes options_getNWorkerThreads to
 * scheduler_new): every worker, including one that was assigned no host, calls
 * getNextTime once per round (scheduler.c:393-394), and the device flush counts
 * exactly those arrivals. */
static gpointer _gpu_create(gpointer arg) {
    GpuPolicyData* d = arg;
    guint nThreads = options_getNWorkerThreads(worker_getOptions());
    sg_policy_params prm = {.n_threads = nThreads ? nThreads : 1, .max_hosts = d->pending->len,
                            .queue_cap = 0, .device = 0};
    SGCHK(sg_policy_create(&prm, &d->p));
    d->pushCount = g_new0(guint64, d->pending->len ? d->pending->len : 1);
    for (guint i = 0; i < d->pending->len; i++) {
        PendingHost* ph = &g_array_index(d->pending, PendingHost, i);
        g_hash_table_insert(d->idToIndex, GUINT_TO_POINTER(ph->id), GUINT_TO_POINTER(i + 1));
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

/* host_single.c:146-165.  Called on each worker at boot and again at shutdown
 * (scheduler.c:78-113); the queue returned last time is freed by the hash
 * table's value-destroy function when the new one replaces it. */
static GQueue* _gpu_getAssignedHosts(SchedulerPolicy* policy) {
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
    g_hash_table_insert(d->threadToHosts, GSIZE_TO_POINTER((gsize)self), q);
    g_mutex_unlock(&d->lock);
    return q;
}

static guint64 _gpu_srcEventID(GpuPolicyData* d, Event* event, GQuark src) {
#ifdef SHADOW_HAS_EVENT_SRCID
    (void)d; (void)src;
    return event_getSrcHostEventID(event);
#else
    (void)event;
    guint idx = GPOINTER_TO_UINT(g_hash_table_lookup(d->idToIndex, GUINT_TO_POINTER(src)));
    utility_assert(idx != 0);
    /* one source host runs on one thread at a time; the atomic only keeps a
     * host that migrates between rounds (host_steal-style) well defined */
    return __atomic_fetch_add(&d->pushCount[idx - 1], 1, __ATOMIC_RELAXED);
#endif
}

/* push takes the caller's reference (scheduler.c:354); the bumped time is written
 * back into the event as host_single.c:181 does. */
static void _gpu_push(SchedulerPolicy* policy, Event* event, Host* srcHost, Host* dstHost,
                      SimulationTime barrier) {
    GpuPolicyData* d = policy->data;
    sg_policy* p = _gpu(policy);
    GQuark src = host_getID(srcHost);
    SimulationTime t = 0;
    SGCHK(sg_policy_push(p, (uint64_t)pthread_self(), (uint64_t)(uintptr_t)event,
                         event_getTime(event), src, host_getID(dstHost),
                         _gpu_srcEventID(d, event, src), barrier, &t));
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
    g_free(d->pushCount);
    g_array_free(d->pending, TRUE);
    g_hash_table_destroy(d->idToHost);
    g_hash_table_destroy(d->idToIndex);
    g_hash_table_destroy(d->threadToHosts); /* frees every queue still held */
    g_mutex_clear(&d->lock);
    g_free(d);
    MAGIC_CLEAR(policy);
    g_free(policy);
}

SchedulerPolicy* schedulerpolicygpu_new(void) {
    GpuPolicyData* d = g_new0(GpuPolicyData, 1);
    d->pending = g_array_new(FALSE, FALSE, sizeof(PendingHost));
    d->idToHost = g_hash_table_new(g_direct_hash, g_direct_equal);
    d->idToIndex = g_hash_table_new(g_direct_hash, g_direct_equal);
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
