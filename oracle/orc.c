/*
 * orc.c — TEST INFRASTRUCTURE, not product code (see orc.h).
 *
 * CPU restatement of the reference's round semantics, written from the
 * reference source (paths under /root/reference/src/main, Shadow 1.14.0):
 *
 *   event order      core/work/event.c:110-153 (time, dst id, src id, srcHostEventID)
 *   queues           utility/priority_queue.c:115-175 (binary min-heap; any correct
 *                    heap yields the same pop sequence because keys are unique)
 *   push / bump      core/scheduler/scheduler.c:339-357,
 *                    scheduler_policy_host_single.c:167-208 (+ host_steal.c:225-272)
 *   pop              scheduler_policy_host_single.c:210-271 (+ host_steal.c:274-418)
 *   next time / MIN  host_single.c:273-305, scheduler.c:386-398, 634-650
 *   windows          core/slave.c:413-466, core/master.c:133-159, 450-480
 *   send             core/worker.c:243-304 (reliability draw, ceil delay, push)
 *   event ids        core/work/event.c:28-43, host/host.c:397-400
 *   RNG              utility/random.c:32-51 over glibc rand_r (glibc 2.35)
 *   PHOLD            src/test/phold/test_phold.c:160-178, 234-239, 310-312
 *   gossip           configs[4]'s body (defined here): PHOLD's
 *                    destination draw and worker_sendPacket per forward
 *   serial policy    scheduler_policy_global_single.c (no bump, one global queue)
 *
 * Per-host independence inside a round (inter-host events are bumped to >= the
 * barrier, so nothing another host does this round can be popped this round)
 * makes the sequential host loop below produce exactly the per-host pop
 * sequences of host_single / host_steal with any worker count and any
 * host-to-thread assignment.
 */
#include "orc.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SIMTIME_MAX (UINT64_MAX - 1)
#define ONE_MS 1000000ULL
#define RAND_MAX_ 2147483647

static __thread char orc_err[256];
const char* orc_error(void) { return orc_err; }

/* ---------------- glibc rand_r + Random (random.c:32-51) ---------------- */
static int32_t orc_rand_r(uint32_t* seed) {
    uint32_t next = *seed;
    int32_t result;
    next *= 1103515245u;
    next += 12345u;
    result = (int32_t)((next / 65536u) % 2048u);
    next *= 1103515245u;
    next += 12345u;
    result <<= 10;
    result ^= (int32_t)((next / 65536u) % 1024u);
    next *= 1103515245u;
    next += 12345u;
    result <<= 10;
    result ^= (int32_t)((next / 65536u) % 1024u);
    *seed = next;
    return result;
}

/* ---------------- event_compare (event.c:110-153) ----------------------- */
/* Host ids are GQuarks assigned in registration order (slave.c:300), so
 * comparing dense indices is host_compare (host.c:439-445). */
static inline int ev_less(const orc_event* a, const orc_event* b) {
    if (a->time != b->time) return a->time < b->time;
    if (a->dst != b->dst) return a->dst < b->dst;
    if (a->src != b->src) return a->src < b->src;
    return a->seq < b->seq;
}

/* ---------------- binary heap (priority_queue.c) ------------------------ */
typedef struct heap {
    orc_event* a;
    uint32_t n, cap;
} heap;

static int heap_push(heap* h, const orc_event* e) {
    if (h->n == h->cap) {
        uint32_t nc = h->cap ? h->cap * 2 : 8;
        orc_event* na = (orc_event*)realloc(h->a, (size_t)nc * sizeof(orc_event));
        if (!na) return -1;
        h->a = na;
        h->cap = nc;
    }
    uint32_t i = h->n++;
    h->a[i] = *e;
    while (i > 0) { /* heapify_up, priority_queue.c:91-97 */
        uint32_t p = (i - 1) / 2;
        if (!ev_less(&h->a[i], &h->a[p])) break;
        orc_event t = h->a[i];
        h->a[i] = h->a[p];
        h->a[p] = t;
        i = p;
    }
    return 0;
}

static void heap_pop(heap* h, orc_event* out) {
    *out = h->a[0];
    h->a[0] = h->a[--h->n];
    uint32_t i = 0; /* heapify_down, priority_queue.c:99-113 */
    for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && ev_less(&h->a[c + 1], &h->a[c])) c++;
        if (!ev_less(&h->a[c], &h->a[i])) break;
        orc_event t = h->a[i];
        h->a[i] = h->a[c];
        h->a[c] = t;
        i = c;
    }
}

/* ---------------- simulation state ------------------------------------- */
struct orc_sim {
    orc_params p;
    uint32_t *vertex, *rng;
    uint64_t* delay;
    int32_t *keep, *wthresh;
    uint32_t* jump;
    /* local hosts */
    heap* q;
    uint64_t *ev, *pops, *digest;
    uint32_t* rng_state;
    heap global; /* serial mode */
    /* outbox */
    orc_event* out;
    size_t n_out, cap_out;
    /* window state (master.c) */
    uint64_t S, E, min_jump, next_min_jump, jmin;
    int booted, done;
    orc_stats st;
    orc_trace_rec* trace;
    /* message-only per-host traces for the probe hash */
    uint64_t* win;
    size_t n_win, cap_win;
    uint64_t* pcount; /* [V*V] path packet counters (topology.c:2053-2063) */
    uint32_t* seen;   /* gossip: [n_local][mw] message bitsets */
    uint32_t mw;
    /* ordered discovery (orc_set_ordered_discovery): the reference's path
     * cache replayed in this oracle's pop order */
    double* pc_lat;
    uint8_t *pc_kind, *pc_have;
    uint32_t* pc_tgt;
    uint32_t pc_ntgt;
    int pc_complete, pc_directed;
    double pc_min; /* topology->minimumPathLatency, 0 = unset */
};

uint64_t orc_digest_mix(uint64_t pos, uint64_t time, uint32_t src, uint64_t seq) {
#define FMIX(z) (z ^= z >> 33, z *= 0xff51afd7ed558ccdULL, z ^= z >> 33, z *= 0xc4ceb9fe1a85ec53ULL, z ^= z >> 33)
    /* test infrastructure: the per-host trace digest term, order-sensitive
       through pos (the device computes the same) */
    uint64_t z = time ^ (pos * 0x9E3779B97F4A7C15ULL);
    FMIX(z);
    z ^= ((uint64_t)src << 40) | seq;
    FMIX(z);
#undef FMIX
    return z;
}

orc_sim* orc_create(const orc_params* p, const uint32_t* host_vertex, const uint32_t* host_rng,
                    const uint64_t* delay_ns, const int32_t* keep_max, const uint32_t* jump_ms,
                    const int32_t* weight_thresh) {
    if (!p || p->n_hosts == 0 || p->n_vertices == 0 || !host_vertex || !host_rng || !delay_ns ||
        !keep_max || !jump_ms || (p->dst_rule == ORC_DST_WEIGHTS && !weight_thresh) ||
        p->first_host + p->n_local > p->n_hosts) {
        snprintf(orc_err, sizeof orc_err, "orc_create: bad arguments");
        return NULL;
    }
    orc_sim* s = (orc_sim*)calloc(1, sizeof *s);
    if (!s) return NULL;
    s->p = *p;
    if (s->p.n_local == 0 && s->p.first_host == 0) s->p.n_local = p->n_hosts;
    size_t N = p->n_hosts, VV = (size_t)p->n_vertices * p->n_vertices, L = s->p.n_local;
    s->vertex = (uint32_t*)malloc(N * 4);
    s->rng = (uint32_t*)malloc(N * 4);
    s->delay = (uint64_t*)malloc(VV * 8);
    s->keep = (int32_t*)malloc(VV * 4);
    s->jump = (uint32_t*)malloc(VV * 4);
    s->wthresh = (int32_t*)malloc(N * 4);
    s->q = (heap*)calloc(L, sizeof(heap));
    s->ev = (uint64_t*)calloc(L, 8);
    s->pops = (uint64_t*)calloc(L, 8);
    s->digest = (uint64_t*)calloc(L, 8);
    s->rng_state = (uint32_t*)malloc(L * 4);
    s->pcount = (uint64_t*)calloc(VV, 8);
    if (p->trace_capacity) s->trace = (orc_trace_rec*)malloc(p->trace_capacity * sizeof(orc_trace_rec));
    if (p->workload == ORC_WORKLOAD_GOSSIP) {
        if (p->gossip_msgs == 0 || p->gossip_msgs > p->n_hosts || p->gossip_msgs > 65536) {
            orc_destroy(s);
            snprintf(orc_err, sizeof orc_err, "orc_create: gossip needs 1 <= messages <= min(hosts, 65536)");
            return NULL;
        }
        s->mw = (p->gossip_msgs + 31) / 32;
        s->seen = (uint32_t*)calloc(L * s->mw, 4);
        if (!s->seen) {
            orc_destroy(s);
            snprintf(orc_err, sizeof orc_err, "orc_create: out of memory");
            return NULL;
        }
    }
    if (!s->vertex || !s->rng || !s->delay || !s->keep || !s->jump || !s->wthresh || !s->q || !s->ev ||
        !s->pops || !s->digest || !s->rng_state || !s->pcount || (p->trace_capacity && !s->trace)) {
        orc_destroy(s);
        snprintf(orc_err, sizeof orc_err, "orc_create: out of memory");
        return NULL;
    }
    memcpy(s->vertex, host_vertex, N * 4);
    memcpy(s->rng, host_rng, N * 4);
    memcpy(s->delay, delay_ns, VV * 8);
    memcpy(s->keep, keep_max, VV * 4);
    memcpy(s->jump, jump_ms, VV * 4);
    if (weight_thresh) memcpy(s->wthresh, weight_thresh, N * 4);
    for (size_t i = 0; i < L; i++) s->rng_state[i] = host_rng[s->p.first_host + i];
    s->jmin = UINT64_MAX;
    s->next_min_jump = (p->window_rule == ORC_WINDOW_FIXED) ? p->fixed_jump : 0;
    return s;
}

void orc_destroy(orc_sim* s) {
    if (!s) return;
    if (s->q)
        for (uint32_t i = 0; i < s->p.n_local; i++) free(s->q[i].a);
    free(s->global.a);
    free(s->q);
    free(s->vertex);
    free(s->rng);
    free(s->delay);
    free(s->keep);
    free(s->jump);
    free(s->wthresh);
    free(s->ev);
    free(s->pops);
    free(s->digest);
    free(s->rng_state);
    free(s->out);
    free(s->trace);
    free(s->win);
    free(s->pcount);
    free(s->seen);
    free(s->pc_lat);
    free(s->pc_kind);
    free(s->pc_have);
    free(s->pc_tgt);
    free(s);
}

/* ---------------- ordered path discovery ---------------------------------- */
/* Test infrastructure: restates the reference's lazy path cache, looked up in
 * the order this oracle pops events (hosts in index order, each host's events
 * in event_compare order: shadow -w 1, host_single.c:210-271). */
int orc_set_ordered_discovery(orc_sim* s, const double* lat, const uint8_t* kind, const uint8_t* attached,
                              int complete, int directed) {
    size_t V = s->p.n_vertices, VV = V * V;
    s->pc_lat = (double*)malloc(VV * sizeof(double));
    s->pc_kind = (uint8_t*)malloc(VV);
    s->pc_have = (uint8_t*)calloc(VV, 1);
    s->pc_tgt = (uint32_t*)malloc(V * 4);
    if (!s->pc_lat || !s->pc_kind || !s->pc_have || !s->pc_tgt) {
        snprintf(orc_err, sizeof orc_err, "orc_set_ordered_discovery: out of memory");
        return -1;
    }
    memcpy(s->pc_lat, lat, VV * sizeof(double));
    memcpy(s->pc_kind, kind, VV);
    s->pc_ntgt = 0;
    for (uint32_t v = 0; v < V; v++) /* _topology_getUniqueVertexTargets */
        if (!attached || attached[v]) s->pc_tgt[s->pc_ntgt++] = v;
    s->pc_complete = complete;
    s->pc_directed = directed;
    s->pc_min = 0;
    return 0;
}

/* _topology_storePathInCache + _topology_shouldStorePath (topology.c:1306-1390) */
static void pc_put(orc_sim* s, uint32_t a, uint32_t b, int direct) {
    size_t V = s->p.n_vertices, ab = (size_t)a * V + b, ba = (size_t)b * V + a;
    int exists = s->pc_have[ab] || s->pc_have[ba];
    int refused = (s->pc_complete && !direct) || (!direct && s->pc_kind[ab] == 0 /* SG_PATH_DIRECT */);
    if (exists || refused) return;
    s->pc_have[ab] = 1;
    if (s->pc_min == 0 || s->pc_lat[ab] < s->pc_min) s->pc_min = s->pc_lat[ab];
}

/* _topology_getPathEntry (topology.c:1969-2051): the V*V index of the path
 * returned, or -1. */
static int64_t pc_entry(orc_sim* s, uint32_t a, uint32_t b) {
    size_t V = s->p.n_vertices, ab = (size_t)a * V + b, ba = (size_t)b * V + a;
    if (s->pc_have[ab]) return (int64_t)ab;
    if (!s->pc_directed && s->pc_have[ba]) return (int64_t)ba;
    if (s->pc_kind[ab] == 0) { /* complete, or preferred and adjacent: the edge */
        pc_put(s, a, b, 1);
    } else if (a == b) { /* _topology_computeShortestPathToSelf, stored as non-direct */
        pc_put(s, a, a, 0);
    } else { /* _topology_computeSourcePaths: every attached target at once */
        for (uint32_t i = 0; i < s->pc_ntgt; i++)
            if (s->pc_tgt[i] != a) pc_put(s, a, s->pc_tgt[i], 0);
    }
    if (s->pc_have[ab]) return (int64_t)ab;
    if (s->pc_have[ba]) return (int64_t)ba;
    return -1;
}

static inline int is_local(const orc_sim* s, uint32_t h) {
    return h >= s->p.first_host && h < s->p.first_host + s->p.n_local;
}

static int outbox_push(orc_sim* s, const orc_event* e) {
    if (s->n_out == s->cap_out) {
        size_t nc = s->cap_out ? s->cap_out * 2 : 1024;
        orc_event* n = (orc_event*)realloc(s->out, nc * sizeof(orc_event));
        if (!n) return -1;
        s->out = n;
        s->cap_out = nc;
    }
    s->out[s->n_out++] = *e;
    return 0;
}

/* scheduler_push (scheduler.c:339-357) + policy push (host_single.c:167-208) */
static int sched_push(orc_sim* s, orc_event* e, uint32_t src_host) {
    if (e->time >= s->p.end_time) { /* scheduler.c:343-346: dropped, id already used */
        s->st.drop_endtime++;
        return 0;
    }
    if (s->p.mode == ORC_MODE_SERIAL) /* global_single.c: no bump */
        return heap_push(&s->global, e);
    uint64_t barrier = s->E; /* currentRound.endTime */
    if (src_host != e->dst && e->time < barrier) { /* host_single.c:180-184 */
        e->time = barrier;
        s->st.bumped++;
    } else if (src_host == e->dst && e->time < barrier && s->booted) {
        s->st.same_round++; /* self event popped later in this same round */
    }
    if (!is_local(s, e->dst)) return outbox_push(s, e);
    return heap_push(&s->q[e->dst - s->p.first_host], e);
}

/* destination draw (test_phold.c:160-178 / survey probe) */
static int choose_dst(orc_sim* s, uint32_t* rng, uint32_t* dst) {
    int32_t x = orc_rand_r(rng);
    uint32_t N = s->p.n_hosts;
    if (s->p.dst_rule == ORC_DST_UNIFORM_FLOOR) {
        double r = (double)x / (double)RAND_MAX_;
        uint32_t d = (uint32_t)floor(r * N);
        if (d >= N) d = N - 1;
        *dst = d;
        return 1;
    }
    /* first i with cumulative(i) >= r  <=>  x <= thresh[i] (thresh non-decreasing) */
    if (x > s->wthresh[N - 1]) return 0;
    uint32_t lo = 0, hi = N - 1; /* smallest i with x <= thresh[i] */
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (x <= s->wthresh[mid]) hi = mid; else lo = mid + 1;
    }
    *dst = lo;
    return 1;
}

/* One PHOLD send from host h at time now (worker_sendPacket, worker.c:243-304). */
static int send_one(orc_sim* s, uint32_t h, uint32_t* rng, uint64_t now, uint64_t* evc, uint32_t msg) {
    uint32_t d;
    if (!choose_dst(s, rng, &d)) { /* no host chosen: the plugin sends nothing */
        s->st.null_dst++;
        return 0;
    }
    s->st.sends++;
    size_t pair = (size_t)s->vertex[h] * s->p.n_vertices + s->vertex[d];
    /* topology_getReliability builds the path (discovery) before the drop test */
    if (s->pc_lat) { /* ordered discovery: the cache's entry and running minimum */
        int64_t k = pc_entry(s, s->vertex[h], s->vertex[d]);
        if (k < 0) {
            snprintf(orc_err, sizeof orc_err, "no path %u -> %u", s->vertex[h], s->vertex[d]);
            return -1;
        }
        pair = (size_t)k;
        if (s->pc_min > 0 && (uint64_t)s->pc_min < s->jmin) s->jmin = (uint64_t)s->pc_min; /* master.c:153 */
    } else if (s->jump[pair] < s->jmin) {
        s->jmin = s->jump[pair];
    }
    int32_t c = orc_rand_r(rng); /* chance = random_nextDouble(host RNG) */
    int bootstrapping = now < s->p.bootstrap_end;
    if (!(bootstrapping || c <= s->keep[pair])) {
        s->st.drop_reliability++;
        return 0;
    }
    s->pcount[pair]++; /* topology_incrementPathPacketCounter, worker.c:279 */
    orc_event e;
    e.time = now + s->delay[pair];
    e.dst = d;
    e.src = h;
    e.seq = (*evc)++; /* event_new_ → host_getNewEventID */
    e.msg = msg;
    e.pad = 0;
    return sched_push(s, &e, h);
}

/* Gossip body (configs[4]).  The reference ships no gossip plugin, so the body
 * is defined here on the reference's own send path:
 *   message m in [0, M) originates at host o(m) = floor(m*N/M) at time
 *   T_m = gossip_start + m*gossip_interval: o(m)'s boot event schedules a self
 *   event carrying m (worker_scheduleTask, worker.c:218-234: src = dst, no
 *   path, no draw; scheduler_push's endTime drop applies);
 *   an event carrying m at host h: if h has seen m, nothing happens (the pop
 *   still commits); otherwise h marks m seen and forwards it to k = load peers,
 *   each one destination draw (test_phold.c:160-178) and one worker_sendPacket
 *   (reliability draw before the drop test, worker.c:267-279). */
static int execute_gossip(orc_sim* s, const orc_event* e, uint32_t li, int boot) {
    const uint32_t h = e->dst;
    if (boot) {
        const uint64_t N = s->p.n_hosts, M = s->p.gossip_msgs;
        const uint64_t m = ((uint64_t)h * M + N - 1) / N; /* smallest m with m*N/M >= h */
        if (m < M && (m * N) / M == h) {
            orc_event o;
            o.time = s->p.gossip_start + m * s->p.gossip_interval;
            o.seq = s->ev[li]++;
            o.dst = o.src = h;
            o.msg = (uint32_t)m;
            o.pad = 0;
            return sched_push(s, &o, h);
        }
        return 0;
    }
    uint32_t* w = &s->seen[(size_t)li * s->mw + (e->msg >> 5)];
    const uint32_t bit = 1u << (e->msg & 31);
    if (*w & bit) return 0; /* duplicate */
    *w |= bit;
    for (uint32_t k = 0; k < s->p.load; k++)
        if (send_one(s, h, &s->rng_state[li], e->time, &s->ev[li], e->msg)) return -1;
    return 0;
}

static int execute(orc_sim* s, const orc_event* e) {
    uint32_t h = e->dst, li = h - s->p.first_host;
    uint64_t pos = s->pops[li]++;
    s->st.pops++;
    s->digest[li] += orc_digest_mix(pos, e->time, e->src, e->seq);
    if (s->trace && s->st.trace_len < s->p.trace_capacity) {
        orc_trace_rec* r = &s->trace[s->st.trace_len++];
        r->time = e->time;
        r->seq = e->seq;
        r->host = h;
        r->src = e->src;
        r->pos = pos;
    }
    int boot = (e->src == h && e->seq == 0);
    if (boot) s->st.boots++;
    if (s->p.workload == ORC_WORKLOAD_GOSSIP) return execute_gossip(s, e, li, boot);
    uint32_t nsend = boot ? s->p.load : 1; /* test_phold.c:234-239 / 310-312 */
    for (uint32_t k = 0; k < nsend; k++)
        if (send_one(s, h, &s->rng_state[li], e->time, &s->ev[li], 0)) return -1;
    return 0;
}

int orc_boot(orc_sim* s) {
    if (s->booted) return -1;
    /* worker_bootHosts: a self event at t=0 per host; event_new_ takes id 0.
     * Pushed before the first round, when currentRound.endTime == endTime. */
    s->E = s->p.end_time;
    for (uint32_t i = 0; i < s->p.n_local; i++) {
        orc_event e = {0, s->ev[i]++, s->p.first_host + i, s->p.first_host + i, 0, 0};
        if (sched_push(s, &e, e.src)) return -1;
    }
    s->S = 0; /* slave.c:431 */
    s->E = 1;
    s->booted = 1;
    return 0;
}

static void record_window(orc_sim* s) {
    if (s->n_win + 2 > s->cap_win) {
        size_t nc = s->cap_win ? s->cap_win * 2 : 1024;
        uint64_t* n = (uint64_t*)realloc(s->win, nc * 8);
        if (!n) return;
        s->win = n;
        s->cap_win = nc;
    }
    s->win[s->n_win++] = s->S;
    s->win[s->n_win++] = s->E;
}

int orc_round_process(orc_sim* s) {
    if (!s->booted) return -1;
    if (s->done) return 0; /* rounds after the end are no-ops, as on the device */
    record_window(s);
    uint64_t E = s->E;
    for (uint32_t li = 0; li < s->p.n_local; li++) {
        heap* q = &s->q[li];
        /* host_single pop loop (host_single.c:237-267): pop while head < barrier;
         * self events created this round with t < barrier are popped too. */
        while (q->n > 0 && q->a[0].time < E) {
            orc_event e;
            heap_pop(q, &e);
            if (execute(s, &e)) return -1;
        }
    }
    s->st.rounds++;
    return 0;
}

size_t orc_outbox(orc_sim* s, const orc_event** out) {
    *out = s->out;
    return s->n_out;
}
void orc_outbox_clear(orc_sim* s) { s->n_out = 0; }

int orc_ingest(orc_sim* s, const orc_event* ev, size_t n) {
    for (size_t i = 0; i < n; i++) {
        if (!is_local(s, ev[i].dst)) return -1;
        if (heap_push(&s->q[ev[i].dst - s->p.first_host], &ev[i])) return -1;
    }
    return 0;
}

uint64_t orc_local_min(orc_sim* s) { /* host_single.c:273-305 */
    uint64_t m = SIMTIME_MAX;
    for (uint32_t li = 0; li < s->p.n_local; li++)
        if (s->q[li].n && s->q[li].a[0].time < m) m = s->q[li].a[0].time;
    return m;
}

uint64_t orc_local_jmin(orc_sim* s) { return s->jmin; }

/* master_slaveFinishedCurrentRound (master.c:450-480). */
int orc_window_apply(orc_sim* s, uint64_t global_min, uint64_t global_jmin) {
    if (s->done) return 0;
    if (s->p.window_rule == ORC_WINDOW_DISCOVERED && global_jmin != UINT64_MAX) {
        /* topology.c:1374-1385 → master_updateMinTimeJump (master.c:148-159):
         * nextMinJumpTime = (SimulationTime)minPathLatency * 1ms; the running
         * minimum of the truncations is the truncation of the running minimum. */
        s->next_min_jump = global_jmin * ONE_MS;
    }
    s->min_jump = s->next_min_jump;
    uint64_t jump;
    if (s->p.window_rule == ORC_WINDOW_FIXED) {
        jump = s->p.fixed_jump;
    } else {
        jump = s->min_jump > 0 ? s->min_jump : 10 * ONE_MS; /* master.c:137 */
        if (s->p.runahead_min > 0 && jump < s->p.runahead_min) jump = s->p.runahead_min;
    }
    uint64_t start = global_min, end = global_min + jump;
    if (end > s->p.end_time) end = s->p.end_time;
    s->S = start;
    s->E = end;
    s->done = !(start < end);
    return !s->done;
}

int64_t orc_run(orc_sim* s, uint64_t max_rounds) {
    if (s->p.n_local != s->p.n_hosts) {
        snprintf(orc_err, sizeof orc_err, "orc_run: sharded sim, use the round primitives");
        return -1;
    }
    uint64_t r = 0;
    while (!s->done && r < max_rounds) {
        if (orc_round_process(s)) return -1;
        r++;
        orc_window_apply(s, orc_local_min(s), s->jmin);
    }
    return (int64_t)r;
}

int orc_run_serial(orc_sim* s) {
    if (s->p.mode != ORC_MODE_SERIAL || !s->booted) return -1;
    /* global_single pop with barrier = endTime (scheduler.c:130, 367) */
    record_window(s);
    while (s->global.n > 0 && s->global.a[0].time < s->p.end_time) {
        orc_event e;
        heap_pop(&s->global, &e);
        if (execute(s, &e)) return -1;
    }
    s->done = 1;
    return 0;
}

int orc_stats_get(orc_sim* s, orc_stats* out) {
    *out = s->st;
    uint64_t pend = s->global.n + s->n_out;
    for (uint32_t li = 0; li < s->p.n_local; li++) pend += s->q[li].n;
    out->pending = pend;
    out->window_start = s->S;
    out->window_end = s->E;
    out->done = (uint64_t)s->done;
    out->min_jump = s->min_jump;
    out->next_min_jump = s->next_min_jump;
    out->jmin_ms = s->jmin;
    return 0;
}

int orc_host_state(orc_sim* s, uint64_t* digest, uint64_t* pops, uint32_t* rng, uint64_t* ev) {
    size_t L = s->p.n_local;
    if (digest) memcpy(digest, s->digest, L * 8);
    if (pops) memcpy(pops, s->pops, L * 8);
    if (rng) memcpy(rng, s->rng_state, L * 4);
    if (ev) memcpy(ev, s->ev, L * 8);
    return 0;
}

size_t orc_trace(orc_sim* s, orc_trace_rec* out, size_t cap) {
    size_t n = s->st.trace_len < cap ? s->st.trace_len : cap;
    if (out && n) memcpy(out, s->trace, n * sizeof(orc_trace_rec));
    return s->st.trace_len;
}

size_t orc_windows(orc_sim* s, uint64_t* out_pairs, size_t cap_pairs) {
    size_t n = s->n_win / 2;
    size_t m = n < cap_pairs ? n : cap_pairs;
    if (out_pairs && m) memcpy(out_pairs, s->win, m * 16);
    return n;
}

static int cmp_trace(const void* a, const void* b) {
    const orc_trace_rec* x = (const orc_trace_rec*)a;
    const orc_trace_rec* y = (const orc_trace_rec*)b;
    if (x->host != y->host) return x->host < y->host ? -1 : 1;
    return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

uint64_t orc_probe_hash(orc_sim* s, uint64_t* n_msgs) {
    /* Per host i in index order, per message pop in pop order:
     *   h = h * 1000003 ^ (t*31 + src*7 + seq + i),  h0 = 5381. */
    size_t n = s->st.trace_len;
    orc_trace_rec* t = (orc_trace_rec*)malloc((n ? n : 1) * sizeof *t);
    if (!t) return 0;
    memcpy(t, s->trace, n * sizeof *t);
    qsort(t, n, sizeof *t, cmp_trace);
    uint64_t h = 5381, m = 0;
    for (size_t k = 0; k < n; k++) {
        if (t[k].src == t[k].host && t[k].seq == 0) continue; /* boot event */
        h = h * 1000003ULL ^ (t[k].time * 31 + (uint64_t)t[k].src * 7 + t[k].seq + t[k].host);
        m++;
    }
    free(t);
    if (n_msgs) *n_msgs = m;
    return h;
}

/* ---------------- setup restatements (cross-check of sg_host.c) --------- */
static double orc_next_double(uint32_t* s) { /* random.c:39-43 */
    return (double)orc_rand_r(s) / (double)RAND_MAX_;
}
static uint32_t orc_next_uint(uint32_t* s) { /* random.c:45-51 */
    double f = orc_next_double(s);
    return (uint32_t)(f * (double)UINT32_MAX);
}
int32_t orc_rand(uint32_t* state) { return orc_rand_r(state); }

void orc_seed_chain(uint32_t seed, uint32_t n, uint32_t* slave_seed, uint32_t* sched_seed,
                    uint32_t* node_seeds) {
    uint32_t m = seed;                 /* master.c:95 */
    uint32_t ss = orc_next_uint(&m);   /* master.c:417 */
    uint32_t sl = ss;                  /* slave.c:182 */
    uint32_t sc = orc_next_uint(&sl);  /* slave.c:198 */
    if (slave_seed) *slave_seed = ss;
    if (sched_seed) *sched_seed = sc;
    for (uint32_t i = 0; i < n; i++) node_seeds[i] = orc_next_uint(&sl); /* slave.c:301 */
}

/* rule 1: topology.c:2327-2333; rule 0: index mod V without a draw */
void orc_attach(uint32_t n, uint32_t V, int rule, const uint32_t* node_seeds, uint32_t* vertex,
                uint32_t* rng) {
    for (uint32_t i = 0; i < n; i++) {
        uint32_t st = node_seeds[i];
        if (rule == 1) {
            double d = orc_next_double(&st);
            int32_t range = (int32_t)V - 1;
            vertex[i] = (uint32_t)(int32_t)round((double)(range * d));
        } else {
            vertex[i] = i % V;
        }
        rng[i] = st;
    }
}

static int32_t orc_prefix(double c) { /* max x with x/RAND_MAX <= c, by linear-free bisection */
    if ((double)RAND_MAX_ / (double)RAND_MAX_ <= c) return RAND_MAX_;
    if (!(0.0 <= c)) return -1;
    int64_t lo = 0, hi = RAND_MAX_;
    while (hi - lo > 1) {
        int64_t mid = (lo + hi) / 2;
        if ((double)mid / (double)RAND_MAX_ <= c) lo = mid; else hi = mid;
    }
    return (int32_t)lo;
}

/* topology.c:1877-1927 + worker.c:275-277 + master.c:153 */
void orc_build_paths(uint32_t V, const double* lat, const double* eloss, const double* vloss,
                     uint64_t* delay, int32_t* keep, uint32_t* jump) {
    for (uint32_t s = 0; s < V; s++)
        for (uint32_t d = 0; d < V; d++) {
            size_t k = (size_t)s * V + d;
            double rel = 1.0;
            if (vloss) {
                rel *= (1.0 - vloss[s]);
                rel *= (1.0 - vloss[d]);
            }
            rel *= (1.0 - eloss[k]);
            double tl = 0.0 + lat[k];
            delay[k] = (uint64_t)ceil(tl * (double)ONE_MS);
            keep[k] = orc_prefix(rel);
            jump[k] = (uint32_t)(uint64_t)tl;
        }
}

/* test_phold.c:160-178 */
void orc_weight_thresholds(uint32_t n, const double* w, int32_t* out) {
    double total = 0.0, cum = 0.0;
    for (uint32_t i = 0; i < n; i++) total += w[i];
    for (uint32_t i = 0; i < n; i++) {
        cum += w[i] / total;
        out[i] = orc_prefix(cum);
    }
}

size_t orc_path_counts(orc_sim* s, uint64_t* out, size_t cap) {
    const size_t n = (size_t)s->p.n_vertices * s->p.n_vertices;
    if (out) memcpy(out, s->pcount, (n < cap ? n : cap) * 8);
    return n;
}
