/*
 * orc.h — TEST INFRASTRUCTURE, not product code.
 *
 * CPU restatement of Shadow 1.14's event-scheduling semantics (the oracle the
 * HIP path is checked against).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  See orc.c for the per-function
 * reference citations and DESIGN.md §Oracle for how it is pinned.
 */
#ifndef ORC_H
#define ORC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_event {
    uint64_t time;  /* SimulationTime */
    uint64_t seq;   /* srcHostEventID */
    uint32_t dst;   /* destination host index (registration order) */
    uint32_t src;   /* source host index */
    uint32_t msg;   /* gossip: message id carried by the packet (0 for PHOLD) */
    uint32_t pad;
} orc_event;

enum { ORC_MODE_HOST = 0, ORC_MODE_SERIAL = 1 };
enum { ORC_WORKLOAD_PHOLD = 0, ORC_WORKLOAD_GOSSIP = 1 };
enum { ORC_DST_UNIFORM_FLOOR = 0, ORC_DST_WEIGHTS = 1 };
enum { ORC_WINDOW_FIXED = 0, ORC_WINDOW_DISCOVERED = 1 };

typedef struct orc_params {
    uint32_t n_hosts, n_vertices, load, dst_rule, window_rule, mode;
    uint32_t first_host, n_local; /* shard: hosts [first_host, first_host+n_local) */
    uint64_t end_time, bootstrap_end, fixed_jump, runahead_min;
    uint64_t trace_capacity;      /* 0 = no per-pop records */
    /* gossip workload (configs[4]); see orc.c execute_gossip */
    uint32_t workload, gossip_msgs;
    uint64_t gossip_start, gossip_interval;
} orc_params;

typedef struct orc_stats {
    uint64_t rounds, pops, boots, sends, null_dst, drop_reliability, drop_endtime;
    uint64_t bumped, same_round, pending;
    uint64_t window_start, window_end, done, min_jump, next_min_jump, jmin_ms;
    uint64_t trace_len;
} orc_stats;

typedef struct orc_trace_rec {
    uint64_t time, seq;
    uint32_t host, src;
    uint64_t pos;
} orc_trace_rec;

typedef struct orc_sim orc_sim;

orc_sim* orc_create(const orc_params* p, const uint32_t* host_vertex, const uint32_t* host_rng,
                    const uint64_t* delay_ns, const int32_t* keep_max, const uint32_t* jump_ms,
                    const int32_t* weight_thresh);
void orc_destroy(orc_sim* s);
const char* orc_error(void);

/* Boot events (t = 0, seq 0) for the local hosts; window [0, 1). */
int orc_boot(orc_sim* s);
/* Unsharded: run rounds until done or max_rounds; returns rounds run (<0 error). */
int64_t orc_run(orc_sim* s, uint64_t max_rounds);
/* Serial global policy (scheduler_policy_global_single.c): pops every event
 * before endTime in global event_compare order, no barrier bump. */
int orc_run_serial(orc_sim* s);

/* Sharded round primitives (the distributed protocol drives these). */
int orc_round_process(orc_sim* s);                 /* current window, local hosts */
size_t orc_outbox(orc_sim* s, const orc_event** out); /* events for other shards */
void orc_outbox_clear(orc_sim* s);
int orc_ingest(orc_sim* s, const orc_event* ev, size_t n);
uint64_t orc_local_min(orc_sim* s);               /* MIN over local queue heads */
uint64_t orc_local_jmin(orc_sim* s);              /* min truncated latency discovered */
int orc_window_apply(orc_sim* s, uint64_t global_min, uint64_t global_jmin); /* 1 = keep running */

int orc_stats_get(orc_sim* s, orc_stats* out);
int orc_host_state(orc_sim* s, uint64_t* digest, uint64_t* pops, uint32_t* rng, uint64_t* ev);
size_t orc_trace(orc_sim* s, orc_trace_rec* out, size_t cap);
/* Per-round windows recorded so far: pairs {start, end}. */
size_t orc_windows(orc_sim* s, uint64_t* out_pairs, size_t cap_pairs);
/* Trace hash of the survey probe (SURVEY.md §0 key finding 2): chained over
 * hosts in index order and each host's message pops in pop order. */
uint64_t orc_probe_hash(orc_sim* s, uint64_t* n_msgs);
/* Kept sends per (source vertex, destination vertex), V*V (topology.c:2053-2063). */
size_t orc_path_counts(orc_sim* s, uint64_t* out, size_t cap);
/* Ordered discovery: sends look their path up in a restatement of the
 * reference's lazy path cache (topology.c:1306-1390, 1655-1875, 1969-2051), in
 * this oracle's pop order, instead of the jump_ms table.  lat / kind are
 * sg_graph_paths' V*V tables (kind 0 = direct), attached the target flags
 * (NULL = all).  Call before orc_boot. */
int orc_set_ordered_discovery(orc_sim* s, const double* lat, const uint8_t* kind, const uint8_t* attached,
                              int complete, int directed);

uint64_t orc_digest_mix(uint64_t pos, uint64_t time, uint32_t src, uint64_t seq);

/* Setup restatements (cross-checks for the product's sg_host.c). */
int32_t orc_rand(uint32_t* state);
void orc_seed_chain(uint32_t seed, uint32_t n, uint32_t* slave_seed, uint32_t* sched_seed,
                    uint32_t* node_seeds);
void orc_attach(uint32_t n, uint32_t V, int rule, const uint32_t* node_seeds, uint32_t* vertex,
                uint32_t* rng);
void orc_build_paths(uint32_t V, const double* lat, const double* eloss, const double* vloss,
                     uint64_t* delay, int32_t* keep, uint32_t* jump);
void orc_weight_thresholds(uint32_t n, const double* w, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif
