/*
 * shadowgpu.h — C-ABI of libshadowgpu, the MI355X (gfx950) event-scheduling core
 * for Shadow 1.14's conservative round scheduler.
 *
 * Plain C, opaque handles, int status returns (0 = SG_OK), no C++ or torch types.
 * Every entry point names the reference interface it replaces (paths relative to
 * the Shadow source tree, src/main/...).  INTEGRATION.md shows the reference-side
 * binding (scheduler_policy_gpu.c) a maintainer adds to use it.
 *
 * Two groups of entry points:
 *   1. Host-side restatements of the reference arithmetic that feeds the device
 *      tables (glibc rand_r streams, the seed chain, host attachment, direct-path
 *      delay/reliability resolution, PHOLD destination weights, window logic).
 *   2. The device engine: an HBM-resident calendar of time buckets; one
 *      conservative round is two kernels.  k_proc: every host pops its events
 *      before the barrier in event_compare order, the PHOLD body runs, delivery
 *      times and drops are resolved, inter-host events get the barrier bump, and
 *      the new events are reserved in their time buckets.  k_scatter: the new
 *      events are written into the buckets, the next window is planned (MIN
 *      next-event time + min-latency runahead → next [start, end)) and its due
 *      events are gathered into the host partitions.  Several shards add one
 *      all-to-all per step (the next k_proc queues the received events).
 */
#ifndef SHADOWGPU_H
#define SHADOWGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_ABI_VERSION 4

typedef uint64_t sg_simtime;                /* SimulationTime, core/support/definitions.h:18 */
#define SG_SIMTIME_INVALID UINT64_MAX       /* definitions.h:28 */
#define SG_SIMTIME_MAX (UINT64_MAX - 1)     /* definitions.h:33 */
#define SG_ONE_MS 1000000ULL                /* SIMTIME_ONE_MILLISECOND, definitions.h:48 */
#define SG_RAND_MAX 2147483647              /* glibc RAND_MAX: rand_r yields 31 bits */

enum sg_status {
    SG_OK = 0,
    SG_ERR_INVAL = 1,     /* bad argument / shape */
    SG_ERR_NOMEM = 2,     /* host or device allocation failed */
    SG_ERR_HIP = 3,       /* a HIP runtime call failed (see sg_last_error) */
    SG_ERR_OVERFLOW = 4,  /* a device queue, outbox or trace buffer ran out of slots */
    SG_ERR_STATE = 5,     /* call out of order (e.g. step before boot) */
    SG_ERR_NODEV = 6      /* no gfx950 device visible */
};

/* Last error message of the calling thread (static storage, never NULL). */
const char* sg_last_error(void);
int sg_abi_version(void);

/* ------------------------------------------------------------------------ */
/* 1. Reference arithmetic (host side)                                      */
/* ------------------------------------------------------------------------ */

/* glibc rand_r (three LCG steps, 31-bit result) on a per-host 32-bit state.
 * Replaces random_rand, utility/random.c:32-37. */
int32_t sg_rand_r(uint32_t* state);
/* random_nextDouble, utility/random.c:39-43: rand_r / RAND_MAX in FP64. */
double sg_random_next_double(uint32_t* state);
/* random_nextUInt, utility/random.c:45-51: (uint)(nextDouble * UINT_MAX). */
uint32_t sg_random_next_uint(uint32_t* state);

/* Seed chain for `-s seed`: master Random(seed) (core/master.c:95) → slave seed
 * (master.c:417) → slave Random (slave.c:182) → scheduler seed (slave.c:198) →
 * one node seed per host in registration order (slave.c:301). */
int sg_seed_chain(uint32_t seed, uint32_t n_hosts, uint32_t* slave_seed,
                  uint32_t* scheduler_seed, uint32_t* node_seeds);

enum sg_attach_rule {
    SG_ATTACH_MODULO = 0, /* vertex = host index mod V, no RNG draw (survey probe) */
    SG_ATTACH_RANDOM = 1  /* routing/topology.c:2327-2333: candidate round((V-1)*nextDouble) */
};
/* Host RNG = Random(nodeSeed) (host/host.c:176); topology_attach may consume one
 * draw (topology.c:2327).  Writes each host's vertex and its RNG state after
 * attachment. */
int sg_attach_hosts(uint32_t n_hosts, uint32_t n_vertices, uint32_t rule,
                    const uint32_t* node_seeds, uint32_t* vertex_out,
                    uint32_t* rng_state_out);

/* Largest x in [0, RAND_MAX] with (double)x / RAND_MAX <= reliability, or -1.
 * Turns worker.c:268-273's FP64 drop test (chance <= reliability) into an exact
 * integer compare on the raw rand_r value. */
int32_t sg_keep_threshold(double reliability);

/* Direct-path resolution for a complete V-vertex graph (topology.c:1877-1927):
 *   reliability = 1 * (1 - loss[src]) * (1 - loss[dst]) * (1 - edge_loss)
 *   delay_ns    = ceil(latency_ms * 1e6)                    (worker.c:275-277)
 *   keep_max    = sg_keep_threshold(reliability)
 *   jump_ms     = (uint64)latency_ms, the truncation of master.c:153
 * latency_ms / edge_loss are V*V row-major (src-major); vertex_loss may be NULL
 * (vertices without a packetloss attribute). */
int sg_build_paths(uint32_t n_vertices, const double* latency_ms,
                   const double* edge_loss, const double* vertex_loss,
                   uint64_t* delay_ns, int32_t* keep_max, uint32_t* jump_ms);

/* PHOLD destination weights (src/test/phold/test_phold.c:160-178): host i is the
 * first with cumulative(i) >= r, r = rand_r / RAND_MAX, cumulative summed in
 * FP64 in host order.  thresh[i] = largest x with x/RAND_MAX <= cumulative(i)
 * (or -1), so "first i with x <= thresh[i]" is the exact integer restatement.
 * An x above thresh[n-1] selects no host (the plugin sends nothing). */
int sg_build_weight_thresholds(uint32_t n, const double* weights, int32_t* thresh_out);

/* Window logic of the master (core/master.c:133-159, 450-480). */
typedef struct sg_window_state {
    sg_simtime min_jump;          /* master->minJumpTime */
    sg_simtime next_min_jump;     /* master->nextMinJumpTime */
    sg_simtime min_jump_config;   /* -r runahead in ns (master.c:97-98); 0 = unset */
    sg_simtime end_time;          /* stoptime in ns */
} sg_window_state;
/* Path discovery during the round lowered the topology minimum latency to
 * latency_ms (topology.c:1374-1385 → master_updateMinTimeJump). */
void sg_window_note_latency(sg_window_state* st, double latency_ms);
/* master_slaveFinishedCurrentRound: returns 1 to keep running. */
int sg_window_next(sg_window_state* st, sg_simtime min_next_event,
                   sg_simtime* start_out, sg_simtime* end_out);

/* Deterministic synthetic topology for the PHOLD configs: symmetric V*V
 * log-normal latency matrix (ms, self-loops included) with minimum min_ms and
 * uniform edge loss.  Input generation only — not reference semantics. */
int sg_topology_lognormal(uint32_t n_vertices, uint64_t seed, double median_ms,
                          double sigma, double min_ms, double edge_loss,
                          double* latency_ms_out, double* edge_loss_out);

/* ------------------------------------------------------------------------ */
/* 1b. Topology: GraphML → per-vertex-pair path tables (sg_topology.c)       */
/* ------------------------------------------------------------------------ */
/* Replaces topology_new / _topology_loadGraph (routing/topology.c:554-800) and
 * the path lookup behind topology_getLatency / topology_getReliability
 * (topology.c:1969-2087), evaluated for every vertex pair up front so the
 * device engine does one table read per send. */
typedef struct sg_graph sg_graph;

typedef struct sg_graph_desc {
    uint32_t n_vertices, n_edges;
    int32_t directed;         /* graph edgedefault="directed" */
    int32_t complete;         /* _topology_isComplete (topology.c:450-552) */
    int32_t prefers_direct;   /* preferdirectpaths graph attribute (topology.c:760-790) */
    double min_edge_latency_ms, max_edge_latency_ms;
} sg_graph_desc;

typedef struct sg_vertex_desc {   /* borrowed strings, NULL when absent */
    const char *id, *ip, *citycode, *countrycode, *geocode, *type;
    double packetloss;
    int32_t has_packetloss;
    uint64_t bandwidth_down, bandwidth_up;
} sg_vertex_desc;

/* Attachment hints of one host (host element attributes iphint, citycodehint,
 * countrycodehint, geocodehint, typehint); NULL = no hint. */
typedef struct sg_attach_hint {
    const char *ip, *citycode, *countrycode, *geocode, *type;
} sg_attach_hint;

enum sg_path_kind {
    SG_PATH_DIRECT = 0,   /* the edge itself (topology.c:1877-1927) */
    SG_PATH_SHORTEST = 1, /* source shortest paths (topology.c:1655-1875, 1407-1523) */
    SG_PATH_SELF = 2      /* shortest path to self (topology.c:1545-1653) */
};

/* Parse GraphML text (topology.c:554-800): keys by attr.name, vertices in
 * <node> order, edges with required latency and packetloss.  A GraphML
 * document embedded in a CDATA section is accepted as is. */
int sg_graphml_load(const char* text, uint64_t len, sg_graph** out);
int sg_graph_free(sg_graph* g);
int sg_graph_info(const sg_graph* g, sg_graph_desc* out);
int sg_graph_vertex(const sg_graph* g, uint32_t index, sg_vertex_desc* out);
int sg_graph_edge(const sg_graph* g, uint32_t index, uint32_t* src, uint32_t* dst,
                  double* latency_ms, double* packetloss);

/* topology_attach (topology.c:2094-2369) for n_hosts hosts in registration
 * order: hint filters, longest-prefix IP match or one random_nextDouble draw
 * from the host's RNG (rng_state[h] is advanced in place).  hints may be NULL
 * (no host has hints: every host draws among all vertices). */
int sg_graph_attach(const sg_graph* g, uint32_t n_hosts, const sg_attach_hint* hints,
                    uint32_t* rng_state, uint32_t* vertex_out);

/* The path every lookup (src vertex, dst vertex) resolves to, V*V row-major:
 * latency (ms) and reliability as _topology_getPathEntry would cache them,
 * the kind of path, and discovered_ms = the minimum path latency the lookup
 * makes known to the window logic (topology.c:1374-1385): the path's own
 * latency for direct and self paths, the minimum over all the source's stored
 * paths for shortest paths (one source run caches every attached target).
 * attached (V flags, NULL = all) selects the shortest-path targets
 * (_topology_getUniqueVertexTargets).  The reference's cache makes
 * incomplete graphs order-dependent (a reverse-direction hit, topology.c:
 * 1986-1990, runs no Dijkstra; directed graphs can get the reverse path,
 * topology.c:1312-1318 / 2034-2036): this is its value when every lookup's
 * source runs its own Dijkstra first.  tests/test_topology_cache_order.py
 * models the cache and shows the cases.  Complete graphs are exact; for the
 * reference's own order use sg_path_cache below. */
int sg_graph_paths(const sg_graph* g, const uint8_t* attached, double* latency_ms,
                   double* reliability, double* discovered_ms, uint8_t* kind);

/* Device tables from path results: delay_ns = ceil(latency * 1e6)
 * (worker.c:275-277), keep_max = sg_keep_threshold(reliability)
 * (worker.c:268-273), jump_ms = (uint64)discovered (master.c:153; latency when
 * discovered_ms is NULL). */
int sg_build_path_tables(uint32_t n_vertices, const double* latency_ms, const double* reliability,
                         const double* discovered_ms, uint64_t* delay_ns, int32_t* keep_max,
                         uint32_t* jump_ms);

/* The reference's lazy path cache in lookup order, for a driver that performs
 * the lookups in the reference's own order (the CPU-worker driver below: one
 * worker pops hosts in their list order, each host's events in event_compare
 * order, host_single.c:210-271).  A miss stores the direct path (complete
 * graph, or preferred and adjacent: topology.c:2013-2024), the self path
 * (topology.c:1545-1653), or every attached target's shortest path from the
 * source (topology.c:1655-1875) under the store rules of topology.c:1306-1336
 * (no entry in either direction; no non-direct path in a complete graph or
 * beside a preferred direct edge); a hit may be the reverse entry (undirected:
 * topology.c:1986-1990; after a miss in either kind of graph: 2033-2036).
 * latency_ms and kind are sg_graph_paths' V*V tables (the latency a store
 * would cache), attached its target flags (NULL = all).  The cache copies
 * them.  Not thread-safe: callers serialise lookups (the reference holds its
 * path-cache lock). */
typedef struct sg_path_cache sg_path_cache;
int sg_path_cache_create(uint32_t n_vertices, const double* latency_ms, const uint8_t* kind,
                         const uint8_t* attached, int complete, int directed, sg_path_cache** out);
int sg_path_cache_destroy(sg_path_cache* c);
/* _topology_getPathEntry(src, dst): *pair_out = the V*V index of the path the
 * reference returns (src*V+dst, or dst*V+src for a reverse entry: its delay
 * and reliability are that entry's); *min_ms_out = topology->minimumPathLatency
 * after the lookup (0 while nothing is stored; topology.c:1374-1385), whose
 * truncation to ms is the window's next jump (master.c:148-159). */
int sg_path_cache_lookup(sg_path_cache* c, uint32_t src_vertex, uint32_t dst_vertex, uint64_t* pair_out,
                         double* min_ms_out);
/* Source runs (Dijkstra) so far and stored entries. */
int sg_path_cache_stats(const sg_path_cache* c, uint64_t* runs, uint64_t* stored);

/* ------------------------------------------------------------------------ */
/* 2. Device engine (synthetic PHOLD-style workload, "Mode S")               */
/* ------------------------------------------------------------------------ */

enum sg_dst_rule {
    SG_DST_UNIFORM_FLOOR = 0, /* dst = floor(r * N), clamped to N-1 (survey probe) */
    SG_DST_WEIGHTS = 1        /* test_phold.c:160-178 via sg_build_weight_thresholds */
};
enum sg_window_rule {
    SG_WINDOW_FIXED = 0,      /* every window is [min, min + fixed_jump) */
    SG_WINDOW_DISCOVERED = 1  /* master.c: runahead = truncated min discovered latency */
};
/* The event body the device executes per committed event. */
enum sg_workload {
    SG_WORKLOAD_PHOLD = 0,    /* test_phold.c: boot sends `load` messages, each receipt sends one */
    SG_WORKLOAD_GOSSIP = 1    /* configs[4] flooding: message m originates at host
                                 floor(m*N/M) at gossip_start + m*gossip_interval (a
                                 self event its boot schedules); a host's first receipt
                                 of m forwards it to `load` (= fan-out) drawn peers
                                 through worker_sendPacket, later receipts are dropped
                                 by a per-host seen set */
};

typedef struct sg_phold_params {
    uint32_t n_hosts;        /* N, global (all shards) */
    uint32_t n_vertices;     /* V */
    uint32_t load;           /* messages each host sends when it boots (test_phold.c:234-239) */
    uint32_t dst_rule;       /* enum sg_dst_rule */
    uint32_t window_rule;    /* enum sg_window_rule */
    uint32_t queue_cap;      /* HBM event capacity per local host: the calendar's
                                chunk pool holds n_local * queue_cap events
                                (0 = default 64); running out is SG_ERR_OVERFLOW */
    uint32_t shard_index;    /* this rank */
    uint32_t shard_count;    /* ranks; hosts are block-partitioned */
    sg_simtime end_time;     /* scheduler endTime (scheduler.c:343) */
    sg_simtime bootstrap_end;/* worker_isBootstrapActive (worker.c:445-453) */
    sg_simtime fixed_jump;   /* SG_WINDOW_FIXED */
    sg_simtime runahead_min; /* -r in ns, SG_WINDOW_DISCOVERED */
    uint64_t trace_capacity; /* pop records kept for trace diffs (0 = off) */
    uint64_t exchange_cap;   /* per-peer outbox slots of the step API (multi-shard;
                                a single shard with exchange_cap != 0 runs the
                                step API too, one rank of a world-1 job) */
    uint32_t workload;       /* enum sg_workload */
    uint32_t gossip_msgs;    /* SG_WORKLOAD_GOSSIP: M messages, 1 <= M <= min(N, 65536) */
    sg_simtime gossip_start; /* origin time of message 0 */
    sg_simtime gossip_interval; /* origin spacing */
} sg_phold_params;

typedef struct sg_phold_tables {        /* host pointers, copied to HBM at create */
    const uint32_t* host_vertex;   /* [n_hosts] attachment vertex of every host */
    const uint32_t* host_rng;      /* [n_hosts] rand_r state after attachment */
    const uint64_t* delay_ns;      /* [V*V] */
    const int32_t* keep_max;       /* [V*V] */
    const uint32_t* jump_ms;       /* [V*V] */
    const int32_t* weight_thresh;  /* [n_hosts]; may be NULL for SG_DST_UNIFORM_FLOOR */
} sg_phold_tables;

typedef struct sg_round_stats {
    uint64_t rounds;          /* windows executed */
    uint64_t pops;            /* committed events (executed pops, worker.c:165-176) */
    uint64_t boots;           /* of which boot events */
    uint64_t sends;           /* send attempts with a destination */
    uint64_t null_dst;        /* destination draws that selected no host */
    uint64_t drop_reliability;/* dropped by the reliability test (PDS_INET_DROPPED) */
    uint64_t drop_endtime;    /* created but dropped at scheduler_push (t >= endTime) */
    uint64_t bumped;          /* inter-host events moved to the barrier */
    uint64_t same_round;      /* self events popped in the round that created them */
    uint64_t overflow;        /* nonzero: a queue / outbox / trace ran out of slots */
    sg_simtime window_start;  /* current window */
    sg_simtime window_end;
    uint64_t done;            /* 1 when start >= end (slave.c:459) */
    sg_simtime min_jump;
    sg_simtime next_min_jump;
    uint64_t jmin_ms;         /* truncated min discovered latency, UINT64_MAX if none */
    uint64_t pending;         /* events queued in HBM after the last round */
    uint64_t trace_len;       /* pop records written */
    uint64_t exchange_steps;  /* multi-shard: exchange steps run (rounds + drain steps) */
    uint64_t phase;           /* multi-shard: 1 while outbox leftovers are being drained */
} sg_round_stats;

typedef struct sg_trace_rec {   /* one executed pop */
    sg_simtime time;
    uint64_t seq;    /* srcHostEventID (event.c:38) */
    uint32_t host;   /* destination host index (global) */
    uint32_t src;    /* source host index (global) */
    uint64_t pos;    /* position in the host's pop sequence */
} sg_trace_rec;

typedef struct sg_engine sg_engine;

/* Allocates the HBM state for this shard's hosts and uploads the tables.
 * hip_stream may be NULL (the engine makes its own) or a hipStream_t. */
int sg_engine_create(const sg_phold_params* params, const sg_phold_tables* tables,
                     int device, void* hip_stream, sg_engine** out);
int sg_engine_destroy(sg_engine* e);
/* host_boot: one self event per local host at t=0 (seq 0) that sends `load`
 * messages, then the first window [0, 1) (slave.c:431). */
int sg_engine_boot(sg_engine* e);
/* Single shard: runs up to max_rounds windows without host round-trips, in
 * batches of `batch` rounds per host synchronisation; stops when done. */
int sg_engine_run(sg_engine* e, uint64_t max_rounds, uint32_t batch);
/* Enqueue one round (k_proc + k_scatter) without synchronising. */
int sg_engine_enqueue_round(sg_engine* e);
/* n rounds without reading the round state back (graph-batched when
 * sg_engine_set_graph is on); at most two batches stay queued on the stream. */
int sg_engine_enqueue_rounds(sg_engine* e, uint64_t n_rounds);
/* Graphs on (sg_engine_set_graph): capture one batch of rounds into the graph
 * now without running it, so that the first replay pays no capture and
 * instantiation (a timed region's first batch).  No-op with graphs off. */
int sg_engine_graph_prepare(sg_engine* e);
int sg_engine_sync(sg_engine* e);
int sg_engine_stats(sg_engine* e, sg_round_stats* out);   /* synchronises */
/* Per local host (index - first_host): trace digest, pops, rng state, event counter. */
int sg_engine_host_state(sg_engine* e, uint64_t* digest, uint64_t* pops,
                         uint32_t* rng, uint64_t* event_counter);
int sg_engine_host_range(sg_engine* e, uint32_t* first_host, uint32_t* n_local);
/* Cumulative hosts-with-pops per round (active host-rounds) and staged events. */
int sg_engine_active_hosts(sg_engine* e, uint64_t* active_host_rounds, uint64_t* emitted);
/* Cumulative record moves of the insert kernels (the per-kernel roofline's
 * algorithmic bytes): events k_proc staged, events k_scatter's gather moved from
 * the calendar into host partitions, received events k_scatter's receive role
 * routed into host partitions (several shards; the received events it leaves
 * for the next k_proc to stage are not counted). */
int sg_engine_event_moves(sg_engine* e, uint64_t* emitted, uint64_t* gathered, uint64_t* received);
/* k_scatter launches whose gather took the due list guessed by the k_proc
 * before (GSpec: the window is one whole bucket, the one after the executed
 * window) and launches that derived it from the bucket words.  SG_GSPEC=0
 * turns the guess off, SG_GSPEC=2 guesses a wrong bucket (the check must
 * reject it); both exist for tests. */
int sg_engine_gather_paths(sg_engine* e, uint64_t* guessed, uint64_t* listed);
/* Test only: between the next round's k_proc and k_scatter, corrupt two of
 * partition 0's staged records (one names a host past the shard, one lies
 * beyond the calendar's horizon).  k_scatter's insert role must clamp both in
 * bounds and set SG overflow flag 128 (an internal inconsistency); the run
 * then stops with SG_ERR_OVERFLOW.  Round-mode engines only. */
int sg_engine_debug_inject(sg_engine* e);
int sg_engine_trace(sg_engine* e, sg_trace_rec* out, uint64_t capacity, uint64_t* n_out);
/* Executed windows {start, end} per round (recorded when trace_capacity > 0). */
int sg_engine_windows(sg_engine* e, uint64_t* out_pairs, uint64_t capacity, uint64_t* n_out);
void* sg_engine_stream(sg_engine* e);

/* Calendar geometry chosen at create. */
typedef struct sg_engine_geom {
    uint64_t bucket_width;    /* W ns: the narrowest window the rules allow */
    uint32_t ring_buckets;    /* R: covers the widest window + the longest delay */
    uint32_t chunk_events;    /* events per pool chunk */
    uint32_t chunks;          /* pool chunks */
    uint32_t partition_hosts; /* HP: hosts per k_proc workgroup */
    uint32_t partitions;      /* P */
    uint32_t partition_cap;   /* due events one partition can take per round */
    uint32_t stage_cap;       /* new events one partition can stage per round */
} sg_engine_geom;
int sg_engine_geometry(sg_engine* e, sg_engine_geom* out);
/* Profiling hook: with SG_STAMPS=1 in the environment at create, k_proc records
 * per workgroup {start, sorted, phase A, phase B, end} s_memrealtime ticks
 * (100 MHz), {due events, active hosts, sends} and finer phase stamps of the
 * last round in a row of 32 u64 per partition, then one spare row and one row
 * per k_scatter workgroup (role, start, setup, events, end);
 * *n_out = 0 when the hook is off. */
int sg_engine_stamps(sg_engine* e, uint64_t* out, uint64_t capacity, uint64_t* n_out);

/* Multi-shard step, driven by the caller around ONE all-to-all per step (no
 * host synchronisation, no all-reduce):
 *   step_send(e, send) — on a process step: pops + PHOLD body + local MIN;
 *       events for other shards go to a per-peer outbox.  On every step: up to
 *       exchange_cap outbox events per peer are written into send, which is
 *       [G][rows][2] int64 (rows = sg_engine_exchange_rows): per peer block four
 *       header rows {n, sender has more, local MIN next time, local min jump ms,
 *       overflow flags, round, time base (the step's window start), 0} then n
 *       16-B event rows {time - time base | destination's index in the
 *       receiving shard << 40, src << 40 | srcHostEventID};
 *   (caller) all_to_all of send → recv, equal [rows][2] blocks per peer;
 *   step_recv(e, recv) — local new events into the queues, received events
 *       due in the new window straight into their hosts' partitions; the next
 *       window from the G received headers (the MIN all-reduce of
 *       scheduler.c:386-408 / master.c:450-480, carried by the all-to-all).
 *       The other received events are queued by the next step_send's kernel,
 *       so recv must stay intact until the next step_send has been enqueued
 *       (the next all-to-all overwrites it only after that).  When any sender
 *       still has outbox leftovers the next step is a drain step (same window,
 *       no processing). */
int sg_engine_exchange_rows(sg_engine* e, uint64_t* rows);
/* Change exchange_cap between steps (every shard must use the same value).  The
 * caller may then reallocate its send / receive buffers: the engine keeps a
 * copy of the last received blocks for the next step_send. */
int sg_engine_set_exchange_cap(sg_engine* e, uint64_t exchange_cap);
/* Largest per-peer outbox of a process step since the last reset. */
int sg_engine_exchange_peak(sg_engine* e, uint64_t* peak, int reset);
int sg_engine_step_send(sg_engine* e, int64_t* send);
int sg_engine_step_recv(sg_engine* e, const int64_t* recv);

/* Native step loop: the whole step (step_send, RCCL all-to-all over xGMI,
 * step_recv) issued from C on the engine stream, so no interpreter sits in the
 * round loop.  A communicator is made from a 128-byte RCCL unique id that rank 0
 * creates (sg_comm_unique_id) and the caller broadcasts; RCCL is opened with
 * dlopen, so the library the process already loaded (e.g. torch's) is the one
 * used.  run_steps enqueues n steps without synchronising; send / recv are
 * device buffers of [G][rows][2] int64.  With sg_engine_set_graph(e, b > 0)
 * (and for sg_engine_run in round mode) every b steps / rounds are captured once
 * into a hipGraph and replayed; a graph is rebuilt when the buffers, the
 * communicator, exchange_cap or the path-counter table change.  set_graph
 * always drops the current graph: call it (e.g. with 0) before destroying a
 * communicator a graph captured, since RCCL frees a captured collective's
 * resources only with its graph.  Errors of the
 * collective are SG_ERR_HIP with the RCCL message in sg_last_error. */
typedef struct sg_comm sg_comm;
/* SG_OK when RCCL can be opened in this process (no collective, no GPU work):
 * every rank probes before the collective sg_comm_create, so a job falls back
 * to another step loop on all ranks or none. */
int sg_comm_available(void);
int sg_comm_unique_id(uint8_t id_out[128]);
int sg_comm_create(const uint8_t id[128], int rank, int world, int device, sg_comm** out);
int sg_comm_destroy(sg_comm* c);
int sg_engine_run_steps(sg_engine* e, sg_comm* c, int64_t* send, int64_t* recv, uint64_t n_steps);
int sg_engine_set_graph(sg_engine* e, uint32_t batch);

/* Native step loop over xGMI peer stores instead of a collective (the same
 * step, the same blocks): every shard exports one region of uncached device
 * memory (arrival counters + double-buffered receive blocks), the caller
 * all-gathers the 128-byte handles in rank order, and each step stores block q
 * straight into shard q's region (k_proc itself by default, SG_XFUSE=0: a copy
 * kernel after it): every storing workgroup waits for its stores — and, when a
 * peer is on another GPU, issues a system-scope release — before it takes a
 * ticket, and the last one adds one arrival to every peer's counter
 * (SG_XFENCE=0/1 forces the release off or on).  The receiving k_scatter
 * waits for every sender's arrivals before it reads their headers (bounded:
 * 5 s, then it flags a time-out, the run stops at the next plan, and every
 * later wait of the link returns at once); shards sharing a device wait in a
 * one-workgroup kernel instead, so spinning workgroups never hold the CUs a
 * peer needs to arrive.
 * Replaces the ncclAllToAll of sg_engine_run_steps; the MIN all-reduce of
 * scheduler.c:386-408 / master.c:450-480 still rides in the block headers.
 *   create   after exchange_cap is final (a later change is refused);
 *   handle   this shard's region and device, to all-gather;
 *   attach   the G handles in rank order (this shard's own is skipped);
 *   selftest n_steps exchanges of a known pattern through the path the steps
 *            take (the fused push: many storing workgroups, release, ticket,
 *            the last one's headers and arrivals), checked on the device:
 *            *bad = mismatched words (+ 2^63 if a wait timed out); every shard
 *            must call it with the same n_steps;
 *   status   synchronises the engine stream; *timed_out = the senders whose
 *            arrival a wait gave up on (bit q: shard q), 0 if none;
 *   info     how the link runs (fenced, fused, shared device) and the last
 *            self-test's result;
 *   destroy  after every shard stopped stepping (the caller's barrier): the
 *            last received blocks are copied back into the engine first.
 *   debug_withhold (tests only): the fused step `step` steps from now does not
 *            arrive at shard `peer`, whose wait then times out. */
#define SG_XLINK_HANDLE_BYTES 128 /* the region's IPC handle + the device's PCI bus id */
typedef struct sg_xlink sg_xlink;
typedef struct sg_xlink_desc {
    uint32_t fenced;          /* a system-scope release by every storing workgroup */
    uint32_t fused;           /* k_proc stores the blocks itself (else k_xpush copies them) */
    uint32_t shared_device;   /* a peer shares this GPU: the arrivals are awaited by k_xwait */
    uint32_t selftest_steps;  /* the last self-test's exchanges */
    uint32_t selftest_fused;  /* ... through the fused push */
    uint32_t pad_;
    uint64_t selftest_bad;    /* ... its mismatched words (+ 2^63: a wait timed out) */
    uint64_t steps;           /* exchanges since attach (self-test included) */
} sg_xlink_desc;
int sg_xlink_create(sg_engine* e, sg_xlink** out);
int sg_xlink_handle(sg_xlink* x, uint8_t out[SG_XLINK_HANDLE_BYTES]);
int sg_xlink_attach(sg_xlink* x, const uint8_t* handles);
int sg_xlink_selftest(sg_xlink* x, uint32_t n_steps, uint64_t* bad);
int sg_xlink_status(sg_xlink* x, uint32_t* timed_out);
int sg_xlink_info(sg_xlink* x, sg_xlink_desc* out);
int sg_xlink_debug_withhold(sg_xlink* x, uint64_t step, uint32_t peer);
int sg_xlink_destroy(sg_xlink* x);
int sg_engine_run_steps_xlink(sg_engine* e, sg_xlink* x, uint64_t n_steps);

/* Kernel timing since sg_engine_set_timing(e, 1) (HIP events on the engine
 * stream): total ms and launches per kernel class, arrays of SG_KCLASSES. */
enum sg_kernel_class {
    SG_K_PROCESS = 0,  /* k_proc: pops + PHOLD body + send resolution + bucket reservations */
    SG_K_INSERT = 1,   /* k_scatter: events into their buckets, the next window planned
                          and gathered (sharded: received events due in it routed) */
    SG_K_PLAN = 2,     /* unused: planning is a k_scatter role now (class kept for ABI stability) */
    SG_K_GATHER = 3,   /* k_spec: the split step's insert, stash refill and guessed gather,
                        * on a second stream beside the all-to-all (several shards) */
    SG_K_EXCHANGE = 4, /* the step's RCCL all-to-all (sg_engine_run_steps): this shard's
                          wait for the slowest shard plus the transfer — the barrier
                          idle time of scheduler.c:380-389 */
    SG_KCLASSES = 5
};
int sg_engine_kernel_times(sg_engine* e, double* ms, uint64_t* launches);
/* enabled != 0 times every class; sg_engine_set_timing_mask times only the
 * classes in mask (bit 1 << class): fewer events, less inflation of the rest. */
int sg_engine_set_timing(sg_engine* e, int enabled);
int sg_engine_set_timing_mask(sg_engine* e, uint32_t mask);

/* Path packet counters (topology_incrementPathPacketCounter, topology.c:2053-2063,
 * counted where worker_sendPacket calls it: every send that passes the
 * reliability test, worker.c:273-279).  enable != 0 allocates a V*V table of
 * kept sends per (source vertex, destination vertex) and zeroes it; counting
 * costs one atomic per kept send, so it is off by default.  The reference keeps
 * one Path per cached direction, so on undirected graphs its count for {s, d}
 * is table[s][d] + table[d][s].  path_counts copies the table (n_out = V*V, or
 * 0 while off); sum the tables of all shards. */
int sg_engine_path_counters(sg_engine* e, int enable);
int sg_engine_path_counts(sg_engine* e, uint64_t* out, uint64_t capacity, uint64_t* n_out);

/* Barrier-idle timers: the Mode S counterpart of the per-worker GTimers that
 * accumulate the wait at the execute-events barrier (scheduler.c:380-389;
 * host_single's push/pop idle timers, scheduler_policy_host_single.c:36-37,
 * 186-200, 242-245, have no counterpart: Mode S takes no locks).  The
 * "worker" here is a host partition's k_proc workgroup: busy = its time from
 * start to its last store, idle = from there to the end of the round's last
 * partition, summed over the rounds since enable (a multi-shard step's wait
 * in the collective is not included).  enable != 0 zeroes them; they cost
 * one extra barrier per partition and a P-entry pass in k_scatter, so they are
 * off by default.  barrier_times copies P entries (n_out = P, or 0 while off). */
int sg_engine_barrier_timers(sg_engine* e, int enable);
int sg_engine_barrier_times(sg_engine* e, uint64_t* busy_ns, uint64_t* idle_ns, uint64_t capacity,
                            uint64_t* n_out);

/* ------------------------------------------------------------------------ */
/* 3. The `gpu` SchedulerPolicy ("Mode P", the drop-in boundary)            */
/* ------------------------------------------------------------------------ */
/* Replaces a SchedulerPolicy's data + function pointers
 * (core/scheduler/scheduler_policy.h:31-51) for a new SP_PARALLEL_GPU type;
 * INTEGRATION.md gives the Shadow-side scheduler_policy_gpu.c that maps
 * Host* / Event* onto these calls.  Threads are identified by an opaque token
 * (pthread_self() in Shadow).  Events are identified by an opaque nonzero
 * handle (the Event* in Shadow); the policy never dereferences it.
 *
 * Per round: push stages inter-host (and future self) events per thread with
 * no lock; self events before the barrier go to a per-host CPU heap (they must
 * be popped in this round, host_single.c:237-267).  The last worker to call
 * next_time flushes the staged events into the device calendar (time buckets
 * of 2^SG_PBUCKET_SHIFT ns, default 2^18; k_cins1 / k_cneed / k_calloc /
 * k_cins2) and reduces the MIN next time on the device (k_cmin).  The first pop
 * of the next round extracts, on the device, every queued event before the new
 * barrier sorted per host in event_compare order, reading only the due buckets
 * (k_xplan / k_hist / k_mscan / k_part / k_local / k_xfinish); pops merge that
 * run with the host's CPU heap. */
typedef struct sg_policy sg_policy;

typedef struct sg_policy_params {
    uint32_t n_threads;   /* worker threads that call push/pop/next_time (nWorkers) */
    uint32_t max_hosts;   /* hosts that will be added */
    uint32_t queue_cap;   /* initial calendar pool, in events per host (0 = 16; grows on demand) */
    int device;           /* HIP device */
} sg_policy_params;

int sg_policy_create(const sg_policy_params* params, sg_policy** out);
int sg_policy_destroy(sg_policy* p);
/* addHost (host_single.c:120-140): host_id is the host's GQuark, which orders
 * hosts in event_compare (host.c:439-445). */
int sg_policy_add_host(sg_policy* p, uint32_t host_id, uint64_t thread_token);
/* getAssignedHosts (host_single.c:146-165): host ids of the thread's hosts. */
int sg_policy_thread_hosts(sg_policy* p, uint64_t thread_token, uint32_t* ids_out,
                           uint32_t capacity, uint32_t* n_out);
/* push (host_single.c:167-208): returns in *time_out the event's time after the
 * barrier bump; the caller stores it in the event (event_setTime). */
int sg_policy_push(sg_policy* p, uint64_t thread_token, uint64_t handle, sg_simtime time,
                   uint32_t src_host_id, uint32_t dst_host_id, uint64_t src_event_id,
                   sg_simtime barrier, sg_simtime* time_out);
/* pop (host_single.c:210-271): *handle_out = 0 when the thread has no event
 * before the barrier. */
int sg_policy_pop(sg_policy* p, uint64_t thread_token, sg_simtime barrier, uint64_t* handle_out);
/* getNextTime (host_single.c:273-305): every worker calls it once per round
 * after the execute barrier; returns the MIN next event time (SG_SIMTIME_MAX
 * when every queue is empty). */
int sg_policy_next_time(sg_policy* p, uint64_t thread_token, sg_simtime* next_out);
/* Events still queued (for unref at free, host_single.c:104). */
int sg_policy_remaining(sg_policy* p, uint64_t* handles_out, uint64_t capacity, uint64_t* n_out);

/* Per-kernel profile of the policy's device half: every launch
 * carries its dispatch packet's start / stop timestamps (no extra packets),
 * and each kernel class accumulates its launches, time and algorithmic bytes
 * (the record bytes its job needs to read and write, counted from the insert
 * and extraction sizes).  skip_rounds: the first extractions (rounds) are not
 * counted (a bench's warmup).  Kernel classes, in order: k_cins1 k_cneed
 * k_calloc k_cins2 k_cmin k_xplan k_hist k_mscan k_part k_local k_xrank k_xlong. */
typedef struct sg_kernel_stat {
    char name[16];
    uint64_t launches;
    double ms;          /* summed kernel time */
    double alg_bytes;   /* summed algorithmic bytes */
} sg_kernel_stat;
int sg_policy_kernel_profile(sg_policy* p, int enable, uint32_t skip_rounds);
/* Up to `cap` classes into out; *n_out = the number of classes. */
int sg_policy_kernel_stats(sg_policy* p, sg_kernel_stat* out, uint32_t cap, uint32_t* n_out);

/* ------------------------------------------------------------------------ */
/* 4. Shadow-style round driver for running a policy outside Shadow          */
/* ------------------------------------------------------------------------ */
/* A C restatement of scheduler.c's round API + worker.c's loop (threads, the
 * execute / collect / prepare barriers, scheduler_push's endTime drop) that
 * drives any policy through the SchedulerPolicy-shaped vtable below, with the
 * synthetic PHOLD body executed by the CPU workers.  In Shadow itself
 * scheduler.c and worker.c play this role. */
typedef struct sg_hevent {
    sg_simtime time;
    uint64_t seq;    /* srcHostEventID */
    uint32_t src;    /* host index */
    uint32_t dst;
} sg_hevent;

typedef struct sg_sched_policy_ops {   /* mirrors struct _SchedulerPolicy */
    void* data;
    void (*add_host)(void* data, uint32_t host, uint64_t thread_token);
    uint32_t (*get_assigned_hosts)(void* data, uint64_t thread_token, uint32_t* out, uint32_t cap);
    void (*push)(void* data, sg_hevent* ev, uint32_t src, uint32_t dst, sg_simtime barrier);
    sg_hevent* (*pop)(void* data, sg_simtime barrier);
    sg_simtime (*get_next_time)(void* data);
    void (*free)(void* data);
} sg_sched_policy_ops;

typedef struct sg_sched_result {
    uint64_t rounds, pops, sends, drop_reliability, drop_endtime, bumped;
    double seconds;          /* wall time of the round loop (worker.c:165-176 semantics) */
    sg_simtime last_window_start, last_window_end;
    /* steady-state split: the only input field.  When mark_round > 0 the rounds
     * after the first mark_round are also reported on their own (a bench's
     * warmup excluded); otherwise the three outputs below are zero. */
    uint64_t mark_round;
    double marked_seconds;
    uint64_t marked_pops, marked_rounds;
    /* CPU time by stage, summed over the workers (input: profile != 0; the
     * rounds after mark_round when it is set, else the whole run): the policy's
     * push / pop / getNextTime calls (pop includes the extraction the first pop
     * of a round runs; getNextTime includes its flush and the wait for the
     * other workers' arrivals), the event bodies without their pushes, and the
     * scheduler barriers (scheduler.c:380-408).  Costs two clock reads per
     * call. */
    uint64_t profile;
    double prof_push_s, prof_pop_s, prof_next_s, prof_exec_s, prof_barrier_s;
    uint64_t prof_pushes, prof_pops;
} sg_sched_result;

/* The gpu policy as a vtable (data = a new sg_policy on `device`); release it
 * with ops->free(ops->data) (the SchedulerPolicy free, scheduler.c:276). */
int sg_policy_ops_gpu(uint32_t n_threads, uint32_t max_hosts, int device, sg_sched_policy_ops* out);
/* First error the gpu vtable's callbacks hit (their signatures return void). */
int sg_policy_ops_gpu_error(const sg_sched_policy_ops* ops);
/* The sg_policy behind a vtable made by sg_policy_ops_gpu (NULL otherwise). */
sg_policy* sg_policy_ops_gpu_policy(const sg_sched_policy_ops* ops);

/* Run the PHOLD workload with n_workers threads (>= 1) under `ops` (not freed).
 * max_rounds bounds the run; per-host digests / pops / rng / event counters
 * are written if the pointers are non-NULL.  Host->thread assignment is the
 * reference's shuffle (scheduler.c:437-531) seeded from the seed chain. */
int sg_sched_run_phold(const sg_phold_params* params, const sg_phold_tables* tables,
                       uint32_t n_workers, uint32_t scheduler_seed, const sg_sched_policy_ops* ops,
                       uint64_t max_rounds, sg_sched_result* result, uint64_t* digest,
                       uint64_t* pops, uint32_t* rng, uint64_t* event_counter);
/* The same with the reference's ordered path discovery: every send looks its
 * path up in `paths` (sg_path_cache_lookup, serialised by the driver) and
 * takes that path's delay and reliability and the cache's minimum latency,
 * instead of the tables' source-wide jump_ms.  With one worker the lookups come
 * in the reference's order (`shadow -w 1`); with several, in the order the
 * workers happen to reach them, as in the reference. */
int sg_sched_run_phold_paths(const sg_phold_params* params, const sg_phold_tables* tables,
                             sg_path_cache* paths, uint32_t n_workers, uint32_t scheduler_seed,
                             const sg_sched_policy_ops* ops, uint64_t max_rounds, sg_sched_result* result,
                             uint64_t* digest, uint64_t* pops, uint32_t* rng, uint64_t* event_counter);

#ifdef __cplusplus
}
#endif
#endif /* SHADOWGPU_H */
