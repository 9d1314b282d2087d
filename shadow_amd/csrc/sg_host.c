/*
 * sg_host.c — host-side restatement of the reference arithmetic that feeds the
 * device tables of libshadowgpu (see include/shadowgpu.h for the contract).
 *
 * Everything here is exact integer / IEEE-754 FP64 code compiled with
 * -ffp-contract=off, so the values equal what the reference computes with the
 * same glibc and the same inputs.
 */
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "shadowgpu.h"

static __thread char g_err[512];

void sg_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

const char* sg_last_error(void) { return g_err; }
int sg_abi_version(void) { return SG_ABI_VERSION; }

/* glibc stdlib/rand_r.c (glibc 2.35): three steps of the LCG
 * next = next * 1103515245 + 12345, keeping 11 + 10 + 10 high bits.
 * Replaces random_rand, utility/random.c:32-37. */
int32_t sg_rand_r(uint32_t* state) {
    uint32_t next = *state;
    uint32_t result;
    next = next * 1103515245u + 12345u;
    result = (next / 65536u) % 2048u;
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (next / 65536u) % 1024u;
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (next / 65536u) % 1024u;
    *state = next;
    return (int32_t)result;
}

/* utility/random.c:39-43 */
double sg_random_next_double(uint32_t* state) {
    int32_t r = sg_rand_r(state);
    return (double)r / (double)SG_RAND_MAX;
}

/* utility/random.c:45-51 */
uint32_t sg_random_next_uint(uint32_t* state) {
    double f = sg_random_next_double(state);
    double max_uint = (double)UINT32_MAX;
    return (uint32_t)(f * max_uint);
}

int sg_seed_chain(uint32_t seed, uint32_t n_hosts, uint32_t* slave_seed,
                  uint32_t* scheduler_seed, uint32_t* node_seeds) {
    uint32_t master = seed;                          /* master.c:95 */
    uint32_t slave_s = sg_random_next_uint(&master); /* master.c:417 */
    uint32_t slave = slave_s;                        /* slave.c:182 */
    uint32_t sched = sg_random_next_uint(&slave);    /* slave.c:198 */
    if (slave_seed) *slave_seed = slave_s;
    if (scheduler_seed) *scheduler_seed = sched;
    if (n_hosts && !node_seeds) {
        sg_set_error("sg_seed_chain: node_seeds is NULL");
        return SG_ERR_INVAL;
    }
    for (uint32_t i = 0; i < n_hosts; i++)
        node_seeds[i] = sg_random_next_uint(&slave); /* slave.c:301, registration order */
    return SG_OK;
}

int sg_attach_hosts(uint32_t n_hosts, uint32_t n_vertices, uint32_t rule,
                    const uint32_t* node_seeds, uint32_t* vertex_out,
                    uint32_t* rng_state_out) {
    if (n_vertices == 0 || !node_seeds || !vertex_out || !rng_state_out) {
        sg_set_error("sg_attach_hosts: bad arguments");
        return SG_ERR_INVAL;
    }
    for (uint32_t i = 0; i < n_hosts; i++) {
        uint32_t rng = node_seeds[i]; /* host.c:176 random_new(nodeSeed) */
        uint32_t v;
        if (rule == SG_ATTACH_RANDOM) {
            /* topology.c:2327-2333: no IP hint, every vertex is a candidate,
             * candidates in vertex order; one nextDouble on the host Random. */
            double rd = sg_random_next_double(&rng);
            int32_t index_range = (int32_t)n_vertices - 1;
            int32_t chosen = (int32_t)round((double)(index_range * rd));
            v = (uint32_t)chosen;
        } else if (rule == SG_ATTACH_MODULO) {
            v = i % n_vertices;
        } else {
            sg_set_error("sg_attach_hosts: unknown rule %u", rule);
            return SG_ERR_INVAL;
        }
        vertex_out[i] = v;
        rng_state_out[i] = rng;
    }
    return SG_OK;
}

/* Predicate x/RAND_MAX <= c is monotone in x (correctly rounded division by a
 * positive constant), so its true set is a prefix [0, X]; find X. */
static int32_t prefix_threshold(double c) {
    if (!((double)SG_RAND_MAX / (double)SG_RAND_MAX <= c)) {
        if (!(0.0 / (double)SG_RAND_MAX <= c)) return -1;
        int64_t lo = 0, hi = SG_RAND_MAX; /* p(lo) true, p(hi) false */
        while (hi - lo > 1) {
            int64_t mid = lo + (hi - lo) / 2;
            if ((double)mid / (double)SG_RAND_MAX <= c) lo = mid; else hi = mid;
        }
        return (int32_t)lo;
    }
    return SG_RAND_MAX;
}

int32_t sg_keep_threshold(double reliability) { return prefix_threshold(reliability); }

int sg_build_paths(uint32_t n_vertices, const double* latency_ms,
                   const double* edge_loss, const double* vertex_loss,
                   uint64_t* delay_ns, int32_t* keep_max, uint32_t* jump_ms) {
    if (n_vertices == 0 || !latency_ms || !edge_loss || !delay_ns || !keep_max || !jump_ms) {
        sg_set_error("sg_build_paths: bad arguments");
        return SG_ERR_INVAL;
    }
    for (uint32_t s = 0; s < n_vertices; s++) {
        for (uint32_t d = 0; d < n_vertices; d++) {
            size_t k = (size_t)s * n_vertices + d;
            double lat = latency_ms[k];
            if (!(lat > 0.0) || !(lat < 4.0e9)) {
                sg_set_error("sg_build_paths: latency[%u][%u]=%g outside (0, 4e9) ms", s, d, lat);
                return SG_ERR_INVAL;
            }
            /* topology.c:1886-1921 */
            double total_latency = 0.0, total_rel = 1.0;
            if (vertex_loss) {
                total_rel *= (1.0 - vertex_loss[s]);
                total_rel *= (1.0 - vertex_loss[d]);
            }
            double edge_rel = (1.0 - edge_loss[k]); /* topology.c:437 */
            total_latency += lat;
            total_rel *= edge_rel;
            /* worker.c:275-277 */
            delay_ns[k] = (uint64_t)ceil(total_latency * (double)SG_ONE_MS);
            keep_max[k] = sg_keep_threshold(total_rel);
            /* master.c:153 truncation of the path latency in ms */
            jump_ms[k] = (uint32_t)(uint64_t)total_latency;
        }
    }
    return SG_OK;
}

int sg_build_weight_thresholds(uint32_t n, const double* weights, int32_t* thresh_out) {
    if (n == 0 || !weights || !thresh_out) {
        sg_set_error("sg_build_weight_thresholds: bad arguments");
        return SG_ERR_INVAL;
    }
    double total = 0.0; /* test_phold.c:344 totalWeight += weights[i] */
    for (uint32_t i = 0; i < n; i++) total += weights[i];
    double cumulative = 0.0; /* test_phold.c:166-170 */
    for (uint32_t i = 0; i < n; i++) {
        double norm = weights[i] / total;
        cumulative += norm;
        thresh_out[i] = prefix_threshold(cumulative);
    }
    return SG_OK;
}

/* master.c:148-159, including its comparison of a latency in ms against a jump
 * stored in ns (it only matters for paths longer than ~83 minutes). */
void sg_window_note_latency(sg_window_state* st, double latency_ms) {
    if (st->next_min_jump == 0 || latency_ms < (double)st->next_min_jump)
        st->next_min_jump = ((sg_simtime)latency_ms) * SG_ONE_MS;
}

/* master.c:133-146 + 450-480 */
int sg_window_next(sg_window_state* st, sg_simtime min_next_event,
                   sg_simtime* start_out, sg_simtime* end_out) {
    st->min_jump = st->next_min_jump;
    sg_simtime jump = st->min_jump > 0 ? st->min_jump : 10 * SG_ONE_MS;
    if (st->min_jump_config > 0 && jump < st->min_jump_config) jump = st->min_jump_config;
    sg_simtime start = min_next_event;
    sg_simtime end = min_next_event + jump; /* unsigned wrap as in the reference */
    if (end > st->end_time) end = st->end_time;
    if (start_out) *start_out = start;
    if (end_out) *end_out = end;
    return start < end ? 1 : 0;
}

/* splitmix64 stream for synthetic inputs */
static uint64_t sm64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static double sm64_unit(uint64_t* s) { /* (0, 1) */
    return ((double)(sm64(s) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

int sg_topology_lognormal(uint32_t n_vertices, uint64_t seed, double median_ms,
                          double sigma, double min_ms, double edge_loss,
                          double* latency_ms_out, double* edge_loss_out) {
    if (n_vertices == 0 || !latency_ms_out || !edge_loss_out || !(median_ms > 0) || !(min_ms > 0)) {
        sg_set_error("sg_topology_lognormal: bad arguments");
        return SG_ERR_INVAL;
    }
    uint64_t s = seed;
    const double two_pi = 6.283185307179586;
    for (uint32_t i = 0; i < n_vertices; i++) {
        for (uint32_t j = i; j < n_vertices; j++) {
            double u1 = sm64_unit(&s), u2 = sm64_unit(&s);
            double z = sqrt(-2.0 * log(u1)) * cos(two_pi * u2);
            double lat = median_ms * exp(sigma * z);
            lat = round(lat * 1000.0) / 1000.0; /* microsecond resolution, like GraphML values */
            if (lat < min_ms) lat = min_ms;
            latency_ms_out[(size_t)i * n_vertices + j] = lat;
            latency_ms_out[(size_t)j * n_vertices + i] = lat;
            edge_loss_out[(size_t)i * n_vertices + j] = edge_loss;
            edge_loss_out[(size_t)j * n_vertices + i] = edge_loss;
        }
    }
    return SG_OK;
}
