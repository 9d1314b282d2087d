/* sg_policy_dev.h — internal interface between the `gpu` policy's host logic
 * (sg_policy.c) and its device kernels (sg_policy_dev.hip). Not part of the
 * public C-ABI. */
#ifndef SG_POLICY_DEV_H
#define SG_POLICY_DEV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sgp_rec {     /* one staged / queued event, 32 B */
    uint64_t time;
    uint64_t seq;            /* srcHostEventID */
    uint64_t handle;         /* opaque Event* */
    uint32_t src_id;         /* source host id (GQuark): event_compare key */
    uint32_t dst;            /* destination host index (policy-dense) */
} sgp_rec;

typedef struct sgp_dev sgp_dev;

int sgp_dev_create(int device, uint32_t n_hosts, uint32_t cap, sgp_dev** out);
int sgp_dev_destroy(sgp_dev* d);
/* Deliver n records into the per-host HBM queues (grows them on demand). */
int sgp_dev_insert(sgp_dev* d, const sgp_rec* recs, uint64_t n);
/* The same for nseg host segments copied back to back (pinned segments DMA
 * straight from where the workers staged them). */
int sgp_dev_insert_segs(sgp_dev* d, const sgp_rec* const* segs, const uint64_t* lens, uint32_t nseg);
/* Pinned host memory for the workers' staging arenas (NULL on failure). */
void* sgp_host_alloc(uint64_t bytes);
void sgp_host_free(void* p);
/* MIN over every queued event time (SIMTIME_MAX if none). */
int sgp_dev_min(sgp_dev* d, uint64_t* min_out);
/* Remove every queued event with time < barrier; returns them in `runs`
 * (pinned host memory owned by d), grouped per host in event_compare order,
 * runs in host order: host h's run is [off[h], off[h + 1]) (off has N + 1
 * entries). */
int sgp_dev_extract(sgp_dev* d, uint64_t barrier, const sgp_rec** runs, const uint32_t** off,
                    uint64_t* total);
/* Per-kernel profile (include/shadowgpu.h sg_policy_kernel_profile). */
int sgp_dev_kprof(sgp_dev* d, int enable, uint32_t skip_rounds);
/* kernel classes: names[i] (static strings), launches, ms, algorithmic bytes */
int sgp_dev_kstats(sgp_dev* d, const char** names, uint64_t* launches, double* ms, double* bytes, uint32_t cap,
                   uint32_t* n_out);
/* Copy out every queued record (teardown). */
int sgp_dev_all(sgp_dev* d, sgp_rec* out, uint64_t capacity, uint64_t* n_out);

#ifdef __cplusplus
}
#endif
#endif
