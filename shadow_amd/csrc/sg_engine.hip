// sg_engine.hip — MI355X (gfx950) device engine of libshadowgpu.
//
// One conservative round of Shadow's host-family scheduler (contract:
// include/shadowgpu.h; design: DESIGN.md) on an HBM-resident calendar:
//
//   events      live in time buckets of width W (a ring of R buckets), each a
//               list of 1024-event chunks.  A round reads only the buckets its
//               window [S, E) covers, never a host's whole queue.
//   k_proc      one workgroup per host partition (HP consecutive slots): LDS
//               counting sort of the partition's due events by host, then the
//               flat pass, one lane per due event: its place in the host's
//               event_compare order (core/work/event.c:110-153), the host's
//               earlier draws replayed, trace digest term, PHOLD destination
//               draw (test_phold.c:160-178), reliability draw + ceil delay
//               (worker.c:243-304), srcHostEventID (event.c:38), endTime drop
//               (scheduler.c:343), barrier bump (host_single.c:180-184).  Hosts
//               the flat pass cannot take (boot events, same-round self events
//               host_single.c:237-267, lossy multi-event hosts, gossip) run
//               phase A, one lane per host, and phases B/C.  New events are
//               staged per partition, counted by bucket in LDS and reserved in
//               the calendar (one atomic per partition and bucket; chunk ids
//               from the partition's stash).
//   k_scatter   the staged events into their reserved slots (due ones routed
//               straight to their partition), the next window planned from the
//               MIN terms (host_single.c:273-305, master.c:450-480) by every
//               workgroup, the new window's due chunks gathered into the host
//               partitions, the minimum beyond the window, the stashes refilled.
//   multi-shard k_proc also writes the events for other shards into per-peer
//               outbox regions; the first xcap rows of each peer's outbox are the
//               exchange block itself, and the last k_proc workgroup to finish
//               writes the block headers (the shard's MIN terms).  After the
//               all-to-all, k_scatter plans from the G headers and routes the
//               received events due in the new window to their partitions; the
//               next k_proc stages the rest with its own new events
//               (stage_received).  On a drain step k_proc copies outbox
//               leftovers into the blocks and stages the received events.
//
// HBM layout: 16-B records everywhere.
//   bucket record     {dst_local << 40 | (t - b*W),  src << 40 | srcHostEventID}
//   partition record  {host_in_partition << 52 | (t - S), key}
//   staged record     {dst_local << 40 | (t - S), key}
// With the destination fixed, event_compare is the lexicographic order of
// (time, src << 40 | srcHostEventID).  Compiled with -ffp-contract=off: the
// only FP is the FP64 floor destination rule, which must round as the
// reference does.
#include <dlfcn.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "shadowgpu.h"

extern "C" void sg_set_error(const char* fmt, ...);

namespace {

constexpr int MAXG = 64;  // max shards
constexpr uint64_t SIMTIME_MAX = UINT64_MAX - 1;
constexpr int SRC_SHIFT = 40;
constexpr uint64_t SEQ_MASK = (1ULL << SRC_SHIFT) - 1;
constexpr uint64_t M40 = (1ULL << 40) - 1;
constexpr uint64_t M52 = (1ULL << 52) - 1;
constexpr uint64_t TOMB = ~0ULL;
constexpr uint32_t EMPTY = 0xFFFFFFFFu;
constexpr int CH_SHIFT = 10;
constexpr uint32_t CH = 1u << CH_SHIFT;  // events per chunk (16 KB)
constexpr uint32_t RMAX = 4096;          // ring buckets (LDS bucket bins)
// Bucket sub-lists: a reserving row appends to sub-list (row mod XS) of a
// bucket, so about P / XS rows contend per counter.  Round 2 measured XS = 1
// fastest (profiles/r02/knobs/xs_ab.log: 58.3 us/round against 61.0 at XS = 2,
// 63.2 at XS = 4).  Round 5, with the rest of the round 20 % shorter, the
// returning adds of 256 rows on one counter (~11 ns each at the memory side)
// were k_proc's reservation tail: XS = 2 takes k_proc 29.4 -> 27.7 us, and
// with the GSpec guess carrying both sub-lists k_scatter stays within 0.5 us
// (configs[3] 7.59 -> 7.87e9 events/s, profiles/r05/xs2).  XS = 4 gains
// nothing more in k_proc and has no guess.
#ifndef SG_XS
#define SG_XS 2
#endif
constexpr uint32_t XS = SG_XS;
// (Two counters per host partition for k_scatter's writers, by workgroup
// parity, were measured in round 5: correct, k_proc +0.6 us, k_scatter
// unchanged, profiles/r05/ph2; removed.)

constexpr uint32_t HPMAX = 4096;         // hosts per partition
constexpr uint32_t PMAX = 4096;          // partitions
constexpr uint32_t G3MAX = 512;          // k_scatter receive-role workgroups (received-block split)
constexpr uint32_t XCAP = 32;            // same-round self events in flight per lane
#ifndef SG_K3T
#define SG_K3T 512  // k_scatter's workgroup size
#endif
constexpr int K2_T = 1024, K3_T = SG_K3T;
constexpr uint32_t RETAINED = 1u << 31;
constexpr uint32_t ST = 16;           // chunk ids in a reserving row's stash
constexpr uint32_t NBMAX = 2046;      // buckets one window spans, at most (bucket width set to fit)
constexpr uint64_t HDR_REC = 1ull << 63;  // k_proc send list: a host's header record
                                          // {evc, HDR_REC | active index << 32 | host}
constexpr uint64_t PAD_REC = 1ull << 62;  // with HDR_REC: a skip record (a draw that selected no host)
// exchange block = HDR header rows + exchange_cap event rows, RW x int64 per
// row.  An event row is 16 B: {time - the sender's window start (40 bits) |
// destination's index in the receiving shard << 40, src << 40 |
// srcHostEventID}; the window start rides in the header (H_BASE), so the
// all-to-all moves two thirds of the bytes of {time, key, destination} rows.
constexpr int HDR = 4;
constexpr int RW = 2;
enum Hdr { H_N = 0, H_MORE, H_MIN, H_JMIN, H_OVF, H_ROUND, H_BASE };
// overflow flags
enum Ovf : uint64_t {
    OV_PROC = 1, OV_PART = 2, OV_POOL = 4, OV_XCHG = 8, OV_STEP = 16, OV_HORIZON = 32,
    OV_BUG = 128,  // internal inconsistency caught by a bounds guard
    // which gossip-skip guard tripped (with OV_BUG)
    GSK_A = 1ull << 20, GSK_B = 1ull << 21, GSK_C = 1ull << 22, GSK_D = 1ull << 23, GSK_E = 1ull << 24
};

enum Ctr {
    C_POPS = 0, C_BOOTS, C_SENDS, C_NULL, C_DROPREL, C_DROPEND, C_BUMPED, C_SAME,
    C_ACTIVE, C_EMIT,
    NPCTR,                  // counters k_proc accumulates; k_scatter's follow
    C_GATHER = NPCTR,       // events the gather role moved from the calendar into partitions
    C_RECV,                 // received events the receive role wrote into partitions (several shards)
    C_GSPEC,                // k_scatter launches whose gather took the GSpec guess
    C_GLIST,                // k_scatter launches whose gather derived the due list (the guess missed)
    NCTR
};

struct Rec {
    uint64_t a;
    uint64_t k;  // src << 40 | srcHostEventID
};
struct Slot {
    uint64_t t;
    uint64_t k;
};
// Streamed records (due-event copies, staged events, host state) use plain
// loads and stores: non-temporal ones (the next kernel re-reads the streamed
// records from HBM: 3.67e9 against 4.60e9 events/s, profiles/r02/knobs/nt.log;
// stores alone 66.8 against 52.5 us per round, profiles/r04/flatb) and
// write-through (sc1) stores (profiles/r04/wt: L2 merges the 16-B records into
// whole lines only when it writes them back) were measured slower and removed.
// SG_PMIN: each reserving row keeps its own minimum time offset per bucket
// (pmin, a plain load / min / store of its own row) instead of a 64-bit
// device-scope atomicMin on the bucket's minimum (bmin); the rmin role takes
// the first non-empty bucket beyond the window and the minimum of its column.
// In isolation (tools/resv_bench.hip, profiles/r05/resv) the atomicMin adds
// 3.4 us to 256 x 300 reservations, the row update 0.6 us.
#ifndef SG_PMIN
#define SG_PMIN 1
#endif
// SG_RS_LANES: k_scatter's planning thread reads the round state from wave
// 0's registers (one readlane per word) instead of from its LDS copy.
// SG_PLAN_TOUCH: k_scatter's planning thread fetches the plan's kernel
// arguments while the round state is in flight (1, default), or inside the
// plan (0)
#ifndef SG_PLAN_TOUCH
#define SG_PLAN_TOUCH 1
#endif
#ifndef SG_RS_LANES
#define SG_RS_LANES 1
#endif
__device__ __forceinline__ Rec ld_stream(const Rec* p) { return *p; }
__device__ __forceinline__ ulonglong2 ld_stream2(const ulonglong2* p) { return *p; }
// A streamed 16-B record store at a byte offset from a wave-uniform array start.
__device__ __forceinline__ void st_rec(void* base, uint64_t off, uint64_t a, uint64_t b) {
    *reinterpret_cast<ulonglong2*>(static_cast<char*>(base) + off) = make_ulonglong2(a, b);
}
struct DueEnt {
    uint32_t id;      // chunk
    uint32_t nflags;  // events in the chunk | RETAINED
    uint64_t base;    // bucket start time b*W
};
struct HostInfo {
    int32_t wt;       // PHOLD weight threshold (test_phold.c:160-178)
    uint32_t vertex;  // attachment vertex
    uint32_t slot;    // global slot: owner shard's first host + the host's place in its
                      // shard's vertex-sorted order
    uint32_t pad;
};
// Per local slot: the host's registration index (its id in event keys and
// traces) and its attachment vertex.  A shard's hosts occupy slots in
// (vertex, index) order, so a partition's hosts share a few vertices and their
// path rows fit in LDS.
struct SlotInfo {
    uint32_t h;
    uint32_t v;
};
struct PairRec {
    uint64_t delay;   // ceil(latency_ms * 1e6)   (worker.c:275-277)
    int32_t keep;     // max rand_r value kept     (worker.c:268-273)
    uint32_t jump;    // (uint64)latency_ms        (master.c:153)
};
// Path-record formats: the narrow ones cut the one random read per send to
// 8 or 4 bytes, so the V*V table stays in an XCD's L2.
enum PairFmt : uint32_t { PAIR_WIDE = 0, PAIR_NARROW = 1, PAIR_DELAY = 2 };

// A host's 32-B record: its state and, so that k_proc reads one record per
// host, its identity (registration index h, attachment vertex, both fixed).
struct HostState {
    uint32_t rng;     // host Random (host.c:176)
    uint32_t h;       // registration index (its id in event keys and traces)
    uint64_t pv;      // pops (low 48 bits) | vertex << 48
    uint64_t digest;
    uint64_t evc;     // eventIDCounter (host.c:397-400); k_proc writes it last (phase C)
};
constexpr uint64_t M48 = (1ULL << 48) - 1;
__device__ __forceinline__ uint64_t hs_w0(uint32_t rng, uint32_t h) { return rng | ((uint64_t)h << 32); }
__device__ __forceinline__ uint64_t hs_w1(uint64_t pops, uint32_t vh) { return pops | ((uint64_t)vh << 48); }
// A host's state while k_proc executes its events.
struct HostWork {
    uint32_t rng;
    uint64_t pops, digest, evc;
};

// Unsigned 32-bit division by a launch constant without a divide:
// Granlund-Montgomery multiply-high with host-made constants, exact for every
// n < 2^32 (the 64-bit divisions it replaces expand to ~70 VALU instructions).
struct Div32 {
    uint32_t m, s1, s2;
};
inline Div32 make_div32(uint64_t dv) {  // 1 <= dv < 2^32
    uint32_t l = 0;
    while ((1ull << l) < dv) ++l;
    return Div32{(uint32_t)(((1ull << 32) * ((1ull << l) - dv)) / dv + 1), l < 1 ? l : 1u, l > 1 ? l - 1 : 0u};
}
__device__ __forceinline__ uint32_t udiv32(const Div32& q, uint32_t n) {
    const uint32_t t = __umulhi(q.m, n);
    return (t + ((n - t) >> q.s1)) >> q.s2;
}

struct RoundState {
    uint64_t S, E, done, rounds;
    uint64_t min_jump, next_min_jump, jmin;
    uint64_t overflow;
    uint64_t trace_len;
    uint64_t ctr[NCTR];
    uint64_t last_min;
    // calendar
    uint64_t bS, bL;         // due bucket range of the current window (absolute indices)
    uint64_t pbS, pbL, pret; // the window before it (its consumed buckets are reset by the next
                             // k_proc) and its straddling bucket, or UINT64_MAX
    uint64_t listed;         // the current window was listed: its k_scatter gathered and routed for it
    uint64_t ret_b;          // retained (straddling) bucket, absolute, or UINT64_MAX
    uint64_t fold;           // k_scatter launches: the values below are current at [fold & 1]; a
                             // k_scatter reads [cur] and writes [cur ^ 1] (bw, rmin2, nfree2, xcarry2)
    uint64_t rmin2[2];       // min time in buckets beyond the window's bL
    uint64_t nfree2[2];      // due chunks the last gather returned to the free ring behind fl_tail
    uint64_t xcarry2[2];     // carry min: what stays in the straddling bucket after the gather and
                             // inserts (k_scatter's atomics)
    uint64_t splan;          // k_scatter workgroups that read the round state this launch: the
                             // last one publishes the next (SG step plan, k_scatter)
    uint64_t fl_head, fl_tail;
    uint64_t ins_local;      // k_proc staged events for k_scatter's insert role this step
    uint64_t ins_S;          // their window start (staged times are relative to it)
    // multi-shard step protocol
    uint64_t phase;      // 0: process step, 1: drain step (outbox leftovers only)
    uint64_t steps;      // exchange steps executed
    uint64_t peak_peer;  // largest per-peer outbox of a process step (since reset)
    uint64_t ticket;     // k_proc workgroups finished this launch (the last one writes the headers)
    uint64_t xacc[2];    // emitted min, discovery min of k_proc's workgroups (atomics)
    uint64_t recv_ok;    // a several-shard k_scatter read the receive buffer: the next k_proc stages it
    uint64_t tail_r, bS_r;  // fl_tail % NCH, bS % R, kept with them (the planner's 64-bit divisions)
};

// The gather's due list, guessed one kernel ahead.  In steady state a window
// is one whole bucket, the one after the window being executed (the barrier
// bump puts events at exactly its end, which becomes the next start), and the
// chunk ids of that bucket's slots written before the step are final when
// k_proc starts.  So one k_proc workgroup copies them here, and k_scatter's
// gather workgroups load their chunk ids beside the round state instead of
// after it (bucket words, a scan, the chunk table: two dependent round trips
// fewer), then check the guess against the window they planned.
constexpr uint32_t NSPEC = 1024;  // chunk ids kept (a million events)
struct GSpec {
    uint64_t fold;  // the step it is for (rs->fold while that k_proc ran); UINT64_MAX: none
    uint64_t b;     // the bucket (absolute, low 48 bits) | its ring row << 48
    uint32_t lo;    // its slots written before the step (bw[fold & 1]); XS = 2: sub-list 0's
    uint32_t nid;   // XS = 1: chunk ids below, ceil(lo / CH); XS = 2: sub-list 1's written slots
    uint32_t ids[NSPEC];  // XS = 2: sub-list 0's ceil(lo / CH) chunk ids, then sub-list 1's
};
static_assert(offsetof(GSpec, ids) == 24, "ids follow three words");
// The guess covers one or two sub-lists per bucket (XS > 2: no guess).
constexpr bool GSPEC_XS = XS <= 2;
struct GSpecLo {
    uint32_t lo0, lo1;  // written slots of sub-lists 0 and 1
    uint32_t nid0, nid; // chunk ids of sub-list 0, of both
};
__device__ __forceinline__ GSpecLo gspec_lo(uint64_t w2) {
    if constexpr (XS == 1) {
        return GSpecLo{(uint32_t)w2, 0u, (uint32_t)(w2 >> 32), (uint32_t)(w2 >> 32)};
    } else {
        const uint32_t lo0 = (uint32_t)w2, lo1 = (uint32_t)(w2 >> 32);
        const uint32_t nid0 = (lo0 + CH - 1) >> CH_SHIFT;
        return GSpecLo{lo0, lo1, nid0, nid0 + ((lo1 + CH - 1) >> CH_SHIFT)};
    }
}

struct Dev {
    uint32_t N, V, L, lo, load, dst_rule, window_rule, G, g;
    // gossip workload (SG_WORKLOAD_GOSSIP): keys carry the message id in their
    // low msg_shift bits (key = src << 40 | srcHostEventID << msg_shift | msg,
    // the same event_compare order since (src, srcHostEventID) is unique)
    uint32_t workload, msg_shift, gossip_msgs, mw;
    uint64_t gossip_start, gossip_interval;
    uint32_t* seen;           // [L][mw] per-host message bitsets
    uint32_t R, NCH, HP, P, CAPP, ECAP, G1, G3;
    Div32 hpdiv;              // a local slot's partition: slot / HP (HP need not be a power of two)
    uint32_t EVL, bin_off, ev_off, proc_lds;  // k_proc LDS: due events kept, bucket bins at,
                                              // events at, dynamic bytes
    uint64_t W;
    Div32 wdiv;                         // n / W for n < 2^32
    bool ring32;                        // R * W < 2^32: bucket offsets from the window's first bucket fit 32 bits
    uint64_t end_time, bootstrap_end, fixed_jump, runahead_min, trace_cap, xcap, xrows;
    uint32_t bounds[MAXG + 1];
    const HostInfo* hinfo;    // [N]
    const uint2* nearw;       // [N + 1] {weight threshold, vertex << slot_bits | global slot}, when dst_near
    uint32_t slot_bits;
    const SlotInfo* sinfo;    // [L] per local slot
    uint32_t lds_rows;        // k_proc stages its partition's path rows in LDS
    const void* prow;         // [V][V] full row-major records (4 or 8 B) the rows are staged from
    uint32_t rows_max, row_off;  // rows per partition at most; their LDS offset
    uint32_t row_pieces;         // 16-B pieces the LDS rows region holds (whole 1 KB wave pieces)
    bool snd_lds;                // k_proc's send records in LDS while they fit
    uint32_t light_max, light_q;  // inline bodies: hosts with <= light_max sends, lanes' first light_q hosts
    uint32_t rec_all;             // a partition with due events + active hosts <= rec_all records every host
    uint32_t flat;                // PHOLD with the due events in LDS: one lane per due event (k_proc flat pass)
    uint32_t grec;                // gossip: hosts record their forwards for phases B / C (SG_GREC, default 1)
    uint32_t gskip_on;            // gossip: their draws after phase A from the jump-ahead table (SG_GSKIP)
    uint32_t gflat;               // gossip: one lane per receipt records the forwards (SG_GFLAT, default 1)
    uint32_t dst_near;        // the uniform-position guess g is the drawn host or g + 1 for every x
                              // (host-checked): records g and g + 1 settle every draw
    uint32_t check;           // SG_CHECK=1: k_scatter's publisher re-derives the sent headers' MIN terms (debug)
    const PairRec* pairs;     // [V*V] full records (PAIR_WIDE), else null
    const uint2* pairs8;      // [V*V] {delay, keep} (PAIR_NARROW)
    const uint32_t* pdelay;   // [V*V] delay only (PAIR_DELAY: every pair keeps every packet)
    const uint32_t* pjump;    // [V*V] discovered ms (narrow formats), read only while it can matter
    uint32_t pair_fmt;        // PAIR_WIDE / PAIR_NARROW / PAIR_DELAY
    uint32_t tri;             // narrow tables hold the lower triangle only (symmetric paths)
    uint64_t gjmin;           // smallest discovered ms of any pair: jmin can fall no lower
    const uint64_t* vself;    // [V] self-path delay of each vertex (the pairs diagonal)
    uint64_t vself_min;       // their minimum: a window no longer than it has no same-round self event
    uint32_t* pcount;         // [V*V] path packet counters (topology.c:2053-2063), or null
    uint64_t* wtime;          // [3][P] barrier timers (scheduler.c:380-389), or null: busy ticks,
                              // idle ticks (waiting for the round's last partition), this round's end
    HostState* hs;            // [L]
    // calendar: bucket rb is XS sub-lists; a reserving row (k_proc partition p)
    // appends to sub-list p % XS
    Rec* pool;                // [NCH][CH]
    uint32_t* btab;           // [XS][R][NCH] chunk ids of each sub-list
    uint32_t* bk;             // [XS][R] slots reserved (k_proc atomics)
    uint32_t* bw;             // [2][XS][R] slots written before the step: k_scatter reads
                              // bw[fold & 1] and copies bk into the other half for the next step
    uint32_t* btomb;          // [R] tombstones
    uint64_t* bmin;           // [R] min live time (SG_PMIN=0)
    uint32_t* pmin;           // [P][R] SG_PMIN: each reserving row's min time offset in each bucket
                              // (UINT32_MAX: none); a bucket's minimum is its column's
    uint32_t* fring;          // [NCH] free chunk ring (head: rs->fl_head, taken atomically)
    uint32_t* stash;          // [P + G3][ST] chunk ids each reserving row keeps at hand
    uint32_t* stn;            // [P + G3] ids in the row's stash
    uint32_t* wbase;          // [P + G3][R] reserved base per (row, bucket) in the row's sub-list
    GSpec* gspec;             // the next gather's guessed due list (k_proc -> k_scatter)
    uint64_t* tick;           // [8] k_scatter's plan arrivals per workgroup shard blockIdx & 7 (SG_TICK8)
    uint32_t gspec_mode;      // SG_GSPEC: 1 guess (default), 0 never, 2 a wrong bucket (tests the check)
    // partitions
    uint32_t* pcnt;           // [P] due events of the partition this round
    Rec* part;                // [P][CAPP]
    Rec* part2;               // [P][CAPP] sorted by host
    Rec* extras;              // [P][K2_T][XCAP]
    uint32_t* rcnt;           // [P] staged local events
    Rec* loc;                 // [P][ECAP]
    Rec* sends;               // [P][ECAP] k_proc's per-send records (phases A-C)
    // per-workgroup partials
    uint64_t* p2min;          // [2][P] emitted min, discovery min
    uint64_t* pcum;           // [NCTR][P] cumulative counters
    // multi-shard
    uint32_t* remn;           // [P] staged events for other shards
    Slot* rem;                // [P][ECAP]
    uint32_t* rem_dst;        // [P][ECAP]
    int64_t* xsend;           // [G][xrows][RW] this step's exchange blocks (set by step_send)
    const int64_t* xrecv;     // [G][xrows_in][RW] the previous step's received blocks (k_proc stages
                              // what k_scatter did not route), or null
    uint64_t xrows_in, xcap_in;  // their layout (the exchange cap may have changed since)
    int64_t* outq;            // [G][oreg][RW] per-peer outbox regions (rows < xcap go
                              // straight into xsend on a process step)
    uint64_t oreg;            // rows per peer region (P * ECAP: every staged event fits)
    uint64_t* outn;           // [G]
    uint64_t* sent;           // [G]
    // debug
    uint64_t* stamps;         // [P][SG_STAMP_W] k_proc phase stamps + one spare row + one row
                              // per k_scatter workgroup (SG_STAMPS=1), else null
    sg_trace_rec* trace;
    uint64_t* wlog;           // [wlog_cap][2] executed windows {start, end}
    uint64_t wlog_cap;
    RoundState* rs;
    // sg_xlink: k_scatter's wave 0 waits for every sender's arrivals before it
    // reads the received headers (null: the blocks were in place at launch)
    const uint64_t* xwait;    // [G] arrival counters in this shard's exchange region
    uint64_t xwait_target;
    uint32_t* xwait_err;      // a wait that gave up (5 s) sets it, and OV_XCHG
    // sg_xlink, fused push: k_proc stores block q straight into shard q's
    // region (null: into xsend, for a copy or a collective after the kernel)
    // flat pass: an event's earlier events in its host consumed two draws
    // each unless one selected no host (rare; detected, that host replayed in
    // phase A), so the LCG is skipped ahead instead of replayed
    const uint2* skip;        // [nskip] {A, C}: the state after 2k draws is A * s + C (null: replay)
    uint32_t nskip;
    int64_t* const* xpeer;    // [G] each shard's region in this process
    uint64_t xoff;            // int64 offset of this shard's block of this step in every region
    uint32_t xfence;          // SG_XFENCE: the peer-region stores system-coherent (sc0 sc1, xst)
    uint32_t xskip;           // test only (sg_xlink_debug_withhold): peer + 1 whose arrival this step withholds
};

// The path record of vertex pair (sv, dv).  want_jump: the discovery minimum
// can still fall (rs->jmin > gjmin); otherwise the jump field is not read
// (UINT32_MAX: it could not lower the minimum anyway).  When every path equals
// its reverse (undirected topology, host-checked) the narrow tables keep the
// lower triangle only: half the bytes, so more of each table stays in an
// XCD's 4 MB L2 under the per-send random reads.
__device__ __forceinline__ size_t pair_index(const Dev& d, uint32_t sv, uint32_t dv) {
    if (!d.tri) return (size_t)sv * d.V + dv;
    const uint32_t lo = sv < dv ? sv : dv, hi = sv < dv ? dv : sv;
    return (size_t)hi * (hi + 1) / 2 + lo;
}
__device__ __forceinline__ PairRec load_pair(const Dev& d, uint32_t sv, uint32_t dv, bool want_jump) {
    if (d.pair_fmt == PAIR_WIDE) return d.pairs[(size_t)sv * d.V + dv];
    const size_t idx = pair_index(d, sv, dv);
    PairRec pr;
    if (d.pair_fmt == PAIR_NARROW) {
        const uint2 v = d.pairs8[idx];
        pr.delay = v.x;
        pr.keep = (int32_t)v.y;
    } else {
        pr.delay = d.pdelay[idx];
        pr.keep = SG_RAND_MAX;
    }
    pr.jump = want_jump ? d.pjump[idx] : UINT32_MAX;
    return pr;
}

__device__ __forceinline__ uint32_t wdiv(const Dev& d, uint32_t n) { return udiv32(d.wdiv, n); }
__device__ __forceinline__ uint32_t part_of(const Dev& d, uint32_t dl) { return udiv32(d.hpdiv, dl); }

__device__ __forceinline__ int32_t dev_rand_r(uint32_t& state) {
    // glibc rand_r, utility/random.c:32-37
    uint32_t next = state;
    uint32_t result;
    next = next * 1103515245u + 12345u;
    result = (next >> 16) % 2048u;
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (next >> 16) % 1024u;
    next = next * 1103515245u + 12345u;
    result <<= 10;
    result ^= (next >> 16) % 1024u;
    state = next;
    return (int32_t)result;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t z) {
    z ^= z >> 33;
    z *= 0xff51afd7ed558ccdULL;
    z ^= z >> 33;
    z *= 0xc4ceb9fe1a85ec53ULL;
    z ^= z >> 33;
    return z;
}

// Per-host trace digest term (order-sensitive through pos); same as the oracle.
__device__ __forceinline__ uint64_t digest_mix(uint64_t pos, uint64_t t, uint32_t src, uint64_t seq) {
    uint64_t z = fmix64(t ^ (pos * 0x9E3779B97F4A7C15ULL));
    return fmix64(z ^ (((uint64_t)src << 40) | seq));  // seq < 2^40 (SRC_SHIFT)
}

// Destination draw; returns the chosen host's global slot, or N when no host
// is selected (test_phold.c:176-177), and its vertex.  Weights rule: the first i with
// x <= wt[i] (non-decreasing thresholds); the uniform-position guess and its
// two neighbours are loaded together, which settles near-uniform weights in
// one round trip, and anything else is bisected.  Split in three steps
// (guess, probe loads, resolve) so a lane can have several draws' loads in
// flight at once.
struct Probe {
    HostInfo cur, prev, next;
};
__device__ __forceinline__ uint32_t dst_guess(const Dev& d, int32_t x) {
    const uint32_t N = d.N;
    if (d.dst_rule == SG_DST_UNIFORM_FLOOR) {
        double r = (double)x / 2147483647.0;
        double f = floor(r * (double)N);
        uint32_t dd = (uint32_t)f;
        return dd >= N ? N - 1 : dd;
    }
    uint32_t g = (uint32_t)(((uint64_t)(uint32_t)x * N) >> 31);
    return g >= N ? N - 1 : g;
}
__device__ __forceinline__ Probe dst_probe(const Dev& d, uint32_t g) {
    Probe pb;
    pb.cur = d.hinfo[g];
    if (d.dst_rule != SG_DST_UNIFORM_FLOOR) {
        pb.prev = d.hinfo[g > 0 ? g - 1 : 0];
        pb.next = d.hinfo[g + 1 < d.N ? g + 1 : d.N - 1];
    }
    return pb;
}
// Keeps a value in a register at this point: stops the compiler from merging
// per-branch values into a load through a selected address (which demotes
// the sources to scratch and the loads to flat).
template <class T>
__device__ __forceinline__ T opaque(T v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t dst_resolve(const Dev& d, int32_t x, uint32_t g, const Probe& pb,
                                                uint32_t& vert) {
    if (d.dst_rule == SG_DST_UNIFORM_FLOOR) {
        vert = pb.cur.vertex;
        return pb.cur.slot;
    }
    const uint32_t N = d.N;
    const HostInfo* w = d.hinfo;
    uint32_t lo, hi;
    if (x <= pb.cur.wt) {
        if (g == 0 || x > pb.prev.wt) {
            vert = opaque(pb.cur.vertex);
            return opaque(pb.cur.slot);
        }
        lo = 0;
        hi = g - 1;  // x <= wt[g-1]: the answer is in [0, g-1]
    } else {
        if (g + 1 < N && x <= pb.next.wt) {
            vert = opaque(pb.next.vertex);
            return opaque(pb.next.slot);
        }
        if (g + 1 >= N || x > w[N - 1].wt) return N;
        lo = g + 2;
        hi = N - 1;  // x > wt[g+1] and x <= wt[N-1]
    }
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (x <= w[mid].wt) hi = mid; else lo = mid + 1;
    }
    vert = opaque(w[lo].vertex);
    return opaque(w[lo].slot);
}
__device__ __forceinline__ uint32_t choose_dst(const Dev& d, int32_t x, HostInfo& info) {
    const uint32_t g = dst_guess(d, x);
    uint32_t v = 0;
    const uint32_t r = dst_resolve(d, x, g, dst_probe(d, g), v);
    info.vertex = v;
    return r;
}
// The shard that owns global slot h: shard g holds [floor(g*N/G), floor((g+1)*N/G)),
// so the owner is the largest g with floor(g*N/G) <= h, i.e. floor(((h+1)*G - 1)/N).
// (Arithmetic, not a search over d.bounds: a dynamic index into the by-value
// kernel argument would make the compiler copy all of Dev to scratch.)
__device__ __forceinline__ uint32_t owner_of(const Dev& d, uint32_t h) {
    return (uint32_t)((((uint64_t)h + 1) * d.G - 1) / d.N);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// DPP wave reductions (row_shr 1/2/4/8, row_bcast 15/31; gfx9 wave64): VALU
// only, no LDS traffic.  Every lane of the wave must be active; the result is
// wave-uniform.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    uint32_t w;
    w = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x111, 0xf, 0xf, false);
    v = w < v ? w : v;
    w = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x112, 0xf, 0xf, false);
    v = w < v ? w : v;
    w = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x114, 0xf, 0xf, false);
    v = w < v ? w : v;
    w = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x118, 0xf, 0xf, false);
    v = w < v ? w : v;
    w = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xa, 0xf, false);
    v = w < v ? w : v;
    w = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x143, 0xc, 0xf, false);
    v = w < v ? w : v;
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
    const uint32_t hi = wave_min_u32((uint32_t)(v >> 32));
    const uint32_t lo = wave_min_u32((uint32_t)(v >> 32) == hi ? (uint32_t)v : 0xFFFFFFFFu);
    return ((uint64_t)hi << 32) | lo;
}

// Workgroup-wide reductions through a [16] LDS scratch (blocks of <= 1024);
// every thread of the block must call them.  The wave partials come back one
// per lane and are combined across the wave (DPP / shuffles), so a thread
// issues one LDS read instead of sixteen.
__device__ __forceinline__ uint64_t block_min(uint64_t v, uint64_t* s16) {
    v = wave_min(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (lane == 0) s16[wid] = v;
    __syncthreads();
    return wave_min(lane < nw ? s16[lane] : UINT64_MAX);
}
__device__ __forceinline__ uint64_t block_sum(uint64_t v, uint64_t* s16) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (lane == 0) s16[wid] = v;
    __syncthreads();
    return wave_sum(lane < nw ? s16[lane] : (uint64_t)0);
}
// A workgroup barrier for LDS data only: it waits for this wave's LDS
// operations but not for its global stores and loads in flight, which a
// __syncthreads() (vmcnt(0) in its release fence) would drain.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// A workgroup's {min, sum, sum} for thread 0 alone, at the end of a role: wave
// reductions, then one barrier that waits for LDS only, so the workgroup's
// stores drain while the reduction and thread 0's atomics proceed (nothing in
// the kernel reads those stores back).
__device__ __forceinline__ void block_tail3(uint64_t& m, uint64_t& a, uint64_t& b) {
    __shared__ uint64_t s_r[3][16];
    m = wave_min(m);
    a = wave_sum(a);
    b = wave_sum(b);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if (lane == 0) {
        s_r[0][w] = m;
        s_r[1][w] = a;
        s_r[2][w] = b;
    }
    lds_barrier();
    if (threadIdx.x == 0)
        for (uint32_t k = 1; k < nw; ++k) {
            m = s_r[0][k] < m ? s_r[0][k] : m;
            a += s_r[1][k];
            b += s_r[2][k];
        }
}

// Inclusive scan of a u32 over the wave with DPP row shifts and broadcasts
// (no LDS round trips).
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}
// Exclusive scan across the workgroup of two packed u32 counts (hi << 32 | lo;
// neither total may overflow 32 bits); *total gets the sums.
template <bool LDS_ONLY = false>
__device__ __forceinline__ uint64_t block_excl_scan_2x32(uint64_t v, uint64_t* s16, uint64_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const uint32_t lo = wave_incl_scan_u32((uint32_t)v), hi = wave_incl_scan_u32((uint32_t)(v >> 32));
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    if (LDS_ONLY) lds_barrier(); else __syncthreads();  // s16 may still be read by a previous use
    if (lane == 63) s16[wid] = x;
    if (LDS_ONLY) lds_barrier(); else __syncthreads();
    // the wave totals one per lane, scanned across the wave: lane w holds the
    // sum of waves 0..w (each half stays within 32 bits by the contract)
    const uint64_t y = lane < nw ? s16[lane] : 0;
    const uint32_t ylo = wave_incl_scan_u32((uint32_t)y), yhi = wave_incl_scan_u32((uint32_t)(y >> 32));
    const int w0 = __builtin_amdgcn_readfirstlane(wid);
    uint64_t add = 0;
    if (w0 > 0)
        add = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)yhi, w0 - 1) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)ylo, w0 - 1);
    *total = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)yhi, nw - 1) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((int)ylo, nw - 1);
    return x - v + add;
}
// Exclusive scan of u32 counts whose workgroup total fits 32 bits.
template <bool LDS_ONLY = false>
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* s16, uint64_t* total) {
    return block_excl_scan_2x32<LDS_ONLY>((uint32_t)v, s16, total);
}

// Wave-aggregated LDS reservations: one atomic per wave instead of one per
// lane (same-address LDS atomics serialise across the workgroup's lanes).
// wave_reserve: n slots per lane, every lane of the wave must call it.
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* ctr, uint32_t n) {
    const int lane = threadIdx.x & 63;
    uint32_t x = n;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(x, o, 64);
        if (lane >= o) x += u;
    }
    uint32_t base = 0;
    if (lane == 63 && x) base = atomicAdd(ctr, x);
    base = __shfl(base, 63, 64);
    return base + x - n;
}
// wave_slot: one slot for each ACTIVE lane (divergent code allowed).
__device__ __forceinline__ uint32_t wave_slot(uint32_t* ctr) {
    const uint64_t m = __ballot(1);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    const uint32_t rank = (uint32_t)__builtin_popcountll(m & ((1ULL << lane) - 1));
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(ctr, (uint32_t)__builtin_popcountll(m));
    base = __shfl(base, (int)leader, 64);
    return base + rank;
}

// wave_slots: n in {0, 1, 2} consecutive slots for each ACTIVE lane, one
// atomic per wave (divergent code allowed).
__device__ __forceinline__ uint32_t wave_slots(uint32_t* ctr, uint32_t n) {
    const uint64_t m1 = __ballot(n >= 1), m2 = __ballot(n >= 2), act = __ballot(1);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lt = (1ULL << lane) - 1;
    const uint32_t rank = (uint32_t)(__builtin_popcountll(m1 & lt) + __builtin_popcountll(m2 & lt));
    const uint32_t total = (uint32_t)(__builtin_popcountll(m1) + __builtin_popcountll(m2));
    const uint32_t leader = (uint32_t)__builtin_ctzll(act);
    uint32_t base = 0;
    if (lane == leader && total) base = atomicAdd(ctr, total);
    base = __shfl(base, (int)leader, 64);
    return base + rank;
}

// event_compare with equal dst (event.c:122-148) on (time, src<<40|seq).
// Bitwise, not short-circuit, and the running minimum is updated through one
// select mask: ROCm 7.2 mis-compiled the branchy form inside a selection
// loop (the winning index was not updated on a time tie).
__device__ __forceinline__ bool key_less(uint64_t t, uint64_t k, uint64_t bt, uint64_t bk) {
    return (t < bt) | ((t == bt) & (k < bk));
}
struct Best {
    uint64_t t, k;
    uint32_t slot;
};
__device__ __forceinline__ void best_take(Best& b, uint64_t t, uint64_t k, uint32_t slot) {
    const bool take = key_less(t, k, b.t, b.k);
    b.t = take ? t : b.t;
    b.k = take ? k : b.k;
    b.slot = take ? slot : b.slot;
}

__device__ __forceinline__ void flag(const Dev& d, uint64_t f) {
    atomicOr((unsigned long long*)&d.rs->overflow, (unsigned long long)f);
}

// ----------------------------------------------------------------- boot ----
// worker_bootHosts: one self event per host at t=0 carrying id 0 (event.c:38),
// all in bucket 0 (chunks 0.. in order); the free ring holds the rest.
__global__ void k_boot(Dev d) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nb0 = (d.L + CH - 1) >> CH_SHIFT;
    if (i < d.L) {
        const uint32_t h = d.sinfo[i].h;  // slot i's host
        d.pool[i] = Rec{(uint64_t)i << 40, (uint64_t)h << SRC_SHIFT};
        HostState s = d.hs[i];
        s.evc = 1;
        s.pv &= ~M48;  // pops 0, the vertex stays
        s.digest = 0;
        d.hs[i] = s;
    }
    if (i < d.NCH) d.fring[i] = i;
    if (d.seen)
        for (size_t j = i; j < (size_t)d.L * d.mw; j += (size_t)gridDim.x * blockDim.x) d.seen[j] = 0;
    if (i < nb0) d.btab[i] = i;  // bucket 0 is ring slot 0, its sub-list 0
    for (uint32_t j = i; j < XS * d.R; j += gridDim.x * blockDim.x) {
        d.bk[j] = j == 0 ? d.L : 0u;
        d.bw[j] = d.bw[(size_t)XS * d.R + j] = j == 0 ? d.L : 0u;
    }
    if (i < d.R) {
        d.btomb[i] = 0;
        d.bmin[i] = i == 0 ? 0 : UINT64_MAX;
    }
    for (size_t j = i; j < (size_t)d.P * d.R; j += (size_t)gridDim.x * blockDim.x) d.pmin[j] = UINT32_MAX;
    if (i < d.P + d.G3) d.stn[i] = 0;  // k_scatter's refill role fills the stashes
    if (i < 8) d.tick[i] = 0;
    if (i < d.P) {
        d.pcnt[i] = 0;
        d.rcnt[i] = 0;
        if (d.remn) d.remn[i] = 0;
        for (int c = 0; c < NCTR; ++c) d.pcum[(size_t)c * d.P + i] = 0;
    }
    if (i == 0) {
        RoundState* rs = d.rs;
        rs->S = 0;  // slave.c:431
        rs->E = 1;
        rs->done = 0;
        rs->rounds = 0;
        rs->min_jump = 0;
        rs->next_min_jump = d.window_rule == SG_WINDOW_FIXED ? d.fixed_jump : 0;
        rs->jmin = UINT64_MAX;
        rs->overflow = 0;
        rs->trace_len = 0;
        for (int c = 0; c < NCTR; ++c) rs->ctr[c] = 0;
        rs->last_min = 0;
        // the first window [0, 1) (slave.c:431) is listed: bucket 0, straddling
        // E = 1 (the bucket width is at least 1 ms); the boot k_scatter gathers it
        rs->bS = rs->bL = 0;
        rs->pbS = rs->pbL = rs->pret = UINT64_MAX;
        rs->listed = 1;
        rs->ret_b = 1 < d.W ? 0 : UINT64_MAX;
        rs->fold = 0;
        rs->splan = 0;
        for (int q = 0; q < 2; ++q) {
            rs->rmin2[q] = SIMTIME_MAX;
            rs->nfree2[q] = 0;
            rs->xcarry2[q] = UINT64_MAX;
        }
        rs->fl_head = nb0;
        rs->fl_tail = d.NCH;
        rs->tail_r = 0;  // fl_tail % NCH
        rs->bS_r = 0;    // bS % R
        rs->ins_local = 0;
        rs->ins_S = 0;
        rs->phase = 0;
        rs->steps = 0;
        rs->peak_peer = 0;
        rs->ticket = 0;
        rs->xacc[0] = UINT64_MAX;
        rs->xacc[1] = UINT64_MAX;
        rs->recv_ok = 0;
    }
    if (i < d.G && d.outn) {
        d.outn[i] = 0;
        d.sent[i] = 0;
    }
}

// --------------------------------------------------------------- gather ----
// Due chunks → partition regions: two passes over the workgroup's chunks
// (LDS histogram + one reservation per partition, then the scatter).  The
// workgroup's due entries are staged in LDS so that every event load of a
// pass is independent of the others.
constexpr uint32_t GDMAX = 32;   // due entries staged per batch
constexpr int GUNR = 4;          // events in flight per thread (two-pass path)

template <bool SCATTER, int GT>
__device__ __forceinline__ void gather_pass(const Dev& d, const DueEnt* s_de, uint32_t nb,
                                            uint64_t S, uint64_t E, uint32_t* s_cnt, uint32_t* s_cur,
                                            uint64_t& cmin, uint64_t& ntomb, uint64_t& ng) {
    const uint32_t tot = nb * CH;
    for (uint32_t e0 = threadIdx.x; e0 < tot; e0 += GT * GUNR) {
        Rec r[GUNR];
        bool v[GUNR];
#pragma unroll
        for (int q = 0; q < GUNR; ++q) {
            const uint32_t e = e0 + q * GT;
            const DueEnt de = s_de[(e < tot ? e : 0) >> CH_SHIFT];
            v[q] = e < tot && de.id < d.NCH && (e & (CH - 1)) < (de.nflags & 0xFFFFu);
            r[q] = v[q] ? ld_stream(&d.pool[((size_t)de.id << CH_SHIFT) + (e & (CH - 1))]) : Rec{TOMB, 0};
        }
#pragma unroll
        for (int q = 0; q < GUNR; ++q) {
            if (!v[q] || r[q].a == TOMB) continue;
            const uint32_t e = e0 + q * GT;
            const DueEnt de = s_de[e >> CH_SHIFT];
            const uint64_t t = de.base + (r[q].a & M40);
            const uint32_t dl = (uint32_t)(r[q].a >> 40);
            if (dl >= d.L) {
                if (!SCATTER) flag(d, OV_BUG);
                continue;
            }
            if (t >= E) {
                if (!SCATTER) cmin = t < cmin ? t : cmin;
                continue;
            }
            const uint32_t p = part_of(d, dl);
            if (!SCATTER) {
                atomicAdd(&s_cnt[p], 1u);
                continue;
            }
            const uint32_t slot = s_cnt[p] + atomicAdd(&s_cur[p], 1u);
            ++ng;
            if (slot < d.CAPP)
                st_rec(d.part, ((size_t)p * d.CAPP + slot) * 16, ((uint64_t)(dl - p * d.HP) << 52) | (t - S), r[q].k);
            if (de.nflags & RETAINED) {
                d.pool[((size_t)de.id << CH_SHIFT) + (e & (CH - 1))].a = TOMB;
                ++ntomb;
            }
        }
    }
}

// The listed window's due chunks as one list of segments, derived by every
// gather workgroup from the bucket words (no listing pass): each fully due
// bucket's sub-lists (all their chunks; the slots written before this step
// hold its events), then the previous window's straddling bucket if the new
// window left it behind (spent: its chunks only go back to the ring), then
// the new window's straddling bucket (retained: the chunks holding written
// slots; its events at or after E stay).  The first nfree entries go back to
// the free ring.  Written slots come from bw[fold & 1]; this launch's inserts
// fill the slots reserved since (and route the due ones themselves).
// What one k_scatter launch works with (step_view): the window it routes and
// gathers for, computed by thread 0 of every workgroup from the round state
// the previous kernels left, before anything in the launch changes it.
struct Window {
    uint64_t S, E, done, min_jump, next_min_jump;
};
struct StepView {
    uint64_t S, E;           // the new window (or, drain step / boot, the current one)
    uint64_t bS, bL, ret;    // its buckets and straddling bucket
    uint64_t pbS, pbL, pret; // the window before it (consumed) and its straddling bucket
    uint64_t tail;           // the free ring's usable end with the plan applied
    uint64_t nfree0, carry0, rmin0;  // the current [cur] values (carried over on a drain step)
    uint64_t ins_S;          // staged local events' time base (k_proc's window start)
    uint64_t m, j, ovf;      // the MIN terms and overflow flags of the plan
    uint64_t fold, rounds0, S0, E0;
    Window w;
    uint32_t cur, listed, ins_local, round_done, more, done, quit;
    uint32_t tail_r, bSr;    // tail % NCH, bS % R (64-bit divisions done once, by the planner)
};
constexpr uint32_t SEGMAX = (NBMAX + 2) * XS;  // segments, at most
// Segment j is bucket sub-list x = j % XS of the list's k-th bucket, k = j / XS:
// k < nfull: bucket bS + k (taken whole); then the spent bucket, if any; then
// the straddling bucket bL (retained).  LDS keeps each segment's first list
// index and written slots.
struct DueList {
    uint64_t bS, bL, pret, W;
    uint32_t nfull, nseg, R;
    bool spent;
    __device__ __forceinline__ void seg(uint32_t j, uint64_t& b, uint32_t& x, uint32_t& flags, bool& events) const {
        const uint32_t k = j / XS;
        x = j % XS;
        b = bL;
        flags = RETAINED;
        events = true;
        if (k < nfull) {
            b = bS + k;
            flags = 0;
        } else if (spent && k == nfull) {
            b = pret;
            flags = 0;
            events = false;
        }
    }
};
template <int GT>
__device__ uint32_t due_segments(const Dev& d, const StepView& sv, DueList& dl, uint32_t* s_start, uint32_t* s_lo,
                                 uint64_t* s16, uint64_t* nfree_out) {
    dl.bS = sv.bS;
    dl.bL = sv.bL;
    dl.pret = sv.pret;
    dl.W = d.W;
    dl.R = d.R;
    const uint64_t ret = sv.ret;
    const uint32_t cur = sv.cur;
    dl.spent = dl.pret != UINT64_MAX && dl.pret < dl.bS;
    const uint32_t nb = (uint32_t)(dl.bL - dl.bS + 1);
    dl.nfull = nb - (ret != UINT64_MAX ? 1u : 0u);
    dl.nseg = (dl.nfull + (dl.spent ? 1u : 0u) + (ret != UINT64_MAX ? 1u : 0u)) * XS;
    const uint32_t per = (dl.nseg + GT - 1) / GT, j0 = threadIdx.x * per;
    const uint32_t j1 = j0 + per < dl.nseg ? j0 + per : dl.nseg;
    uint32_t nc = 0, ncf = 0;
    for (uint32_t j = j0; j < j1; ++j) {
        uint64_t b;
        uint32_t x, flags;
        bool events;
        dl.seg(j, b, x, flags, events);
        const uint32_t row = x * dl.R + (uint32_t)(b % dl.R);
        const uint32_t hi = d.bk[row], lo = events ? d.bw[(size_t)cur * XS * dl.R + row] : 0u;
        const uint32_t n = ((flags ? lo : hi) + CH - 1) >> CH_SHIFT;
        s_lo[j] = lo;
        s_start[j] = n;  // the count for now
        nc += n;
        ncf += flags ? 0u : n;
    }
    uint64_t tot;
    uint64_t off = block_excl_scan_2x32(((uint64_t)ncf << 32) | nc, s16, &tot);  // barriers inside
    uint32_t o = (uint32_t)off;
    for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t n = s_start[j];
        s_start[j] = o;
        o += n;
    }
    __syncthreads();
    *nfree_out = tot >> 32;
    return (uint32_t)tot;
}
// List entry i: its chunk id (from the table), events, flags and bucket base.
__device__ __forceinline__ DueEnt due_entry(const Dev& d, const DueList& dl, const uint32_t* s_start,
                                            const uint32_t* s_lo, uint32_t i) {
    uint32_t lo = 0, hi = dl.nseg - 1;  // the last segment starting at or before i
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_start[mid] <= i) lo = mid; else hi = mid - 1;
    }
    uint64_t b;
    uint32_t x, flags;
    bool events;
    dl.seg(lo, b, x, flags, events);
    const uint32_t ci = i - s_start[lo], w = s_lo[lo];
    const uint32_t left = w > (ci << CH_SHIFT) ? w - (ci << CH_SHIFT) : 0u;
    const size_t row = (size_t)x * dl.R + (uint32_t)(b % dl.R);
    return DueEnt{d.btab[row * d.NCH + ci], (left < CH ? left : CH) | flags, b * dl.W};
}

// Gather role of k_scatter's workgroups [g0, g0 + nw): the due chunks of the
// new window [S, E) into the host partitions.  GR events per thread in
// registers on the one-pass path (4 chunks per workgroup).  The counts cover
// only the slots written before this launch ("old" slots); the same launch's
// insert workgroups route the new due events themselves, so the two never
// touch the same slot.
constexpr size_t GDE_OFF = (2 * PMAX) * 4;  // s_de's offset in the gather role's LDS
constexpr size_t GATHER_LDS = GDE_OFF + GDMAX * sizeof(DueEnt) + 16 * 8 + 2 * SEGMAX * 4;
constexpr uint32_t GSPEC_N = 4;  // chunks per gather workgroup on the GSpec path (the one-pass capacity)
// Gather workgroup w of nw, its wave 1 at launch (beside the round state): the
// GSpec header words into s_gsw and the workgroup's entries w + k * nw (k <
// GSPEC_N) of the guessed due list into s_de, one load per lane.
__device__ __forceinline__ void gspec_load(const Dev& d, uint32_t w, uint32_t nw, uint64_t* s_gsw, DueEnt* s_de) {
    const uint32_t k = threadIdx.x & 63;
    const uint32_t i = w + (k >= 3 ? k - 3 : 0) * nw, ic = i < NSPEC ? i : 0u;
    const uint32_t wi = k < 3 ? k : (k < 3 + GSPEC_N ? 3 + (ic >> 1) : 0u);
    const uint64_t v = reinterpret_cast<const uint64_t*>(d.gspec)[wi];
    const uint64_t b = __shfl(v, 1, 64), ln = __shfl(v, 2, 64);
    if (k < 3) {
        s_gsw[k] = v;
    } else if (k < 3 + GSPEC_N) {
        const GSpecLo gl = gspec_lo(ln);
        const bool ok = i < gl.nid && i < NSPEC;
        // entry i: sub-list 0's chunk i, or (XS = 2) sub-list 1's chunk i - nid0
        const uint32_t left = !ok ? 0u : i < gl.nid0 ? gl.lo0 - i * CH : gl.lo1 - (i - gl.nid0) * CH;
        s_de[k - 3] = DueEnt{ok ? (uint32_t)(v >> ((ic & 1) * 32)) : EMPTY, left < CH ? left : CH,
                             (b & ((1ull << 48) - 1)) * d.W};
    }
}
// The guessed list when the plan confirms it, else the list path.
template <int GT>
__device__ void gather_role(const Dev& d, const StepView& sv, uint32_t w, uint32_t nw, unsigned char* lds,
                            const uint64_t* s_gsw, uint64_t* st) {
    constexpr int GR = 4 * (int)CH / GT;
    static_assert(GR * GT == (int)(GSPEC_N * CH), "the one-pass path holds GSPEC_N chunks");
    uint32_t* s_cnt = (uint32_t*)lds;                      // [PMAX]
    uint32_t* s_cur = s_cnt + PMAX;                        // [PMAX]
    DueEnt* s_de = (DueEnt*)(lds + GDE_OFF);               // [GDMAX]
    uint64_t* s16 = (uint64_t*)(s_de + GDMAX);             // [16]
    uint32_t* s_start = (uint32_t*)(s16 + 16);             // [SEGMAX] the due list's segments
    uint32_t* s_lo = s_start + SEGMAX;                     // [SEGMAX]
    const uint64_t S = sv.S, E = sv.E;
    const uint32_t P = d.P;
    // The window's chunks outside the retained bucket go back to the free ring
    // behind the tail as the entries are staged below (the next step's plan
    // advances the tail; nothing allocates before it).
    const uint32_t tail_r = sv.tail_r;
    uint32_t* pc = d.pcnt;
    for (uint32_t p = threadIdx.x; p < P; p += GT) {
        s_cnt[p] = 0;
        s_cur[p] = 0;
    }
    uint64_t cmin = UINT64_MAX, ntomb = 0, ng = 0;  // ng: events moved (C_GATHER)
    auto reserve = [&]() {  // one reservation per partition this workgroup feeds
        for (uint32_t p = threadIdx.x; p < P; p += GT) {
            const uint32_t c = s_cnt[p];
            if (c) {
                const uint32_t base = atomicAdd(&pc[p], c);
                if (base + c > d.CAPP) flag(d, OV_PART);
                s_cnt[p] = base;
            }
        }
    };
    // The workgroup's chunks s_de[0, nb) (nb <= GSPEC_N, visible to every
    // thread) in registers: load once, count, reserve, scatter.  mid() runs
    // between the count and the reservations.
    auto one_pass = [&](uint32_t nb, auto&& mid) __attribute__((always_inline)) {
        const uint32_t tot = nb * CH;
        Rec r[GR];
        uint32_t pp[GR];  // partition of the event, UINT32_MAX: not gathered
#pragma unroll
        for (int q = 0; q < GR; ++q) {  // every load unconditional (clamped address)
            const uint32_t e = threadIdx.x + q * GT;
            const DueEnt de = s_de[(e < tot ? e : 0) >> CH_SHIFT];
            const bool v = e < tot && de.id < d.NCH && (e & (CH - 1)) < (de.nflags & 0xFFFFu);
            r[q] = ld_stream(&d.pool[v ? ((size_t)de.id << CH_SHIFT) + (e & (CH - 1)) : 0]);
            if (!v) r[q].a = TOMB;
        }
        lds_barrier();  // s_cnt / s_cur zeroed
#pragma unroll
        for (int q = 0; q < GR; ++q) {
            pp[q] = UINT32_MAX;
            if (r[q].a == TOMB) continue;
            const uint32_t e = threadIdx.x + q * GT;
            const uint64_t t = s_de[e >> CH_SHIFT].base + (r[q].a & M40);
            const uint32_t dl = (uint32_t)(r[q].a >> 40);
            if (dl >= d.L) {
                flag(d, OV_BUG);
                continue;
            }
            if (t >= E) {
                cmin = t < cmin ? t : cmin;
                continue;
            }
            pp[q] = part_of(d, dl);
            r[q].a = ((uint64_t)(dl - pp[q] * d.HP) << 52) | (t - S);  // the partition record
            atomicAdd(&s_cnt[pp[q]], 1u);
        }
        lds_barrier();
        if (st) st[2] = __builtin_amdgcn_s_memrealtime();
        mid();
        reserve();
        lds_barrier();
        if (st) st[6] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int q = 0; q < GR; ++q) {
            if (pp[q] == UINT32_MAX) continue;
            const uint32_t p = pp[q];
            const uint32_t slot = s_cnt[p] + atomicAdd(&s_cur[p], 1u);
            ++ng;
            if (slot < d.CAPP) st_rec(d.part, ((size_t)p * d.CAPP + slot) * 16, r[q].a, r[q].k);
            const uint32_t e = threadIdx.x + q * GT;
            const DueEnt de = s_de[e >> CH_SHIFT];
            if (de.nflags & RETAINED) {
                d.pool[((size_t)de.id << CH_SHIFT) + (e & (CH - 1))].a = TOMB;
                ++ntomb;
            }
        }
    };
    // The GSpec path: the window is the one whole bucket the k_proc before
    // guessed, and s_de holds this workgroup's entries w + k * nw of its
    // written chunks already.  Every chunk of the bucket (the slots reserved
    // since included: their due events were routed by the insert role) goes
    // back to the ring, entry i at tail + i, as the list path would put it.
    const uint64_t gb = s_gsw[1] & ((1ull << 48) - 1);
    const GSpecLo gl = gspec_lo(s_gsw[2]);
    const uint32_t gnid = gl.nid;
    const bool spent = sv.pret != UINT64_MAX && sv.pret < sv.bS;
    if (GSPEC_XS && s_gsw[0] == sv.fold && sv.bS == gb && sv.bL == gb &&
        sv.ret == UINT64_MAX && !spent && gnid <= GSPEC_N * nw) {  // uniform
        const uint32_t row = (uint32_t)(s_gsw[1] >> 48);
        // in flight under the pool loads: the sub-lists' reserved slots
        const uint32_t hi = d.bk[row], hi1 = XS == 2 ? d.bk[d.R + row] : 0u;
        if (st) st[1] = __builtin_amdgcn_s_memrealtime();
        one_pass(GSPEC_N, [&]() __attribute__((always_inline)) {
            // ring order as the list path's: sub-list 0's chunks, then sub-list 1's
            const uint32_t nd0 = (hi + CH - 1) >> CH_SHIFT, nd = nd0 + ((hi1 + CH - 1) >> CH_SHIFT);
            if (w == 0 && threadIdx.x == 0) {
                d.rs->nfree2[sv.cur ^ 1] = nd;
                atomicAdd((unsigned long long*)&d.pcum[(size_t)C_GSPEC * d.P], 1ull);
            }
            if (st) {
                st[5] = nd;
                st[7] = 1;
            }
            for (uint32_t i = w + threadIdx.x * nw; i < nd; i += GT * nw) {
                // entry i of the guess is sub-list 0's chunk i while i < nid0
                // (s_de[k] holds entry w + k * nw); the rest from the chunk table
                const bool x1 = XS == 2 && i >= nd0;
                const uint32_t id = threadIdx.x < GSPEC_N && i < gl.nid0
                                        ? s_de[threadIdx.x].id
                                        : d.btab[((size_t)(x1 ? d.R : 0u) + row) * d.NCH + (x1 ? i - nd0 : i)];
                // as the list path's free_chunk: an id past the pool (a slot
                // whose reservation found the pool exhausted, OV_POOL) never
                // enters the ring
                if (id >= d.NCH) continue;
                const uint32_t pos = tail_r + i;  // i < NCH: one wrap at most
                d.fring[pos >= d.NCH ? pos - d.NCH : pos] = id;
            }
        });
    } else {
    DueList dl;
    uint64_t nfree;
    const uint64_t nd = due_segments<GT>(d, sv, dl, s_start, s_lo, s16, &nfree);
    if (w == 0 && threadIdx.x == 0) {
        d.rs->nfree2[sv.cur ^ 1] = nfree;
        atomicAdd((unsigned long long*)&d.pcum[(size_t)C_GLIST * d.P], 1ull);
    }
    if (st) {  // the list's shape (SG_STAMPS)
        st[5] = nd;
        st[7] = dl.nseg;
        st[8] = nfree;
        st[9] = sv.bS;
        st[10] = sv.bL;
        st[11] = sv.ret;
        st[12] = sv.pret;
        st[13] = sv.S;
        st[14] = sv.E;
    }
    const uint64_t c0 = nd * w / nw, c1 = nd * (w + 1) / nw;
    auto free_chunk = [&](const DueEnt& de, uint64_t i) {
        if (i >= nfree || (de.nflags & RETAINED) || de.id >= d.NCH) return;  // not in the prefix
        const uint64_t pos = tail_r + i;  // i < NCH: one wrap at most
        d.fring[pos >= d.NCH ? pos - d.NCH : pos] = de.id;
    };
    if ((c1 - c0) * CH <= (uint64_t)GR * GT) {
        // the workgroup's chunks fit in registers: load once, count, reserve, scatter
        const uint32_t nb = (uint32_t)(c1 - c0);
        if (threadIdx.x < nb) {
            const DueEnt de = due_entry(d, dl, s_start, s_lo, (uint32_t)(c0 + threadIdx.x));
            s_de[threadIdx.x] = de;
            free_chunk(de, c0 + threadIdx.x);
        }
        lds_barrier();
        if (st) st[1] = __builtin_amdgcn_s_memrealtime();
        one_pass(nb, []() {});
    } else {
        // more chunks than registers hold (the boot round): two passes over them
        for (uint64_t cb = c0; cb < c1; cb += GDMAX) {
            const uint32_t nb = (uint32_t)(c1 - cb < GDMAX ? c1 - cb : GDMAX);
            __syncthreads();
            if (threadIdx.x < nb) s_de[threadIdx.x] = due_entry(d, dl, s_start, s_lo, (uint32_t)(cb + threadIdx.x));
            __syncthreads();
            gather_pass<false, GT>(d, s_de, nb, S, E, s_cnt, s_cur, cmin, ntomb, ng);
        }
        __syncthreads();
        reserve();
        for (uint64_t cb = c0; cb < c1; cb += GDMAX) {
            const uint32_t nb = (uint32_t)(c1 - cb < GDMAX ? c1 - cb : GDMAX);
            __syncthreads();
            if (threadIdx.x < nb) {
                const DueEnt de = due_entry(d, dl, s_start, s_lo, (uint32_t)(cb + threadIdx.x));
                s_de[threadIdx.x] = de;
                free_chunk(de, cb + threadIdx.x);
            }
            __syncthreads();
            gather_pass<true, GT>(d, s_de, nb, S, E, s_cnt, s_cur, cmin, ntomb, ng);
        }
    }
    }  // the list path
    uint64_t m = cmin, nt = ntomb, gn = ng;
    block_tail3(m, nt, gn);
    if (threadIdx.x == 0) {
        if (gn) atomicAdd((unsigned long long*)&d.pcum[(size_t)C_GATHER * d.P + w % d.P], (unsigned long long)gn);
        if (m != UINT64_MAX) atomicMin((unsigned long long*)&d.rs->xcarry2[sv.cur ^ 1], (unsigned long long)m);
        if (sv.ret != UINT64_MAX) {
            const uint32_t rb = (uint32_t)(sv.ret % d.R);
            if (nt) atomicAdd(&d.btomb[rb], (uint32_t)nt);
            if (m != UINT64_MAX) atomicMin((unsigned long long*)&d.bmin[rb], (unsigned long long)m);
        }
    }
}

// ----------------------------------------------------------------- proc ----
struct Acc {
    uint32_t ctr[NPCTR];
    uint64_t jmin;   // min truncated latency of attempted sends
    uint64_t emin;   // min time of staged (emitted) events
    bool overflow;
};

struct HostCtx {
    uint32_t h, vh;   // registration index, vertex
    uint32_t sg;      // global slot (destinations are slots)
    HostWork s;
};
__device__ __forceinline__ void host_load(HostCtx& c, ulonglong2 w01, ulonglong2 w23) {
    c.s.rng = (uint32_t)w01.x;
    c.h = (uint32_t)(w01.x >> 32);
    c.s.pops = w01.y & M48;
    c.vh = (uint32_t)(w01.y >> 48);
    c.s.digest = w23.x;
    c.s.evc = w23.y;
}

struct ProcShared {
    uint32_t nloc, nrem;
    uint32_t peer[MAXG];
};

// Stage one event for another shard's host (the outbox, several shards only).
__device__ __forceinline__ void stage_remote(const Dev& d, uint32_t part, ProcShared& sh, Acc& a, uint32_t dst,
                                             uint64_t tn, uint64_t key) {
    const uint32_t slot = wave_slot(&sh.nrem);
    if (slot < d.ECAP) {
        const size_t so = (size_t)part * d.ECAP + slot;
        d.rem[so] = Slot{tn, key};
        d.rem_dst[so] = dst;
        atomicAdd(&sh.peer[owner_of(d, dst)], 1u);
    } else {
        a.overflow = true;
    }
}

// Stage one new event (time already bumped) for the calendar (this shard's
// hosts; k_proc counts them by bucket after phase C) or for the outbox (other
// shards).
__device__ __forceinline__ bool stage_event(const Dev& d, uint64_t S, uint32_t part, ProcShared& sh,
                                            Acc& a, uint32_t dst, uint64_t tn, uint64_t key) {
    const uint32_t dl = dst - d.lo;
    a.emin = tn < a.emin ? tn : a.emin;
    ++a.ctr[C_EMIT];
    if (dl < d.L) {
        const uint32_t slot = wave_slot(&sh.nloc);
        if (slot < d.ECAP) st_rec(d.loc, ((size_t)part * d.ECAP + slot) * 16, ((uint64_t)dl << 40) | (tn - S), key);
        else a.overflow = true;
        return true;
    }
    stage_remote(d, part, sh, a, dst, tn, key);
    return false;
}

// Execute one popped event (worker.c:165-176 + the PHOLD body + worker_sendPacket).
// Self events that fall inside the window go to the lane's same-round list
// through `append`; everything else is staged.
template <class Append, class Count>
__device__ __forceinline__ void execute_event(const Dev& d, uint64_t S, uint64_t E, uint32_t part,
                                              HostCtx& c, Acc& a, uint64_t bt, uint64_t bk,
                                              ProcShared& sh, Append append, Count count) {
    const uint32_t bsrc = (uint32_t)(bk >> SRC_SHIFT);
    const uint64_t bseq = (bk & SEQ_MASK) >> d.msg_shift;
    const uint32_t msg = (uint32_t)(bk & ((1ULL << d.msg_shift) - 1));
    c.s.digest += digest_mix(c.s.pops, bt, bsrc, bseq);
    if (d.trace) {
        const uint64_t ts = atomicAdd((unsigned long long*)&d.rs->trace_len, 1ULL);
        if (ts < d.trace_cap) {
            sg_trace_rec r;
            r.time = bt;
            r.seq = bseq;
            r.host = c.h;
            r.src = bsrc;
            r.pos = c.s.pops;
            d.trace[ts] = r;
        } else {
            a.overflow = true;
        }
    }
    ++c.s.pops;
    ++a.ctr[C_POPS];
    const bool boot = (bsrc == c.h && bseq == 0);
    a.ctr[C_BOOTS] += boot;
    uint32_t nsend = boot ? d.load : 1u;  // test_phold.c:234-239 / 310-312
    if (d.workload == SG_WORKLOAD_GOSSIP) {
        // configs[4] body (oracle/orc.c execute_gossip): the boot event schedules
        // the host's origin self event (worker_scheduleTask, worker.c:218-234); a
        // message's first receipt forwards it to `load` peers, later ones are
        // dropped by the seen set
        nsend = 0;
        const uint32_t lh = c.sg - d.lo;
        if (boot) {
            const uint64_t N = d.N, M = d.gossip_msgs;
            const uint64_t m = ((uint64_t)c.h * M + N - 1) / N;
            if (m < M && (m * N) / M == c.h) {
                const uint64_t tn = d.gossip_start + m * d.gossip_interval;
                const uint64_t sq = c.s.evc++;
                if (sq >> (SRC_SHIFT - d.msg_shift)) a.overflow = true;
                const uint64_t key = ((uint64_t)c.h << SRC_SHIFT) | (sq << d.msg_shift) | m;
                if (tn >= d.end_time) {
                    ++a.ctr[C_DROPEND];
                } else if (tn < E) {
                    ++a.ctr[C_SAME];
                    if (!append(tn - S, key)) a.overflow = true;
                } else if (stage_event(d, S, part, sh, a, c.sg, tn, key)) {
                    count(tn);
                }
            }
        } else {
            uint32_t* w = d.seen + (size_t)lh * d.mw + (msg >> 5);
            const uint32_t bit = 1u << (msg & 31), wv = *w;
            if (!(wv & bit)) {
                *w = wv | bit;
                nsend = d.load;
            }
        }
    }
    for (uint32_t m = 0; m < nsend; ++m) {
        const int32_t x = dev_rand_r(c.s.rng);
        HostInfo di;
        const uint32_t dst = choose_dst(d, x, di);
        if (dst >= d.N) {
            ++a.ctr[C_NULL];
            continue;
        }
        ++a.ctr[C_SENDS];
        const PairRec pr = load_pair(d, c.vh, di.vertex, d.rs->jmin > d.gjmin);
        a.jmin = pr.jump < a.jmin ? pr.jump : a.jmin;  // path discovery (topology.c:1374-1385)
        const int32_t ch = dev_rand_r(c.s.rng);          // worker.c:268-269
        if (!(bt < d.bootstrap_end || ch <= pr.keep)) {
            ++a.ctr[C_DROPREL];
            continue;
        }
        if (d.pcount) atomicAdd(&d.pcount[(size_t)c.vh * d.V + di.vertex], 1u);  // worker.c:279
        uint64_t tn = bt + pr.delay;        // worker.c:275-277
        const uint64_t sq = c.s.evc++;      // event.c:38
        if (sq >> (SRC_SHIFT - d.msg_shift)) a.overflow = true;
        if (tn >= d.end_time) {             // scheduler.c:343-346
            ++a.ctr[C_DROPEND];
            continue;
        }
        const uint64_t key = ((uint64_t)c.h << SRC_SHIFT) | (sq << d.msg_shift) | msg;
        if (dst == c.sg && tn < E) {
            ++a.ctr[C_SAME];
            if (!append(tn - S, key)) a.overflow = true;
            continue;
        }
        if (dst != c.sg && tn < E) {  // host_single.c:180-184
            tn = E;
            ++a.ctr[C_BUMPED];
        }
        if (stage_event(d, S, part, sh, a, dst, tn, key)) count(tn);
    }
}

// A resolved send of a host whose sends cannot land in this window at the host
// itself: reliability test (worker.c:268-273), delivery time (worker.c:275-277),
// srcHostEventID (event.c:38), endTime drop (scheduler.c:343-346), barrier
// bump (host_single.c:180-184). False when the send is dropped.
__device__ __forceinline__ bool send_tests(const Dev& d, uint64_t E, HostCtx& c, Acc& a, uint64_t bt, int32_t ch,
                                           uint32_t dst, uint32_t vd, const PairRec& pr, uint64_t& tn, uint64_t& key) {
    a.jmin = pr.jump < a.jmin ? pr.jump : a.jmin;  // path discovery (topology.c:1374-1385)
    if (!(bt < d.bootstrap_end || ch <= pr.keep)) {  // worker.c:268-273
        ++a.ctr[C_DROPREL];
        return false;
    }
    if (d.pcount) atomicAdd(&d.pcount[(size_t)c.vh * d.V + vd], 1u);  // worker.c:279
    tn = bt + pr.delay;                 // worker.c:275-277
    const uint64_t sq = c.s.evc++;      // event.c:38
    if (tn >= d.end_time) {             // scheduler.c:343-346
        ++a.ctr[C_DROPEND];
        return false;
    }
    if (dst == c.sg && tn < E) a.overflow = true;  // excluded by the caller's self-path test
    if (dst != c.sg && tn < E) {        // host_single.c:180-184
        tn = E;
        ++a.ctr[C_BUMPED];
    }
    key = ((uint64_t)c.h << SRC_SHIFT) | sq;
    return true;
}
// The light path's two resolved sends (the first nsd are real): the tests for
// each, then one staging reservation per wave for both local events.
template <class Count>
__device__ __forceinline__ void commit_two(const Dev& d, uint64_t S, uint64_t E, uint32_t part, HostCtx& c, Acc& a,
                                           ProcShared& sh, uint32_t nsd, uint64_t bt0, int32_t ch0, uint32_t dst0,
                                           uint32_t vd0, const PairRec& pr0, uint64_t bt1, int32_t ch1,
                                           uint32_t dst1, uint32_t vd1, const PairRec& pr1, Count count) {
    uint64_t tn0 = 0, tn1 = 0, k0 = 0, k1 = 0;
    const bool g0 = nsd > 0 && send_tests(d, E, c, a, bt0, ch0, dst0, vd0, pr0, tn0, k0);
    const bool g1 = nsd > 1 && send_tests(d, E, c, a, bt1, ch1, dst1, vd1, pr1, tn1, k1);
    const uint32_t dl0 = dst0 - d.lo, dl1 = dst1 - d.lo;
    const bool l0 = g0 && dl0 < d.L, l1 = g1 && dl1 < d.L;
    const uint32_t base = wave_slots(&sh.nloc, (uint32_t)l0 + (uint32_t)l1);
    Rec* loc = d.loc + (size_t)part * d.ECAP;
    if (l0) {
        if (base < d.ECAP) st_rec(d.loc, ((size_t)part * d.ECAP + base) * 16, ((uint64_t)dl0 << 40) | (tn0 - S), k0);
        else a.overflow = true;
        count(tn0);
    }
    if (l1) {
        const uint32_t sl = base + (l0 ? 1u : 0u);
        if (sl < d.ECAP) st_rec(d.loc, ((size_t)part * d.ECAP + sl) * 16, ((uint64_t)dl1 << 40) | (tn1 - S), k1);
        else a.overflow = true;
        count(tn1);
    }
    if (g0) {
        a.emin = tn0 < a.emin ? tn0 : a.emin;
        ++a.ctr[C_EMIT];
    }
    if (g1) {
        a.emin = tn1 < a.emin ? tn1 : a.emin;
        ++a.ctr[C_EMIT];
    }
    if (g0 && !l0) stage_remote(d, part, sh, a, dst0, tn0, k0);
    if (g1 && !l1) stage_remote(d, part, sh, a, dst1, tn1, k1);
}

// Pop a host's sorted segment (worker.c:165-176): trace digest, counters and
// the PHOLD body's draws (test_phold.c:160-178, worker.c:268-269); every send
// with a destination goes to on_send(x, chance, time offset).
template <class OnSend>
__device__ __forceinline__ void pop_segment(const Dev& d, RoundState* rs, uint64_t S, HostCtx& c, Acc& a,
                                            const Rec* seg, uint32_t cnt, int32_t last, OnSend on_send) {
    for (uint32_t i = 0; i < cnt; ++i) {
        const Rec ev = seg[i];
        const uint64_t trel = ev.a & M52, bt = S + trel;
        const uint32_t bsrc = (uint32_t)(ev.k >> SRC_SHIFT);
        const uint64_t bseq = ev.k & SEQ_MASK;
        c.s.digest += digest_mix(c.s.pops, bt, bsrc, bseq);
        if (d.trace) {
            const uint64_t ts = atomicAdd((unsigned long long*)&rs->trace_len, 1ULL);
            if (ts < d.trace_cap) {
                sg_trace_rec tr;
                tr.time = bt;
                tr.seq = bseq;
                tr.host = c.h;
                tr.src = bsrc;
                tr.pos = c.s.pops;
                d.trace[ts] = tr;
            } else {
                a.overflow = true;
            }
        }
        ++c.s.pops;
        ++a.ctr[C_POPS];
        const bool boot = (bsrc == c.h) & (bseq == 0);
        a.ctr[C_BOOTS] += boot;
        const uint32_t nsend = boot ? d.load : 1u;  // test_phold.c:234-239 / 310-312
        for (uint32_t m = 0; m < nsend; ++m) {
            const int32_t x = dev_rand_r(c.s.rng);
            if (x > last) {  // no host selected (test_phold.c:176-177)
                ++a.ctr[C_NULL];
                continue;
            }
            const int32_t ch = dev_rand_r(c.s.rng);  // worker.c:268-269
            ++a.ctr[C_SENDS];
            on_send(x, ch, trel);
        }
    }
}

// Sort a host's due segment by (time, key): event_compare with equal dst.
// Selection sort; segments are short (a few events per host per window).
__device__ __forceinline__ void sort_segment(Rec* seg, uint32_t cnt) {
    for (uint32_t i = 0; i + 1 < cnt; ++i) {
        Best b{UINT64_MAX, 0, i};
        for (uint32_t k = i; k < cnt; ++k) {
            const Rec r = seg[k];
            best_take(b, r.a & M52, r.k, k);
        }
        if (b.slot != i) {
            const Rec t = seg[i];
            seg[i] = seg[b.slot];
            seg[b.slot] = t;
        }
    }
}

// Flat pass (k_proc): one lane per due event instead of one per host.  A
// lane finds its event's place in the host's pop order by comparing it with
// the host's other due events (seg, cnt records in LDS, any order): rank,
// the host's earliest time and whether a boot event is among them.
struct SegScan {
    uint32_t rank;
    uint64_t tmin;
    bool boot;  // srcHostEventID 0: only a boot event carries it (event.c:38, worker_bootHosts)
};
__device__ __forceinline__ SegScan seg_scan(const Rec* seg, uint32_t cnt, uint64_t et, uint64_t ek) {
    SegScan s{0, et, (ek & SEQ_MASK) == 0};
    if (cnt > 1) {
#pragma unroll 4
        for (uint32_t k = 0; k < cnt; ++k) {
            const Rec r = seg[k];
            const uint64_t rt = r.a & M52;
            s.rank += key_less(rt, r.k, et, ek) ? 1u : 0u;
            s.tmin = rt < s.tmin ? rt : s.tmin;
            s.boot |= (r.k & SEQ_MASK) == 0;
        }
    }
    return s;
}
// A host the flat pass executes: every event is a PHOLD message event with one
// send (no boot event: test_phold.c:310-312), so an event's draws follow the
// draws of the events before it; every send kept unless the host has one event
// (lossy records: a send's srcHostEventID counts the kept sends before it,
// event.c:38 after worker.c:268-273); no self event can land inside the window
// (host_single.c:237-267 would pop it this round).  Every lane of the host
// computes the same answer; the others run phase A.
// Events of one host the flat pass takes at most (each lane scans its host's
// events in LDS and replays the draws of those before it, so a lane's work
// grows with it).  configs[1] (10k hosts, 16 events each, 50 ms windows) has
// Poisson(16) events per host per round: at 16, 43 % of its hosts fell back to
// phase A, one lane per host (k_proc 85 us per round; profiles/r05/stamps).
#ifndef SG_FLAT_CMAX
#define SG_FLAT_CMAX 64
#endif
constexpr uint32_t FLAT_CMAX = SG_FLAT_CMAX;
constexpr uint32_t NULL_DRAW = 1u << 31;  // s_n mark: a flat-pass host whose skip-ahead miscounted
constexpr uint32_t GF_DONE = 1u << 30;    // s_n mark: a host the gossip flat pass recorded (s_n = mark | j)
__device__ __forceinline__ bool flat_ok(const Dev& d, uint32_t cnt, const SegScan& s, bool self_possible, uint64_t S,
                                        uint64_t E, uint32_t vh) {
    if (s.boot || cnt > FLAT_CMAX || (cnt > 1 && d.pair_fmt != PAIR_DELAY)) return false;
    return !self_possible || S + s.tmin + d.vself[vh] >= E;
}

// Diagnostics (SG_STAMPS): a timestamp once this wave's outstanding memory
// operations have landed.
constexpr uint32_t SG_STAMP_W = 32;  // stamp slots per workgroup row
__device__ __forceinline__ uint64_t wait_stamp() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    return __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------- reservations ----
// A reserving row's staged events by ring slot (s_bc counts, s_bm min offsets
// in the bucket; slot (bSr + o) % R is bucket bS + o) into the calendar: one
// reservation per (row, bucket) in the row's sub-list x, the bucket minima,
// and the chunks whose first slot falls inside one of the row's reservations.
// Those come from the row's stash (sid: this lane's stash entry, sn: the
// stash count, both loaded at launch), beyond it from the free ring (one
// reservation of its head; avail: the ring's usable end at launch).  k_scatter
// writes the events into the reserved slots and refills the stashes.  Every
// thread of the block (T threads) calls it.
template <int T, bool STASH_LOOP = false>
__device__ __forceinline__ void reserve_buckets(const Dev& d, uint32_t row, uint32_t x, const uint32_t* s_bc, const uint32_t* s_bm,
                                uint64_t bS, uint32_t bSr, uint32_t sid, uint32_t sn, uint64_t avail,
                                uint32_t* s_ids, uint64_t* s_h, uint64_t* s16) {
    constexpr uint32_t PER = RMAX / T;
    const uint32_t R = d.R, NCH = d.NCH, tid = threadIdx.x;
    const uint64_t W = d.W;
    uint32_t* bkx = d.bk + (size_t)x * R;
    uint32_t* wb = d.wbase + (size_t)row * R;
    if (tid < ST) s_ids[tid] = sid;  // read after the scan's barriers
    uint32_t first[PER], nn[PER];
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t rb = tid + q * T;
        nn[q] = 0;
        first[q] = 0;
        const uint32_t c = rb < R ? s_bc[rb] : 0u;
        if (!c) continue;
#if SG_PMIN
        uint32_t* pm = d.pmin + (size_t)row * R + rb;  // this row's own entry: no other row writes it
        const uint32_t pold = *pm;
#endif
        const uint32_t base = atomicAdd(&bkx[rb], c);
        wb[rb] = base;
#if SG_PMIN
        *pm = s_bm[rb] < pold ? s_bm[rb] : pold;
#else
        const uint64_t b = bS + (rb >= bSr ? rb - bSr : rb + R - bSr);  // absolute bucket of slot rb
        atomicMin((unsigned long long*)&d.bmin[rb], (unsigned long long)(b * W + s_bm[rb]));
#endif
        const uint32_t f = (base + CH - 1) >> CH_SHIFT, l = (base + c - 1) >> CH_SHIFT;
        first[q] = f;
        nn[q] = l + 1 > f ? l + 1 - f : 0u;
        mine += nn[q];
    }
    uint64_t total;
    // LDS-only barriers: nothing here reads another lane's global stores, so
    // the caller's stores keep draining
    uint64_t off = block_excl_scan<true>(mine, s16, &total);
    if (total > sn) {  // uniform: beyond the stash, one ring reservation for the row
        if (tid == 0) *s_h = atomicAdd((unsigned long long*)&d.rs->fl_head, (unsigned long long)(total - sn));
        lds_barrier();
    }
    if (STASH_LOOP && total <= sn) {  // uniform: every chunk from the stash (LDS only)
        // (a separate loop: with the ring's global load in the same loop, its
        // id register made every LDS-path iteration wait vmcnt(0), i.e. for
        // all of the wave's outstanding stores, before its btab store;
        // configs[3] k_proc -0.4 us.  The PHOLD instantiations only: in the
        // gossip one, at its register limit, the extra loop moved spills into
        // hot code, +2 us on configs[4], profiles/r06/g30)
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) {
            const uint32_t rb = tid + q * T;
            for (uint32_t k = 0; k < nn[q]; ++k, ++off) {
                const uint32_t ci = first[q] + k, id = s_ids[off];
                if (ci < NCH) d.btab[((size_t)x * R + rb) * NCH + ci] = id;
                else flag(d, OV_POOL);
            }
        }
    } else {
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
        const uint32_t rb = tid + q * T;
        for (uint32_t k = 0; k < nn[q]; ++k, ++off) {
            uint32_t id = EMPTY;
            if (off < sn) {
                id = s_ids[off];
            } else {
                const uint64_t pos = *s_h + (off - sn);
                if (pos < avail) id = d.fring[pos % NCH];
                else flag(d, OV_POOL);
            }
            const uint32_t ci = first[q] + k;
            if (ci < NCH) d.btab[((size_t)x * R + rb) * NCH + ci] = id;
            else flag(d, OV_POOL);
        }
    }
    }
    const uint32_t left = total < sn ? sn - (uint32_t)total : 0u;
    if (tid < left) d.stash[(size_t)row * ST + tid] = s_ids[total + tid];
    if (tid == 0) d.stn[row] = left;
}

// ------------------------------------------------------------ plan ----
// The end of a step is planned by k_scatter itself (step_view): thread 0 of
// every workgroup reads the round state and the MIN terms the previous
// kernels left (k_proc's accumulators, or, several shards, the G exchange
// headers: the MIN all-reduce of scheduler.c:386-408 rides on the
// all-to-all) and computes master_slaveFinishedCurrentRound
// (master.c:450-480), so every workgroup routes and gathers for the same new
// window.  Each workgroup then takes a ticket; the last one publishes the plan
// for the next kernels (publish_step).  Nothing in the launch writes the
// state the workgroups read before the last ticket, and nothing waits.
// The next window from the global MIN and the discovery minimum (ms), given
// the round state's jump fields (computed in registers; the caller stores).
__device__ Window next_window(const Dev& d, uint64_t minNext, uint64_t jmin, uint64_t mj0, uint64_t nmj0) {
    Window w;
    w.next_min_jump = nmj0;
    w.min_jump = mj0;
    uint64_t jump;
    if (d.window_rule == SG_WINDOW_FIXED) {
        jump = d.fixed_jump;
    } else {
        if (jmin != UINT64_MAX) w.next_min_jump = jmin * SG_ONE_MS;  // master.c:153
        w.min_jump = w.next_min_jump;                                // master.c:459
        jump = w.min_jump > 0 ? w.min_jump : 10 * SG_ONE_MS;         // master.c:137
        if (d.runahead_min > 0 && jump < d.runahead_min) jump = d.runahead_min;
    }
    const uint64_t start = minNext;
    uint64_t end = minNext + jump;  // unsigned wrap as in the reference
    if (end > d.end_time) end = d.end_time;
    w.S = start;
    w.E = end;
    w.done = start < end ? 0 : 1;
    return w;
}

__device__ __forceinline__ uint64_t rmw_read(uint64_t* p) {
    return atomicAdd((unsigned long long*)p, 0ull);
}

// A 64-bit value of lane i (wave-uniform i), and a round state field's word.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t i) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), (int)i) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)i);
}
#define RSF(f) ((uint32_t)(offsetof(RoundState, f) / 8))

// Forces the scalar loads of the Dev fields step_view / next_window read (an
// input-only asm operand needs the value in a register here).
template <class T>
__device__ __forceinline__ void touch_s(const T& v) {
    asm volatile("" ::"s"(v));
}
__device__ __forceinline__ void touch_plan_args(const Dev& d) {
    touch_s(d.W);
    touch_s((uint32_t)d.window_rule);
    touch_s(d.fixed_jump);
    touch_s(d.runahead_min);
    touch_s(d.end_time);
    touch_s((uint32_t)d.ring32);
    touch_s(d.R);
    touch_s(d.NCH);
    touch_s(d.G);
    touch_s(d.wdiv.m);
    touch_s(d.wdiv.s1);
    touch_s(d.wdiv.s2);
}
// mode 0: one shard, after k_proc; 1: several shards, after the all-to-all
// (hdr: the G blocks' HDR_W header words, LDS); 2: boot (the first window is
// listed already).  One thread, from the LDS copy of the round state
// (load_round_state), so no load of it waits for another.
constexpr uint32_t HDR_W = HDR * RW;  // header words per exchange block
constexpr uint32_t RSW = sizeof(RoundState) / 8;
static_assert(sizeof(RoundState) % 8 == 0 && RSW <= 64, "one word per lane of a wave");
__device__ __forceinline__ void step_view(const Dev& d, int mode, const RoundState* rs, const int64_t* hdr,
                                          StepView& sv, uint64_t h0 = 0, bool h_lanes = false) {
    const uint64_t W = d.W;
    sv.quit = rs->done != 0;
    sv.fold = rs->fold;
    sv.cur = (uint32_t)(sv.fold & 1);
    sv.S0 = rs->S;
    sv.E0 = rs->E;
    sv.rounds0 = rs->rounds;
    const uint64_t nmj0 = rs->next_min_jump, mj0 = rs->min_jump, jmin0 = rs->jmin;
    const uint64_t tail0 = rs->fl_tail;
    // (selects, not indices: a register copy of the state stays in registers)
    sv.nfree0 = sv.cur ? rs->nfree2[1] : rs->nfree2[0];
    sv.carry0 = sv.cur ? rs->xcarry2[1] : rs->xcarry2[0];
    sv.rmin0 = sv.cur ? rs->rmin2[1] : rs->rmin2[0];
    sv.ins_S = rs->ins_S;
    sv.ins_local = (uint32_t)rs->ins_local;
    // the current window (kept on a drain step and at boot)
    sv.S = sv.S0;
    sv.E = sv.E0;
    sv.bS = rs->bS;
    sv.bL = rs->bL;
    sv.ret = rs->ret_b;
    sv.pbS = rs->pbS;
    sv.pbL = rs->pbL;
    sv.pret = rs->pret;
    sv.tail = tail0;
    sv.listed = mode == 2 ? (uint32_t)rs->listed : 0u;
    sv.round_done = 0;
    sv.more = 0;
    sv.done = 0;
    uint64_t m = UINT64_MAX, j = UINT64_MAX, ovf = rs->overflow;
    if (mode == 0) {
        // the local MIN terms: carry min, k_proc's emitted and discovery minima
        // (device-scope atomics, a kernel ago), the buckets beyond the window
        const uint64_t em = rs->xacc[0], jm = rs->xacc[1];
        m = sv.carry0 < em ? sv.carry0 : em;
        m = sv.rmin0 < m ? sv.rmin0 : m;
        m = m < SIMTIME_MAX ? m : SIMTIME_MAX;
        j = jmin0 < jm ? jmin0 : jm;
    } else if (mode == 1) {
        uint64_t more = 0;
        // the header words from wave 0's registers when the G blocks' words fit
        // one per lane (h_lanes: G <= 8), else from their LDS copy
        auto hw = [&](uint32_t p, uint32_t f) __attribute__((always_inline)) {
            return h_lanes ? readlane64(h0, p * HDR_W + f) : (uint64_t)hdr[(size_t)p * HDR_W + f];
        };
        for (uint32_t p = 0; p < d.G; ++p) {
            more |= hw(p, H_MORE);
            const uint64_t bm = hw(p, H_MIN), bj = hw(p, H_JMIN);
            m = bm < m ? bm : m;
            j = bj < j ? bj : j;
            ovf |= hw(p, H_OVF);
            if (hw(p, H_ROUND) != sv.rounds0) ovf |= OV_STEP;  // shards out of step
        }
        sv.more = more != 0;
    }
    sv.m = m;
    sv.j = j;
    sv.ovf = ovf;
    sv.tail_r = (uint32_t)rs->tail_r;
    sv.bSr = (uint32_t)rs->bS_r;
    if (mode == 2 || sv.more) return;
    sv.round_done = 1;
    const Window w = next_window(d, m, j, mj0, nmj0);
    sv.w = w;
    sv.done = (w.done | (ovf ? 1u : 0u)) != 0;  // a capacity ran out: stop, the host reports it
    sv.S = w.S;
    sv.E = w.E;
    sv.tail = tail0 + sv.nfree0;  // the last gather's chunks are in the ring now
    sv.tail_r += (uint32_t)sv.nfree0;  // nfree0 <= NCH: one wrap at most
    sv.tail_r -= sv.tail_r >= d.NCH ? d.NCH : 0u;
    // the executed window: its consumed buckets are skipped by rmin until the
    // next k_proc resets them; its straddling bucket is spent unless the new
    // window starts in it
    sv.pbS = sv.bS;
    sv.pbL = sv.bL;
    sv.pret = sv.ret;
    if (!sv.done) {
        sv.listed = 1;
        // the buckets from the old first bucket (S >= its start): one 32-bit
        // multiply-high division while the offsets fit, as in steady state
        const uint64_t bS0 = sv.bS, x = w.S - bS0 * W;
        const uint64_t o = d.ring32 && x < (1ull << 32) ? wdiv(d, (uint32_t)x) : w.S / W - bS0;
        sv.bS = bS0 + o;
        const uint64_t y = w.E - 1 - sv.bS * W;
        sv.bL = sv.bS + (d.ring32 && y < (1ull << 32) ? wdiv(d, (uint32_t)y) : y / W);
        sv.ret = w.E < (sv.bL + 1) * W ? sv.bL : UINT64_MAX;
        if (o < d.R) {
            sv.bSr += (uint32_t)o;
            sv.bSr -= sv.bSr >= d.R ? d.R : 0u;
        } else {
            sv.bSr = (uint32_t)(sv.bS % d.R);
        }
    }
}

// The round state as the previous kernels left it and, with several shards,
// the G blocks' header words, copied into LDS with one load per lane (a chain
// of dependent scalar loads of the round state cost about a microsecond per
// link).  Every lane of wave 0.
constexpr uint64_t XWAIT_TICKS = 500000000;  // 5 s of the 100 MHz clock: a peer that never arrives

// sg_xlink: one lane per sender waits until its arrival counter reaches the
// step's target (the peer's rows were performed before its counter moved), or
// gives up after XWAIT_TICKS and flags the exchange.  The blocks live in
// uncached memory, so the loads issued after the loop read what the peers
// stored; the compiler barrier keeps them after it.
// Fail fast: once any wait of this link has given up (err != 0), no later wait
// waits at all.  A sender that never arrives then costs one time-out, not one
// per step: the run flags OV_XCHG, stops at the next plan, and the host raises
// at its next status check (sg_xlink_status), naming the senders in err's bits.
__device__ __forceinline__ void xlink_wait(const uint64_t* flags, uint32_t G, uint64_t target, uint32_t* err,
                                           uint64_t* ovf) {
    const uint32_t q = threadIdx.x;
    if (q < G) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(flags + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
            if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                if (ovf) atomicOr((unsigned long long*)ovf, (unsigned long long)OV_XCHG);
                break;  // an earlier wait gave up: the link is broken
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > XWAIT_TICKS) {
                atomicOr(err, 1u << (q & 31));
                if (ovf) atomicOr((unsigned long long*)ovf, (unsigned long long)OV_XCHG);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint64_t load_round_state(const Dev& d, int mode, const int64_t* recv, uint64_t* s_rsw,
                                                     int64_t* s_hdr, uint64_t* h0 = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t v = reinterpret_cast<const uint64_t*>(d.rs)[lane < RSW ? lane : 0u];
    constexpr uint32_t HPL = (MAXG * HDR_W + 63) / 64;  // header words per lane, at most
    int64_t h[HPL];
    if (mode == 1) {  // uniform
        // sg_xlink: the peers' arrivals before their headers are read (the
        // round-state load above is in flight meanwhile)
        if (d.xwait) xlink_wait(d.xwait, d.G, d.xwait_target, d.xwait_err, &d.rs->overflow);
        const uint32_t nh = d.G * HDR_W;
#pragma unroll
        for (uint32_t q = 0; q < HPL; ++q) {
            const uint32_t i = lane + q * 64, j = i < nh ? i : 0u;
            // system-scope loads (sc0 sc1): the headers a peer handed off
            // with system-coherent stores (xst) are read past every cache
            h[q] = __hip_atomic_load(&recv[(size_t)(j / HDR_W) * d.xrows * RW + j % HDR_W], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
        }
#pragma unroll
        for (uint32_t q = 0; q < HPL; ++q)
            if (lane + q * 64 < nh) s_hdr[lane + q * 64] = h[q];
        if (h0) *h0 = (uint64_t)h[0];
    }
    // (with SG_RS_LANES the LDS copy is not read: its store would wait for the
    // load before thread 0 fetches the plan's kernel arguments)
    if ((!SG_RS_LANES || !SG_PLAN_TOUCH) && lane < RSW) s_rsw[lane] = v;
    return v;  // the lane's word: thread 0 reads the state by readlane (SG_RS_LANES)
}

// The last workgroup to read the round state writes the plan (one thread).
// rmin2 / nfree2 / xcarry2 [cur ^ 1] are written by their producers (the rmin
// role, gather workgroup 0, the carry atomics); on a step without a new window
// they carry over here.
__device__ void publish_step(const Dev& d, int mode, const StepView& sv, const int64_t* recv) {
    RoundState* rs = d.rs;
    const uint32_t cur = sv.cur;
    if (sv.ovf) atomicOr((unsigned long long*)&rs->overflow, (unsigned long long)sv.ovf);
    rs->fold = sv.fold + 1;
    rs->splan = 0;
    if (mode == 1) {
        rs->recv_ok = 1;  // the next k_proc stages what this launch did not route
        if (d.check) {
            // debug (SG_CHECK=1): the MIN terms k_proc's last workgroup put in
            // this shard's headers, from device-scope atomics it read without a
            // fence, must equal the same terms re-derived here from the
            // workgroups' plain partials; the own block comes back in recv.
            // (The carry min and rmin are this step's values, at [cur].)
            uint64_t lm = sv.carry0, lj = UINT64_MAX;
            for (uint32_t i = 0; i < d.P; ++i) {
                const uint64_t x = d.p2min[i], y = d.p2min[d.P + i];
                lm = x < lm ? x : lm;
                lj = y < lj ? y : lj;
            }
            lm = sv.rmin0 < lm ? sv.rmin0 : lm;
            lm = lm < SIMTIME_MAX ? lm : SIMTIME_MAX;
            lj = rs->jmin < lj ? rs->jmin : lj;
            const int64_t* own = recv + (size_t)d.g * d.xrows * RW;
            if ((uint64_t)own[H_MIN] != lm || (uint64_t)own[H_JMIN] != lj) flag(d, OV_BUG);
        }
        rs->steps += 1;
        for (uint32_t q = 0; q < d.G; ++q) {
            if (sv.listed) {  // the next step processes: the outboxes refill
                d.outn[q] = 0;
                d.sent[q] = 0;
            } else {
                const uint64_t left = d.outn[q] - d.sent[q];
                d.sent[q] += left < d.xcap ? left : d.xcap;
            }
        }
    }
    if (mode == 0) {
        rs->xacc[0] = UINT64_MAX;  // k_proc's next launch accumulates again
        rs->xacc[1] = UINT64_MAX;
    }
    rs->xcarry2[cur] = UINT64_MAX;  // the next launch's carry atomics go here
    if (!sv.listed) {               // no gather: nothing new in these
        rs->xcarry2[cur ^ 1] = sv.carry0;
        rs->nfree2[cur ^ 1] = sv.nfree0;
    }
    if (mode == 2) return;
    if (sv.more) {  // drain step: same window, more exchange
        rs->phase = 1;
        rs->listed = 0;
        return;
    }
    const Window& w = sv.w;
    rs->phase = 0;
    rs->jmin = sv.j;
    if (d.wlog && sv.rounds0 < d.wlog_cap) {  // the window just executed
        d.wlog[2 * sv.rounds0] = sv.S0;
        d.wlog[2 * sv.rounds0 + 1] = sv.E0;
    }
    rs->rounds = sv.rounds0 + 1;
    rs->last_min = sv.m;
    rs->next_min_jump = w.next_min_jump;
    rs->min_jump = w.min_jump;
    rs->S = sv.S;
    rs->E = sv.E;
    rs->done = sv.done;
    rs->fl_tail = sv.tail;
    rs->tail_r = sv.tail_r;
    rs->bS_r = sv.bSr;
    rs->pbS = sv.pbS;
    rs->pbL = sv.pbL;
    rs->pret = sv.pret;
    rs->bS = sv.bS;
    rs->bL = sv.bL;
    rs->ret_b = sv.ret;
    rs->listed = sv.listed;
}

// Resets the buckets the window before the current one consumed (fully due,
// or a straddling bucket the current window left behind): no reservation can
// reach them (new events are at or after the current window's start), and
// k_scatter's gather and rmin of the previous step are done with them.
// Threads [0, XS * nb) of one workgroup at launch.
__device__ __forceinline__ void reset_consumed(const Dev& d) {
    const RoundState* rs = d.rs;
    const uint64_t pbS = rs->pbS, pbL = rs->pbL, pret = rs->pret, bS = rs->bS;
    if (pbS == UINT64_MAX) return;
    const uint32_t R = d.R, nb = (uint32_t)(pbL - pbS + 1);
    for (uint32_t i = threadIdx.x; i < nb * XS; i += blockDim.x) {
        const uint64_t b = pbS + i / XS;
        if (b == pret && pret >= bS) continue;  // still live: the current window starts in it
        const uint32_t x = i % XS, rb = (uint32_t)(b % R), row = x * R + rb;
        atomicExch(&d.bk[row], 0u);
        d.bw[row] = 0;
        d.bw[(size_t)XS * R + row] = 0;
        if (x == 0) {
            atomicExch(&d.btomb[rb], 0u);
            atomicExch((unsigned long long*)&d.bmin[rb], (unsigned long long)UINT64_MAX);
        }
    }
#if SG_PMIN
    // the consumed buckets' columns of every row's minima (the rows reserve in
    // buckets at or after the current window only, so none writes these now)
    for (uint32_t i = threadIdx.x; i < nb * d.P; i += blockDim.x) {
        const uint64_t b = pbS + i / d.P;
        if (b == pret && pret >= bS) continue;
        d.pmin[(size_t)(i % d.P) * R + (uint32_t)(b % R)] = UINT32_MAX;
    }
#endif
}

// One workgroup per partition of HP hosts.
//   sort     the partition's due events by host (LDS counting sort into an LDS
//            image of the events when they fit, else into part2) and list the
//            active hosts;
//   phase A  per active host: pop order (event_compare), trace digest, and the
//            host's rand_r draws, which are pure arithmetic: one record
//            {time, x, c} per send with a destination.  A host that could
//            create an event for itself inside this window (its earliest event
//            + its self-path delay < barrier) runs the whole sequential body
//            here instead (same-round self events, host_single.c:237-267);
//   phase B  one lane per send, two sends in flight per lane: destination,
//            path record, reliability test, delivery time;
//   phase C  one lane per send record: srcHostEventID, endTime drop, barrier
//            bump, staging (with delay-only path records every send is kept,
//            so phases B and C run as one pass without the barrier);
//   count    the staged local events by calendar bucket (LDS bins over the
//            dead event image) and one reservation per (partition, bucket).
constexpr uint32_t HPT = HPMAX / K2_T;     // active hosts per lane, at most
constexpr uint32_t EVLMAX = 6144;          // due events sorted in LDS, at most
constexpr uint32_t EPT = EVLMAX / K2_T;    // of them per lane

// --------------------------------------------------------- multi-shard ----
// Exchange blocks: per peer, HDR header rows {n, sender has more, MIN next,
// min jump, overflow, round} then up to xcap outbox rows.  The MIN terms are
// this shard's reduce_local of the step's process partials (unchanged on drain
// steps, so a drain step repeats them).  One workgroup (every thread calls it).
__device__ __forceinline__ void reduce_local(const Dev& d, uint64_t* s16, uint64_t& m, uint64_t& j);
__device__ __forceinline__ uint64_t atomic_read(uint64_t* a) {
    return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// outn / overflow are read atomically: the last k_proc workgroup reads what
// the others' device-scope atomics performed (their L2 lines may be stale here).
// Peer q's exchange block of this step: in xsend, or (fused xGMI push) in
// shard q's own region.
__device__ __forceinline__ int64_t* xblock(const Dev& d, uint32_t q) {
    return d.xpeer ? d.xpeer[q] + d.xoff : d.xsend + (size_t)q * d.xrows * RW;
}
// Fused push, the protocol every storing workgroup follows (k_proc's process
// and drain steps, and k_xfused, the self-test that exercises it):
//   1. store its rows into the peers' regions (xst);
//   2. xlink_release: every wave drains its stores (vmcnt(0)), then the
//      workgroup takes a device-scope ticket;
//   3. the last workgroup writes the G headers, drains them the same way and
//      adds one arrival to each peer's counter (xlink_arrive).
// Across GPUs (xfence) every store of the handed-off bytes is system-coherent
// (sc0 sc1: written through to the owner's memory at system scope) and drained
// before the ticket / arrival — MI355X_MICROARCH.md "Correctness boundaries",
// the valid form that replaces a release by the producers (a system-scope
// release, __threadfence_system, is an L2 write-back + invalidate per wave:
// it took k_proc 20.8 -> 39 us per 125k-host step, profiles/r06/g1); the
// receiver's header loads are system-scope too.  Within one device the
// blocks are uncached local memory and plain stores drained by vmcnt(0)
// already order the rows before the arrival (measured).
// (through a global-address-space pointer: a generic one — these come from
// a table of peer regions or a select between two arrays — compiles to flat
// stores, which count on lgkmcnt too and make later LDS accesses wait vmcnt(0))
typedef __attribute__((address_space(1))) int64_t gint64_t;
__device__ __forceinline__ void xst(uint32_t sys, int64_t* p, int64_t v) {
    gint64_t* g = (gint64_t*)p;  // (a C-style cast: reinterpret_cast cannot change address spaces)
    if (sys) __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *g = v;
}
__device__ __forceinline__ void xlink_release() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void xlink_arrive(int64_t* const* peer, uint32_t G, uint32_t g, uint32_t skip) {
    xlink_release();
    __syncthreads();
    if (threadIdx.x < G && threadIdx.x + 1 != skip)
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(peer[threadIdx.x]) + g, 1ull,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void xlink_signal(const Dev& d) { xlink_arrive(d.xpeer, d.G, d.g, d.xskip); }
__device__ __forceinline__ void write_headers(const Dev& d, uint64_t m, uint64_t j) {
    RoundState* rs = d.rs;
    const uint32_t sys = d.xpeer ? d.xfence : 0u;
    if (threadIdx.x < d.G) {
        const uint32_t p = threadIdx.x;
        const uint64_t left = atomic_read(&d.outn[p]) - d.sent[p];
        int64_t* blk = xblock(d, p);
        xst(sys, blk + H_N, (int64_t)(left < d.xcap ? left : d.xcap));
        xst(sys, blk + H_BASE, (int64_t)rs->S);  // the rows' time base: the step's window start
        xst(sys, blk + H_MIN, (int64_t)m);
        xst(sys, blk + H_JMIN, (int64_t)j);
        xst(sys, blk + H_OVF, (int64_t)atomic_read(&rs->overflow));
        xst(sys, blk + H_ROUND, (int64_t)rs->rounds);
    }
    if (threadIdx.x == 0) {
        uint64_t more = 0, peak = rs->peak_peer;
        for (uint32_t q = 0; q < d.G; ++q) {
            const uint64_t on = atomic_read(&d.outn[q]);
            more |= (on - d.sent[q] > d.xcap) ? 1u : 0u;
            peak = q != d.g && on > peak ? on : peak;
        }
        for (uint32_t q = 0; q < d.G; ++q) xst(sys, xblock(d, q) + H_MORE, (int64_t)more);
        rs->peak_peer = peak;
    }
}
// Drain step: the next xcap leftovers of every peer's outbox into its block,
// spread over nblk workgroups; workgroup 0 also writes the headers.
__device__ __forceinline__ void fill_blocks(const Dev& d, uint32_t blk, uint32_t nblk, uint64_t* s16) {
    for (uint32_t p = 0; p < d.G; ++p) {
        const uint64_t left = d.outn[p] - d.sent[p];
        const uint64_t n = left < d.xcap ? left : d.xcap;
        int64_t* dst = xblock(d, p) + HDR * RW;
        const int64_t* src = d.outq + ((uint64_t)p * d.oreg + d.sent[p]) * RW;
        const uint32_t sys = d.xpeer ? d.xfence : 0u;
        for (uint64_t i = (uint64_t)blk * blockDim.x + threadIdx.x; i < n * RW; i += (uint64_t)nblk * blockDim.x)
            xst(sys, dst + i, src[i]);
    }
    if (blk == 0) {
        uint64_t m, j;
        reduce_local(d, s16, m, j);  // barriers inside
        write_headers(d, m, j);
    }
}
// Fused push on a drain step: the last workgroup to finish arrives at the
// peers.  Every workgroup calls it at its very end, after it staged the
// previous step's received events: the arrival releases the peers' k_scatter
// of this step, and their next k_proc stores into the parity buffer that
// stage_received reads here (an arrival sent as soon as the copies
// were done raced with that read).
__device__ __forceinline__ void drain_arrive(const Dev& d, uint32_t nblk) {
    __shared__ bool s_last;
    xlink_release();  // this wave's rows performed at the peers
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd((unsigned long long*)&d.rs->ticket, 1ULL) == nblk - 1;
    __syncthreads();
    if (s_last) {
        if (threadIdx.x == 0) d.rs->ticket = 0;
        xlink_signal(d);
    }
}

// The path record of (sv, dv) from the partition's LDS rows (sv in
// [vlo, vlo + rows)); the discovered-ms field from HBM while it can matter.
__device__ __forceinline__ PairRec lds_pair(const Dev& d, const unsigned char* rows, uint32_t vlo, uint32_t sv,
                                            uint32_t dv, bool want_jump) {
    const size_t i = (size_t)(sv - vlo) * d.V + dv;
    PairRec pr;
    if (d.pair_fmt == PAIR_NARROW) {
        const uint2 v = reinterpret_cast<const uint2*>(rows)[i];
        pr.delay = v.x;
        pr.keep = (int32_t)v.y;
    } else {
        pr.delay = reinterpret_cast<const uint32_t*>(rows)[i];
        pr.keep = SG_RAND_MAX;
    }
    pr.jump = want_jump ? d.pjump[pair_index(d, sv, dv)] : UINT32_MAX;
    return pr;
}

// A draw x whose host is its guess g or g + 1 (d.dst_near): a = record g,
// b = record g + 1 (adjacent: one line); the first host with x <= threshold.
__device__ __forceinline__ void near_resolve(const Dev& d, int32_t x, uint2 a, uint2 b, uint32_t& vd, uint32_t& dst) {
    const bool first = d.dst_rule == SG_DST_UNIFORM_FLOOR || x <= (int32_t)a.x;
    const uint32_t w = first ? a.y : b.y;
    vd = w >> d.slot_bits;
    dst = w & ((1u << d.slot_bits) - 1);
}

// EXACT: d.dst_near (a destination is two adjacent 8-byte records per send);
// the other instantiation resolves destinations through the weight probes
// (and bisection).  ROWS: d.lds_rows (path records from the partition's LDS rows).
// Exclusive offsets of the received blocks' event counts (own block: 0) and
// the blocks' time bases.  rows / cap: the blocks' layout (HDR + cap rows per peer).
__device__ __forceinline__ uint64_t recv_offsets(const Dev& d, const int64_t* recv, uint64_t rows, uint64_t cap,
                                                 uint32_t* s_off, uint64_t* s_rbase, uint64_t* s16, bool check) {
    const uint32_t s = threadIdx.x;
    uint64_t c = 0, base = 0;
    if (s < d.G && s != d.g) {
        const int64_t* blk = recv + (size_t)s * rows * RW;
        const uint64_t n = (uint64_t)blk[H_N];
        base = (uint64_t)blk[H_BASE];
        if (n <= cap) c = n;
        else if (check) flag(d, OV_XCHG);
    }
    uint64_t total;
    const uint64_t run = block_excl_scan(c, s16, &total);
    if (s < d.G) {
        s_off[s] = (uint32_t)run;
        s_rbase[s] = base;
    }
    __syncthreads();
    return total;
}

// Received event `idx` of the concatenated blocks: t, key, dst_local.
__device__ __forceinline__ bool recv_event(const Dev& d, const int64_t* recv, uint64_t rows, const uint32_t* s_off,
                                           const uint64_t* s_rbase, uint32_t idx, uint64_t& t, uint64_t& k,
                                           uint32_t& dl) {
    uint32_t lo = 0, hi = d.G - 1;  // last block with s_off <= idx
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_off[mid] <= idx) lo = mid; else hi = mid - 1;
    }
    const int64_t* row = recv + ((size_t)lo * rows + HDR + (idx - s_off[lo])) * RW;
    const uint64_t w0 = (uint64_t)row[0];
    t = s_rbase[lo] + (w0 & M40);
    k = (uint64_t)row[1];
    dl = (uint32_t)(w0 >> 40);
    return dl < d.L;
}

// A staged event at time t into a reserving row's LDS bucket bins (bucket bS
// + o is ring slot (bSr + o) % R): count and min offset in the bucket.  False
// (and no bin) when t lies outside the calendar's horizon.
__device__ __forceinline__ bool bin_time(const Dev& d, uint64_t t, uint64_t bS, uint64_t bSW, uint32_t bSr,
                                         uint32_t* s_bc, uint32_t* s_bm) {
    const uint32_t R = d.R;
    const uint64_t W = d.W;
    uint32_t o, off;
    if (d.ring32) {  // launch-uniform: no 64-bit division
        const uint64_t rel = t - bSW;
        o = wdiv(d, (uint32_t)rel);
        off = (uint32_t)rel - o * (uint32_t)W;
        if (t < bSW || (rel >> 32) || o >= R) return false;
    } else {
        const uint64_t b = t / W;
        if (b < bS || b - bS >= R) return false;
        o = (uint32_t)(b - bS);
        off = (uint32_t)(t - b * W);
    }
    uint32_t rb = bSr + o;
    rb = rb >= R ? rb - R : rb;
    atomicAdd(&s_bc[rb], 1u);
    atomicMin(&s_bm[rb], off);
    return true;
}

// Several shards: k_proc stages its share of the events the previous step
// received (recv: that step's blocks, intact until this step's all-to-all)
// like local events — into loc and the bucket bins, reserved with them —
// except those k_scatter already routed into this window's partitions
// (routed: it planned this window, and t < E).  This is the insert of
// received events (scheduler_push on the receiving side, scheduler.c:339-357):
// no kernel of its own.  Every thread calls it (barrier inside).  Returns the
// minimum time staged (UINT64_MAX: none).
template <class Count>
__device__ __forceinline__ uint64_t stage_received(const Dev& d, const int64_t* recv, uint32_t part, uint32_t nparts,
                                                   bool routed, uint64_t S, uint64_t E, ProcShared& sh, bool& ovf,
                                                   uint32_t* s_off, uint64_t* s16, Count count) {
    __shared__ uint64_t s_rbase[MAXG];  // the received blocks' time bases
    const uint64_t total = recv_offsets(d, recv, d.xrows_in, d.xcap_in, s_off, s_rbase, s16, true);  // barrier inside
    const uint64_t lo = total * part / nparts, hi = total * (part + 1) / nparts;
    uint64_t mn = UINT64_MAX;
    for (uint64_t i0 = lo; i0 < hi; i0 += blockDim.x) {
        const uint64_t idx = i0 + threadIdx.x;
        uint64_t t = 0, k = 0;
        uint32_t dl = 0;
        bool v = idx < hi;
        if (v && !recv_event(d, recv, d.xrows_in, s_off, s_rbase, (uint32_t)idx, t, k, dl)) {
            flag(d, OV_XCHG);
            v = false;
        }
        if (v && routed && t < E) v = false;  // k_scatter put it in its partition
        if (v) {
            const uint32_t slot = wave_slot(&sh.nloc);
            if (slot < d.ECAP) st_rec(d.loc, ((size_t)part * d.ECAP + slot) * 16, ((uint64_t)dl << 40) | (t - S), k);
            else ovf = true;
            count(t);
            mn = t < mn ? t : mn;
        }
    }
    return mn;
}

// The next gather's guessed due list (GSpec): when this window ends on a
// bucket boundary, the next one most likely is that bucket, whole.  Its slots
// written before the step are bw[fold & 1] (the last k_scatter's copy) and
// their chunks were allocated before that k_scatter, so their ids are final
// now (this launch's reservations append beyond them).  One workgroup, every
// thread; the loads go out together.
__device__ __forceinline__ void gspec_write(const Dev& d, uint64_t fold, uint64_t E) {
    const uint64_t b = E / d.W + (d.gspec_mode == 2 ? 1u : 0u);
    const bool guess = GSPEC_XS && (b - (d.gspec_mode == 2 ? 1u : 0u)) * d.W == E && d.gspec_mode != 0;
    const uint32_t row = (uint32_t)(b % d.R), i = threadIdx.x, ic = i < d.NCH ? i : 0u;
    const uint32_t* bw = d.bw + (size_t)(fold & 1) * XS * d.R;
    const uint32_t lo = bw[row];
    const uint32_t id = d.btab[(size_t)row * d.NCH + ic];
    // XS = 2: sub-list 1's count and chunk i, loaded beside sub-list 0's
    const uint32_t lo1 = XS == 2 ? bw[d.R + row] : 0u;
    const uint32_t id1 = XS == 2 ? d.btab[((size_t)d.R + row) * d.NCH + ic] : 0u;
    const uint32_t nid0 = (lo + CH - 1) >> CH_SHIFT, nid = nid0 + ((lo1 + CH - 1) >> CH_SHIFT);
    GSpec* g = d.gspec;
    if (guess && i < nid0 && i < NSPEC) g->ids[i] = id;
    if (XS == 2 && guess && nid0 + i < nid && nid0 + i < NSPEC) g->ids[nid0 + i] = id1;
    if (i == 0) {
        g->fold = guess && nid <= NSPEC ? fold : UINT64_MAX;
        g->b = b | ((uint64_t)row << 48);
        g->lo = lo;
        g->nid = XS == 2 ? lo1 : nid;
    }
}

// SG_INS_PRE: k_scatter's insert role loads its first staged events and its
// reservation bases at launch, beside the plan (1, default), or after it (0).
// With the gather dispatched after the inserts, 0 was faster (51.1-51.4
// against 51.6-52.0 us per round, profiles/r04/insert_pre); with the gather
// first (SG_GFIRST) the insert role is the long pole and 1 wins (48.9-49.1
// against 49.7-50.0, profiles/r04/inspre2).
#ifndef SG_GFIRST
#define SG_GFIRST 1
#endif
#ifndef SG_INS_PRE
#define SG_INS_PRE 1
#endif
// SG_LATE_TICKET: k_scatter's workgroups arrive on the plan counter at their
// end (1) or right after planning (0).  Arriving early, the 386 arrivals land
// together on one counter (fan-in ~11 ns each), and wave 0 of every role then
// waits for its arrival at its first load-use (vmcnt counts in order): the
// stamps showed 7 us from entry to role start (profiles/r05/stamps).
#ifndef SG_LATE_TICKET
#define SG_LATE_TICKET 1
#endif
// SG_FLAT_LDSB: the barrier after the flat pass orders LDS only (default;
// profiles/r04/flatb: 52.2 against 52.5-53.3 us/round, interleaved).
#ifndef SG_FLAT_LDSB
#define SG_FLAT_LDSB 1
#endif
// SG_TICK8: k_scatter's plan arrival in two levels, one counter per workgroup
// shard blockIdx & 7 and then the plan counter (1, default), or every
// workgroup on the plan counter (0): k_scatter 17.6 -> 17.1 us, configs[3]
// 7.68 -> 7.80e9 events/s (profiles/r05/tick).
#ifndef SG_TICK8
#define SG_TICK8 1
#endif
// SG_SORT_LB: the PHOLD instantiations' barriers from the partition's loads to
// its scatter wait for LDS only (1, default), or for every outstanding access (0):
// configs[3] k_proc 29.5 -> 29.1 us (profiles/r06/g13)
#ifndef SG_SORT_LB
#define SG_SORT_LB 1
#endif
// k_proc's static LDS, at most (the dynamic region is sized around it;
// sg_engine_boot checks every instantiation against it)
constexpr uint32_t PROC_LDS_STATIC = 5u << 10;
// SG_SGET_WAIT: a send record read from HBM (past the LDS share) is waited
// for at its load (1, default), or at its first use (0)
#ifndef SG_SGET_WAIT
#define SG_SGET_WAIT 1
#endif
// SG_SKIP_LDS: the flat pass reads its skip-ahead table from an LDS copy (1,
// default) or from global memory (0)
#ifndef SG_SKIP_LDS
#define SG_SKIP_LDS 1
#endif
// SG_ROWS_GLDS: k_proc's path rows go global -> LDS by global_load_lds (1),
// or through 8 VGPRs per lane held through the sort (0)
#ifndef SG_ROWS_GLDS
#define SG_ROWS_GLDS 1
#endif
// FLAT: d.flat (PHOLD): a partition with at most SPEC due events per lane runs
// the flat pass; its event image holds only those (EPTF registers per lane), a
// bigger one sorts through part2 and runs phase A.
template <bool EXACT, bool ROWS, bool FLAT>
__global__ __launch_bounds__(K2_T) void k_proc(Dev d) {
    RoundState* rs = d.rs;
    const uint32_t p = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    // One batch of loads before anything waits: the round state, one word per
    // lane of every wave (its fields then come by readlane), and what the
    // partition needs from nothing else (its first records, count, chunk
    // stash, slot range).  Read field by field, the round state was a chain of
    // dependent scalar loads in front of the partition's loads.
    const uint64_t rsv = reinterpret_cast<const uint64_t*>(rs)[(tid & 63) < RSW ? (tid & 63) : 0u];
    const Rec* part = d.part + (size_t)p * d.CAPP;
    // the first SPEC records per lane are loaded before the count arrives
    // (CAPP >= K2_T; records past the count are ignored).  A lane's record q
    // is entry tid + q * K2_T of the partition.
    constexpr uint32_t SPEC = 2;
    constexpr uint32_t EPTF = FLAT ? SPEC : EPT;
    auto rq_idx = [&](uint32_t q) __attribute__((always_inline)) { return tid + q * K2_T; };
    Rec rr[EPTF];
#pragma unroll
    for (uint32_t q = 0; q < SPEC; ++q) rr[q] = ld_stream(&part[rq_idx(q)]);
    const uint32_t n_a = d.pcnt[p];  // the window's due events of the partition
    // the partition's chunk stash (reserve_buckets), loaded now, used at the end
    const uint32_t stash_id = d.stash[(size_t)p * ST + (tid & (ST - 1))], stash_n = d.stn[p];
    uint32_t v_first = 0, v_last = 0;  // ROWS: the partition's first and last slots' vertices
    if constexpr (ROWS) {
        const uint32_t s0 = p * d.HP, s1 = (p + 1) * d.HP < d.L ? (p + 1) * d.HP : d.L;
        v_first = d.sinfo[s0].v;
        v_last = d.sinfo[s1 - 1].v;
    }
    auto rsf = [&](uint32_t w) __attribute__((always_inline)) { return readlane64(rsv, w); };
    // a use of those loads on the paths that do not need them keeps the
    // compiler from sinking them below the branches (and so behind the wait)
    auto pin = [&]() __attribute__((always_inline)) {
        asm volatile("" ::"v"(rr[0].a), "v"(rr[1].a), "v"(n_a), "v"(stash_id), "v"(stash_n), "v"(v_first),
                     "v"(v_last));
    };
    if (rsf(RSF(done))) {
        pin();
        if (d.xpeer && p == 0) xlink_signal(d);  // the peers' k_scatter still waits for this step
        return;
    }
    const uint64_t rs_fold = rsf(RSF(fold)), rs_bS = rsf(RSF(bS));
    extern __shared__ __align__(16) unsigned char dyn[];
    const uint32_t HP = d.HP, R = d.R;
    uint32_t* s_n = (uint32_t*)dyn;             // [HP] events per host
    uint32_t* s_c = s_n + HP;                   // [HP] start offset, then end (scatter cursor)
    uint32_t* s_vh = s_c + HP;                  // [HP] active host j: vertex | phase C sends << 16
    uint32_t* s_sb = s_vh + HP;                 // [HP] active host j: first phase B/C send, or UINT32_MAX
    uint16_t* s_act = (uint16_t*)(s_sb + HP);   // [HP] active hosts, ascending
    uint32_t* s_bc = (uint32_t*)(dyn + d.bin_off);  // [R] staged local events per bucket
    uint32_t* s_bm = s_bc + R;                      // [R] their min time offset in the bucket
    Rec* s_ev = (Rec*)(dyn + d.ev_off);             // [EVL] due events grouped by host
    const unsigned char* s_rows = dyn + d.row_off;  // [rows][V] path records of the partition's vertices
    __shared__ uint32_t s_nsend;
    __shared__ int32_t s_last;         // last weight threshold: x above it selects no host
    __shared__ ProcShared sh;
    __shared__ uint64_t s16[16];
    __shared__ uint64_t s_red[K2_T / 64][NPCTR + 2];
    __shared__ uint32_t s_obase[MAXG], s_oslot[MAXG];
    __shared__ uint32_t s_roff[MAXG];  // received blocks' offsets (stage_received)
    __shared__ uint32_t s_ids[ST];
    __shared__ uint64_t s_h;
    const uint64_t S = rsf(RSF(S)), E = rsf(RSF(E));
    // several shards: stage the previous step's received events this step
    // (k_scatter routed those due in this window when it planned it: listed)
    const bool stage_recv = d.xrecv && rsf(RSF(recv_ok));
    const bool recv_routed = rsf(RSF(listed)) != 0;
    const bool want_jump = rsf(RSF(jmin)) > d.gjmin;  // discovery can still lower the window's jump
    const uint64_t ring_end = rsf(RSF(fl_tail)) + rsf(RSF(nfree2) + (uint32_t)(rs_fold & 1));  // the last gather freed nfree more
    if (rsf(RSF(phase))) {
        pin();
        // drain step: outbox leftovers into the exchange blocks; the previous
        // step's received events staged and reserved (no window was planned,
        // so none was routed).  The headers repeat the process step's MIN
        // terms, whose emitted minima cover the staged events.
        if (d.xsend) fill_blocks(d, p, gridDim.x, s16);
        if (tid == 0 && p == 0) {
            rs->ins_local = stage_recv ? 1 : 0;
            rs->ins_S = S;
        }
        if (!stage_recv) {  // uniform
            if (d.xpeer) drain_arrive(d, gridDim.x);
            return;
        }
        const uint32_t R = d.R;
        const uint64_t bS = rs_bS, bSW = bS * d.W;
        const uint32_t bSr = (uint32_t)(bS % R);
        uint32_t* s_bc = (uint32_t*)(dyn + d.bin_off);
        uint32_t* s_bm = s_bc + R;
        for (uint32_t rb = tid; rb < R; rb += K2_T) {
            s_bc[rb] = 0;
            s_bm[rb] = UINT32_MAX;
        }
        if (tid == 0) sh.nloc = 0;
        __syncthreads();
        bool ovf = false, hz = false;
        (void)stage_received(d, d.xrecv, p, gridDim.x, false, S, E, sh, ovf, s_roff, s16, [&](uint64_t t) {
            if (!bin_time(d, t, bS, bSW, bSr, s_bc, s_bm)) hz = true;
        });
        if (ovf) flag(d, OV_PROC);
        if (hz) flag(d, OV_HORIZON);
        __syncthreads();
        reserve_buckets<K2_T>(d, p, p % XS, s_bc, s_bm, bS, bSr, stash_id, stash_n, ring_end, s_ids, &s_h, s16);
        if (tid == 0) {
            if (sh.nloc > d.ECAP) flag(d, OV_PROC);
            d.rcnt[p] = sh.nloc < d.ECAP ? sh.nloc : d.ECAP;
        }
        if (d.xpeer) drain_arrive(d, gridDim.x);  // after every read of the received blocks
        return;
    }
    uint64_t* stamp = d.stamps ? d.stamps + (size_t)p * SG_STAMP_W : nullptr;
    if (stamp && tid == 0) stamp[0] = __builtin_amdgcn_s_memrealtime();
    const uint64_t t_start = d.wtime ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t n = n_a < d.CAPP ? n_a : d.CAPP;  // the partition's due events
    // lane record q holds an event; entry i of the partition (0 <= i < n)
    auto rq_ok = [&](uint32_t q) __attribute__((always_inline)) { return tid + q * K2_T < n; };
    auto pidx = [&](uint32_t i) __attribute__((always_inline)) { return i; };
    // flat pass: a host's digest terms of its events but the last, summed in
    // LDS over s_vh / s_sb (phase A's arrays, free until phase A runs)
    unsigned long long* s_dig = reinterpret_cast<unsigned long long*>(s_vh);
    for (uint32_t h = tid; h < HP; h += K2_T) {
        s_n[h] = 0;
        if constexpr (FLAT) s_dig[h] = 0;
    }
    for (uint32_t rb = tid; rb < R; rb += K2_T) {
        s_bc[rb] = 0;
        s_bm[rb] = UINT32_MAX;
    }
    if (tid == 0) {
        sh.nloc = 0;
        sh.nrem = 0;
        s_nsend = 0;
        s_last = d.dst_rule == SG_DST_WEIGHTS ? d.hinfo[d.N - 1].wt : INT32_MAX;
        if (p == 0) {  // k_scatter takes this step's staged local events
            rs->ins_local = 1;
            rs->ins_S = S;
        }
    }
    if (tid < MAXG) sh.peer[tid] = 0;
#if SG_SKIP_LDS
    // the flat pass's skip-ahead table (ranks below FLAT_CMAX) in LDS: read once
    // per lane there, behind its rank scan (a global load on that chain before)
    __shared__ uint2 s_skipf[FLAT_CMAX];
    if (FLAT && d.skip && tid < FLAT_CMAX) s_skipf[tid] = d.skip[tid < d.nskip ? tid : 0u];
#endif
    Rec* part2 = d.part2 + (size_t)p * d.CAPP;
    const bool in_lds = n <= d.EVL && (!FLAT || n <= SPEC * K2_T);
    // Flat pass (PHOLD, events in LDS, at most SPEC per lane; see below): the
    // states of the hosts of the lane's two due events are loaded as soon as
    // the records arrive.  Every lane's state reads have returned before the
    // barrier after the scatter (vmcnt(0)) and every state write comes after
    // it, so a host's last event cannot overwrite the state its other events
    // read.
    const bool flat = FLAT && in_lds;
    ulonglong2 pre_a0, pre_b0, pre_a1 = make_ulonglong2(0, 0), pre_b1 = make_ulonglong2(0, 0);
    if (in_lds) {
#pragma unroll
        for (uint32_t q = SPEC; q < EPTF; ++q) rr[q] = rq_ok(q) ? ld_stream(&part[rq_idx(q)]) : Rec{0, 0};
    }
    // the partition's hosts share a few vertices (slots are vertex-sorted):
    // their path rows (<= 32 KB: RQ words per lane) are loaded now into
    // registers, every load unconditional so the sort below waits for none of
    // them, and stored into LDS after the scatter
    constexpr uint32_t RQ = (32u << 10) / 4 / K2_T;
    uint32_t vlo = 0, nwords = 0;
#if !SG_ROWS_GLDS
    uint32_t rw[RQ];
#endif
    if constexpr (ROWS) {
        vlo = v_first;
        const uint32_t nrow = v_last - vlo + 1;
        const uint32_t wpe = d.pair_fmt == PAIR_NARROW ? 2u : 1u;  // words per record
        nwords = (nrow < d.rows_max ? nrow : d.rows_max) * d.V * wpe;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(d.prow) + (size_t)vlo * d.V * wpe;
#if SG_ROWS_GLDS
        // straight into LDS (global_load_lds_dwordx4, 16 B a lane, each wave
        // instruction 1 KB lane-linear): no VGPRs held through the sort.  The
        // LDS region holds whole 1 KB wave pieces (row_pieces); pieces past the
        // rows re-read their last one (prow is padded to a whole piece)
        const uint32_t lastp = (nwords + 3) / 4 - 1;
#pragma unroll
        for (uint32_t q = 0; q < RQ / 4; ++q) {
            const uint32_t w0 = (tid & ~63u) + q * K2_T;  // the wave's first piece
            if (w0 >= d.row_pieces) continue;                // wave-uniform
            const uint32_t i = tid + q * K2_T, ic = i < lastp ? i : lastp;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 4 * (size_t)ic),
                                             (__attribute__((address_space(3))) void*)(dyn + d.row_off + (size_t)w0 * 16),
                                             16, 0, 0);
        }
#else
        // clamped to the partition's own rows (nwords >= V): the loads past
        // them re-read its last word instead of fetching rows nobody uses
        const uint32_t last = nwords - 1;
#pragma unroll
        for (uint32_t q = 0; q < RQ; ++q) {
            const uint32_t i = tid + q * K2_T;
            rw[q] = src[i < last ? i : last];
        }
#endif
        if (nrow > d.rows_max && tid == 0) flag(d, OV_BUG);  // the host sized rows_max
    }
    auto pair_of = [&](uint32_t sv, uint32_t dv, bool wj) __attribute__((always_inline)) {
        if constexpr (ROWS) return lds_pair(d, s_rows, vlo, sv, dv, wj);
        else return load_pair(d, sv, dv, wj);
    };
    static_assert(K2_T >= NSPEC, "one GSpec id per thread");
    if (p == d.P - 1) gspec_write(d, rs_fold, E);  // the lightest partition; loads beside the rows
    if (stamp && tid == 0) stamp[20] = __builtin_amdgcn_s_memrealtime();
    // the flat pass's host states, loaded as soon as the records are in (the
    // histogram; issued after the scan instead, under the scatter only, the
    // scatter took what the histogram gave back: profiles/r06/g5)
    auto flat_prefetch = [&]() __attribute__((always_inline)) {
        if (flat) {  // uniform
            const ulonglong2* hsw = reinterpret_cast<const ulonglong2*>(d.hs);
            uint32_t l0 = p * HP + (uint32_t)(rr[0].a >> 52), l1 = p * HP + (uint32_t)(rr[1].a >> 52);
            l0 = l0 < d.L ? l0 : d.L - 1;  // a record past the count: any valid slot
            l1 = l1 < d.L ? l1 : d.L - 1;
            pre_a0 = ld_stream2(&hsw[2 * (size_t)l0]);
            pre_b0 = ld_stream2(&hsw[2 * (size_t)l0 + 1]);
            if (rq_ok(1)) {  // most lanes have one event
                pre_a1 = ld_stream2(&hsw[2 * (size_t)l1]);
                pre_b1 = ld_stream2(&hsw[2 * (size_t)l1 + 1]);
            }
        }
    };
    // Barriers up to the scatter wait for LDS only (SG_SORT_LB): no lane reads
    // another's global data before the vmcnt(0) after the scatter, so the path
    // rows' DMA and the flat pass's state loads stay in flight under the
    // histogram and the scan
    auto sort_barrier = [&]() __attribute__((always_inline)) {
        if (SG_SORT_LB && FLAT) lds_barrier();  // (the gossip path measured +0.5 us: profiles/r06/g13)
        else __syncthreads();
    };
    sort_barrier();
    if (in_lds) {
#pragma unroll
        for (uint32_t q = 0; q < EPTF; ++q) {
            if (!rq_ok(q)) continue;
            const uint32_t hl = (uint32_t)(rr[q].a >> 52);
            if (hl < HP) atomicAdd(&s_n[hl], 1u);
            else flag(d, OV_BUG);
        }
        flat_prefetch();
        // the records are in registers now: re-defining them through asm keeps
        // the scatter below from waiting on the state prefetch (vmcnt(0))
#pragma unroll
        for (uint32_t q = 0; q < EPTF; ++q) {
            rr[q].a = opaque(rr[q].a);
            rr[q].k = opaque(rr[q].k);
        }
    } else {
        for (uint32_t i = tid; i < n; i += K2_T) {
            const uint32_t hl = (uint32_t)(part[pidx(i)].a >> 52);
            if (hl < HP) atomicAdd(&s_n[hl], 1u);
            else flag(d, OV_BUG);
        }
    }
    sort_barrier();  // the counts
    if (stamp && tid == 0) stamp[21] = __builtin_amdgcn_s_memrealtime();
    // gossip (configs[4]): hosts take the record path (phases B / C resolve
    // their sends one lane each) while the message ids fit the record's 12 bits
    // and the host's seen set GMW registers
    constexpr uint32_t GMW = 4;
    // (the flat pass is PHOLD's: its instantiations carry none of this)
    const bool gossip_rec = !FLAT && d.workload == SG_WORKLOAD_GOSSIP && d.gossip_msgs <= 4096 &&
                            d.mw <= GMW && d.grec;
    // lossy links (phases B and C apart): phase A leaves the record path's
    // draws to a pass of one lane per send (send s of a host: draws 2s, 2s + 1
    // after its state, by the jump-ahead table); a draw selecting no host
    // marks the host, which one lane then redraws in order (skip_fix)
    const bool gskip = gossip_rec && d.skip && d.pair_fmt != PAIR_DELAY && d.nskip > d.load * GMW * 32 &&
                       d.gskip_on;
    // the gossip flat pass (below): one lane per receipt, up to GFE per lane;
    // in the event image's last records, per host (by partition slot) its
    // digest terms' sum, first receipts, the messages it received and its
    // active index, and per receipt (by host and rank) a first-receipt flag
    constexpr uint32_t GFE = 2;
    const uint32_t gfrec = (32 * HP + 4 * n + 15) / 16;
    const bool gflat = gskip && in_lds && d.gflat && n <= GFE * K2_T && d.EVL >= n + gfrec;
    unsigned long long* s_hdig = reinterpret_cast<unsigned long long*>(s_ev + d.EVL) - (gflat ? HP : 0u);
    uint32_t* s_hcnt = reinterpret_cast<uint32_t*>(s_hdig) - (gflat ? HP : 0u);
    uint32_t* s_jof = s_hcnt - (gflat ? HP : 0u);
    uint32_t* s_hsw = s_jof - (gflat ? GMW * HP : 0u);  // [HP][GMW]
    uint32_t* s_ef = s_hsw - (gflat ? n : 0u);
    // exclusive scan of (count, active) over the HP hosts, HP/K2_T per thread
    const uint32_t per = (HP + K2_T - 1) / K2_T;
    const uint32_t h0 = tid * per, hs = 1;  // (strided hosts measured: no change, profiles/r04/insert_pre)
    uint64_t mine = 0;
    for (uint32_t j = 0; j < per; ++j) {
        const uint32_t h = h0 + j * hs;
        if (h < HP) {
            const uint32_t c = s_n[h];
            mine += ((uint64_t)c << 32) | (c ? 1u : 0u);
        }
    }
    uint64_t tot;
    uint64_t run = block_excl_scan_2x32<SG_SORT_LB != 0 && FLAT>(mine, s16, &tot);
    for (uint32_t j = 0; j < per; ++j) {
        const uint32_t h = h0 + j * hs;
        if (h < HP) {
            const uint32_t c = s_n[h];
            s_c[h] = (uint32_t)(run >> 32);
            if (c) s_act[(uint32_t)run] = (uint16_t)h;
            if (gflat) {  // uniform: the gossip flat pass's per-host words
                s_jof[h] = (uint32_t)run;
                s_hdig[h] = 0;
                s_hcnt[h] = 0;
#pragma unroll
                for (uint32_t w = 0; w < GMW; ++w) s_hsw[h * GMW + w] = 0;
            }
            run += ((uint64_t)c << 32) | (c ? 1u : 0u);
        }
    }
    const uint32_t nact = (uint32_t)tot;
    sort_barrier();
    if (stamp && tid == 0) stamp[22] = __builtin_amdgcn_s_memrealtime();
    const uint32_t sbase = p * HP;  // the partition's first local slot
    // phase A's first host of every lane: state loads issued now, under the
    // LDS scatter below (profiles/r02/knobs/prefetch_ab.log: 57.6 against 58.3
    // us/round with conditional loads of the first two hosts)
    // the lane's first host only (the second is rare), loaded unconditionally
    // from a clamped slot: a conditional load is waited for where it is issued
    constexpr uint32_t NPRE = 1;
    if (!flat) {  // uniform
        const ulonglong2* hsw = reinterpret_cast<const ulonglong2*>(d.hs);
        uint32_t l0 = sbase + s_act[tid < nact ? tid : 0u];
        l0 = l0 < d.L ? l0 : d.L - 1;
        pre_a0 = ld_stream2(&hsw[2 * (size_t)l0]);
        pre_b0 = ld_stream2(&hsw[2 * (size_t)l0 + 1]);
    }
    if (tid == 0) d.pcnt[p] = 0;  // consumed; the next k_scatter's gather refills it
    if (p == d.P - 1) reset_consumed(d);  // stores only (the last partition is the lightest)
    if (in_lds) {
#pragma unroll
        for (uint32_t q = 0; q < EPTF; ++q) {
            if (!rq_ok(q)) continue;
            const uint32_t hl = (uint32_t)(rr[q].a >> 52);
            if (hl >= HP) continue;
            const uint32_t pos = atomicAdd(&s_c[hl], 1u);
            if (pos < n) s_ev[pos] = rr[q];
        }
    } else {
        for (uint32_t i = tid; i < n; i += K2_T) {
            const Rec r = part[pidx(i)];
            const uint32_t hl = (uint32_t)(r.a >> 52);
            if (hl >= HP) continue;
            const uint32_t pos = atomicAdd(&s_c[hl], 1u);
            if (pos < n) part2[pos] = r;
        }
    }
#if SG_ROWS_GLDS
    // the rows' LDS-DMA (and the flat pass's state reads) have landed
    if (ROWS || flat) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
    if constexpr (ROWS) {
#pragma unroll
        for (uint32_t q = 0; q < RQ; ++q) {
            const uint32_t i = tid + q * K2_T;
            if (i < nwords) reinterpret_cast<uint32_t*>(dyn + d.row_off)[i] = rw[q];
        }
    }
    if (flat) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the flat pass's state reads have returned
#endif
    __syncthreads();  // the grouped events (and rows) are read back by other lanes
    if (stamp && tid == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();

    Acc a;
#pragma unroll
    for (int i = 0; i < NPCTR; ++i) a.ctr[i] = 0;
    a.jmin = UINT64_MAX;
    a.emin = SIMTIME_MAX;
    a.overflow = false;
    Rec* xs = d.extras + ((size_t)p * K2_T + tid) * XCAP;
    Rec* snd = d.sends + (size_t)p * d.ECAP;
    // Send records (phase A writes, phase B resolves, phase C commits) live in
    // the event image's unused tail while they fit, in HBM beyond it: phases
    // B and C then read them at LDS latency.
    Rec* s_snd = s_ev + (in_lds ? n : 0u);
    const uint32_t lcap = d.snd_lds ? (in_lds ? d.EVL - n - (gflat ? gfrec : 0u) : d.EVL) : 0u;
    // The HBM side uses a different instruction (non-temporal) from the LDS
    // side, so the compiler cannot merge the two into one flat access: a flat
    // store counts on vmcnt as well, and every later LDS access then waited
    // vmcnt(0) — for all of the wave's outstanding global stores — behind it
    // (2-3 us of the gossip flat pass and phases B / C, profiles/r06/g8).
    typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
    // The HBM side's load is waited for where it is issued: left pending, its
    // register made every use of sget's result wait vmcnt(0) on the LDS side
    // too, i.e. for all of the wave's outstanding stores.
    auto sget = [&](uint32_t i) __attribute__((always_inline)) {
        if (i < lcap) return s_snd[i];
        const u64x2_t v = __builtin_nontemporal_load(reinterpret_cast<const u64x2_t*>(snd + i));
        if (SG_SGET_WAIT) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (expcnt, lgkmcnt left)
        return Rec{v.x, v.y};
    };
    auto sput = [&](uint32_t i, const Rec& r) __attribute__((always_inline)) {
        if (i < lcap) {
            s_snd[i] = r;
        } else {
            u64x2_t v;
            v.x = r.a;
            v.y = r.k;
            __builtin_nontemporal_store(v, reinterpret_cast<u64x2_t*>(snd + i));
        }
    };
    const int32_t last = s_last;

    // ---- phase A (segments in LDS or in part2: two instantiations)
    const uint64_t W = d.W, bS = rs_bS;
    const uint32_t bSr = (uint32_t)(bS % R);
    const bool self_possible = E - S > d.vself_min;
    // few due events (a small shard): every host records its sends and the
    // fused pass resolves them one lane each (shorter than the inline chain)
    const uint32_t lmax = d.pair_fmt == PAIR_DELAY && n + nact <= d.rec_all ? 0u : d.light_max;
    bool horizon = false;
    const uint64_t bSW = bS * W;
    auto count_local = [&](uint64_t t) {  // one staged local event into the bucket bins
        if (!bin_time(d, t, bS, bSW, bSr, s_bc, s_bm)) horizon = true;
    };
    uint32_t nacta = nact;  // the hosts phase A takes: s_act[0, nacta)

    uint32_t gsw[GMW];
    // A seen word by a runtime index, as selects of register values: left to
    // itself the compiler turned the select chain into an indexed private
    // array, i.e. a scratch store of the four words and a scratch load per
    // access — a memory round trip per receipt in phase A's gossip loops.
    // opaque() keeps every word a register value.
    static_assert(GMW == 4, "four seen words");
    auto gword = [](const uint32_t (&w)[GMW], uint32_t i) __attribute__((always_inline)) {
        const uint32_t w0 = opaque(w[0]), w1 = opaque(w[1]), w2 = opaque(w[2]), w3 = opaque(w[3]);
        return i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
    };
    auto gset = [](uint32_t (&w)[GMW], uint32_t i, uint32_t v) __attribute__((always_inline)) {
        w[0] = opaque(i == 0 ? v : w[0]);
        w[1] = opaque(i == 1 ? v : w[1]);
        w[2] = opaque(i == 2 ? v : w[2]);
        w[3] = opaque(i == 3 ? v : w[3]);
    };
    auto phase_a = [&](auto seg_in_lds) __attribute__((always_inline)) {
        Rec* segs = decltype(seg_in_lds)::value ? s_ev : part2;
#pragma unroll 1
        for (uint32_t q = 0; q < HPT; ++q) {
            const uint32_t j = tid + q * K2_T;
            if (__builtin_amdgcn_readfirstlane(tid & ~63u) + q * K2_T >= nacta) break;  // wave-uniform
            bool go = false;  // this lane records sends (phase B/C path)
            uint32_t ns = 0, cnt = 0, lh = 0;
            Rec* seg = nullptr;
            HostCtx c;
            const bool st0 = stamp && tid == 0 && q == 0;
            if (stamp && tid == 0 && q == 1) stamp[23] = __builtin_amdgcn_s_memrealtime();
            if (j < nacta && !(s_n[s_act[j]] & GF_DONE)) {  // (the gossip flat pass's hosts are done)
                s_sb[j] = UINT32_MAX;
                const uint32_t hl = s_act[j];
                cnt = s_n[hl] & ~NULL_DRAW;
                seg = segs + (s_c[hl] - cnt);
                lh = sbase + hl;  // local slot
                c.sg = d.lo + lh;
                if (lh >= d.L) {
                    a.overflow = true;
                } else {
                    if (q < NPRE && !flat) {  // selects of values, not of addresses
                        host_load(c, make_ulonglong2(opaque(pre_a0.x), opaque(pre_a0.y)),
                                  make_ulonglong2(opaque(pre_b0.x), opaque(pre_b0.y)));
                    } else {
                        const ulonglong2* hw = reinterpret_cast<const ulonglong2*>(d.hs + lh);
                        host_load(c, hw[0], hw[1]);
                    }
                    s_vh[j] = c.vh;
                    // the vertex's self delay only when some vertex's could land
                    // inside this window (uniform; never in steady C4 rounds)
                    const uint64_t self_delay = self_possible ? d.vself[c.vh] : 0;
                    ++a.ctr[C_ACTIVE];
                    if (st0) stamp[8] = wait_stamp();
                    sort_segment(seg, cnt);  // pop order
                    if (st0) stamp[9] = wait_stamp();
                    // gossip hosts record their forwards for phases B / C (their
                    // loads one lane per send) unless a boot event or a same-round
                    // self event needs the sequential body
                    bool gos = gossip_rec && !(self_possible && S + (seg[0].a & M52) + self_delay < E);
                    for (uint32_t i = 0; gos && i < cnt; ++i) {
                        const uint64_t bk = seg[i].k;
                        gos = !(((uint32_t)(bk >> SRC_SHIFT) == c.h) & ((bk & SEQ_MASK) == 0));
                    }
                    if (gos) {
                        // forwards, at most: a message's first receipt (in the
                        // host's seen set as the round leaves it so far) sends to
                        // `load` peers; the record path pads the draws that select
                        // no host.  The seen words stay in registers until the
                        // host's records are written.
#pragma unroll
                        for (uint32_t w = 0; w < GMW; ++w) gsw[w] = w < d.mw ? d.seen[(size_t)lh * d.mw + w] : 0u;
                        uint32_t tmp[GMW];
#pragma unroll
                        for (uint32_t w = 0; w < GMW; ++w) tmp[w] = gsw[w];
                        for (uint32_t i = 0; i < cnt; ++i) {
                            const uint32_t msg = (uint32_t)(seg[i].k & 0xFFFFu), bit = 1u << (msg & 31);
                            const uint32_t wv = gword(tmp, msg >> 5);
                            ns += wv & bit ? 0u : d.load;
                            gset(tmp, msg >> 5, wv | bit);
                        }
                        go = true;
                    } else if (d.workload != SG_WORKLOAD_PHOLD ||
                               (self_possible && S + (seg[0].a & M52) + self_delay < E)) {
                        // sequential body: a self event may land inside this window
                        uint32_t nx = 0;
                        auto append = [&](uint64_t trel, uint64_t key) -> bool {
                            if (nx >= XCAP) return false;
                            xs[nx++] = Rec{trel, key};
                            return true;
                        };
                        uint32_t nl = cnt, i0 = 0;
                        for (;;) {
                            Best b{UINT64_MAX, 0, UINT32_MAX};
                            for (uint32_t i = i0; i < nl; ++i) {
                                const Rec r = seg[i];
                                best_take(b, r.a & M52, r.k, i);
                            }
                            for (uint32_t i = 0; i < nx; ++i) {
                                const Rec r = xs[i];
                                best_take(b, r.a, r.k, 0x80000000u | i);
                            }
                            if (b.slot == UINT32_MAX) break;
                            if (b.slot & 0x80000000u) {
                                const uint32_t i = b.slot & 0x7FFFFFFFu;
                                --nx;
                                if (i != nx) xs[i] = xs[nx];
                            } else {
                                --nl;
                                if (b.slot != nl) seg[b.slot] = seg[nl];
                            }
                            execute_event(d, S, E, p, c, a, S + b.t, b.k, sh, append, count_local);
                        }
                        reinterpret_cast<ulonglong2*>(d.hs + lh)[0] =
                            make_ulonglong2(hs_w0(c.s.rng, c.h), hs_w1(c.s.pops, c.vh));
                        reinterpret_cast<ulonglong2*>(d.hs + lh)[1] = make_ulonglong2(c.s.digest, c.s.evc);
                    } else {
                        // this host's sends, at most: a draw that selects no host
                        // (test_phold.c:176-177) sends nothing, so the path is
                        // picked without the draws; the record path pads for them
                        for (uint32_t i = 0; i < cnt; ++i) {
                            const uint64_t bk = seg[i].k;
                            const bool boot = ((uint32_t)(bk >> SRC_SHIFT) == c.h) & ((bk & SEQ_MASK) == 0);
                            ns += boot ? d.load : 1u;
                        }
                        if (ns <= lmax && q < d.light_q) {
                            // light host (most hosts in steady state): the whole
                            // body here, both sends' loads in flight together
                            int32_t x0 = 0, x1 = 0, c0 = 0, c1 = 0;
                            uint64_t t0 = 0, t1 = 0;
                            uint32_t nsd = 0;
                            pop_segment(d, rs, S, c, a, seg, cnt, last, [&](int32_t x, int32_t ch, uint64_t trel) {
                                if (nsd == 0) {
                                    x0 = x;
                                    c0 = ch;
                                    t0 = trel;
                                } else {
                                    x1 = x;
                                    c1 = ch;
                                    t1 = trel;
                                }
                                ++nsd;
                            });
                            if (st0) stamp[16] = wait_stamp();
                            // loads issued unconditionally (unused sends read host 0's
                            // record): a load under a runtime condition makes hipcc
                            // branch around it and wait for it before the next one
                            const uint32_t g0 = dst_guess(d, x0), g1 = dst_guess(d, x1);
                            uint32_t vd0 = 0, vd1 = 0, dst0 = 0, dst1 = 0;
                            if constexpr (EXACT) {  // records g and g + 1: threshold, vertex, slot
                                const uint2 a0 = d.nearw[g0], b0 = d.nearw[g0 + 1];
                                const uint2 a1 = d.nearw[g1], b1 = d.nearw[g1 + 1];
                                near_resolve(d, x0, a0, b0, vd0, dst0);
                                near_resolve(d, x1, a1, b1, vd1, dst1);
                            } else {
                                const Probe pb0 = dst_probe(d, g0), pb1 = dst_probe(d, g1);
                                dst0 = nsd > 0 ? dst_resolve(d, x0, g0, pb0, vd0) : 0;
                                dst1 = nsd > 1 ? dst_resolve(d, x1, g1, pb1, vd1) : 0;
                            }
                            if (st0) stamp[17] = wait_stamp();
                            asm volatile("" ::: "memory");  // both pair loads after both resolves
                            const PairRec pr0 = pair_of(c.vh, vd0, want_jump);
                            const PairRec pr1 = pair_of(c.vh, vd1, want_jump);
                            if (st0) stamp[18] = wait_stamp();
                            commit_two(d, S, E, p, c, a, sh, nsd, S + t0, c0, dst0, vd0, pr0, S + t1, c1, dst1, vd1, pr1,
                                       count_local);
                            ulonglong2* hp = reinterpret_cast<ulonglong2*>(d.hs + lh);
                            st_rec(d.hs, (size_t)lh * 32, hs_w0(c.s.rng, c.h), hs_w1(c.s.pops, c.vh));
                            if (st0) stamp[19] = wait_stamp();
                            st_rec(d.hs, (size_t)lh * 32 + 16, c.s.digest, c.s.evc);
                            ns = 0;
                        } else {
                            go = true;
                        }
                    }
                }
            }
            if (st0) stamp[10] = wait_stamp();
            // a header record {evc, HDR | host} then the sends: phase C needs no
            // state load
            const uint32_t base = wave_reserve(&s_nsend, go ? ns + 1 : 0u);  // wave converged here
            if (st0) stamp[11] = wait_stamp();
            if (stamp && tid == 0 && q == 1) stamp[25] = wait_stamp();
            if (!go) continue;
            if (base + ns + 1 > d.ECAP) {
                a.overflow = true;
                continue;
            }
            if (ns > 0xFFFFu) {
                a.overflow = true;
                continue;
            }
            s_sb[j] = base;
            s_vh[j] = c.vh | (ns << 16);
            // (gskip: the header also keeps the state before the draws, bits 32-63)
            sput(base, Rec{c.s.evc | (gskip ? (uint64_t)c.s.rng << 32 : 0ull), HDR_REC | ((uint64_t)j << 32) | c.h});
            uint32_t k = base + 1;
            if (gossip_rec) {  // (a lane on this path with gossip took the gossip record path)
                // the gossip body's draws (orc.c execute_gossip): trace digest,
                // then per first receipt `load` sends, each a destination draw and,
                // when it selects a host, the reliability draw (worker.c:268-269);
                // the message id rides in the record (bits 40-51)
                if (st0) stamp[16] = __builtin_amdgcn_s_memrealtime();  // (the light path's slots: unused here)
                const uint32_t rng0 = c.s.rng;
                for (uint32_t i = 0; i < cnt; ++i) {
                    const Rec ev = seg[i];
                    const uint64_t trel = ev.a & M52, bt = S + trel;
                    const uint32_t bsrc = (uint32_t)(ev.k >> SRC_SHIFT);
                    const uint64_t bseq = (ev.k & SEQ_MASK) >> d.msg_shift;
                    const uint32_t msg = (uint32_t)(ev.k & 0xFFFFu), bit = 1u << (msg & 31);
                    c.s.digest += digest_mix(c.s.pops, bt, bsrc, bseq);
                    if (d.trace) {
                        const uint64_t ts = atomicAdd((unsigned long long*)&rs->trace_len, 1ULL);
                        if (ts < d.trace_cap) {
                            sg_trace_rec tr;
                            tr.time = bt;
                            tr.seq = bseq;
                            tr.host = c.h;
                            tr.src = bsrc;
                            tr.pos = c.s.pops;
                            d.trace[ts] = tr;
                        } else {
                            a.overflow = true;
                        }
                    }
                    ++c.s.pops;
                    ++a.ctr[C_POPS];
                    const uint32_t wv = gword(gsw, msg >> 5);
                    if (wv & bit) continue;  // a duplicate: the pop still commits
                    gset(gsw, msg >> 5, wv | bit);
                    if (gskip) {  // {state before the draws, send index}: drawn after phase A
                        for (uint32_t m = 0; m < d.load; ++m, ++k)
                            sput(k, Rec{((uint64_t)j << 52) | ((uint64_t)msg << 40) | trel,
                                        (uint64_t)rng0 | ((uint64_t)(k - base - 1) << 32)});
                        a.ctr[C_SENDS] += d.load;
                        continue;
                    }
                    for (uint32_t m = 0; m < d.load; ++m) {
                        const int32_t x = dev_rand_r(c.s.rng);
                        if (x > last) {  // no host selected (test_phold.c:176-177)
                            ++a.ctr[C_NULL];
                            continue;
                        }
                        const int32_t ch = dev_rand_r(c.s.rng);  // worker.c:268-269
                        ++a.ctr[C_SENDS];
                        sput(k++, Rec{((uint64_t)j << 52) | ((uint64_t)msg << 40) | trel,
                                      (uint64_t)(uint32_t)x | ((uint64_t)(uint32_t)ch << 32)});
                    }
                }
                if (gskip) {  // the state after every send's two draws (skip_fix redoes a null)
                    const uint32_t si = k - base - 1;
                    if (si >= d.nskip) flag(d, OV_BUG | GSK_A);
                    const uint2 sk = d.skip[si < d.nskip ? si : 0u];
                    c.s.rng = sk.x * rng0 + sk.y;
                }
                if (st0) stamp[17] = __builtin_amdgcn_s_memrealtime();
#pragma unroll
                for (uint32_t w = 0; w < GMW; ++w)
                    if (w < d.mw) d.seen[(size_t)lh * d.mw + w] = gsw[w];
            } else {
                pop_segment(d, rs, S, c, a, seg, cnt, last, [&](int32_t x, int32_t ch, uint64_t trel) {
                    sput(k++, Rec{((uint64_t)j << 52) | trel, (uint64_t)(uint32_t)x | ((uint64_t)(uint32_t)ch << 32)});
                });
            }
            const uint32_t nreal = k - base - 1;  // sends with a destination
            for (; k <= base + ns; ++k) sput(k, Rec{0, HDR_REC | PAD_REC});  // draws that selected no host
            // {rng, pops, digest} now; evc now too when every send is kept, else
            // after phase C
            HostState* hp = d.hs + lh;
            reinterpret_cast<ulonglong2*>(hp)[0] = make_ulonglong2(hs_w0(c.s.rng, c.h), hs_w1(c.s.pops, c.vh));
            if (d.pair_fmt == PAIR_DELAY) {  // every send kept: the final counter is known now
                reinterpret_cast<ulonglong2*>(hp)[1] = make_ulonglong2(c.s.digest, c.s.evc + nreal);
            } else {
                hp->digest = c.s.digest;
            }
            if (st0 && gossip_rec) stamp[18] = __builtin_amdgcn_s_memrealtime();
            if (st0) stamp[12] = wait_stamp();
            if (stamp && tid == 0 && q == 1) stamp[24] = wait_stamp();
        }
    };
    // ---- flat pass: one lane per due event (the lane's own records, still in
    // registers).  A host's events are independent once each knows its rank
    // in the host's pop order: the rand_r draws of the events before it are
    // replayed (pure arithmetic, one send per event, test_phold.c:310-312;
    // a draw selecting no host consumes one draw, not two), its trace digest
    // term is additive given its position, and its srcHostEventID is the
    // host's counter plus the kept sends before it.  The host's last event
    // writes the state; a host with several events adds the digest terms
    // with atomics.  Hosts flat_ok rejects are listed (their rank-0 event's
    // lane appends them to s_act, which only phase A reads from here on) and
    // run phase A.  A lane's two events are resolved together: both
    // destination loads in flight at once.
    __shared__ uint32_t s_nser;
    bool ser = !flat;
    if (flat) {
        // skip-ahead pays where hosts carry several due events (configs[1]:
        // 16 each); with about one per host (configs[3]) the barrier the
        // null-draw check needs costs more than the few replays it saves
        const bool use_skip = d.skip && n >= 2 * nact;  // uniform
        if (tid == 0) s_nser = 0;
        __syncthreads();
        // what stage 3 needs of an event, kept small (two are live at once)
        enum : uint32_t { F_OK = 1, F_SND = 2, F_LAST = 4, F_MULTI = 8, F_FIRST = 16 };
        struct FlatEv {
            uint32_t hl, h, vh, rng, g, flags;
            int32_t x, ch;
            uint64_t bt;
            uint64_t pops_end;  // the host's pops after the round (its last event writes it)
            uint64_t sq;        // this send's srcHostEventID
            uint64_t term;      // digest term; one-event host: the new digest
        };
        // stage 1: place in the host's order, replay, draws (LDS and ALU only)
        auto flat_draw = [&](const Rec& ev, bool valid, ulonglong2 w01, ulonglong2 w23)
            __attribute__((always_inline)) {
            FlatEv f;
            f.hl = (uint32_t)(ev.a >> 52);
            f.flags = 0;
            f.x = 0;
            f.g = 0;
            f.vh = 0;
            if (!valid || f.hl >= HP) return f;  // past the count / flagged by the histogram
            const uint32_t cnt = s_n[f.hl] & ~NULL_DRAW;  // (the skip path's mark: below)
            const uint64_t et = ev.a & M52;
            const SegScan sc = seg_scan(s_ev + (s_c[f.hl] - cnt), cnt, et, ev.k);
            f.h = (uint32_t)(w01.x >> 32);
            f.vh = (uint32_t)(w01.y >> 48);
            if (!flat_ok(d, cnt, sc, self_possible, S, E, f.vh)) {
                if (sc.rank == 0) s_act[atomicAdd(&s_nser, 1u)] = (uint16_t)f.hl;  // phase A takes it
                return f;
            }
            f.flags = F_OK | (sc.rank + 1 == cnt ? F_LAST : 0u) | (cnt > 1 ? F_MULTI : 0u) |
                      (sc.rank == 0 ? F_FIRST : 0u);
            uint32_t rng = (uint32_t)w01.x;
            const uint64_t pops0 = w01.y & M48;
            f.pops_end = pops0 + cnt;
            uint32_t before = 0;  // sends of the host's earlier events (all kept: flat_ok)
            if (use_skip) {  // two draws per earlier event, skipped in one step
#if SG_SKIP_LDS
                const uint2 sk = s_skipf[sc.rank];  // rank < cnt <= FLAT_CMAX (flat_ok)
#else
                const uint2 sk = d.skip[sc.rank];
#endif
                rng = sk.x * rng + sk.y;
                before = sc.rank;
            } else {
                for (uint32_t k = 0; k < sc.rank; ++k) {
                    if (dev_rand_r(rng) <= last) {
                        (void)dev_rand_r(rng);
                        ++before;
                    }
                }
            }
            f.sq = w23.y + before;  // event.c:38: the counter plus the kept sends before
            f.bt = S + et;
            const uint32_t bsrc = (uint32_t)(ev.k >> SRC_SHIFT);
            const uint64_t bseq = ev.k & SEQ_MASK;
            f.term = digest_mix(pops0 + sc.rank, f.bt, bsrc, bseq);
            if (sc.rank + 1 == cnt) f.term += w23.x;  // the last event: the old digest + its term
            if (d.trace) {
                const uint64_t ts = atomicAdd((unsigned long long*)&rs->trace_len, 1ULL);
                if (ts < d.trace_cap) {
                    sg_trace_rec tr;
                    tr.time = f.bt;
                    tr.seq = bseq;
                    tr.host = f.h;
                    tr.src = bsrc;
                    tr.pos = pops0 + sc.rank;
                    d.trace[ts] = tr;
                } else {
                    a.overflow = true;
                }
            }
            ++a.ctr[C_POPS];
            a.ctr[C_ACTIVE] += sc.rank == 0 ? 1u : 0u;
            f.x = dev_rand_r(rng);
            const bool snd = f.x <= last;  // test_phold.c:176-177
            f.flags |= snd ? F_SND : 0u;
            // skip path: a draw selecting no host shifts every later event's
            // draws by one; the host is marked (and replayed in phase A)
            if (use_skip && !snd && sc.rank + 1 < cnt) atomicOr(&s_n[f.hl], NULL_DRAW);
            f.ch = 0;
            if (snd) f.ch = dev_rand_r(rng);  // worker.c:268-269
            f.rng = rng;
            f.g = dst_guess(d, f.x);
            return f;
        };
        // stage 3: the send's tests and staging, the host's state (stores and
        // LDS atomics only: nothing after it waits for a global load)
        auto flat_send = [&](const FlatEv& f, uint32_t vd, uint32_t dst, const PairRec& pr)
            __attribute__((always_inline)) {
            if (!(f.flags & F_OK)) return;
            bool kept = false;
            if (f.flags & F_SND) {
                ++a.ctr[C_SENDS];
                kept = f.bt < d.bootstrap_end || f.ch <= pr.keep;  // worker.c:268-273
                if (!kept) {
                    ++a.ctr[C_DROPREL];
                } else {
                    if (d.pcount) atomicAdd(&d.pcount[(size_t)f.vh * d.V + vd], 1u);  // worker.c:279
                    uint64_t tn = f.bt + pr.delay;        // worker.c:275-277
                    const uint64_t sq = f.sq;             // event.c:38
                    if (sq >> SRC_SHIFT) a.overflow = true;
                    if (tn >= d.end_time) {               // scheduler.c:343-346
                        ++a.ctr[C_DROPEND];
                    } else {
                        const uint32_t sg = d.lo + sbase + f.hl;
                        if (dst == sg && tn < E) a.overflow = true;  // excluded by flat_ok
                        if (dst != sg && tn < E) {                   // host_single.c:180-184
                            tn = E;
                            ++a.ctr[C_BUMPED];
                        }
                        if (stage_event(d, S, p, sh, a, dst, tn, ((uint64_t)f.h << SRC_SHIFT) | sq)) count_local(tn);
                    }
                }
            } else {
                ++a.ctr[C_NULL];
            }
            HostState* hp = d.hs + sbase + f.hl;
            if (f.flags & F_LAST) {  // the host's last event: its state after the round
                const uint64_t evc = f.sq + (kept ? 1u : 0u);
                ulonglong2* hw = reinterpret_cast<ulonglong2*>(hp);
                st_rec(d.hs, (size_t)(sbase + f.hl) * 32, hs_w0(f.rng, f.h), hs_w1(f.pops_end, f.vh));
                if (!(f.flags & F_MULTI)) st_rec(d.hs, (size_t)(sbase + f.hl) * 32 + 16, f.term, evc);
                else hp->evc = evc;  // the digest after the barrier below
            } else {  // an earlier event of a multi-event host (ok: F_MULTI)
                atomicAdd(&s_dig[f.hl], (unsigned long long)f.term);
            }
        };
        const bool stf = stamp && tid == 0;
        if (stf) stamp[16] = __builtin_amdgcn_s_memrealtime();
        FlatEv f0 = flat_draw(rr[0], rq_ok(0), pre_a0, pre_b0);
        FlatEv f1 = flat_draw(rr[1], rq_ok(1), pre_a1, pre_b1);
        if (use_skip) {
            // a host whose draws the skip-ahead miscounted goes to phase A
            // (its rank-0 lane lists it), its events here are dropped
            lds_barrier();  // every mark is in
            auto unflat = [&](FlatEv& f) __attribute__((always_inline)) {
                if (!(f.flags & F_OK) || !(s_n[f.hl] & NULL_DRAW)) return;
                --a.ctr[C_POPS];
                if (f.flags & F_FIRST) {
                    --a.ctr[C_ACTIVE];
                    s_act[atomicAdd(&s_nser, 1u)] = (uint16_t)f.hl;
                }
                f.flags = 0;
            };
            unflat(f0);
            unflat(f1);
        }
        if (stf) stamp[17] = wait_stamp();
        // stage 2: both events' destination records in flight together
        // (unconditional loads; an unused one reads record 0's line), resolved
        // and pinned here: a value resolved after the first store would wait
        // for that store too (vmcnt counts in order)
        uint32_t vd0 = 0, vd1 = 0, dst0 = 0, dst1 = 0;
        if constexpr (EXACT) {
            const uint2 a0 = d.nearw[f0.g], b0 = d.nearw[f0.g + 1];
            const uint2 a1 = d.nearw[f1.g], b1 = d.nearw[f1.g + 1];
            near_resolve(d, f0.x, a0, b0, vd0, dst0);
            near_resolve(d, f1.x, a1, b1, vd1, dst1);
        } else {
            const Probe pb0 = dst_probe(d, f0.g), pb1 = dst_probe(d, f1.g);
            dst0 = (f0.flags & F_OK) && (f0.flags & F_SND) ? dst_resolve(d, f0.x, f0.g, pb0, vd0) : 0u;
            dst1 = (f1.flags & F_OK) && (f1.flags & F_SND) ? dst_resolve(d, f1.x, f1.g, pb1, vd1) : 0u;
        }
        vd0 = opaque(vd0);
        vd1 = opaque(vd1);
        dst0 = opaque(dst0);
        dst1 = opaque(dst1);
        const PairRec pr0 = pair_of(f0.vh, vd0, want_jump), pr1 = pair_of(f1.vh, vd1, want_jump);
        // path discovery (topology.c:1374-1385) folded here, before the stores
        // (the discovered-ms loads run only while the minimum can still fall)
        constexpr uint32_t F_SENDS = F_OK | F_SND;
        if ((f0.flags & F_SENDS) == F_SENDS) a.jmin = pr0.jump < a.jmin ? pr0.jump : a.jmin;
        if ((f1.flags & F_SENDS) == F_SENDS) a.jmin = pr1.jump < a.jmin ? pr1.jump : a.jmin;
        a.jmin = opaque(a.jmin);
        if (stf) stamp[18] = wait_stamp();
        flat_send(f0, vd0, dst0, pr0);
        flat_send(f1, vd1, dst1, pr1);
        if (stf) stamp[19] = wait_stamp();
#if SG_FLAT_LDSB
        // LDS only (s_dig, s_nser): no lane reads another's global stores from
        // here on (phase A takes hosts the flat pass did not write), so the
        // staging and state stores drain under the rest of the kernel
        lds_barrier();
#else
        __syncthreads();
#endif
        // a multi-event host's digest: the last event's lane adds the others'
        // terms (LDS; global atomics on the state's line next to the state
        // stores cost about 10 us per round, profiles/r03/flat)
        if ((f0.flags & (F_LAST | F_MULTI)) == (F_LAST | F_MULTI))
            d.hs[sbase + f0.hl].digest = f0.term + s_dig[f0.hl];
        if ((f1.flags & (F_LAST | F_MULTI)) == (F_LAST | F_MULTI))
            d.hs[sbase + f1.hl].digest = f1.term + s_dig[f1.hl];
        nacta = s_nser;
        ser = nacta != 0;
        if (ser) __syncthreads();  // phase A reuses s_vh / s_sb
        if (stf) stamp[30] = __builtin_amdgcn_s_memrealtime();
    }
    // ---- gossip flat pass (configs[4]): one lane per receipt, where phase A
    // takes one lane per host (the heaviest host of a wave sets its time, and
    // ~400 hosts fill 6 of 16 waves).  A receipt's place in its host's order
    // is independent of the others once it knows (orc.c execute_gossip,
    // worker.c:268-273, event.c:38):
    //   its rank in the host's pop order (event_compare over the host's due
    //   events in LDS), hence its trace position pops + rank and digest term;
    //   whether it is the host's first receipt of its message (not in the seen
    //   set as the round found it, no lower-ranked receipt of it) — a first
    //   receipt forwards to `load` peers;
    //   the forwards ranked before it (load x the first receipts of lower
    //   rank), hence its sends' indices: send s of the host draws 2s, 2s + 1
    //   after the host's state (the jump-ahead table, drawn after this pass as
    //   on the record path).
    // Pass 1 ranks and classifies (s_ef); pass 2: each host's rank-0 lane
    // reserves its records (a header and load x firsts sends, exactly the
    // record path's layout) and publishes them through s_n / s_c; pass 3
    // writes the send records, and the host's last lane its state (rng after
    // the draws, pops, digest) and seen set.  A host with a boot event, or
    // one whose self event could land inside the window (host_single.c:
    // 237-267), keeps phase A's sequential body (s_nser counts them).
    if constexpr (!FLAT) {
        if (gflat) {  // uniform
            if (tid == 0) s_nser = 0;
            // Every global load is issued at the start (a host's {digest,
            // counter} and seen words by each of its lanes: the one that finds
            // itself rank 0 uses them); nothing after pass 1 waits for memory.
            // A host's state after its draws (rng) is written by the lane that
            // draws its last send (the draws pass after this one); a host with
            // no forwards keeps its rng.
            struct GfEv {
                Rec ev;
                uint32_t hl, cnt, start, rank;
                uint32_t rng0, h, vh, seenw;
                uint64_t pops0;
                bool valid, ok, first;
            };
            GfEv g[GFE];
            ulonglong2 w23x[GFE];
            uint32_t swx[GFE][GMW];
            const ulonglong2* hsw = reinterpret_cast<const ulonglong2*>(d.hs);
            const bool stf = stamp && tid == 0;
#pragma unroll
            for (uint32_t q = 0; q < GFE; ++q) {  // loads first, every one unconditional (clamped)
                const uint32_t i = tid + q * K2_T;
                g[q].valid = i < n;
                g[q].ev = s_ev[g[q].valid ? i : 0u];
                g[q].hl = (uint32_t)(g[q].ev.a >> 52);
                const uint32_t hl = g[q].hl < HP ? g[q].hl : 0u, lh = sbase + hl < d.L ? sbase + hl : 0u;
                const ulonglong2 w01 = hsw[2 * (size_t)lh];
                w23x[q] = hsw[2 * (size_t)lh + 1];
                g[q].rng0 = (uint32_t)w01.x;
                g[q].h = (uint32_t)(w01.x >> 32);
                g[q].pops0 = w01.y & M48;
                g[q].vh = (uint32_t)(w01.y >> 48);
#pragma unroll
                for (uint32_t w = 0; w < GMW; ++w) swx[q][w] = d.seen[(size_t)lh * d.mw + (w < d.mw ? w : 0u)];
            }
            // pass 1: rank, first receipt, the host's eligibility
#pragma unroll
            for (uint32_t q = 0; q < GFE; ++q) {
                GfEv& f = g[q];
                f.ok = f.first = false;
                f.rank = 0;
                if (!f.valid) continue;
                if (f.hl >= HP) {
                    flag(d, OV_BUG);
                    f.valid = false;
                    continue;
                }
                f.cnt = s_n[f.hl] & ~NULL_DRAW;
                f.start = s_c[f.hl] - f.cnt;
                const uint64_t et = f.ev.a & M52, ek = f.ev.k;
                const uint32_t msg = (uint32_t)(ek & 0xFFFFu);
                uint64_t tmin = et;
                bool boot = (ek & SEQ_MASK) == 0, dup = false;
                for (uint32_t k = 0; k < f.cnt; ++k) {
                    const Rec r = s_ev[f.start + k];
                    const uint64_t rt = r.a & M52;
                    const bool lt = key_less(rt, r.k, et, ek);
                    f.rank += lt ? 1u : 0u;
                    dup |= lt & ((uint32_t)(r.k & 0xFFFFu) == msg);
                    tmin = rt < tmin ? rt : tmin;
                    boot |= (r.k & SEQ_MASK) == 0;
                }
                f.ok = !boot && !(self_possible && S + tmin + d.vself[f.vh] < E);
                f.first = f.ok && !dup && !(gword(swx[q], msg >> 5) & (1u << (msg & 31)));
                // by rank: the host's receipts in pop order; the host's sums by
                // LDS atomics (its rank-0 lane reads them after the barrier)
                s_ef[f.start + f.rank] = f.first ? 1u : 0u;
                atomicAdd(&s_hdig[f.hl], (unsigned long long)digest_mix(f.pops0 + f.rank, S + et, (uint32_t)(ek >> SRC_SHIFT),
                                                                         (ek & SEQ_MASK) >> d.msg_shift));
                if (f.first) atomicAdd(&s_hcnt[f.hl], 1u);
                atomicOr(&s_hsw[f.hl * GMW + (msg >> 5) % GMW], 1u << (msg & 31));
            }
            if (stf) stamp[16] = __builtin_amdgcn_s_memrealtime();
            lds_barrier();
            if (stf) stamp[31] = __builtin_amdgcn_s_memrealtime();
            // pass 2: each host's rank-0 lane reserves its records, writes the
            // header and the host's state but the rng.  The start's loads are
            // taken into registers first, before any store: a use of them
            // after the stores made the compiler wait vmcnt(0), i.e. for those
            // stores too (vmcnt counts in order)
#pragma unroll
            for (uint32_t q = 0; q < GFE; ++q) {
                w23x[q].x = opaque(w23x[q].x);
                w23x[q].y = opaque(w23x[q].y);
#pragma unroll
                for (uint32_t w = 0; w < GMW; ++w) swx[q][w] = opaque(swx[q][w]);
            }
            // The records are reserved in converged code: a DPP scan of the
            // lane's two counts and one LDS atomic per wave (the compiler's
            // own aggregation of a divergent atomic walks the active lanes).
            uint32_t nres[GFE], tot = 0;
            bool anyser = false;
#pragma unroll
            for (uint32_t q = 0; q < GFE; ++q) {
                const GfEv& f = g[q];
                const bool lead = f.valid && f.rank == 0;
                const uint32_t nf = s_hcnt[f.hl < HP ? f.hl : 0u];
                nres[q] = lead && f.ok ? nf * d.load + 1u : 0u;
                anyser |= lead && !f.ok;  // phase A's sequential body takes it
                tot += nres[q];
            }
            if (anyser) s_nser = 1u;
            const uint32_t incl = wave_incl_scan_u32(tot);
            uint32_t rbase = 0;
            if ((tid & 63) == 63 && incl) rbase = atomicAdd(&s_nsend, incl);
            rbase = (uint32_t)__builtin_amdgcn_readlane((int)rbase, 63) + incl - tot;
#pragma unroll
            for (uint32_t q = 0; q < GFE; ++q) {
                const GfEv& f = g[q];
                if (nres[q] == 0) continue;
                const uint32_t base = rbase, ns = nres[q] - 1u;
                rbase += nres[q];
                const uint64_t dig = s_hdig[f.hl];
                uint32_t sw[GMW];
#pragma unroll
                for (uint32_t w = 0; w < GMW; ++w) sw[w] = swx[q][w] | s_hsw[f.hl * GMW + w];
                const uint32_t j = s_jof[f.hl];  // the host's active index
                const bool bad = j >= nact || s_act[j < nact ? j : 0u] != f.hl || ns > 0xFFFFu ||
                                 ns >= d.nskip || base + ns + 1 > d.ECAP;
                if (bad) {
                    a.overflow = true;
                    if (j < nact) s_sb[j] = UINT32_MAX;
                } else {
                    s_sb[j] = base;
                    s_vh[j] = f.vh | (ns << 16);
                    sput(base, Rec{w23x[q].y | ((uint64_t)f.rng0 << 32), HDR_REC | ((uint64_t)j << 32) | f.h});
                }
                ++a.ctr[C_ACTIVE];
                s_c[f.hl] = bad ? UINT32_MAX : base;
                s_n[f.hl] = GF_DONE | j;
                // the state after the round: pops, digest, seen set; the rng
                // here only when the host draws nothing (the last send's lane
                // writes it otherwise), the counter with phase C
                const uint32_t lh = sbase + f.hl;
                HostState* hp = d.hs + lh;
                if (ns == 0) reinterpret_cast<ulonglong2*>(hp)[0] = make_ulonglong2(hs_w0(f.rng0, f.h), hs_w1(f.pops0 + f.cnt, f.vh));
                else reinterpret_cast<uint64_t*>(hp)[1] = hs_w1(f.pops0 + f.cnt, f.vh);
                hp->digest = w23x[q].x + dig;
#pragma unroll
                for (uint32_t w = 0; w < GMW; ++w)
                    if (w < d.mw) d.seen[(size_t)lh * d.mw + w] = sw[w];
            }
            if (stf) stamp[17] = __builtin_amdgcn_s_memrealtime();
            lds_barrier();
            if (stf) stamp[18] = __builtin_amdgcn_s_memrealtime();
            // pass 3: the sends of every first receipt, and the trace
#pragma unroll
            for (uint32_t q = 0; q < GFE; ++q) {
                const GfEv& f = g[q];
                if (!f.valid || !f.ok) continue;
                const uint32_t base = s_c[f.hl], j = s_n[f.hl] & 0xFFFFu;
                const uint64_t trel = f.ev.a & M52, bt = S + trel;
                if (d.trace) {
                    const uint64_t ts = atomicAdd((unsigned long long*)&rs->trace_len, 1ULL);
                    if (ts < d.trace_cap) {
                        sg_trace_rec tr;
                        tr.time = bt;
                        tr.seq = (f.ev.k & SEQ_MASK) >> d.msg_shift;
                        tr.host = f.h;
                        tr.src = (uint32_t)(f.ev.k >> SRC_SHIFT);
                        tr.pos = f.pops0 + f.rank;
                        d.trace[ts] = tr;
                    } else {
                        a.overflow = true;
                    }
                }
                ++a.ctr[C_POPS];
                if (base == UINT32_MAX || !f.first) continue;  // (UINT32_MAX: overflow, flagged)
                uint32_t fb = 0;  // first receipts before this one
                for (uint32_t k = 0; k < f.rank; ++k) fb += s_ef[f.start + k];
                const uint64_t msg = f.ev.k & 0xFFFu;
                for (uint32_t m = 0; m < d.load; ++m) {
                    const uint32_t si = fb * d.load + m;  // the send's index in the host's list
                    sput(base + 1 + si, Rec{((uint64_t)j << 52) | (msg << 40) | trel,
                                            (uint64_t)f.rng0 | ((uint64_t)si << 32)});
                }
                a.ctr[C_SENDS] += d.load;
            }
            if (stf) stamp[19] = __builtin_amdgcn_s_memrealtime();
            lds_barrier();  // s_nsend, s_nser, the records
            if (stf) stamp[30] = __builtin_amdgcn_s_memrealtime();
            ser = s_nser != 0;
        }
    }
    if (!ser) {
    } else if (in_lds) phase_a(std::true_type{});
    else phase_a(std::false_type{});
    if (stamp && (tid & 63) == 0) stamp[26 + (tid >> 8)] = wait_stamp();  // waves 0, 4, 8, 12 done
    __syncthreads();
    if (stamp && tid == 0) stamp[2] = __builtin_amdgcn_s_memrealtime();

    // ---- phase B: one lane per send, two in flight (header records skipped)
    const uint32_t nsend = s_nsend < d.ECAP ? s_nsend : d.ECAP;
    // Delay-only path records (no loss): every send is kept, so a send's
    // srcHostEventID is its host's counter plus its place in the host's list
    // and phases B and C run as one pass (no barrier, no walk back).
    if (d.pair_fmt == PAIR_DELAY) {
        if (stamp && tid == 0) stamp[3] = __builtin_amdgcn_s_memrealtime();  // no phase B of its own
        for (uint32_t i = tid; i < nsend; i += K2_T) {
            const Rec r = sget(i);
            const int32_t x = (int32_t)(uint32_t)r.k;
            const uint32_t g = dst_guess(d, x);
            uint32_t vd = 0, dst = 0;
            if constexpr (EXACT) {
                const uint2 a0 = d.nearw[g], b0 = d.nearw[g + 1];
                near_resolve(d, x, a0, b0, vd, dst);
            } else {
                const Probe pb = dst_probe(d, g);
                dst = dst_resolve(d, x, g, pb, vd);
            }
            if (r.k & HDR_REC) continue;  // header and pad records: phase A wrote the counter
            const uint32_t j = (uint32_t)(r.a >> 52);
            const PairRec pr = pair_of(s_vh[j] & 0xFFFFu, vd, want_jump);
            const uint32_t sb = s_sb[j];
            const Rec hd = sget(sb);
            a.jmin = pr.jump < a.jmin ? pr.jump : a.jmin;  // topology.c:1374-1385
            if (d.pcount) atomicAdd(&d.pcount[(size_t)(s_vh[j] & 0xFFFFu) * d.V + vd], 1u);  // worker.c:279
            const uint64_t sq = hd.a + (i - sb - 1);   // event.c:38: the host's real sends precede its pads
            // gossip records carry the message id in bits 40-51 (the key's low bits)
            const uint64_t msg = gossip_rec ? (r.a >> 40) & 0xFFFu : 0u;
            uint64_t tn = S + (r.a & (gossip_rec ? M40 : M52)) + pr.delay;  // worker.c:275-277
            if (tn >= d.end_time) {                    // scheduler.c:343-346
                ++a.ctr[C_DROPEND];
                continue;
            }
            const uint32_t sg = d.lo + sbase + s_act[j];
            if (dst == sg && tn < E) a.overflow = true;  // excluded by the phase A test
            if (dst != sg && tn < E) {                   // host_single.c:180-184
                tn = E;
                ++a.ctr[C_BUMPED];
            }
            const uint32_t h = (uint32_t)hd.k;
            if (sq >> (SRC_SHIFT - d.msg_shift)) a.overflow = true;
            if (stage_event(d, S, p, sh, a, dst, tn, ((uint64_t)h << SRC_SHIFT) | (sq << d.msg_shift) | msg))
                count_local(tn);
        }
    } else {
        if (gskip) {  // uniform
            // the gossip records' draws, one lane per send (bounds-checked:
            // GSK_* name a guard that tripped)
            for (uint32_t i = tid; i < nsend; i += K2_T) {
                const Rec r = sget(i);
                if (r.k & HDR_REC) continue;
                const uint32_t si = (uint32_t)(r.k >> 32), jr = (uint32_t)(r.a >> 52);
                if (si >= d.nskip || jr >= nacta) {
                    flag(d, OV_BUG | (si >= d.nskip ? GSK_B : GSK_C));
                    sput(i, Rec{0, HDR_REC | PAD_REC});  // nothing undrawn reaches phase B
                    continue;
                }
                const uint2 sk = d.skip[si];
                uint32_t st = sk.x * (uint32_t)r.k + sk.y;
                const int32_t x = dev_rand_r(st);
                if (x > last) {  // no host selected: this host's later draws shift by one
                    atomicOr(&s_sb[jr], NULL_DRAW);
                    continue;
                }
                const int32_t ch = dev_rand_r(st);  // worker.c:268-269
                sput(i, Rec{r.a, (uint64_t)(uint32_t)x | ((uint64_t)(uint32_t)ch << 32)});
                // the host's last send: its rng after every draw (the gossip
                // flat pass leaves it to this lane; skip_fix redoes a host
                // with a null draw)
                if (si + 1 == (s_vh[jr] >> 16)) {
                    const uint32_t sb = s_sb[jr] & ~NULL_DRAW, ha = s_act[jr];
                    if (ha < HP) reinterpret_cast<uint64_t*>(d.hs + sbase + ha)[0] = hs_w0(st, (uint32_t)sget(sb).k);
                }
            }
            __syncthreads();
            // skip_fix: a marked host's sends drawn again in order (test_phold.c:
            // 176-177: a draw selecting no host sends nothing and takes no
            // reliability draw), real sends first, pads after, as phase A lays
            // them out; its state after the draws rewritten
            for (uint32_t j = tid; j < nacta; j += K2_T) {
                const uint32_t sbm = s_sb[j];
                if (sbm == UINT32_MAX || !(sbm & NULL_DRAW)) continue;
                const uint32_t sb = sbm & ~NULL_DRAW, ns = s_vh[j] >> 16;
                if (sb + ns >= nsend) {
                    flag(d, OV_BUG | GSK_D);
                    for (uint32_t k = sb + 1; k < nsend && k <= sb + ns; ++k) sput(k, Rec{0, HDR_REC | PAD_REC});
                    s_sb[j] = sb;
                    continue;
                }
                const Rec hd = sget(sb);
                uint32_t st = (uint32_t)(hd.a >> 32);
                uint32_t out = sb + 1, nulls = 0;
                for (uint32_t k = sb + 1; k <= sb + ns; ++k) {
                    const uint64_t ra = sget(k).a;  // read before any write at or below k
                    const int32_t x = dev_rand_r(st);
                    if (x > last) {
                        ++nulls;
                        continue;
                    }
                    const int32_t ch = dev_rand_r(st);
                    sput(out++, Rec{ra, (uint64_t)(uint32_t)x | ((uint64_t)(uint32_t)ch << 32)});
                }
                for (; out <= sb + ns; ++out) sput(out, Rec{0, HDR_REC | PAD_REC});
                a.ctr[C_SENDS] -= nulls;
                a.ctr[C_NULL] += nulls;
                const uint32_t ha = s_act[j];
                if (ha >= HP) flag(d, OV_BUG | GSK_E);
                else reinterpret_cast<uint64_t*>(d.hs + sbase + ha)[0] = hs_w0(st, (uint32_t)hd.k);
                s_sb[j] = sb;
            }
            __syncthreads();
        }
        for (uint32_t i0 = tid; i0 < nsend; i0 += 2 * K2_T) {
            const uint32_t i1 = i0 + K2_T;
            const bool v1 = i1 < nsend;
            const Rec r0 = sget(i0);
            const Rec r1 = sget(v1 ? i1 : i0);  // an index select, not a conditional load
            const int32_t x0 = (int32_t)(uint32_t)r0.k, x1 = (int32_t)(uint32_t)r1.k;
            const uint32_t g0 = dst_guess(d, x0), g1 = dst_guess(d, x1);
            uint32_t vd0 = 0, vd1 = 0, dst0 = 0, dst1 = 0;
            if constexpr (EXACT) {
                const uint2 a0 = d.nearw[g0], b0 = d.nearw[g0 + 1];
                const uint2 a1 = d.nearw[g1], b1 = d.nearw[g1 + 1];
                near_resolve(d, x0, a0, b0, vd0, dst0);
                near_resolve(d, x1, a1, b1, vd1, dst1);
            } else {
                const Probe pb0 = dst_probe(d, g0), pb1 = dst_probe(d, g1);
                dst0 = dst_resolve(d, x0, g0, pb0, vd0);
                dst1 = dst_resolve(d, x1, g1, pb1, vd1);
            }
            asm volatile("" ::: "memory");  // both pair loads after both resolves (see phase A)
            // a header record's .a is its counter (gskip: and the host's state in
            // bits 32-63): no active index, so its path lookup uses host 0's
            const uint32_t j0 = (r0.k & HDR_REC) ? 0u : (uint32_t)(r0.a >> 52);
            const uint32_t j1 = (r1.k & HDR_REC) ? 0u : (uint32_t)(r1.a >> 52);
            const PairRec pr0 = pair_of(s_vh[j0] & 0xFFFFu, vd0, want_jump);
            const PairRec pr1 = pair_of(s_vh[j1] & 0xFFFFu, vd1, want_jump);
            // gossip records carry the message id in bits 40-51; it moves to
            // the resolved record's high word beside the destination
            const uint64_t tmask = gossip_rec ? M40 : M52;
            if (!(r0.k & HDR_REC)) {
                const uint64_t bt = S + (r0.a & tmask);
                const int32_t ch = (int32_t)(uint32_t)(r0.k >> 32);
                a.jmin = pr0.jump < a.jmin ? pr0.jump : a.jmin;            // topology.c:1374-1385
                const bool keep = bt < d.bootstrap_end || ch <= pr0.keep;  // worker.c:268-273
                if (keep && d.pcount) atomicAdd(&d.pcount[(size_t)(s_vh[j0] & 0xFFFFu) * d.V + vd0], 1u);
                const uint64_t rel = bt + pr0.delay - S;  // worker.c:275-277
                if (rel >> 40) a.overflow = true;
                const uint64_t msg = gossip_rec ? (r0.a >> 40) & 0xFFFu : 0u;
                sput(i0, Rec{((uint64_t)keep << 63) | ((uint64_t)j0 << 40) | rel, dst0 | (msg << 32)});
            }
            if (v1 && !(r1.k & HDR_REC)) {
                const uint64_t bt = S + (r1.a & tmask);
                const int32_t ch = (int32_t)(uint32_t)(r1.k >> 32);
                a.jmin = pr1.jump < a.jmin ? pr1.jump : a.jmin;
                const bool keep = bt < d.bootstrap_end || ch <= pr1.keep;
                if (keep && d.pcount) atomicAdd(&d.pcount[(size_t)(s_vh[j1] & 0xFFFFu) * d.V + vd1], 1u);
                const uint64_t rel = bt + pr1.delay - S;
                if (rel >> 40) a.overflow = true;
                const uint64_t msg = gossip_rec ? (r1.a >> 40) & 0xFFFu : 0u;
                sput(i1, Rec{((uint64_t)keep << 63) | ((uint64_t)j1 << 40) | rel, dst1 | (msg << 32)});
            }
        }
        __syncthreads();
        if (stamp && tid == 0) stamp[3] = __builtin_amdgcn_s_memrealtime();

        // ---- phase C: one lane per send record.  A send's srcHostEventID is its
        // host's counter plus the kept sends before it in the host's order
        // (worker.c:268-279, event.c:38), from a block-wide exclusive scan of
        // the records' keep bits: each thread takes a contiguous run of
        // records, a host's header records the scan's value at it (s_c by
        // host, free since phase A), and a send counts the kept sends between
        // its header and itself from the two (a walk back over the host's
        // records, as before, was quadratic in its sends); then endTime drop,
        // barrier bump, staging.  A host's kept sends are also counted into
        // s_n by host (free since phase A): its header writes its counter.
        for (uint32_t j = tid; j < nacta; j += K2_T) s_n[s_act[j]] = 0;
        __syncthreads();
        const uint32_t cper = (nsend + K2_T - 1) / K2_T, ci0 = tid * cper < nsend ? tid * cper : nsend;
        const uint32_t ci1 = ci0 + cper < nsend ? ci0 + cper : nsend;
        uint32_t kc = 0;
        for (uint32_t i = ci0; i < ci1; ++i) {
            const Rec r = sget(i);
            if (!(r.k & HDR_REC) && (r.a >> 63)) {
                ++kc;
                atomicAdd(&s_n[s_act[(uint32_t)(r.a >> 40) & 0xFFFFu]], 1u);
            }
        }
        uint64_t ktot;
        const uint32_t kpre = (uint32_t)block_excl_scan_2x32((uint64_t)kc, s16, &ktot);  // barriers inside
        {
            uint32_t pre = kpre;
            for (uint32_t i = ci0; i < ci1; ++i) {
                const Rec r = sget(i);
                if (r.k & HDR_REC) {
                    if (!(r.k & PAD_REC)) s_c[s_act[(uint32_t)(r.k >> 32) & 0xFFFFu]] = pre;
                } else {
                    pre += (uint32_t)(r.a >> 63);
                }
            }
        }
        __syncthreads();  // every header's scan value
        uint32_t pre = kpre;
        for (uint32_t i = ci0; i < ci1; ++i) {
            const Rec r = sget(i);
            if (r.k & HDR_REC) {
                if (r.k & PAD_REC) continue;
                // a host's header: its counter after all its kept sends
                const uint32_t ha = s_act[(uint32_t)(r.k >> 32) & 0xFFFFu];
                d.hs[sbase + ha].evc = (gskip ? r.a & 0xFFFFFFFFull : r.a) + s_n[ha];
                continue;
            }
            const uint32_t kept_before = pre;
            const bool keep = (r.a >> 63) != 0;
            pre += keep ? 1u : 0u;
            const uint32_t j = (uint32_t)(r.a >> 40) & 0xFFFFu;
            const uint32_t sb = s_sb[j], ha = s_act[j];
            const Rec hd = sget(sb);
            const uint64_t evc0 = gskip ? hd.a & 0xFFFFFFFFull : hd.a;  // the counter when phase A recorded the sends
            const uint64_t evc = evc0 + (kept_before - s_c[ha]);
            if (!keep) {
                ++a.ctr[C_DROPREL];
                continue;
            }
            const uint64_t sq = evc;                // event.c:38
            uint64_t tn = S + (r.a & M40);
            if (tn >= d.end_time) {                 // scheduler.c:343-346
                ++a.ctr[C_DROPEND];
                continue;
            }
            const uint32_t dst = (uint32_t)r.k;
            const uint64_t msg = r.k >> 32;  // gossip: the message id (0 for PHOLD)
            const uint32_t sg = d.lo + sbase + ha;
            if (dst == sg && tn < E) a.overflow = true;  // excluded by the phase A test
            if (dst != sg && tn < E) {              // host_single.c:180-184
                tn = E;
                ++a.ctr[C_BUMPED];
            }
            const uint32_t h = (uint32_t)hd.k;
            if (sq >> (SRC_SHIFT - d.msg_shift)) a.overflow = true;
            if (stage_event(d, S, p, sh, a, dst, tn, ((uint64_t)h << SRC_SHIFT) | (sq << d.msg_shift) | msg))
                count_local(tn);
        }
    }
    if (stage_recv) {  // uniform; a barrier inside
        const uint64_t m = stage_received(d, d.xrecv, p, gridDim.x, recv_routed, S, E, sh, a.overflow, s_roff, s16,
                                          count_local);
        a.emin = m < a.emin ? m : a.emin;  // in this shard's MIN terms from now on
    }
    // staging done: sh.nloc final, bins complete (LDS); several shards: the
    // outbox copy below reads other lanes' staged records from HBM
    if (d.outn) __syncthreads();
    else lds_barrier();
    if (d.outn) {
        // multi-shard: the partition's events for other shards into their peers'
        // outbox regions, one reservation per peer
        if (tid < d.G) {
            s_oslot[tid] = 0;
            s_obase[tid] = sh.peer[tid] ? (uint32_t)atomicAdd((unsigned long long*)&d.outn[tid],
                                                              (unsigned long long)sh.peer[tid]) : 0u;
        }
        __syncthreads();
        const uint32_t nr = sh.nrem < d.ECAP ? sh.nrem : d.ECAP;
        const bool xsys = d.xpeer && d.xfence;
        for (uint32_t i = tid; i < nr; i += K2_T) {
            const size_t so = (size_t)p * d.ECAP + i;
            const uint32_t dst = d.rem_dst[so];
            const uint32_t q = owner_of(d, dst);
            const uint64_t r = s_obase[q] + atomicAdd(&s_oslot[q], 1u);
            const Slot ev = d.rem[so];
            const bool inblk = r < d.xcap;
            int64_t* o = inblk ? xblock(d, q) + (HDR + r) * RW : d.outq + ((uint64_t)q * d.oreg + r) * RW;
            const uint64_t rel = ev.t - S;  // new events are at or after the window's end
            if (rel >> 40) a.overflow = true;  // beyond 2^40 ns (18 min) of the window start
            const int64_t w0 = (int64_t)((rel & M40) | ((uint64_t)(dst - d.bounds[q]) << 40)), w1 = (int64_t)ev.k;
            if (xsys && inblk) {  // into a peer on another GPU: system-coherent stores
                xst(1u, o, w0);
                xst(1u, o + 1, w1);
            } else {
                gint64_t* og = (gint64_t*)o;
                og[0] = w0;
                og[1] = w1;
            }
        }
    }
    if (stamp && tid == 0) stamp[13] = __builtin_amdgcn_s_memrealtime();
    const uint32_t nl = sh.nloc < d.ECAP ? sh.nloc : d.ECAP;
    if (horizon) flag(d, OV_HORIZON);

    // workgroup partials: cumulative counters, this round's two minima
    const int lane = tid & 63, wid = tid >> 6;
    uint64_t v[NPCTR + 2];
#pragma unroll
    // a wave's sum as a signed 32-bit value: a lane's counter may be negative
    // (the gossip flat pass counts a host's sends on its receipts' lanes, the
    // null-draw fix takes them back on the host's lane), the wave's never is
    for (int i = 0; i < NPCTR; ++i) v[i] = (uint64_t)(int64_t)(int32_t)wave_sum_u32(a.ctr[i]);
    v[NPCTR] = wave_min(a.emin);
    v[NPCTR + 1] = wave_min(a.jmin);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NPCTR + 2; ++i) s_red[wid][i] = v[i];
    }
    if (a.overflow) flag(d, OV_PROC);
    lds_barrier();  // s_red
    if (stamp && tid == 0) stamp[14] = __builtin_amdgcn_s_memrealtime();
    // wave 0: the partials and the MIN accumulators (the last workgroup reads
    // them), before the reservations (after them measured k_proc +1.0 us,
    // profiles/r05/tick)
    auto partials = [&]() __attribute__((always_inline)) {
        if (tid < NPCTR + 2) {
            const int i = tid;
            uint64_t r = s_red[0][i];
            for (int w = 1; w < K2_T / 64; ++w) {
                const uint64_t x = s_red[w][i];
                r = i < NPCTR ? r + x : (x < r ? x : r);
            }
            // the workgroup's own slot: an atomic add needs no load (wave 0 joins
            // the reservations' barrier without waiting for one)
            if (i < NPCTR) atomicAdd((unsigned long long*)&d.pcum[(size_t)i * d.P + p], (unsigned long long)r);
            else d.p2min[(size_t)(i - NPCTR) * d.P + p] = r;
            if (i >= NPCTR && r != UINT64_MAX) atomicMin((unsigned long long*)&rs->xacc[i - NPCTR], (unsigned long long)r);
        }
    };
    partials();
    reserve_buckets<K2_T, FLAT>(d, p, p % XS, s_bc, s_bm, bS, bSr, stash_id, stash_n, ring_end, s_ids, &s_h, s16);
    if (stamp && tid == 0) stamp[15] = wait_stamp();
    if (tid == 0) {
        if (sh.nloc > d.ECAP || sh.nrem > d.ECAP || s_nsend > d.ECAP) flag(d, OV_PROC);
        d.rcnt[p] = nl;
        if (d.remn) d.remn[p] = sh.nrem < d.ECAP ? sh.nrem : d.ECAP;
    }
    if (d.xsend) {
        // Several shards: the last workgroup to finish writes the exchange
        // block headers (this shard's MIN terms; one shard, k_scatter plans
        // the next window from the accumulators after the kernel boundary).
        // No fences (an L2 write-back per workgroup costs more than a launch):
        // what it reads from the others was performed by device-scope atomics
        // (MIN accumulators, outbox counts), which the issuing wave waits for
        // (vmcnt(0)) before the workgroup takes its ticket: wave 0 for the MIN
        // accumulators; every wave's outbox reservations returned their value.
        // An overflow flag another workgroup sets may reach the next step's
        // headers instead; the run still stops and reports it.  No workgroup
        // waits for another.
        __shared__ bool s_lastwg;
        __shared__ uint64_t s_mj[2];
        // fused push: every wave's rows are performed (and, across GPUs,
        // released at system scope) at the peers before the workgroup takes
        // its ticket; the last one signals them (xlink_release / xlink_arrive)
        if (d.xpeer) xlink_release();
        else if (wid == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // (a two-level ticket here, as k_scatter's plan arrival, hung the
        // two-process xGMI test in round 5; on round 6's tree it passed:
        // profiles/r05/ptick8/README.md)
        if (tid == 0)
            s_lastwg = atomicAdd((unsigned long long*)&rs->ticket, 1ULL) == gridDim.x - 1;
        __syncthreads();
        if (s_lastwg) {
            if (tid == 0) {
                const uint32_t cur = (uint32_t)(rs->fold & 1);
                const uint64_t em = rmw_read(&rs->xacc[0]), jm = rmw_read(&rs->xacc[1]);
                uint64_t m = rs->xcarry2[cur];  // carry min (k_scatter's atomics, a kernel ago)
                m = em < m ? em : m;
                m = rs->rmin2[cur] < m ? rs->rmin2[cur] : m;
                m = m < SIMTIME_MAX ? m : SIMTIME_MAX;
                s_mj[0] = m;
                s_mj[1] = rs->jmin < jm ? rs->jmin : jm;
                rs->ticket = 0;
                rs->xacc[0] = UINT64_MAX;
                rs->xacc[1] = UINT64_MAX;
            }
            __syncthreads();
            write_headers(d, s_mj[0], s_mj[1]);
            if (d.xpeer) xlink_signal(d);
        }
    }
    if (stamp && tid == 0) {
        stamp[4] = __builtin_amdgcn_s_memrealtime();
        stamp[5] = n;
        stamp[6] = nact;
        stamp[7] = s_nsend;
    }
    if (d.wtime) {  // this partition's busy time; k_scatter's rmin workgroup charges the wait for the last one
        __syncthreads();
        if (tid == 0) {
            const uint64_t t_end = wait_stamp();
            d.wtime[p] += t_end - t_start;
            d.wtime[2 * (size_t)d.P + p] = t_end;
        }
    }
}

// --------------------------------------------------------------- insert ----
// Events → calendar buckets.  Staged events (a partition's new events and,
// several shards, its share of the previous step's received events) were
// counted and reserved per (partition, bucket) by k_proc; k_scatter writes
// them into the chunks the reserving rows allocated, one workgroup per
// partition.

// k_scatter: new (and received) events into the calendar, fused with the
// gather of the window it plans.  Workgroup roles:
//   [0, P)          partition blk's staged local events (process step)
//   [P, P + G3)     the received blocks' events (multi-shard), split evenly
//   [g0, g0 + G1)   gather: the listed due chunks into the host partitions
//   last            rmin: first live bucket beyond the new window, its min
// An inserted event due in the new window (t < E) is routed straight to its
// host partition instead: its slot stays empty in a fully due bucket (whose
// chunks were not grown and k_scatter's gather returns to the ring) or
// becomes a tombstone in the straddling bucket.  Events that stay in the
// straddling bucket add to the carry min (the next MIN term), as the
// gather's leftovers do.
constexpr int SU = 2048 / K3_T;  // events per thread in flight (2048 per insert batch)
constexpr size_t INS_LDS = (RMAX + 2 * PMAX) * 4 + 16 * 8 + MAXG * 4;
constexpr size_t REFILL_LDS = 16 * 8 + 8 + 2 * (PMAX + G3MAX) * 4;
constexpr size_t SCAT_LDS0 = INS_LDS > GATHER_LDS ? INS_LDS : GATHER_LDS;
constexpr size_t SCAT_LDS = SCAT_LDS0 > REFILL_LDS ? SCAT_LDS0 : REFILL_LDS;

struct Route {
    bool listed;
    uint32_t cur;         // the step's parity (carry min goes to xcarry2[cur ^ 1])
    uint64_t S, E, ret;   // the new window, its straddling bucket (UINT64_MAX: none)
    uint64_t bS, bSW;     // the window's first bucket and its start: every event inserted is at or
                          // after it and within R buckets of it (k_proc's horizon check)
    uint32_t bSr;         // bS % R
};

// One batch of up to SU events per thread (every thread of the workgroup
// calls it): slot from the (partition, bucket) reservation cursor, chunk
// from the reserving row's allocation; due events routed.  Returns nothing; carry min
// and tombstones accumulate in smin / ntomb.
__device__ __forceinline__ void insert_batch(const Dev& d, const Route& ro, uint32_t x, uint32_t* s_cur, uint32_t* s_pc,
                                             uint32_t* s_pk, const bool (&v)[SU], const uint64_t (&t)[SU],
                                             const uint64_t (&k)[SU], const uint32_t (&dl)[SU], uint64_t& smin,
                                             uint64_t& ntomb) {
    const uint64_t W = d.W;
    const uint32_t R = d.R;
    uint32_t rb[SU], pos[SU], off[SU];
    bool due[SU], write[SU];
#pragma unroll
    for (int q = 0; q < SU; ++q) {
        uint64_t b;
        if (d.ring32) {  // launch-uniform: offsets from the window's first bucket, no 64-bit division
            const uint64_t rel = t[q] - ro.bSW;
            const uint32_t o = wdiv(d, (uint32_t)rel);
            b = ro.bS + o;
            off[q] = (uint32_t)rel - o * (uint32_t)W;
            const uint32_t r0 = ro.bSr + o;
            if (v[q] && (t[q] < ro.bSW || (rel >> 32) || o >= R)) flag(d, OV_BUG);  // beyond k_proc's horizon
            const uint32_t r1 = r0 >= R ? r0 - R : r0;
            rb[q] = v[q] && r1 < R ? r1 : 0u;  // clamped: a bad record writes in bounds, flagged
        } else {
            b = t[q] / W;
            off[q] = (uint32_t)(t[q] - b * W);
            rb[q] = v[q] ? (uint32_t)(b % R) : 0u;
        }
        pos[q] = v[q] ? atomicAdd(&s_cur[rb[q]], 1u) : 0u;
        due[q] = v[q] && ro.listed && t[q] < ro.E;
        const bool in_ret = ro.listed && b == ro.ret;
        write[q] = v[q] && (!due[q] || in_ret);  // fully due buckets: the slot stays empty
        if (v[q] && !due[q] && in_ret) smin = t[q] < smin ? t[q] : smin;
        if (due[q]) atomicAdd(&s_pc[part_of(d, dl[q])], 1u);
    }
    uint32_t id[SU];
    const uint32_t* tab = d.btab + (size_t)x * R * d.NCH;
#pragma unroll
    for (int q = 0; q < SU; ++q) {
        const uint32_t ci = pos[q] >> CH_SHIFT;
        id[q] = tab[(size_t)rb[q] * d.NCH + (ci < d.NCH ? ci : d.NCH - 1)];
    }
#pragma unroll
    for (int q = 0; q < SU; ++q) {
        // no chunk only when the pool ran out (reserve_buckets flagged it)
        if (!write[q] || (pos[q] >> CH_SHIFT) >= d.NCH || id[q] >= d.NCH) continue;
        Rec r{due[q] ? TOMB : (((uint64_t)dl[q] << 40) | off[q]), k[q]};
        ntomb += due[q];
        st_rec(d.pool, (((size_t)id[q] << CH_SHIFT) + (pos[q] & (CH - 1))) * 16, r.a, r.k);
    }
    if (!ro.listed) return;  // launch-uniform
    // due events: one reservation per (workgroup, partition), then the copies.
    // The barriers order LDS only: the calendar and partition stores drain
    // while the workgroup goes on (nothing in the launch reads them back).
    lds_barrier();
    uint32_t* pc = d.pcnt;
    for (uint32_t p = threadIdx.x; p < d.P; p += blockDim.x) {
        const uint32_t c = s_pc[p];
        s_pk[p] = 0;
        if (c) {
            const uint32_t base = atomicAdd(&pc[p], c);
            if (base + c > d.CAPP) flag(d, OV_PART);
            s_pc[p] = base;
        }
    }
    lds_barrier();
#pragma unroll
    for (int q = 0; q < SU; ++q) {
        if (!due[q]) continue;
        const uint32_t p = part_of(d, dl[q]);
        const uint32_t slot = s_pc[p] + atomicAdd(&s_pk[p], 1u);
        if (slot < d.CAPP)
            st_rec(d.part, ((size_t)p * d.CAPP + slot) * 16, ((uint64_t)(dl[q] - p * d.HP) << 52) | (t[q] - ro.S), k[q]);
    }
    lds_barrier();
    for (uint32_t p = threadIdx.x; p < d.P; p += blockDim.x) s_pc[p] = 0;
    lds_barrier();
}

__device__ __forceinline__ void insert_finish(const Dev& d, const Route& ro, uint64_t smin, uint64_t ntomb,
                                              uint64_t* s16) {
    if (!ro.listed || ro.ret == UINT64_MAX) return;  // launch-uniform
    (void)s16;
    uint64_t m = smin, nt = ntomb, unused = 0;
    block_tail3(m, nt, unused);
    if (threadIdx.x == 0) {
        const uint32_t rb = (uint32_t)(ro.ret % d.R);
        if (nt) atomicAdd(&d.btomb[rb], (uint32_t)nt);
        if (m != UINT64_MAX) {
            atomicMin((unsigned long long*)&d.rs->xcarry2[ro.cur ^ 1], (unsigned long long)m);
            atomicMin((unsigned long long*)&d.bmin[rb], (unsigned long long)m);
        }
    }
}

// Refill role (one workgroup, every thread): bk copied into bw[nx] (every slot
// reserved so far is written once this launch's inserts are, so the next
// step's gather may read them all), then every reserving row's stash back to
// ST chunk ids from the free ring, usable up to avail.
__device__ __forceinline__ void refill_role(const Dev& d, uint32_t nx, uint64_t avail, unsigned char* lds,
                                            uint64_t* st) {
    RoundState* rs = d.rs;
    const uint32_t R = d.R, tid = threadIdx.x;
    // fold: every slot reserved so far is written by this launch, so the
    // next step's gather may read them all
    {
        // (nx: the other half of bw, read by the next step)
        constexpr uint32_t CPT = XS * RMAX / K3_T;
        uint32_t cv[CPT];  // every load in flight at once
#pragma unroll
        for (uint32_t q = 0; q < CPT; ++q) {
            const uint32_t i = tid + q * K3_T;
            cv[q] = d.bk[i < XS * R ? i : 0u];
        }
#pragma unroll
        for (uint32_t q = 0; q < CPT; ++q)
            if (tid + q * K3_T < XS * R) d.bw[(size_t)nx * XS * R + tid + q * K3_T] = cv[q];
    }
    // stash refill: every reserving row back to ST chunk ids, one ring
    // reservation for all of them; the ring is usable up to the tail the
    // plan set (this launch's gather frees more behind it).  The ids are
    // copied as one flat list of (row, slot) entries, every load of a
    // batch in flight together.
    constexpr uint32_t RPT = (PMAX + G3MAX + K3_T - 1) / K3_T;
    constexpr int FU = 8;
    uint64_t* s16 = (uint64_t*)lds;
    uint64_t* s_hh = s16 + 16;
    uint32_t* s_have = (uint32_t*)(s_hh + 1);  // [PMAX + G3MAX]
    uint32_t* s_roff = s_have + PMAX + G3MAX;  // [PMAX + G3MAX] first list entry of each row
    const uint32_t rows = d.P, NCH = d.NCH;  // the reserving rows: k_proc's partitions
    
    uint32_t have[RPT];
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t q = 0; q < RPT; ++q) {
        const uint32_t r = tid + q * K3_T;
        have[q] = r < rows ? d.stn[r] : ST;
        mine += ST - have[q];
    }
    uint64_t total;
    uint32_t off = (uint32_t)block_excl_scan(mine, s16, &total);  // barriers inside
    if (total == 0) return;  // uniform
#pragma unroll
    for (uint32_t q = 0; q < RPT; ++q) {
        const uint32_t r = tid + q * K3_T;
        if (r < rows) {
            s_have[r] = have[q];
            s_roff[r] = off;
        }
        off += ST - have[q];
    }
    if (tid == 0) *s_hh = atomicAdd((unsigned long long*)&rs->fl_head, (unsigned long long)total);
    __syncthreads();
    const uint64_t h = *s_hh;
    const uint32_t hr = (uint32_t)(h % NCH);
    if (h + total > avail && tid == 0) flag(d, OV_POOL);
    for (uint32_t f0 = 0; f0 < rows * ST; f0 += K3_T * FU) {
        uint32_t id[FU], dst[FU];
        bool v[FU];
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const uint32_t f = f0 + tid + u * K3_T, r = f / ST < rows ? f / ST : 0u, k = f % ST;
            const uint32_t e = s_roff[r] + (k - s_have[r]);  // list entry (when k >= have)
            v[u] = f < rows * ST && k >= s_have[r] && h + e < avail;
            const uint32_t pos = hr + (v[u] ? e : 0u);  // e < total <= NCH: one wrap at most
            id[u] = d.fring[pos >= NCH ? pos - NCH : pos];  // unconditional (clamped)
            dst[u] = r * ST + k;
        }
#pragma unroll
        for (int u = 0; u < FU; ++u)
            if (v[u]) d.stash[dst[u]] = id[u];
    }
#pragma unroll
    for (uint32_t q = 0; q < RPT; ++q) {
        const uint32_t r = tid + q * K3_T;
        if (r >= rows || have[q] == ST) continue;
        const uint64_t e0 = h + s_roff[r];  // the row's first entry's ring position
        const uint64_t got = e0 >= avail ? 0 : std::min<uint64_t>(avail - e0, ST - have[q]);
        d.stn[r] = have[q] + (uint32_t)got;
    }
    if (st) st[3] = __builtin_amdgcn_s_memrealtime();
}

// mode: 0 one shard (after k_proc), 1 several shards (after the all-to-all; recv the
// exchange blocks), 2 boot.  Every workgroup plans the step (step_view) from
// the state as the previous kernels left it, then arrives on a counter once its
// reads of that state have returned; the last to arrive publishes the plan
// (publish_step).  Nothing waits for anything: no workgroup depends on another
// being resident, whatever the order the hardware dispatches them in.
__global__ __launch_bounds__(K3_T) void k_scatter(Dev d, const int64_t* recv, int mode) {
    const uint64_t t_in = d.stamps ? __builtin_amdgcn_s_memrealtime() : 0;  // SG_STAMPS: the workgroup's entry
    RoundState* rs = d.rs;
    __shared__ __align__(16) unsigned char lds[SCAT_LDS];
    __shared__ StepView sv;
    __shared__ uint64_t s_rsw[RSW];              // the round state as the previous kernels left it
    __shared__ int64_t s_hdr[MAXG * HDR_W];      // several shards: the received blocks' headers
    __shared__ uint64_t s_gsw[3];                // gather: the GSpec header
    __shared__ uint32_t s_routed;
    __shared__ uint64_t s_rbase[MAXG];           // receive role: the received blocks' time bases
    // role order [insert P][receive G3][gather][refill][rmin] over the
    // workgroups; SG_GFIRST dispatches the gather workgroups (the launch's long
    // pole) first
    const uint32_t nv = gridDim.x;
    const uint32_t g0 = d.P + (recv ? d.G3 : 0), gx = nv - 2;  // gather workgroups [g0, gx)
    const uint32_t ng = gx - g0, bi = blockIdx.x;
    const uint32_t blk = SG_GFIRST ? (bi < ng ? g0 + bi : bi < gx ? bi - ng : bi) : bi;
    const uint32_t R = d.R, tid = threadIdx.x;
    // wave 0: the round state (and headers) in one batch of loads, then thread
    // 0 plans the step from LDS and arrives.  The arrival's return is not
    // waited for until the workgroup's end: the last to arrive publishes then.
    uint64_t ticket = 0, rsv = 0, h0 = 0, t_rs = 0, t_sv = 0;
    if (tid < 64) rsv = load_round_state(d, mode, recv, s_rsw, s_hdr, &h0);
    asm volatile("" ::: "memory");  // the copy's stores before thread 0's reads of it
    if (tid == 0) {
        // the kernel arguments the plan reads, fetched while the round state is
        // in flight: read first inside the plan, each scalar-cache miss was a
        // round trip after it (the plan took 1.2 us, profiles/r06/g14)
        if (SG_PLAN_TOUCH) touch_plan_args(d);
        if (d.stamps) t_rs = wait_stamp();  // SG_STAMPS: the round state is in
#if SG_RS_LANES
        // the round state from wave 0's registers (one readlane per word), not
        // through a chain of LDS reads
        RoundState rl;
        uint64_t* rw = reinterpret_cast<uint64_t*>(&rl);
#pragma unroll
        for (uint32_t i = 0; i < RSW; ++i) rw[i] = readlane64(rsv, i);
        step_view(d, mode, &rl, s_hdr, sv, h0, d.G * HDR_W <= 64);
#else
        step_view(d, mode, reinterpret_cast<const RoundState*>(s_rsw), s_hdr, sv);
#endif
        if (d.stamps) t_sv = __builtin_amdgcn_s_memrealtime();  // the step is planned
        // every read of the round state has returned (they are in LDS).  The
        // address is made opaque (divergent to the compiler): for a uniform one
        // the atomic optimizer reads the result back at once, which would wait
        // for the arrival's round trip here.
#if !SG_LATE_TICKET
        const uint32_t z = opaque(tid) - tid;  // 0
        if (!sv.quit) ticket = atomicAdd((unsigned long long*)&rs->splan + z, 1ull);
#endif
    }
    // gather workgroups, wave 1: the guessed due list (GSpec) beside the round state
    if (blk >= g0 && blk < gx && (tid >> 6) == 1) gspec_load(d, blk - g0, gx - g0, s_gsw, (DueEnt*)(lds + GDE_OFF));
    // Insert role: what does not depend on the window is loaded while thread 0
    // plans (waves 1.. at once; wave 0 after its plan): the partition's count,
    // its first SU staged events per thread and its reservation bases.
    Rec pre[SU];
    uint32_t pre_n = 0;
    // the partition's reservation bases into LDS (every load in flight at once, R <= RMAX)
    auto load_bases = [&]() __attribute__((always_inline)) {
        uint32_t* s_cur = (uint32_t*)lds;
        uint32_t* s_pc = s_cur + RMAX;
        const uint32_t* wb = d.wbase + (size_t)blk * R;
        constexpr uint32_t WPT = RMAX / K3_T;
        uint32_t wv[WPT];
#pragma unroll
        for (uint32_t q = 0; q < WPT; ++q) {
            const uint32_t rb = tid + q * K3_T;
            wv[q] = wb[rb < R ? rb : 0u];
        }
        for (uint32_t p = tid; p < d.P; p += K3_T) s_pc[p] = 0;
#pragma unroll
        for (uint32_t q = 0; q < WPT; ++q)
            if (tid + q * K3_T < R) s_cur[tid + q * K3_T] = wv[q];
    };
    if (blk < d.P) {  // uniform
        pre_n = d.rcnt[blk];
#if SG_INS_PRE
        const Rec* src = d.loc + (size_t)blk * d.ECAP;  // ECAP >= SU * K3_T (host-checked)
#pragma unroll
        for (int q = 0; q < SU; ++q) pre[q] = ld_stream(&src[threadIdx.x + q * K3_T]);
        load_bases();
#endif
    }
    lds_barrier();  // the plan, the headers, the guess and the bases are in LDS
    if (sv.quit) return;  // uniform: the run ended (no workgroup took a ticket)
    do {  // the roles (break: this workgroup's role is done)
    Route ro;
    ro.listed = sv.listed != 0;
    ro.cur = sv.cur;
    ro.S = sv.S;
    ro.E = sv.E;
    ro.ret = sv.ret;
    ro.bS = sv.bS;
    ro.bSW = ro.bS * d.W;
    ro.bSr = sv.bSr;
    // SG_STAMPS: {start, after setup, after the events, end, role, events}
    uint64_t* st = d.stamps && tid == 0 ? d.stamps + (size_t)(d.P + 1 + blk) * SG_STAMP_W : nullptr;
    if (st) {
        st[0] = __builtin_amdgcn_s_memrealtime();
        st[4] = blk == nv - 1 ? 3 : blk == nv - 2 ? 4 : blk >= g0 ? 2 : blk >= d.P ? 1 : 0;
        st[1] = st[2] = st[3] = st[6] = st[0];
        st[5] = 0;
        st[16] = t_in;
        st[17] = t_rs;
        st[18] = t_sv;
    }
    if (blk == nv - 1) {
        uint64_t* s16 = (uint64_t*)lds;
        if (d.wtime && sv.round_done) {
            // barrier wait (scheduler.c:380-389): each partition idles from its
            // end to the round's last partition end
            uint64_t mx = 0;
            for (uint32_t p = tid; p < d.P; p += K3_T) {
                const uint64_t t = d.wtime[2 * (size_t)d.P + p];
                mx = t > mx ? t : mx;
            }
            mx = ~block_min(~mx, s16);  // max; barriers inside
            for (uint32_t p = tid; p < d.P; p += K3_T) d.wtime[(size_t)d.P + p] += mx - d.wtime[2 * (size_t)d.P + p];
        }
        // rmin for the listed window: the min time of the buckets beyond it,
        // (bL, bS + R), but those of the window before it (consumed, reset by
        // the next k_proc).  The rest hold no tombstones or were reset, and this
        // launch changes only the straddling bucket's minimum, so the minima
        // read are final.  No new window: the current value carries over.
        if (!sv.listed) {
            if (tid == 0) rs->rmin2[sv.cur ^ 1] = sv.rmin0;
            break;
        }
        const uint64_t bS = sv.bS, bL = sv.bL, pbS = sv.pbS, pbL = sv.pbL;
        const uint32_t span = (uint32_t)(bL - bS), bLr = (uint32_t)(bL % R);
        constexpr uint32_t OPT = RMAX / K3_T;
#if SG_PMIN
        // the first bucket beyond the window holding events (reserved slots),
        // then the minimum of its column of the rows' minima
        uint32_t kv[OPT];  // every count in flight at once (clamped slots)
#pragma unroll
        for (uint32_t q = 0; q < OPT; ++q) {
            const uint32_t o = tid + 1 + q * K3_T;
            const uint32_t rb = o + span < R ? (bLr + o >= R ? bLr + o - R : bLr + o) : 0u;
            uint32_t c = 0;
#pragma unroll
            for (uint32_t x = 0; x < XS; ++x) c += d.bk[(size_t)x * R + rb];
            kv[q] = c;
        }
        uint64_t fo = UINT64_MAX;
#pragma unroll
        for (uint32_t q = 0; q < OPT; ++q) {
            const uint32_t o = tid + 1 + q * K3_T;
            const uint64_t b = bL + o - R;  // the ring slot's consumed bucket, if any
            const bool live = o + span < R && !(pbS != UINT64_MAX && b >= pbS && b <= pbL);
            fo = live && kv[q] && o < fo ? o : fo;
        }
        fo = block_min(fo, s16);  // barriers inside
        uint64_t mn = UINT64_MAX;
        if (fo != UINT64_MAX) {  // uniform
            const uint32_t rb = bLr + (uint32_t)fo >= R ? bLr + (uint32_t)fo - R : bLr + (uint32_t)fo;
            uint32_t m = UINT32_MAX;
            for (uint32_t p = tid; p < d.P; p += K3_T) {
                const uint32_t v = d.pmin[(size_t)p * R + rb];
                m = v < m ? v : m;
            }
            const uint64_t bm = block_min((uint64_t)m, s16);
            mn = bm != UINT32_MAX ? (bL + fo) * d.W + bm : UINT64_MAX;
        }
#else
        uint64_t bv[OPT];  // every minimum in flight at once (clamped slots)
#pragma unroll
        for (uint32_t q = 0; q < OPT; ++q) {
            const uint32_t o = tid + 1 + q * K3_T;
            const uint32_t rb = o + span < R ? (bLr + o >= R ? bLr + o - R : bLr + o) : 0u;
            bv[q] = d.bmin[rb];
        }
        uint64_t mn = UINT64_MAX;
#pragma unroll
        for (uint32_t q = 0; q < OPT; ++q) {
            const uint32_t o = tid + 1 + q * K3_T;
            const uint64_t b = bL + o - R;  // the ring slot's consumed bucket, if any
            const bool live = o + span < R && !(pbS != UINT64_MAX && b >= pbS && b <= pbL);
            mn = live && bv[q] < mn ? bv[q] : mn;
        }
        mn = block_min(mn, s16);  // barriers inside
#endif
        if (tid == 0) {
            rs->rmin2[sv.cur ^ 1] = mn < SIMTIME_MAX ? mn : SIMTIME_MAX;
            if (st) st[3] = __builtin_amdgcn_s_memrealtime();
        }
        break;
    }
    if (blk == nv - 2) {
        // the plan's tail: this launch's gather frees more behind it
        refill_role(d, sv.cur ^ 1, sv.tail, lds, st);
        break;
    }
    if (blk >= g0) {
        if (ro.listed) gather_role<K3_T>(d, sv, blk - g0, gx - g0, lds, s_gsw, st);
        if (st) st[3] = wait_stamp();
        break;
    }
    uint32_t* s_cur = (uint32_t*)lds;    // [RMAX] slot cursor per bucket
    uint32_t* s_pc = s_cur + RMAX;       // [PMAX] routed events per partition, then their base
    uint32_t* s_pk = s_pc + PMAX;        // [PMAX] cursor within it
    uint64_t* s16 = (uint64_t*)(s_pk + PMAX);
    uint32_t* s_off = (uint32_t*)(s16 + 16);  // [MAXG] received blocks' offsets
    uint64_t smin = UINT64_MAX, ntomb = 0;
    if (blk < d.P) {  // partition blk's staged local events (bases and first batch loaded above)
        const Rec* src = d.loc + (size_t)blk * d.ECAP;
        Rec r[SU];
        if (!sv.ins_local) break;
        const uint32_t n = pre_n;
        if (n == 0) break;  // uniform: nothing routed, nothing to finish
        const uint64_t S = sv.ins_S;
        if (st) {
            st[1] = __builtin_amdgcn_s_memrealtime();
            st[5] = n;
        }
#if !SG_INS_PRE
        load_bases();  // after the plan: the gather's first loads go out ahead of these
        lds_barrier();
#endif
        for (uint32_t i0 = 0; i0 < n; i0 += K3_T * SU) {
#if SG_INS_PRE
            if (i0 == 0) {  // uniform
#pragma unroll
                for (int q = 0; q < SU; ++q) r[q] = pre[q];
            } else
#endif
            {
#pragma unroll
                for (int q = 0; q < SU; ++q) {
                    const uint32_t i = i0 + threadIdx.x + q * K3_T;
                    r[q] = ld_stream(&src[i < n ? i : 0]);
                }
            }
            bool v[SU];
            uint64_t t[SU], k[SU];
            uint32_t dl[SU];
#pragma unroll
            for (int q = 0; q < SU; ++q) {
                v[q] = i0 + threadIdx.x + q * K3_T < n;
                t[q] = S + (r[q].a & M40);
                k[q] = r[q].k;
                dl[q] = (uint32_t)(r[q].a >> 40);
                if (v[q] && dl[q] >= d.L) {  // a staged record is always a local host: clamped, flagged
                    flag(d, OV_BUG);
                    dl[q] = 0;
                }
            }
            insert_batch(d, ro, blk % XS, s_cur, s_pc, s_pk, v, t, k, dl, smin, ntomb);
        }
        if (st) st[2] = wait_stamp();
        insert_finish(d, ro, smin, ntomb, s16);
        if (st) st[3] = wait_stamp();
        break;
    }
    // the received blocks' events due in the new window, split evenly over G3
    // workgroups, routed straight to their host partitions (one reservation
    // per (workgroup, partition)); the next k_proc stages the rest
    // (stage_received): no slot is reserved for an event about to be popped
    const uint32_t g3 = d.G3, w = blk - d.P;
    uint32_t* pc = d.pcnt;
    if (tid == 0) s_routed = 0;
    for (uint32_t p = threadIdx.x; p < d.P; p += K3_T) {
        s_pc[p] = 0;
        s_pk[p] = 0;
    }
    const uint64_t total = recv_offsets(d, recv, d.xrows, d.xcap, s_off, s_rbase, s16, false);  // barrier inside
    const uint64_t lo = total * w / g3, hi = total * (w + 1) / g3;
    if (!ro.listed) break;  // uniform: no new window, nothing is due
    for (uint64_t i = lo + threadIdx.x; i < hi; i += K3_T) {
        uint64_t t, k;
        uint32_t dl;
        if (recv_event(d, recv, d.xrows, s_off, s_rbase, (uint32_t)i, t, k, dl) && t < ro.E)
            atomicAdd(&s_pc[part_of(d, dl)], 1u);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < d.P; p += K3_T) {
        const uint32_t c = s_pc[p];
        if (c) {
            const uint32_t base = atomicAdd(&pc[p], c);
            if (base + c > d.CAPP) flag(d, OV_PART);
            s_pc[p] = base;
            atomicAdd(&s_routed, c);
        }
    }
    __syncthreads();
    if (tid == 0 && s_routed)  // C_RECV: received events this workgroup writes into partitions
        atomicAdd((unsigned long long*)&d.pcum[(size_t)C_RECV * d.P + w % d.P], (unsigned long long)s_routed);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += K3_T) {
        uint64_t t, k;
        uint32_t dl;
        if (!recv_event(d, recv, d.xrows, s_off, s_rbase, (uint32_t)i, t, k, dl) || t >= ro.E) continue;
        const uint32_t p = part_of(d, dl);
        const uint32_t slot = s_pc[p] + atomicAdd(&s_pk[p], 1u);
        if (slot < d.CAPP) st_rec(d.part, ((size_t)p * d.CAPP + slot) * 16, ((uint64_t)(dl - p * d.HP) << 52) | (t - ro.S), k);
    }
    } while (0);
    // the last workgroup to arrive publishes the plan for the next kernels
#if SG_LATE_TICKET
    if (tid == 0) {
        const uint32_t z = opaque(tid) - tid;  // 0
#if SG_TICK8
        // two levels (SG_TICK8): the workgroups of shard blk & 7 arrive on its
        // own counter, the last of each on the plan counter; the last of those
        // publishes.  Each counter takes <= 49 adds instead of one taking 386.
        const uint32_t k = blockIdx.x & 7u, nsh = gridDim.x < 8 ? gridDim.x : 8u;
        const uint64_t in_k = (gridDim.x - k + 7) / 8;  // workgroups b < gridDim.x with b & 7 == k
        ticket = 0;
        if (atomicAdd((unsigned long long*)&d.tick[k] + z, 1ull) == in_k - 1) {
            atomicExch((unsigned long long*)&d.tick[k], 0ull);  // every arrival of the shard is in
            if (atomicAdd((unsigned long long*)&rs->splan + z, 1ull) == nsh - 1) ticket = gridDim.x - 1;
        }
#else
        ticket = atomicAdd((unsigned long long*)&rs->splan + z, 1ull);
#endif
    }
#endif
    if (tid == 0 && ticket == gridDim.x - 1) publish_step(d, mode, sv, recv);
}

// ----------------------------------------------------------------- plan ----
// The local MIN terms of a round: carry min (k_scatter's gather and inserts),
// emitted min and discovery min (k_proc), and the buckets beyond the window
// (rmin).
__device__ __forceinline__ void reduce_local(const Dev& d, uint64_t* s16, uint64_t& m, uint64_t& j) {
    const uint32_t cur = (uint32_t)(d.rs->fold & 1);
    uint64_t mm = d.rs->xcarry2[cur], jj = UINT64_MAX;
    for (uint32_t i = threadIdx.x; i < d.P; i += blockDim.x) {
        const uint64_t x = d.p2min[i], y = d.p2min[d.P + i];
        mm = x < mm ? x : mm;
        jj = y < jj ? y : jj;
    }
    m = block_min(mm, s16);
    j = block_min(jj, s16);
    const RoundState* rs = d.rs;
    m = rs->rmin2[cur] < m ? rs->rmin2[cur] : m;
    m = m < SIMTIME_MAX ? m : SIMTIME_MAX;
    j = rs->jmin < j ? rs->jmin : j;
}

// Cumulative counters (stats on demand) and pending events.
__global__ __launch_bounds__(1024) void k_stats(Dev d, unsigned long long* pending) {
    __shared__ uint64_t s16[16];
    uint64_t c[NCTR];
    for (int i = 0; i < NCTR; ++i) c[i] = 0;
    for (uint32_t b = threadIdx.x; b < d.P; b += 1024)
        for (int i = 0; i < NCTR; ++i) c[i] += d.pcum[(size_t)i * d.P + b];
    // pending: live calendar events outside the current window's buckets (the
    // straddling one's stay; the window's events are in the host partitions,
    // gathered or routed by k_scatter and not yet popped, or, when none was
    // listed, popped) and outside the window before it (consumed, reset by the
    // next k_proc)
    const RoundState* rs = d.rs;
    const bool listed = rs->listed != 0;
    const uint64_t bS = rs->bS, span = rs->bL - rs->bS;
    const uint32_t bSr = (uint32_t)(bS % d.R);
    const uint32_t retr = rs->ret_b != UINT64_MAX ? (uint32_t)(rs->ret_b % d.R) : UINT32_MAX;
    const uint64_t pbS = rs->pbS, pbL = rs->pbL;
    uint64_t pend = 0;
    for (uint32_t rb = threadIdx.x; rb < d.R; rb += 1024) {
        const uint64_t o = rb >= bSr ? rb - bSr : rb + d.R - bSr;
        if (o <= span && rb != retr) continue;  // listed (gathered), or, none listed, consumed
        const uint64_t past = bS + o - d.R;  // the slot's bucket before the window (wraps when none)
        if (pbS != UINT64_MAX && past >= pbS && past <= pbL) continue;  // consumed, reset by the next k_proc
        for (uint32_t x = 0; x < XS; ++x) pend += d.bk[(size_t)x * d.R + rb];
        pend -= d.btomb[rb];
    }
    if (listed)
        for (uint32_t p = threadIdx.x; p < d.P; p += 1024) pend += d.pcnt[p];
    for (int i = 0; i < NCTR; ++i) {
        const uint64_t t = block_sum(c[i], s16);
        if (threadIdx.x == 0) d.rs->ctr[i] = t;
    }
    pend = block_sum(pend, s16);
    if (threadIdx.x == 0) *pending = pend;
}

// Test only (sg_engine_debug_inject): corrupts two of partition 0's staged
// records between a k_proc and its k_scatter, as a corrupt calendar or a
// staging bug would (profiles/r04/ablation/README.md: the round-4 fault): one
// names a host past the shard, one lies beyond the calendar's horizon.  The
// insert role must clamp both in bounds and flag OV_BUG.  One thread.
__global__ void k_inject(Dev d) {
    const uint32_t n = d.rcnt[0];
    if (n < 2) return;
    Rec* r = d.loc;
    r[0].a = (r[0].a & M40) | ((uint64_t)(d.L + 7) << 40);         // an impossible host
    r[1].a = (r[1].a & ~M40) | ((uint64_t)2 * d.R * d.W & M40);   // beyond R buckets of the window
}

}  // namespace

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
struct sg_engine {
    sg_phold_params p;
    Dev d;
    std::vector<uint32_t> host_of_slot;  // local slot -> registration index
    int device;
    hipStream_t stream;
    bool own_stream;
    bool booted;
    std::vector<void*> allocs;
    uint32_t* pcount_buf = nullptr;  // path packet counters, once enabled
    uint64_t* wtime_buf = nullptr;   // barrier timers, once enabled
    RoundState* h_rs;  // pinned
    unsigned long long* d_pend;
    bool timing;
    uint32_t timing_mask;  // kernel classes timed while timing is on
    bool debug_sync;  // SG_DEBUG_SYNC=1: synchronise after every launch, name the faulting class
    struct Pair { hipEvent_t a, b; int cls; };
    std::vector<Pair> pending_ev;
    std::vector<hipEvent_t> free_ev;
    double ms[SG_KCLASSES];
    uint64_t launches[SG_KCLASSES];
    // hipGraph replay of batches of rounds / steps (sg_engine_set_graph)
    uint32_t graph_batch = 0;
    uint64_t gen = 0;  // bumped whenever a kernel argument captured in a graph changes
    bool inject = false;  // sg_engine_debug_inject: corrupt the next round's staged records
    hipGraphExec_t gexec = nullptr;
    hipEvent_t batch_ev[2] = {nullptr, nullptr};  // sg_engine_enqueue_rounds' queue bound
    const int64_t* last_recv = nullptr;  // the last step_recv's buffer (read by the next k_proc)
    uint64_t last_rows = 0, last_cap = 0;  // its layout
    int64_t* recv_hold = nullptr;          // a copy of it kept across set_exchange_cap
    size_t recv_hold_bytes = 0;
    struct GraphKey {
        uint64_t gen;
        const void *send, *recv, *comm;
        const void* staged;  // the receive buffer the batch's first k_proc stages from
        uint32_t n;
        bool operator==(const GraphKey& o) const {
            return gen == o.gen && send == o.send && recv == o.recv && comm == o.comm && staged == o.staged &&
                   n == o.n;
        }
    } gkey{};
};

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t _e = (x);                                                           \
        if (_e != hipSuccess) {                                                        \
            sg_set_error("%s failed: %s (%s:%d)", #x, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                    \
            return SG_ERR_HIP;                                                         \
        }                                                                              \
    } while (0)

template <typename T>
static int dalloc(sg_engine* e, T** p, size_t n) {
    void* ptr = nullptr;
    if (n == 0) n = 1;
    hipError_t err = hipMalloc(&ptr, n * sizeof(T));
    if (err != hipSuccess) {
        sg_set_error("hipMalloc(%zu bytes) failed: %s", n * sizeof(T), hipGetErrorString(err));
        return SG_ERR_NOMEM;
    }
    e->allocs.push_back(ptr);
    *p = (T*)ptr;
    return SG_OK;
}

static hipEvent_t get_event(sg_engine* e) {
    if (!e->free_ev.empty()) {
        hipEvent_t ev = e->free_ev.back();
        e->free_ev.pop_back();
        return ev;
    }
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return nullptr;
    return ev;
}

// launch(a, b) enqueues the work; with timing on for its class, a and b are
// events for it to stamp.  Kernels take them as the dispatch packet's own
// start / stop timestamps (hipExtLaunchKernelGGL, SG_LAUNCH): no extra packets
// around the kernel, so the measured duration is the kernel's.  The RCCL
// exchange records them on the stream around the collective.
template <typename F>
static int timed_launch(sg_engine* e, int cls, F&& launch) {
    hipEvent_t a = nullptr, b = nullptr;
    const bool timed = e->timing && (e->timing_mask >> cls & 1u);
    if (timed) {
        a = get_event(e);
        b = get_event(e);
        if (!a || !b) a = b = nullptr;
    }
    launch(a, b);
    HIPCHK(hipGetLastError());
    if (e->debug_sync) {
        const hipError_t err = hipStreamSynchronize(e->stream);
        if (err != hipSuccess) {
            static const char* names[SG_KCLASSES] = {"process", "insert", "plan", "gather", "exchange"};
            sg_set_error("kernel class %s (launch %llu) failed: %s", names[cls],
                         (unsigned long long)e->launches[cls], hipGetErrorString(err));
            return SG_ERR_HIP;
        }
    }
    if (a && b) e->pending_ev.push_back({a, b, cls});
    e->launches[cls]++;
    return SG_OK;
}

#define SG_LAUNCH(kernel, grid, block, shmem, stream, ev_a, ev_b, ...)                              \
    do {                                                                                          \
        if (ev_a) hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, ev_a, ev_b, 0, __VA_ARGS__); \
        else hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                \
    } while (0)

static void harvest_timing(sg_engine* e) {
    for (auto& pr : e->pending_ev) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pr.a, pr.b) == hipSuccess) e->ms[pr.cls] += ms;
        e->free_ev.push_back(pr.a);
        e->free_ev.push_back(pr.b);
    }
    e->pending_ev.clear();
}

static uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* s = getenv(name);
    if (!s || !*s) return dflt;
    const long v = strtol(s, nullptr, 10);
    return v > 0 ? (uint32_t)v : dflt;
}
// As env_u32, but 0 is a value (debug switches whose 0 setting means something).
static uint32_t env_u32z(const char* name, uint32_t dflt) {
    const char* s = getenv(name);
    if (!s || !*s) return dflt;
    const long v = strtol(s, nullptr, 10);
    return v >= 0 ? (uint32_t)v : dflt;
}

extern "C" {

int sg_engine_create(const sg_phold_params* params, const sg_phold_tables* t, int device,
                     void* hip_stream, sg_engine** out) {
    if (!params || !t || !out) {
        sg_set_error("sg_engine_create: NULL argument");
        return SG_ERR_INVAL;
    }
    *out = nullptr;
    const sg_phold_params& p = *params;
    const uint32_t G = p.shard_count ? p.shard_count : 1;
    if (p.n_hosts == 0 || p.n_hosts > (1u << (64 - SRC_SHIFT)) || p.n_vertices == 0 || p.n_vertices > 0xFFFFu || G > MAXG ||
        p.shard_index >= G || G > p.n_hosts || !t->host_vertex || !t->host_rng || !t->delay_ns ||
        !t->keep_max || !t->jump_ms || (p.dst_rule == SG_DST_WEIGHTS && !t->weight_thresh) ||
        p.dst_rule > 1 || p.window_rule > 1 || p.load == 0 || p.workload > SG_WORKLOAD_GOSSIP) {
        sg_set_error("sg_engine_create: invalid parameters (n_hosts must be in [1, 2^24], n_vertices in [1, 65535])");
        return SG_ERR_INVAL;
    }
    if (p.workload == SG_WORKLOAD_GOSSIP &&
        (p.gossip_msgs == 0 || p.gossip_msgs > p.n_hosts || p.gossip_msgs > 65536)) {
        sg_set_error("sg_engine_create: gossip needs 1 <= gossip_msgs <= min(n_hosts, 65536)");
        return SG_ERR_INVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || device < 0 || device >= ndev) {
        sg_set_error("sg_engine_create: no HIP device %d (count %d)", device, ndev);
        return SG_ERR_NODEV;
    }
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        sg_set_error("sg_engine_create: device %d is %s, need gfx950", device, prop.gcnArchName);
        return SG_ERR_NODEV;
    }
    HIPCHK(hipSetDevice(device));

    Dev d;
    memset(&d, 0, sizeof d);
    d.N = p.n_hosts;
    d.V = p.n_vertices;
    d.G = G;
    d.g = p.shard_index;
    for (uint32_t i = 0; i <= G; ++i) d.bounds[i] = (uint32_t)(((uint64_t)i * p.n_hosts) / G);
    d.lo = d.bounds[d.g];
    d.L = d.bounds[d.g + 1] - d.lo;
    if (d.L == 0) {
        sg_set_error("sg_engine_create: shard has no hosts");
        return SG_ERR_INVAL;
    }
    for (uint32_t i = 0; G > 1 && i < G; ++i)
        if (d.bounds[i + 1] - d.bounds[i] >= (1u << 24)) {  // a 16-B exchange row keeps 24 bits of it
            sg_set_error("sg_engine_create: shard %u has %u hosts, at most 2^24 with several shards", i,
                         d.bounds[i + 1] - d.bounds[i]);
            return SG_ERR_INVAL;
        }
    d.load = p.load;
    d.workload = p.workload;
    if (p.workload == SG_WORKLOAD_GOSSIP) {
        d.msg_shift = 16;  // srcHostEventID keeps 24 bits: 16M sends per host
        d.gossip_msgs = p.gossip_msgs;
        d.mw = (p.gossip_msgs + 31) / 32;
        d.gossip_start = p.gossip_start;
        d.gossip_interval = p.gossip_interval;
    }
    d.dst_rule = p.dst_rule;
    d.window_rule = p.window_rule;
    d.end_time = p.end_time;
    d.bootstrap_end = p.bootstrap_end;
    d.fixed_jump = p.fixed_jump;
    d.runahead_min = p.runahead_min;
    d.trace_cap = p.trace_capacity;
    d.xcap = p.exchange_cap ? p.exchange_cap : 4096;
    d.xrows = HDR + d.xcap;

    // Calendar geometry: bucket width W = the narrowest window the rules allow
    // after the first, ring R covering the widest window plus the longest delay.
    const size_t VV = (size_t)d.V * d.V;
    uint64_t max_delay = 0, max_jump_ms = 0;
    for (size_t i = 0; i < VV; ++i) {
        max_delay = std::max<uint64_t>(max_delay, t->delay_ns[i]);
        max_jump_ms = std::max<uint64_t>(max_jump_ms, t->jump_ms[i]);
    }
    uint64_t W, max_jump;
    if (p.window_rule == SG_WINDOW_FIXED) {
        W = std::max<uint64_t>(p.fixed_jump, 1);
        max_jump = p.fixed_jump;
    } else {
        W = std::max<uint64_t>(p.runahead_min, SG_ONE_MS);
        max_jump = std::max<uint64_t>(std::max<uint64_t>(10 * SG_ONE_MS, p.runahead_min),
                                      max_jump_ms * SG_ONE_MS);
    }
    uint64_t span = max_jump + max_delay + 2;
    if (p.workload == SG_WORKLOAD_GOSSIP) {  // origin self events are scheduled at boot
        const uint64_t last = p.gossip_start + (uint64_t)(p.gossip_msgs - 1) * p.gossip_interval;
        span = std::max<uint64_t>(span, std::min<uint64_t>(last, p.end_time) + 2);
    }
    if (span >= (1ULL << 39)) {
        sg_set_error("sg_engine_create: window + delay span %llu ns exceeds 2^39 ns",
                     (unsigned long long)span);
        return SG_ERR_INVAL;
    }
    // a window spans at most max_jump / W + 2 buckets: at most NBMAX (the
    // gather's due segments)
    if (max_jump / W + 2 > NBMAX) W = max_jump / (NBMAX - 2) + 1;
    if (span / W + 3 > RMAX) W = (span + RMAX - 4) / (RMAX - 3);
    if (W >= (1ULL << 32)) {
        sg_set_error("sg_engine_create: bucket width %llu ns too large", (unsigned long long)W);
        return SG_ERR_INVAL;
    }
    d.W = W;
    d.R = (uint32_t)(span / W + 3);
    // SG_NO_RING32=1 (tests): the 64-bit bucket arithmetic everywhere, as for a
    // calendar whose horizon passes 2^32 ns
    d.ring32 = (uint64_t)d.R * W < (1ull << 32) && env_u32("SG_NO_RING32", 0) == 0;
    d.wdiv = make_div32(W);
    // the receive role's workgroups: none on one shard (a world-1 step receives
    // only its own header block)
    d.G3 = env_u32("SG_INS_GRID", p.shard_count > 1 ? 128 : 0);
    // default event slots per host: PHOLD keeps `load` events per host in flight;
    // gossip floods keep about ten fan-outs' worth (configs[4]: 82 per host at peak)
    const uint64_t qc = p.queue_cap ? p.queue_cap
                                    : p.workload == SG_WORKLOAD_GOSSIP ? std::max<uint64_t>(64, 24ull * p.load) : 64;
    const uint64_t base_ch = ((uint64_t)d.L * qc + CH - 1) / CH;
    if (d.G3 > G3MAX) {
        sg_set_error("sg_engine_create: SG_INS_GRID %u exceeds %u", d.G3, G3MAX);
        return SG_ERR_INVAL;
    }
    d.G1 = env_u32("SG_GATHER_GRID", 128);
    d.gspec_mode = env_u32z("SG_GSPEC", 1);
    d.xfence = 0;  // set per exchange link (sg_xlink_attach: SG_XFENCE, else fenced across devices)
    d.check = env_u32("SG_CHECK", 0) != 0;
    d.snd_lds = env_u32("SG_SND_LDS", 1) != 0;
    // host partitions: HP hosts per k_proc workgroup, about one partition per
    // CU: HP = ceil(L / 256) rounded up to a multiple of 16 (P = 245 at 1M
    // hosts with powers of two left 11 CUs idle).  A shard above 64k hosts
    // keeps at least 2048 hosts per partition: at 125k and 250k hosts (one of
    // eight or four shards of configs[3]) every kernel is at its latency
    // floor, and fewer workgroups cut the contention on the shared bucket and
    // partition counters: world-1 steps 44.8-45.7 -> 39.5-40.2 us at 125k,
    // 48.9-49.1 -> 44.8-46.2 us at 250k (profiles/r04/hp125k).  The floor
    // applies from 64k hosts up, so 500k gets 2048 as well (245 partitions;
    // 3907 was slower there).  It was measured on the world-1 step path; a
    // single-shard round of 64k-500k hosts runs with it unmeasured.  PHOLD
    // only: configs[4]'s gossip hosts carry ~3 due events each, and 49
    // partitions of 2048 left 200 CUs idle (k_proc 136 us per round).
    const uint32_t hp_env = env_u32("SG_HP", 0);
    uint32_t hp_auto = ((d.L + 255) / 256 + 15) / 16 * 16;
    if (d.L > 65536 && hp_auto < 2048 && p.workload == SG_WORKLOAD_PHOLD) hp_auto = 2048;
    d.HP = std::min<uint32_t>(HPMAX, std::max<uint32_t>(64, hp_env ? hp_env : hp_auto));
    d.hpdiv = make_div32(d.HP);
    d.P = (d.L + d.HP - 1) / d.HP;
    if (d.P > PMAX) {
        sg_set_error("sg_engine_create: %u partitions exceed %u", d.P, PMAX);
        return SG_ERR_INVAL;
    }
    {
        // every live sub-list may hold one partly filled chunk; the reserving
        // rows' stashes hold ST chunks each
        const uint64_t nch = base_ch + (uint64_t)XS * d.R + 64 + (uint64_t)(d.P + d.G3) * ST;
        if (nch >= (1ULL << 31) || (uint64_t)XS * d.R * nch > (1ULL << 31)) {
            sg_set_error("sg_engine_create: calendar too large (R=%u chunks=%llu); lower queue_cap",
                         d.R, (unsigned long long)nch);
            return SG_ERR_INVAL;
        }
        d.NCH = (uint32_t)nch;
    }
    // Slots: every shard's hosts in (vertex, index) order.  Every shard knows
    // every host's global slot (the destination of a send is a slot).
    for (size_t i = 0; i < p.n_hosts; ++i)
        if (t->host_vertex[i] >= d.V) {
            sg_set_error("sg_engine_create: host %zu attached to vertex %u >= %u", i, t->host_vertex[i], d.V);
            return SG_ERR_INVAL;
        }
    std::vector<uint32_t> slot_of(p.n_hosts), host_of_slot(d.L);
    {
        std::vector<uint32_t> ord;
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t b0 = d.bounds[g], b1 = d.bounds[g + 1];
            ord.resize(b1 - b0);
            for (uint32_t i = 0; i < b1 - b0; ++i) ord[i] = b0 + i;
            std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
                return t->host_vertex[x] < t->host_vertex[y];
            });
            for (uint32_t i = 0; i < b1 - b0; ++i) {
                slot_of[ord[i]] = b0 + i;
                if (g == d.g) host_of_slot[i] = ord[i];
            }
        }
    }
    // path-record format: delays below 2^32 ns fit the narrow records
    uint64_t max_delay_all = 0, gjmin = UINT64_MAX;
    bool all_keep = true;
    for (size_t i = 0; i < VV; ++i) {
        max_delay_all = std::max<uint64_t>(max_delay_all, t->delay_ns[i]);
        gjmin = std::min<uint64_t>(gjmin, t->jump_ms[i]);
        all_keep &= t->keep_max[i] >= SG_RAND_MAX;
    }
    d.pair_fmt = max_delay_all >> 32 ? PAIR_WIDE : all_keep ? PAIR_DELAY : PAIR_NARROW;
    {
        const uint32_t fmt_env = env_u32z("SG_PAIR_FMT", 99);  // debugging: force a wider format
        if (fmt_env < d.pair_fmt) d.pair_fmt = fmt_env;
    }
    // a partition's path rows in LDS when they fit (vertex span x V records)
    d.rows_max = 0;
    for (uint32_t q = 0; q < d.P; ++q) {
        const uint32_t s0 = q * d.HP, s1 = std::min<uint32_t>(d.L, s0 + d.HP);
        const uint32_t nrow = t->host_vertex[host_of_slot[s1 - 1]] - t->host_vertex[host_of_slot[s0]] + 1;
        d.rows_max = std::max(d.rows_max, nrow);
    }
    const uint32_t resz = d.pair_fmt == PAIR_NARROW ? 8 : 4;
    const uint64_t row_bytes = (uint64_t)d.rows_max * d.V * resz;
    d.lds_rows = d.pair_fmt != PAIR_WIDE && row_bytes <= (32u << 10) && env_u32("SG_NO_LDS_ROWS", 0) == 0;
    // k_proc dynamic LDS: per-host arrays (18 B per host), the bucket bins
    // (2 x R u32), the partition's path rows, then the event image (EVL due
    // events, 16 B each).  Two workgroups per CU when there are more
    // partitions than CUs.
    d.bin_off = (d.HP * 18 + 15) & ~15u;
    d.row_off = d.bin_off + ((8 * d.R + 15) & ~15u);
    // (the rows region in whole 1 KB pieces: one global_load_lds wave
    // instruction fills 1 KB)
    const uint32_t row_region = d.lds_rows ? (uint32_t)((row_bytes + 1023) & ~1023ull) : 0u;
    d.row_pieces = row_region / 16;
    d.ev_off = d.row_off + row_region;
    {
        uint32_t wgs = d.P > 256 ? 2 : 1, evl = 0;
        for (;;) {
            const uint32_t dyn = (160u << 10) / wgs - PROC_LDS_STATIC;
            evl = dyn > d.ev_off ? (dyn - d.ev_off) / 16 : 0;
            if (wgs == 1 || evl >= 1024) break;
            wgs = 1;
        }
        evl = std::min<uint32_t>(std::min<uint32_t>(evl, EVLMAX), env_u32("SG_EVL", EVLMAX));
        d.EVL = evl;
        d.proc_lds = d.ev_off + evl * 16;
        if (d.proc_lds > (156u << 10)) {
            sg_set_error("sg_engine_create: k_proc needs %u B of LDS (HP=%u, R=%u)", d.proc_lds, d.HP, d.R);
            return SG_ERR_INVAL;
        }
    }
    const uint32_t per_host = std::max<uint32_t>(32, 2 * d.load);
    d.CAPP = d.HP * per_host;
    d.ECAP = d.HP * per_host + 1024;

    sg_engine* e = new sg_engine();
    e->p = p;
    e->device = device;
    e->timing = false;
    e->debug_sync = env_u32("SG_DEBUG_SYNC", 0) != 0;
    for (int i = 0; i < SG_KCLASSES; ++i) {
        e->ms[i] = 0;
        e->launches[i] = 0;
    }
    e->d = d;
    Dev& D = e->d;

    int rc = SG_OK;
    const size_t N = D.N, L = D.L, P = D.P;
#define ALLOC(ptr, n)                                  \
    do {                                               \
        if ((rc = dalloc(e, &(ptr), (n))) != SG_OK) {  \
            sg_engine_destroy(e);                      \
            return rc;                                 \
        }                                              \
    } while (0)
    HostInfo* hinfo;
    uint2* nearw = nullptr;
    SlotInfo* sinfo;
    PairRec* pairs = nullptr;
    uint2* pairs8 = nullptr;
    uint32_t *pdelay = nullptr, *pjump = nullptr;
    ALLOC(hinfo, N);
    ALLOC(sinfo, L);
    D.sinfo = sinfo;
    e->host_of_slot = host_of_slot;
    D.gjmin = gjmin;
    bool sym = D.pair_fmt != PAIR_WIDE && env_u32("SG_NO_TRI", 0) == 0;
    for (size_t a = 0; sym && a < D.V; ++a)
        for (size_t b = 0; sym && b < a; ++b) {
            const size_t i = a * D.V + b, j = b * D.V + a;
            sym = t->delay_ns[i] == t->delay_ns[j] && t->keep_max[i] == t->keep_max[j] &&
                  t->jump_ms[i] == t->jump_ms[j];
        }
    D.tri = sym ? 1 : 0;
    const size_t NT = D.tri ? (size_t)D.V * (D.V + 1) / 2 : VV;  // narrow table entries
    if (D.pair_fmt == PAIR_WIDE) {
        ALLOC(pairs, VV);
    } else {
        if (D.pair_fmt == PAIR_NARROW) ALLOC(pairs8, NT);
        else ALLOC(pdelay, NT);
        ALLOC(pjump, NT);
    }
    D.pairs8 = pairs8;
    D.pdelay = pdelay;
    D.pjump = pjump;
    void* prow = nullptr;
    if (D.lds_rows) {
        unsigned char* pr_ = nullptr;
        ALLOC(pr_, VV * resz + 16);  // + a 16-B piece: k_proc's row pieces may read past the last row
        prow = pr_;
    }
    D.prow = prow;
    uint64_t* vself;
    ALLOC(vself, D.V);
    D.hinfo = hinfo;
    // exact guess: with the weights rule, every host's x range [wt[i-1]+1, wt[i]]
    // must map to i under the (monotone) guess, so checking both ends suffices
    // a lane's later light hosts record their sends for phase B instead: their
    // chains then overlap every other lane's instead of running after them
    D.light_q = env_u32z("SG_LIGHT_Q", 1);
    D.light_max = std::min<uint32_t>(env_u32z("SG_LIGHT_MAX", 2), 2);
    D.rec_all = env_u32z("SG_REC_ALL", 2 * K2_T);
    D.flat = env_u32z("SG_FLAT", 1) != 0 && D.workload == SG_WORKLOAD_PHOLD;
    D.grec = env_u32z("SG_GREC", 1) != 0 ? 1u : 0u;
    D.gskip_on = env_u32z("SG_GSKIP", 1) != 0 ? 1u : 0u;
    D.gflat = env_u32z("SG_GFLAT", 1) != 0 ? 1u : 0u;
    // near guess: with the weights rule, every host's x range [wt[i-1]+1, wt[i]]
    // must map to i - 1 or i under the (monotone) guess, so checking both ends
    // suffices; the floor rule's guess is its answer
    D.dst_near = 0;
    if (D.V <= 65536 && env_u32("SG_NO_EXACT_DST", 0) == 0) {
        bool ok = true;
        if (p.dst_rule == SG_DST_WEIGHTS) {
            auto guess = [&](int64_t x) {
                const uint64_t g = ((uint64_t)x * N) >> 31;
                return g >= N ? N - 1 : g;
            };
            auto near = [&](uint64_t g, size_t i) { return g == i || g + 1 == i; };
            int64_t prev = -1;
            for (size_t i = 0; i < N && ok; ++i) {
                const int64_t hi = t->weight_thresh ? t->weight_thresh[i] : 0;
                if (hi > prev && hi >= 0) {
                    const int64_t lo = prev + 1 > 0 ? prev + 1 : 0;
                    const int64_t hc = hi < SG_RAND_MAX ? hi : SG_RAND_MAX;
                    if (lo <= hc) ok = near(guess(lo), i) && near(guess(hc), i);
                }
                prev = hi > prev ? hi : prev;
            }
            ok = ok && t->weight_thresh != nullptr;
        }
        D.dst_near = ok ? 1 : 0;
    }
    // vertex and global slot in one word
    D.slot_bits = 1;
    while (D.slot_bits < 32 && (1ull << D.slot_bits) < N) ++D.slot_bits;
    {
        uint32_t vbits = 1;
        while ((1ull << vbits) < D.V) ++vbits;
        if (D.slot_bits + vbits > 32) D.dst_near = 0;  // the probe path carries slots instead
    }
    if (D.dst_near) ALLOC(nearw, N + 1);
    D.nearw = nearw;
    D.pairs = pairs;
    D.vself = vself;
    ALLOC(D.hs, L);
    if (D.workload == SG_WORKLOAD_GOSSIP) ALLOC(D.seen, L * D.mw);
    ALLOC(D.pool, (size_t)D.NCH * CH);
    ALLOC(D.btab, (size_t)XS * D.R * D.NCH);
    ALLOC(D.bk, (size_t)XS * D.R);
    ALLOC(D.bw, (size_t)2 * XS * D.R);
    ALLOC(D.btomb, D.R);
    ALLOC(D.bmin, D.R);
    ALLOC(D.pmin, (size_t)D.P * D.R);
    ALLOC(D.fring, D.NCH);
    ALLOC(D.stash, (size_t)(D.P + D.G3) * ST);
    ALLOC(D.stn, D.P + D.G3);
    ALLOC(D.wbase, (size_t)(D.P + D.G3) * D.R);
    ALLOC(D.gspec, 1);
    ALLOC(D.tick, 8);
    ALLOC(D.pcnt, P);
    ALLOC(D.part, P * D.CAPP);
    ALLOC(D.part2, P * D.CAPP);
    ALLOC(D.extras, P * K2_T * XCAP);
    ALLOC(D.rcnt, P);
    ALLOC(D.loc, P * D.ECAP);
    ALLOC(D.sends, P * D.ECAP);
    ALLOC(D.p2min, 2 * P);
    ALLOC(D.pcum, NCTR * P);
    {
        // rand_r skip-ahead for the flat pass (its ranks stay below FLAT_CMAX):
        // glibc's LCG s -> 1103515245 s + 12345 runs three steps per draw, so an
        // event's two draws are six steps; {A, C} composes 6k of them.  An
        // earlier event whose destination draw selects no host (x above the
        // last weight threshold, e.g. x = RAND_MAX when the cumulative weight
        // rounds below 1) consumed one draw, not two: k_proc detects it and
        // sends that host to phase A's replay.  Off with a trace (the flat
        // pass writes an event's trace record before the check).
        D.skip = nullptr;
        if (env_u32z("SG_SKIP", 1) && !p.trace_capacity) {
            // gossip's record path draws up to load x 128 sends per host (the
            // first receipts of at most 128 messages) from the same table
            const uint32_t n = std::max<uint32_t>(FLAT_CMAX, p.workload == SG_WORKLOAD_GOSSIP ? p.load * 128 + 1 : 0);
            D.nskip = n;
            std::vector<uint2> sk(n);
            uint32_t A = 1, C = 0;
            for (uint32_t k = 0; k < n; ++k) {
                sk[k] = make_uint2(A, C);
                for (int i = 0; i < 6; ++i) {  // compose one more LCG step: s -> a (A s + C) + c
                    A = 1103515245u * A;
                    C = 1103515245u * C + 12345u;
                }
            }
            uint2* dsk = nullptr;
            ALLOC(dsk, n);
            HIPCHK(hipMemcpy(dsk, sk.data(), n * sizeof(uint2), hipMemcpyHostToDevice));
            D.skip = dsk;
        }
    }
    if (G > 1 || p.exchange_cap) {  // step API (a single shard may use it too: exchange_cap != 0)
        ALLOC(D.remn, P);
        ALLOC(D.rem, P * D.ECAP);
        ALLOC(D.rem_dst, P * D.ECAP);
        D.oreg = (uint64_t)P * D.ECAP;
        ALLOC(D.outq, (size_t)G * D.oreg * RW);
        ALLOC(D.outn, G);
        ALLOC(D.sent, G);
    }
    ALLOC(D.rs, 1);
    ALLOC(e->d_pend, 1);
    if (D.trace_cap) ALLOC(D.trace, D.trace_cap);
    if (env_u32("SG_STAMPS", 0)) ALLOC(D.stamps, (2 * P + D.G3 + D.G1 + 3) * SG_STAMP_W);  // + a spare row, k_scatter's
    D.wlog_cap = D.trace_cap ? 1u << 20 : 0;
    if (D.wlog_cap) ALLOC(D.wlog, 2 * D.wlog_cap);
#undef ALLOC

    if (hip_stream) {
        e->stream = (hipStream_t)hip_stream;
        e->own_stream = false;
    } else {
        if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
            sg_engine_destroy(e);
            sg_set_error("hipStreamCreate failed");
            return SG_ERR_HIP;
        }
        e->own_stream = true;
    }
    if (hipHostMalloc((void**)&e->h_rs, sizeof(RoundState), hipHostMallocDefault) != hipSuccess) {
        e->h_rs = nullptr;
        sg_engine_destroy(e);
        sg_set_error("hipHostMalloc failed");
        return SG_ERR_NOMEM;
    }
    // pack the tables on the host
    std::vector<HostInfo> hi(N);
    for (size_t i = 0; i < N; ++i) {
        hi[i].vertex = t->host_vertex[i];
        hi[i].wt = t->weight_thresh ? t->weight_thresh[i] : 0;
        hi[i].slot = slot_of[i];
        hi[i].pad = 0;
    }
    std::vector<PairRec> pr(D.pair_fmt == PAIR_WIDE ? VV : 0);
    std::vector<uint2> pr8(D.pair_fmt == PAIR_NARROW ? NT : 0);
    std::vector<uint32_t> pd(D.pair_fmt == PAIR_DELAY ? NT : 0), pj(D.pair_fmt != PAIR_WIDE ? NT : 0);
    for (size_t i = 0; i < VV; ++i) {
        const size_t a = i / D.V, b = i % D.V;
        if (D.tri && b > a) continue;  // the lower triangle (a >= b) holds every pair
        const size_t o = D.tri ? a * (a + 1) / 2 + b : i;  // pair_index
        if (D.pair_fmt == PAIR_WIDE) pr[i] = PairRec{t->delay_ns[i], t->keep_max[i], t->jump_ms[i]};
        else if (D.pair_fmt == PAIR_NARROW) pr8[o] = make_uint2((uint32_t)t->delay_ns[i], (uint32_t)t->keep_max[i]);
        else pd[o] = (uint32_t)t->delay_ns[i];
        if (D.pair_fmt != PAIR_WIDE) pj[o] = t->jump_ms[i];
    }
    std::vector<uint64_t> vs(D.V);
    for (size_t v = 0; v < D.V; ++v) vs[v] = t->delay_ns[v * D.V + v];
    D.vself_min = *std::min_element(vs.begin(), vs.end());
    std::vector<HostState> hs(L);
    std::vector<SlotInfo> si(L);
    for (size_t i = 0; i < L; ++i) {
        const uint32_t h = host_of_slot[i];
        hs[i] = HostState{t->host_rng[h], h, (uint64_t)t->host_vertex[h] << 48, 0, 0};  // evc 0 until boot
        si[i] = SlotInfo{h, t->host_vertex[h]};
    }
    hipError_t err = hipSuccess;
    err = err != hipSuccess ? err : hipMemcpy(hinfo, hi.data(), N * sizeof(HostInfo), hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(sinfo, si.data(), L * sizeof(SlotInfo), hipMemcpyHostToDevice);
    if (nearw) {
        std::vector<uint2> vt(N + 1);
        for (size_t i = 0; i < N; ++i)
            vt[i] = make_uint2((uint32_t)hi[i].wt, (hi[i].vertex << D.slot_bits) | slot_of[i]);
        vt[N] = vt[N - 1];  // read as record g + 1 of g = N - 1; never chosen (x > wt[N-1] has no host)
        err = err != hipSuccess ? err : hipMemcpy(nearw, vt.data(), (N + 1) * sizeof(uint2), hipMemcpyHostToDevice);
    }
    if (pairs) err = err != hipSuccess ? err : hipMemcpy(pairs, pr.data(), VV * sizeof(PairRec), hipMemcpyHostToDevice);
    if (pairs8) err = err != hipSuccess ? err : hipMemcpy(pairs8, pr8.data(), NT * sizeof(uint2), hipMemcpyHostToDevice);
    if (pdelay) err = err != hipSuccess ? err : hipMemcpy(pdelay, pd.data(), NT * 4, hipMemcpyHostToDevice);
    if (pjump) err = err != hipSuccess ? err : hipMemcpy(pjump, pj.data(), NT * 4, hipMemcpyHostToDevice);
    if (prow) {  // full row-major copy for k_proc's LDS rows
        if (D.pair_fmt == PAIR_NARROW) {
            std::vector<uint2> f(VV);
            for (size_t i = 0; i < VV; ++i) f[i] = make_uint2((uint32_t)t->delay_ns[i], (uint32_t)t->keep_max[i]);
            err = err != hipSuccess ? err : hipMemcpy(prow, f.data(), VV * 8, hipMemcpyHostToDevice);
        } else {
            std::vector<uint32_t> f(VV);
            for (size_t i = 0; i < VV; ++i) f[i] = (uint32_t)t->delay_ns[i];
            err = err != hipSuccess ? err : hipMemcpy(prow, f.data(), VV * 4, hipMemcpyHostToDevice);
        }
    }
    err = err != hipSuccess ? err : hipMemcpy(vself, vs.data(), D.V * sizeof(uint64_t), hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemcpy(D.hs, hs.data(), L * sizeof(HostState), hipMemcpyHostToDevice);
    err = err != hipSuccess ? err : hipMemset(D.rs, 0, sizeof(RoundState));
    err = err != hipSuccess ? err : hipMemset(D.pcum, 0, NCTR * P * 8);
    if (err != hipSuccess) {
        sg_set_error("table upload failed: %s", hipGetErrorString(err));
        sg_engine_destroy(e);
        return SG_ERR_HIP;
    }
    e->booted = false;
    *out = e;
    return SG_OK;
}

int sg_engine_destroy(sg_engine* e) {
    if (!e) return SG_OK;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (void* p : e->allocs) (void)hipFree(p);
    for (auto& pr : e->pending_ev) {
        (void)hipEventDestroy(pr.a);
        (void)hipEventDestroy(pr.b);
    }
    for (auto ev : e->free_ev) (void)hipEventDestroy(ev);
    if (e->h_rs) (void)hipHostFree(e->h_rs);
    if (e->gexec) (void)hipGraphExecDestroy(e->gexec);
    if (e->recv_hold) (void)hipFree(e->recv_hold);
    for (hipEvent_t ev : e->batch_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return SG_OK;
}

void* sg_engine_stream(sg_engine* e) { return e ? (void*)e->stream : nullptr; }

int sg_engine_host_range(sg_engine* e, uint32_t* first_host, uint32_t* n_local) {
    if (!e) return SG_ERR_INVAL;
    if (first_host) *first_host = e->d.lo;
    if (n_local) *n_local = e->d.L;
    return SG_OK;
}

int sg_engine_geometry(sg_engine* e, sg_engine_geom* out) {
    if (!e || !out) return SG_ERR_INVAL;
    const Dev& d = e->d;
    out->bucket_width = d.W;
    out->ring_buckets = d.R;
    out->chunk_events = CH;
    out->chunks = d.NCH;
    out->partition_hosts = d.HP;
    out->partitions = d.P;
    out->partition_cap = d.CAPP;
    out->stage_cap = d.ECAP;
    return SG_OK;
}

int sg_engine_boot(sg_engine* e) {
    if (!e) return SG_ERR_INVAL;
    if (e->booted) {
        sg_set_error("sg_engine_boot: already booted");
        return SG_ERR_STATE;
    }
    HIPCHK(hipSetDevice(e->device));
    const Dev& d = e->d;
    // each instantiation's dynamic LDS, checked against its static LDS (the
    // sizing above reserves PROC_LDS_STATIC for it): 160 KB per CU in all
    const void* procs[] = {(const void*)k_proc<true, true, false>, (const void*)k_proc<true, false, false>,
                           (const void*)k_proc<false, true, false>, (const void*)k_proc<false, false, false>,
                           (const void*)k_proc<true, true, true>, (const void*)k_proc<true, false, true>,
                           (const void*)k_proc<false, true, true>, (const void*)k_proc<false, false, true>};
    for (const void* f : procs) {
        hipFuncAttributes fa;
        HIPCHK(hipFuncGetAttributes(&fa, f));
        if (fa.sharedSizeBytes > PROC_LDS_STATIC || fa.sharedSizeBytes + d.proc_lds > (160u << 10)) {
            sg_set_error("sg_engine_boot: k_proc needs %zu B of static LDS beside %u B dynamic (reserved %u)",
                         (size_t)fa.sharedSizeBytes, d.proc_lds, PROC_LDS_STATIC);
            return SG_ERR_INVAL;
        }
        HIPCHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)d.proc_lds));
    }
    HIPCHK(hipMemsetAsync(d.btab, 0xFF, (size_t)XS * d.R * d.NCH * sizeof(uint32_t), e->stream));
    HIPCHK(hipMemsetAsync(d.gspec, 0xFF, sizeof(GSpec), e->stream));  // no guess (fold UINT64_MAX)
    const uint32_t n = std::max<uint32_t>(std::max<uint32_t>(d.L, d.NCH),
                                          std::max<uint32_t>(d.R, d.P + d.G3));
    hipLaunchKernelGGL(k_boot, dim3((n + 255) / 256), dim3(256), 0, e->stream, d);
    HIPCHK(hipGetLastError());
    // the first window's gather (k_scatter's gather role; nothing is staged
    // yet) and the first stash refill
    hipLaunchKernelGGL(k_scatter, dim3(d.P + d.G1 + 2), dim3(K3_T), 0, e->stream, d, (const int64_t*)nullptr, 2);
    HIPCHK(hipGetLastError());
    e->booted = true;
    return SG_OK;
}

static int enqueue_process(sg_engine* e) {
    const Dev& d = e->d;
    return timed_launch(e, SG_K_PROCESS, [&](hipEvent_t a, hipEvent_t b) {
        const dim3 g(d.P), t(K2_T);
        if (d.flat) {
            if (d.dst_near && d.lds_rows) SG_LAUNCH((k_proc<true, true, true>), g, t, d.proc_lds, e->stream, a, b, d);
            else if (d.dst_near) SG_LAUNCH((k_proc<true, false, true>), g, t, d.proc_lds, e->stream, a, b, d);
            else if (d.lds_rows) SG_LAUNCH((k_proc<false, true, true>), g, t, d.proc_lds, e->stream, a, b, d);
            else SG_LAUNCH((k_proc<false, false, true>), g, t, d.proc_lds, e->stream, a, b, d);
        } else {
            if (d.dst_near && d.lds_rows) SG_LAUNCH((k_proc<true, true, false>), g, t, d.proc_lds, e->stream, a, b, d);
            else if (d.dst_near) SG_LAUNCH((k_proc<true, false, false>), g, t, d.proc_lds, e->stream, a, b, d);
            else if (d.lds_rows) SG_LAUNCH((k_proc<false, true, false>), g, t, d.proc_lds, e->stream, a, b, d);
            else SG_LAUNCH((k_proc<false, false, false>), g, t, d.proc_lds, e->stream, a, b, d);
        }
    });
}

// k_scatter: the staged events into the calendar, the next window planned and
// gathered; several shards (recv): the received events due in it routed.
// (Round 5 measured a split step — the window-independent half of k_scatter
// on a second stream beside the all-to-all — at 56-57 against 37.5 us per
// 125k-host step: the cross-stream fork and join cost more than the overlap
// saved, profiles/r05/split/; it was removed in round 6.)
static int enqueue_insert_plan(sg_engine* e, const int64_t* recv) {
    const Dev& d = e->d;
    return timed_launch(e, SG_K_INSERT, [&](hipEvent_t a, hipEvent_t b) {
        SG_LAUNCH(k_scatter, dim3(d.P + (recv ? d.G3 : 0) + d.G1 + 2), dim3(K3_T), 0, e->stream, a, b, d, recv,
                  recv ? 1 : 0);
    });
}

int sg_engine_enqueue_round(sg_engine* e) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_enqueue_round: engine not booted");
        return SG_ERR_STATE;
    }
    if (e->d.G != 1 || e->d.outn) {
        sg_set_error("sg_engine_enqueue_round: step-mode engine, use the step API");
        return SG_ERR_STATE;
    }
    int rc;
    if ((rc = enqueue_process(e))) return rc;
    if (e->inject) {  // test only
        e->inject = false;
        hipLaunchKernelGGL(k_inject, dim3(1), dim3(1), 0, e->stream, e->d);
        HIPCHK(hipGetLastError());
    }
    return enqueue_insert_plan(e, nullptr);
}

int sg_engine_debug_inject(sg_engine* e) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_debug_inject: engine not booted");
        return SG_ERR_STATE;
    }
    if (e->d.G != 1 || e->d.outn) {
        sg_set_error("sg_engine_debug_inject: round-mode engines only");
        return SG_ERR_STATE;
    }
    e->inject = true;
    return SG_OK;
}

// Enqueues n iterations of body (one round or one step each) on the engine
// stream.  With graphs on (sg_engine_set_graph) and a full batch, the
// iterations are captured once into a hipGraph and the graph is replayed while
// its key (buffers, communicator, captured kernel arguments) is unchanged.
extern "C++" template <typename F>
static int enqueue_batch(sg_engine* e, const sg_engine::GraphKey& key, uint32_t n, F&& body, bool launch = true) {
    const bool use = e->graph_batch && n == e->graph_batch && !e->timing && !e->debug_sync;
    if (!use) {
        for (uint32_t i = 0; i < n; ++i)
            if (int rc = body()) return rc;
        return SG_OK;
    }
    if (!e->gexec || !(e->gkey == key)) {
        if (e->gexec) {
            HIPCHK(hipGraphExecDestroy(e->gexec));
            e->gexec = nullptr;
        }
        HIPCHK(hipStreamBeginCapture(e->stream, hipStreamCaptureModeRelaxed));
        int rc = SG_OK;
        for (uint32_t i = 0; i < n && rc == SG_OK; ++i) rc = body();
        hipGraph_t g = nullptr;
        const hipError_t ce = hipStreamEndCapture(e->stream, &g);
        if (rc != SG_OK || ce != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            if (rc == SG_OK) sg_set_error("hipStreamEndCapture failed: %s", hipGetErrorString(ce));
            return rc != SG_OK ? rc : SG_ERR_HIP;
        }
        const hipError_t ie = hipGraphInstantiate(&e->gexec, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ie != hipSuccess) {
            e->gexec = nullptr;
            sg_set_error("hipGraphInstantiate failed: %s", hipGetErrorString(ie));
            return SG_ERR_HIP;
        }
        e->gkey = key;
    }
    if (launch) HIPCHK(hipGraphLaunch(e->gexec, e->stream));
    return SG_OK;
}

int sg_engine_graph_prepare(sg_engine* e) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_graph_prepare: engine not booted");
        return SG_ERR_STATE;
    }
    if (e->d.G != 1 || e->d.outn) {
        sg_set_error("sg_engine_graph_prepare: step-mode engine, the step loop captures its own graph");
        return SG_ERR_STATE;
    }
    const uint32_t n = e->graph_batch;
    // graphs off, or a setting under which enqueue_batch launches eagerly
    // (timing, SG_DEBUG_SYNC): nothing to capture, and nothing may run here
    if (!n || e->timing || e->debug_sync) return SG_OK;
    const sg_engine::GraphKey key{e->gen, nullptr, nullptr, nullptr, nullptr, n};
    return enqueue_batch(e, key, n, [&] { return sg_engine_enqueue_round(e); }, false);
}

int sg_engine_enqueue_rounds(sg_engine* e, uint64_t n_rounds) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_enqueue_rounds: engine not booted");
        return SG_ERR_STATE;
    }
    const uint32_t b = e->graph_batch ? e->graph_batch : 32;
    if (!e->batch_ev[0]) {
        HIPCHK(hipEventCreateWithFlags(&e->batch_ev[0], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&e->batch_ev[1], hipEventDisableTiming));
    }
    int rc;
    for (uint32_t k = 0; n_rounds; ++k) {
        const uint32_t n = n_rounds < b ? (uint32_t)n_rounds : b;
        const sg_engine::GraphKey key{e->gen, nullptr, nullptr, nullptr, nullptr, n};
        if ((rc = enqueue_batch(e, key, n, [&] { return sg_engine_enqueue_round(e); }))) return rc;
        n_rounds -= n;
        // at most two batches queued: wait for the one before this
        hipEvent_t& ev = e->batch_ev[k & 1];
        if (k) HIPCHK(hipEventSynchronize(e->batch_ev[(k + 1) & 1]));
        HIPCHK(hipEventRecord(ev, e->stream));
    }
    return SG_OK;
}

int sg_engine_sync(sg_engine* e) {
    if (!e) return SG_ERR_INVAL;
    HIPCHK(hipStreamSynchronize(e->stream));
    if (e->timing) harvest_timing(e);
    return SG_OK;
}

static int read_rs(sg_engine* e) {
    HIPCHK(hipMemcpyAsync(e->h_rs, e->d.rs, sizeof(RoundState), hipMemcpyDeviceToHost, e->stream));
    return sg_engine_sync(e);
}

int sg_engine_run(sg_engine* e, uint64_t max_rounds, uint32_t batch) {
    if (!e || !e->booted) {
        sg_set_error("sg_engine_run: engine not booted");
        return SG_ERR_STATE;
    }
    if (batch == 0) batch = 16;
    int rc = read_rs(e);
    if (rc) return rc;
    uint64_t done_rounds = 0;
    while (done_rounds < max_rounds && !e->h_rs->done) {
        uint64_t n = max_rounds - done_rounds;
        if (n > batch) n = batch;
        const sg_engine::GraphKey key{e->gen, nullptr, nullptr, nullptr, nullptr, (uint32_t)n};
        if ((rc = enqueue_batch(e, key, (uint32_t)n, [&] { return sg_engine_enqueue_round(e); })))
            return rc;
        done_rounds += n;
        if ((rc = read_rs(e))) return rc;
        if (e->h_rs->overflow) {
            sg_set_error("sg_engine_run: device capacity overflow (flags 0x%llx); raise queue_cap",
                         (unsigned long long)e->h_rs->overflow);
            return SG_ERR_OVERFLOW;
        }
    }
    return SG_OK;
}

int sg_engine_stats(sg_engine* e, sg_round_stats* out) {
    if (!e || !out) return SG_ERR_INVAL;
    hipLaunchKernelGGL(k_stats, dim3(1), dim3(1024), 0, e->stream, e->d, e->d_pend);
    HIPCHK(hipGetLastError());
    uint64_t pend = 0;
    HIPCHK(hipMemcpyAsync(&pend, e->d_pend, 8, hipMemcpyDeviceToHost, e->stream));
    int rc = read_rs(e);
    if (rc) return rc;
    const RoundState& r = *e->h_rs;
    memset(out, 0, sizeof *out);
    out->rounds = r.rounds;
    out->pops = r.ctr[C_POPS];
    out->boots = r.ctr[C_BOOTS];
    out->sends = r.ctr[C_SENDS];
    out->null_dst = r.ctr[C_NULL];
    out->drop_reliability = r.ctr[C_DROPREL];
    out->drop_endtime = r.ctr[C_DROPEND];
    out->bumped = r.ctr[C_BUMPED];
    out->same_round = r.ctr[C_SAME];
    out->overflow = r.overflow;
    out->window_start = r.S;
    out->window_end = r.E;
    out->done = r.done;
    out->min_jump = r.min_jump;
    out->next_min_jump = r.next_min_jump;
    out->jmin_ms = r.jmin;
    out->pending = pend;
    out->trace_len = r.trace_len;
    out->exchange_steps = r.steps;
    out->phase = r.phase;
    return SG_OK;
}

int sg_engine_active_hosts(sg_engine* e, uint64_t* active, uint64_t* emitted) {
    if (!e) return SG_ERR_INVAL;
    sg_round_stats s;
    int rc = sg_engine_stats(e, &s);
    if (rc) return rc;
    if (active) *active = e->h_rs->ctr[C_ACTIVE];
    if (emitted) *emitted = e->h_rs->ctr[C_EMIT];
    return SG_OK;
}

int sg_engine_gather_paths(sg_engine* e, uint64_t* guessed, uint64_t* listed) {
    if (!e) return SG_ERR_INVAL;
    sg_round_stats s;
    int rc = sg_engine_stats(e, &s);
    if (rc) return rc;
    if (guessed) *guessed = e->h_rs->ctr[C_GSPEC];
    if (listed) *listed = e->h_rs->ctr[C_GLIST];
    return SG_OK;
}

int sg_engine_event_moves(sg_engine* e, uint64_t* emitted, uint64_t* gathered, uint64_t* received) {
    if (!e) return SG_ERR_INVAL;
    sg_round_stats s;
    int rc = sg_engine_stats(e, &s);
    if (rc) return rc;
    if (emitted) *emitted = e->h_rs->ctr[C_EMIT];
    if (gathered) *gathered = e->h_rs->ctr[C_GATHER];
    if (received) *received = e->h_rs->ctr[C_RECV];
    return SG_OK;
}

int sg_engine_host_state(sg_engine* e, uint64_t* digest, uint64_t* pops, uint32_t* rng,
                         uint64_t* event_counter) {
    if (!e) return SG_ERR_INVAL;
    const size_t L = e->d.L;
    std::vector<HostState> hs(L);
    HIPCHK(hipMemcpyAsync(hs.data(), e->d.hs, L * sizeof(HostState), hipMemcpyDeviceToHost, e->stream));
    int rc = sg_engine_sync(e);
    if (rc) return rc;
    for (size_t sl = 0; sl < L; ++sl) {  // slots back to registration order
        const size_t i = e->host_of_slot[sl] - e->d.lo;
        if (digest) digest[i] = hs[sl].digest;
        if (pops) pops[i] = hs[sl].pv & ((1ull << 48) - 1);
        if (rng) rng[i] = hs[sl].rng;
        if (event_counter) event_counter[i] = hs[sl].evc;
    }
    return SG_OK;
}

int sg_engine_trace(sg_engine* e, sg_trace_rec* out, uint64_t capacity, uint64_t* n_out) {
    if (!e) return SG_ERR_INVAL;
    int rc = read_rs(e);
    if (rc) return rc;
    uint64_t n = e->h_rs->trace_len;
    if (n > e->d.trace_cap) n = e->d.trace_cap;
    if (n_out) *n_out = n;
    if (out && capacity) {
        uint64_t m = n < capacity ? n : capacity;
        if (m) HIPCHK(hipMemcpy(out, e->d.trace, m * sizeof(sg_trace_rec), hipMemcpyDeviceToHost));
    }
    return SG_OK;
}

int sg_engine_windows(sg_engine* e, uint64_t* out_pairs, uint64_t capacity, uint64_t* n_out) {
    if (!e) return SG_ERR_INVAL;
    int rc = read_rs(e);
    if (rc) return rc;
    uint64_t n = e->h_rs->rounds < e->d.wlog_cap ? e->h_rs->rounds : e->d.wlog_cap;
    if (n_out) *n_out = n;
    if (out_pairs && capacity && n) {
        const uint64_t m = n < capacity ? n : capacity;
        HIPCHK(hipMemcpy(out_pairs, e->d.wlog, m * 16, hipMemcpyDeviceToHost));
    }
    return SG_OK;
}

static int need_sharded(sg_engine* e, const char* fn) {
    if (!e || !e->booted) {
        sg_set_error("%s: engine not booted", fn);
        return SG_ERR_STATE;
    }
    if (!e->d.outn) {
        sg_set_error("%s: round-mode engine (one shard, exchange_cap 0), use sg_engine_run / enqueue_round", fn);
        return SG_ERR_STATE;
    }
    return SG_OK;
}

// Copies the last received blocks (which the next k_proc stages from) into
// engine-owned memory, before their buffer is reallocated or unmapped.
static int hold_last_recv(sg_engine* e) {
    if (e->last_recv && e->last_recv != e->recv_hold) {
        const size_t bytes = (size_t)e->d.G * e->last_rows * RW * sizeof(int64_t);
        if (bytes > e->recv_hold_bytes) {
            if (e->recv_hold) HIPCHK(hipFree(e->recv_hold));
            e->recv_hold = nullptr;
            e->recv_hold_bytes = 0;
            HIPCHK(hipMalloc(&e->recv_hold, bytes));
            e->recv_hold_bytes = bytes;
        }
        HIPCHK(hipMemcpyAsync(e->recv_hold, e->last_recv, bytes, hipMemcpyDeviceToDevice, e->stream));
        HIPCHK(hipStreamSynchronize(e->stream));
        e->last_recv = e->recv_hold;
    }
    return SG_OK;
}

int sg_engine_exchange_rows(sg_engine* e, uint64_t* rows) {
    if (!e || !rows) return SG_ERR_INVAL;
    *rows = e->d.xrows;
    return SG_OK;
}

int sg_engine_set_exchange_cap(sg_engine* e, uint64_t exchange_cap) {
    if (!e || exchange_cap == 0) {
        sg_set_error("sg_engine_set_exchange_cap: exchange_cap must be > 0");
        return SG_ERR_INVAL;
    }
    // the last step's received blocks are still to be staged by the next
    // k_proc, and the caller reallocates its buffers for the new cap: keep a
    // copy (in the old layout, which the next k_proc decodes)
    if (int rc = hold_last_recv(e)) return rc;
    e->d.xcap = exchange_cap;
    e->d.xrows = HDR + exchange_cap;
    e->gen++;
    return SG_OK;
}

int sg_engine_exchange_peak(sg_engine* e, uint64_t* peak, int reset) {
    if (!e) return SG_ERR_INVAL;
    int rc = read_rs(e);
    if (rc) return rc;
    if (peak) *peak = e->h_rs->peak_peer;
    if (reset) HIPCHK(hipMemsetAsync(&e->d.rs->peak_peer, 0, 8, e->stream));
    return SG_OK;
}

int sg_engine_step_send(sg_engine* e, int64_t* send) {
    int rc = need_sharded(e, "sg_engine_step_send");
    if (rc) return rc;
    if (!send) {
        sg_set_error("sg_engine_step_send: NULL send buffer");
        return SG_ERR_INVAL;
    }
    e->d.xsend = send;  // k_proc writes the exchange blocks (launch argument)
    e->d.xrecv = e->last_recv;  // and stages what the last step received but did not route
    e->d.xrows_in = e->last_rows;
    e->d.xcap_in = e->last_cap;
    rc = enqueue_process(e);
    e->d.xsend = nullptr;
    e->d.xrecv = nullptr;
    return rc;
}

int sg_engine_step_recv(sg_engine* e, const int64_t* recv) {
    int rc = need_sharded(e, "sg_engine_step_recv");
    if (rc) return rc;
    if (!recv) {
        sg_set_error("sg_engine_step_recv: NULL receive buffer");
        return SG_ERR_INVAL;
    }
    e->last_recv = recv;  // the next step_send's k_proc stages its non-due events
    e->last_rows = e->d.xrows;
    e->last_cap = e->d.xcap;
    return enqueue_insert_plan(e, recv);
}

int sg_engine_stamps(sg_engine* e, uint64_t* out, uint64_t capacity, uint64_t* n_out) {
    if (!e) return SG_ERR_INVAL;
    const uint64_t n = e->d.stamps ? (2ull * e->d.P + e->d.G3 + e->d.G1 + 3) * SG_STAMP_W : 0;
    if (n_out) *n_out = n;
    if (out && capacity && n) {
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipMemcpy(out, e->d.stamps, (n < capacity ? n : capacity) * 8, hipMemcpyDeviceToHost));
    }
    return SG_OK;
}

int sg_engine_path_counters(sg_engine* e, int enable) {
    if (!e) return SG_ERR_INVAL;
    HIPCHK(hipSetDevice(e->device));
    if (!enable) {
        e->d.pcount = nullptr;  // the table stays allocated until destroy
        e->gen++;
        return SG_OK;
    }
    const size_t VV = (size_t)e->d.V * e->d.V;
    if (!e->pcount_buf) {
        int rc = dalloc(e, &e->pcount_buf, VV);
        if (rc) return rc;
    }
    HIPCHK(hipMemsetAsync(e->pcount_buf, 0, VV * sizeof(uint32_t), e->stream));
    e->d.pcount = e->pcount_buf;
    e->gen++;
    return SG_OK;
}

int sg_engine_barrier_timers(sg_engine* e, int enable) {
    if (!e) return SG_ERR_INVAL;
    HIPCHK(hipSetDevice(e->device));
    if (!enable) {
        e->d.wtime = nullptr;  // the buffer stays allocated until destroy
        e->gen++;
        return SG_OK;
    }
    const size_t n = 3 * (size_t)e->d.P;
    if (!e->wtime_buf) {
        int rc = dalloc(e, &e->wtime_buf, n);
        if (rc) return rc;
    }
    HIPCHK(hipMemsetAsync(e->wtime_buf, 0, n * sizeof(uint64_t), e->stream));
    e->d.wtime = e->wtime_buf;
    e->gen++;
    return SG_OK;
}

int sg_engine_barrier_times(sg_engine* e, uint64_t* busy_ns, uint64_t* idle_ns, uint64_t capacity,
                            uint64_t* n_out) {
    if (!e) return SG_ERR_INVAL;
    const uint64_t n = e->d.wtime ? e->d.P : 0;
    if (n_out) *n_out = n;
    if (capacity && n) {
        const uint64_t m = n < capacity ? n : capacity;
        std::vector<uint64_t> tmp(2 * (size_t)n);
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipMemcpy(tmp.data(), e->d.wtime, 2 * n * sizeof(uint64_t), hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < m; ++i) {  // s_memrealtime ticks at 100 MHz
            if (busy_ns) busy_ns[i] = tmp[i] * 10;
            if (idle_ns) idle_ns[i] = tmp[n + i] * 10;
        }
    }
    return SG_OK;
}

int sg_engine_path_counts(sg_engine* e, uint64_t* out, uint64_t capacity, uint64_t* n_out) {
    if (!e) return SG_ERR_INVAL;
    const uint64_t n = e->d.pcount ? (uint64_t)e->d.V * e->d.V : 0;
    if (n_out) *n_out = n;
    if (out && capacity && n) {
        const uint64_t m = n < capacity ? n : capacity;
        std::vector<uint32_t> tmp(m);
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipMemcpy(tmp.data(), e->d.pcount, m * sizeof(uint32_t), hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < m; ++i) out[i] = tmp[i];
    }
    return SG_OK;
}

int sg_engine_set_timing(sg_engine* e, int enabled) {
    return sg_engine_set_timing_mask(e, enabled ? (1u << SG_KCLASSES) - 1 : 0u);
}

int sg_engine_set_timing_mask(sg_engine* e, uint32_t mask) {
    if (!e) return SG_ERR_INVAL;
    if (e->timing) {  // events of the previous setting are harvested first
        const int rc = sg_engine_sync(e);
        if (rc) return rc;
    }
    e->timing = mask != 0;
    e->timing_mask = mask;
    for (int i = 0; i < SG_KCLASSES; ++i) {
        e->ms[i] = 0;
        e->launches[i] = 0;
    }
    return SG_OK;
}

int sg_engine_kernel_times(sg_engine* e, double* ms, uint64_t* launches) {
    if (!e) return SG_ERR_INVAL;
    int rc = sg_engine_sync(e);
    if (rc) return rc;
    for (int i = 0; i < SG_KCLASSES; ++i) {
        if (ms) ms[i] = e->ms[i];
        if (launches) launches[i] = e->launches[i];
    }
    return SG_OK;
}

}  // extern "C"

// ------------------------------------------------------- native step loop ----
// RCCL through dlopen: the copy the process already loaded (torch links one)
// is reused, so this library neither links RCCL nor brings a second copy.
namespace {
struct Rccl {
    bool ok = false;
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*allToAll)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*errStr)(ncclResult_t) = nullptr;
};
Rccl g_rccl;

int rccl_open() {
    if (g_rccl.ok) return SG_OK;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) {
        sg_set_error("RCCL not found (dlopen librccl.so.1): %s", dlerror());
        return SG_ERR_STATE;
    }
    g_rccl.getUniqueId = (decltype(g_rccl.getUniqueId))dlsym(h, "ncclGetUniqueId");
    g_rccl.commInitRank = (decltype(g_rccl.commInitRank))dlsym(h, "ncclCommInitRank");
    g_rccl.commDestroy = (decltype(g_rccl.commDestroy))dlsym(h, "ncclCommDestroy");
    g_rccl.allToAll = (decltype(g_rccl.allToAll))dlsym(h, "ncclAllToAll");
    g_rccl.errStr = (decltype(g_rccl.errStr))dlsym(h, "ncclGetErrorString");
    if (!g_rccl.getUniqueId || !g_rccl.commInitRank || !g_rccl.commDestroy || !g_rccl.allToAll ||
        !g_rccl.errStr) {
        sg_set_error("librccl.so.1 lacks an ncclGetUniqueId / ncclCommInitRank / ncclAllToAll symbol");
        return SG_ERR_STATE;
    }
    g_rccl.ok = true;
    return SG_OK;
}
}  // namespace

#define RCCLCHK(x)                                                                      \
    do {                                                                                \
        ncclResult_t _r = (x);                                                          \
        if (_r != ncclSuccess) {                                                        \
            sg_set_error("%s failed: %s (%s:%d)", #x, g_rccl.errStr(_r), __FILE__, __LINE__); \
            return SG_ERR_HIP;                                                          \
        }                                                                               \
    } while (0)

struct sg_comm {
    ncclComm_t comm;
    int rank, world, device;
};

// ------------------------------------------------ xGMI peer exchange ----
// sg_xlink: the step's all-to-all as direct stores into the peers' receive
// blocks over xGMI (hipIpc-mapped memory), with no collective.  Each rank owns
// one region of uncached device memory, so a peer's stores and this GPU's
// loads meet in HBM, never in a stale L2 line:
//   [XFLAG_BYTES]         arrival counters, one u64 per sender;
//   [2][G][xrows][RW]     receive blocks, double-buffered by step parity.
// Step k's blocks are read by its k_scatter and by step k + 1's k_proc (the
// events it did not route); a sender writes parity k & 1 again only in step
// k + 2, after its k_xwait(k + 1) saw this rank's push(k + 1), which this rank
// issues after its k_proc(k + 1).  Per step: step_send (k_proc writes the
// blocks into the local send buffer), k_xpush (XNW workgroups per peer copy
// the header and n rows into the peer's parity buffer, release at system
// scope, one arrival each), k_xwait (one lane per sender waits, bounded),
// step_recv on the parity buffer.  The MIN all-reduce of scheduler.c:386-408
// still rides in the block headers.
constexpr size_t XFLAG_BYTES = 4096;  // the counters' page

// workgroups per destination block: 256 in all (64 at most per peer), so one
// shard's whole block (world 1) is copied as fast as eight peers' slices
static uint32_t xlink_nw(uint32_t G) { return std::max<uint32_t>(4, std::min<uint32_t>(64, 256 / G)); }

struct XArgs {
    int64_t* peer[MAXG];  // each shard's region in this process (this shard's own for q == g)
    const int64_t* send;  // [G][xrows][RW]
    uint64_t xrows;
    uint64_t buf_off;     // int64 offset of this step's parity buffer (after the counters)
    uint32_t G, g, nw, fence;
};

__global__ __launch_bounds__(256) void k_xpush(XArgs a) {
    static_assert(RW == 2, "one exchange row is 16 bytes");
    const uint32_t XNW = a.nw, q = blockIdx.x / XNW, w = blockIdx.x % XNW;
    const int64_t* src = a.send + (size_t)q * a.xrows * RW;
    const uint64_t n = (uint64_t)src[H_N], cap = a.xrows - HDR;  // n <= xcap (write_headers)
    const uint64_t rows = HDR + (n < cap ? n : cap);
    int64_t* dst = a.peer[q] + a.buf_off + (size_t)a.g * a.xrows * RW;
    const longlong2* s2 = reinterpret_cast<const longlong2*>(src);
    longlong2* d2 = reinterpret_cast<longlong2*>(dst);
    for (uint64_t i = (uint64_t)w * blockDim.x + threadIdx.x; i < rows; i += (uint64_t)XNW * blockDim.x) {
        if (a.fence) {  // another GPU: system-coherent stores (xst)
            const longlong2 v = s2[i];
            xst(1u, dst + 2 * i, v.x);
            xst(1u, dst + 2 * i + 1, v.y);
        } else {
            d2[i] = s2[i];
        }
    }
    // the rows are performed at the peer (uncached memory) before its counter moves
    xlink_release();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(a.peer[q]) + a.g, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
}

// The self-test's wait as a kernel of its own (k_scatter waits in its
// prologue on real steps): the kernel always ends.
__global__ __launch_bounds__(64) void k_xwait(const uint64_t* flags, uint32_t G, uint64_t target, uint32_t* err) {
    xlink_wait(flags, G, target, err, nullptr);
}

// Self-test pattern: block q of sender g, row r, word c = a value only (g, q,
// r, c, step) gives; k_xcheck counts the received words that differ.
__device__ __forceinline__ int64_t xpattern(uint32_t g, uint32_t q, uint64_t r, uint32_t c, uint64_t step) {
    return (int64_t)(((uint64_t)g << 56) ^ ((uint64_t)q << 48) ^ (r << 8) ^ ((uint64_t)c << 4) ^ (step * 0x9E3779B97F4A7C15ull));
}
__global__ void k_xfill(int64_t* send, uint64_t xrows, uint32_t G, uint32_t g, uint64_t n, uint64_t step) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)G * xrows * RW;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t q = (uint32_t)(i / (xrows * RW));
        const uint64_t r = (i / RW) % xrows;
        const uint32_t c = (uint32_t)(i % RW);
        send[i] = r == 0 && c == 0 ? (int64_t)n : xpattern(g, q, r, c, step);
    }
}
// The self-test of the fused push, the protocol real steps take (k_proc with
// d.xpeer): XFW workgroups each store a slice of every peer's pattern rows
// straight into the peer's region, release (xlink_release: vmcnt(0), and the
// system-scope release when fenced) and take a device-scope ticket; the last
// writes the G headers and arrives at every peer (xlink_arrive).
constexpr uint32_t XFW = 128;
struct XFArgs {
    int64_t* peer[MAXG];  // each shard's region in this process
    unsigned long long* ticket;
    uint64_t xrows, buf_off, n, step;
    uint32_t G, g, fence;
};
__global__ __launch_bounds__(256) void k_xfused(XFArgs a) {
    const size_t own = a.buf_off + (size_t)a.g * a.xrows * RW;  // this sender's block in every region
    for (uint32_t q = 0; q < a.G; ++q) {
        int64_t* dst = a.peer[q] + own + HDR * RW;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n * RW;
             i += (uint64_t)gridDim.x * blockDim.x)
            xst(a.fence, dst + i, xpattern(a.g, q, HDR + i / RW, (uint32_t)(i % RW), a.step));
    }
    __shared__ bool s_last;
    xlink_release();
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(a.ticket, 1ull) == gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;  // uniform in the workgroup
    if (threadIdx.x == 0) atomicExch(a.ticket, 0ull);
    for (uint32_t i = threadIdx.x; i < a.G * HDR_W; i += blockDim.x) {
        const uint32_t q = i / HDR_W, j = i % HDR_W, r = j / RW, c = j % RW;
        xst(a.fence, a.peer[q] + own + j, r == 0 && c == 0 ? (int64_t)a.n : xpattern(a.g, q, r, c, a.step));
    }
    xlink_arrive(a.peer, a.G, a.g, 0);
}
__global__ void k_xcheck(const int64_t* recv, uint64_t xrows, uint32_t G, uint32_t g, uint64_t n, uint64_t step,
                         unsigned long long* bad) {
    uint32_t nb = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)G * xrows * RW;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(i / (xrows * RW));
        const uint64_t r = (i / RW) % xrows;
        const uint32_t c = (uint32_t)(i % RW);
        if (r >= HDR + n) continue;
        const int64_t want = r == 0 && c == 0 ? (int64_t)n : xpattern(s, g, r, c, step);
        nb += recv[i] != want;
    }
    if (nb) atomicAdd(bad, (unsigned long long)nb);
}

struct sg_xlink {
    sg_engine* e = nullptr;
    uint32_t G = 0, g = 0;
    uint64_t xrows = 0;
    int64_t* region = nullptr;  // this shard's (uncached)
    size_t region_bytes = 0;
    int64_t* send = nullptr;    // [G][xrows][RW], ordinary device memory
    int64_t* peer[MAXG] = {};
    bool opened[MAXG] = {};
    uint32_t* err = nullptr;    // k_xwait's timeout flags (device)
    uint64_t steps = 0;         // steps pushed since attach
    bool attached = false;
    // another shard runs on this device: the arrivals are awaited by k_xwait
    // (one workgroup), not in k_scatter's prologue, whose spinning workgroups
    // would hold the CUs the peer's kernels need to arrive at all
    bool shared = false;
    // system-coherent stores (sc0 sc1) of every handed-off row and header,
    // drained before each ticket and arrival (xst).  Between shards of one
    // device (and at world 1) the blocks are uncached local memory and a plain
    // store's acknowledgement orders it; a peer on another GPU gets the
    // system-scope form the memory model guarantees across xGMI.
    // SG_XFENCE=0 / 1 forces either.
    bool fence = false;
    // fused push (SG_XFUSE, default 1): k_proc stores the blocks into the peers'
    // regions and its last workgroup signals them; 0: k_xpush copies x->send
    bool fuse = true;
    int64_t** d_peer = nullptr;  // device copy of peer[] (k_proc's xblock)
    uint64_t expect = 0;         // arrivals every sender's counter holds once the last step is in
    unsigned long long* ticket = nullptr;  // k_xfused's workgroup ticket (device)
    // the last self-test: steps, mismatched words, which path it exercised
    uint32_t st_steps = 0, st_fused = 0;
    uint64_t st_bad = 0;
    // test only (sg_xlink_debug_withhold): the fused step with this number
    // (since attach) withholds its arrival at peer withhold_peer
    uint64_t withhold_step = 0;
    uint32_t withhold_peer = 0;
};

extern "C" {

int sg_comm_available(void) { return rccl_open(); }

int sg_comm_unique_id(uint8_t id_out[128]) {
    if (!id_out) return SG_ERR_INVAL;
    int rc = rccl_open();
    if (rc) return rc;
    ncclUniqueId id;
    RCCLCHK(g_rccl.getUniqueId(&id));
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    memcpy(id_out, &id, sizeof id);
    return SG_OK;
}

int sg_comm_create(const uint8_t id_in[128], int rank, int world, int device, sg_comm** out) {
    if (!id_in || !out || world < 1 || rank < 0 || rank >= world) {
        sg_set_error("sg_comm_create: bad arguments (rank %d, world %d)", rank, world);
        return SG_ERR_INVAL;
    }
    int rc = rccl_open();
    if (rc) return rc;
    HIPCHK(hipSetDevice(device));
    ncclUniqueId id;
    memcpy(&id, id_in, sizeof id);
    ncclComm_t comm = nullptr;
    RCCLCHK(g_rccl.commInitRank(&comm, world, id, rank));
    *out = new sg_comm{comm, rank, world, device};
    return SG_OK;
}

int sg_comm_destroy(sg_comm* c) {
    if (!c) return SG_OK;
    if (g_rccl.ok && c->comm) (void)g_rccl.commDestroy(c->comm);
    delete c;
    return SG_OK;
}

int sg_engine_set_graph(sg_engine* e, uint32_t batch) {
    if (!e) return SG_ERR_INVAL;
    e->graph_batch = batch;
    // drop the captured graph: RCCL keeps resources of captured collectives
    // until their graph is destroyed, and a communicator is destroyed only after
    if (e->gexec) {
        HIPCHK(hipStreamSynchronize(e->stream));
        HIPCHK(hipGraphExecDestroy(e->gexec));
        e->gexec = nullptr;
    }
    return SG_OK;
}

int sg_engine_run_steps(sg_engine* e, sg_comm* c, int64_t* send, int64_t* recv, uint64_t n_steps) {
    int rc = need_sharded(e, "sg_engine_run_steps");
    if (rc) return rc;
    if (!c || !send || !recv) {
        sg_set_error("sg_engine_run_steps: NULL communicator or buffer");
        return SG_ERR_INVAL;
    }
    if ((uint32_t)c->world != e->d.G || (uint32_t)c->rank != e->d.g) {
        sg_set_error("sg_engine_run_steps: communicator rank %d of %d, engine shard %u of %u", c->rank,
                     c->world, e->d.g, e->d.G);
        return SG_ERR_INVAL;
    }
    const size_t per_peer = (size_t)e->d.xrows * RW;  // int64 elements per peer block
    auto step = [&]() -> int {
        int r = sg_engine_step_send(e, send);
        if (r) return r;
        ncclResult_t nr = ncclSuccess;
        r = timed_launch(e, SG_K_EXCHANGE, [&](hipEvent_t a, hipEvent_t b) {
            if (a) (void)hipEventRecord(a, e->stream);
            nr = g_rccl.allToAll(send, recv, per_peer, ncclInt64, c->comm, e->stream);
            if (b) (void)hipEventRecord(b, e->stream);
        });
        if (r) return r;
        RCCLCHK(nr);
        return sg_engine_step_recv(e, recv);
    };
    const uint32_t b = e->graph_batch ? e->graph_batch : 32;
    while (n_steps) {
        const uint32_t n = n_steps < b ? (uint32_t)n_steps : b;
        const sg_engine::GraphKey key{e->gen, send, recv, c, e->last_recv, n};
        if ((rc = enqueue_batch(e, key, n, step))) return rc;
        n_steps -= n;
    }
    return SG_OK;
}

static int xlink_fail(sg_xlink* x, const char* what, hipError_t err) {
    sg_set_error("%s failed: %s", what, hipGetErrorString(err));
    (void)sg_xlink_destroy(x);
    return SG_ERR_HIP;
}

int sg_xlink_create(sg_engine* e, sg_xlink** out) {
    if (!out) return SG_ERR_INVAL;
    *out = nullptr;
    int rc = need_sharded(e, "sg_xlink_create");
    if (rc) return rc;
    HIPCHK(hipSetDevice(e->device));
    sg_xlink* x = new sg_xlink();
    x->e = e;
    x->G = e->d.G;
    x->g = e->d.g;
    x->xrows = e->d.xrows;
    const size_t blk = (size_t)x->G * x->xrows * RW * sizeof(int64_t);
    x->region_bytes = XFLAG_BYTES + 2 * blk;
    // uncached by default; SG_XLINK_MEM=1 takes fine-grained memory instead
    const unsigned flags = env_u32z("SG_XLINK_MEM", 0) == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached;
    hipError_t err = hipExtMallocWithFlags((void**)&x->region, x->region_bytes, flags);
    if (err != hipSuccess) return xlink_fail(x, "hipExtMallocWithFlags (exchange region)", err);
    if ((err = hipMemset(x->region, 0, x->region_bytes)) != hipSuccess) return xlink_fail(x, "hipMemset", err);
    if ((err = hipMalloc(&x->send, blk)) != hipSuccess) return xlink_fail(x, "hipMalloc (send blocks)", err);
    if ((err = hipMalloc(&x->err, sizeof(uint32_t))) != hipSuccess) return xlink_fail(x, "hipMalloc", err);
    if ((err = hipMemset(x->err, 0, sizeof(uint32_t))) != hipSuccess) return xlink_fail(x, "hipMemset", err);
    if ((err = hipDeviceSynchronize()) != hipSuccess) return xlink_fail(x, "hipDeviceSynchronize", err);
    if ((err = hipMalloc(&x->d_peer, MAXG * sizeof(int64_t*))) != hipSuccess) return xlink_fail(x, "hipMalloc", err);
    if ((err = hipMalloc(&x->ticket, sizeof *x->ticket)) != hipSuccess) return xlink_fail(x, "hipMalloc", err);
    if ((err = hipMemset(x->ticket, 0, sizeof *x->ticket)) != hipSuccess) return xlink_fail(x, "hipMemset", err);
    x->peer[x->g] = x->region;
    x->fuse = env_u32z("SG_XFUSE", 1) != 0;
    *out = x;
    return SG_OK;
}

// handle = the region's IPC handle, then the device's PCI bus id (ranks that
// share a device are told apart at attach)
constexpr size_t XBUS = SG_XLINK_HANDLE_BYTES - sizeof(hipIpcMemHandle_t);
static_assert(XBUS >= 16, "room for a PCI bus id");

int sg_xlink_handle(sg_xlink* x, uint8_t out[SG_XLINK_HANDLE_BYTES]) {
    if (!x || !out) return SG_ERR_INVAL;
    hipIpcMemHandle_t h;
    HIPCHK(hipIpcGetMemHandle(&h, x->region));
    memset(out, 0, SG_XLINK_HANDLE_BYTES);
    memcpy(out, &h, sizeof h);
    HIPCHK(hipDeviceGetPCIBusId((char*)out + sizeof h, (int)XBUS - 1, x->e->device));
    return SG_OK;
}

int sg_xlink_attach(sg_xlink* x, const uint8_t* handles) {
    if (!x || !handles) return SG_ERR_INVAL;
    if (x->attached) {
        sg_set_error("sg_xlink_attach: already attached");
        return SG_ERR_STATE;
    }
    HIPCHK(hipSetDevice(x->e->device));
    const uint8_t* own = handles + (size_t)x->g * SG_XLINK_HANDLE_BYTES + sizeof(hipIpcMemHandle_t);
    for (uint32_t q = 0; q < x->G; ++q) {
        if (q == x->g) continue;
        const uint8_t* hq = handles + (size_t)q * SG_XLINK_HANDLE_BYTES;
        if (memcmp(hq + sizeof(hipIpcMemHandle_t), own, XBUS) == 0) x->shared = true;
        hipIpcMemHandle_t h;
        memcpy(&h, hq, sizeof h);
        void* p = nullptr;
        const hipError_t err = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (err != hipSuccess) {
            sg_set_error("sg_xlink_attach: hipIpcOpenMemHandle (shard %u) failed: %s", q, hipGetErrorString(err));
            return SG_ERR_HIP;
        }
        x->peer[q] = (int64_t*)p;
        x->opened[q] = true;
    }
    HIPCHK(hipMemcpy(x->d_peer, x->peer, MAXG * sizeof(int64_t*), hipMemcpyHostToDevice));
    bool remote = false;
    for (uint32_t q = 0; q < x->G; ++q)
        if (q != x->g && memcmp(handles + (size_t)q * SG_XLINK_HANDLE_BYTES + sizeof(hipIpcMemHandle_t), own, XBUS))
            remote = true;
    const char* fe = getenv("SG_XFENCE");
    x->fence = fe && *fe ? strtol(fe, nullptr, 10) != 0 : remote;
    x->attached = true;
    return SG_OK;
}

// Enqueues one push of the blocks in x->send into the peers' regions; returns
// the receive buffer of this step's parity and the arrival count every
// sender's counter reaches (the caller's k_scatter, or k_xwait, waits for it).
static int xlink_push(sg_engine* e, sg_xlink* x, const int64_t** recv, uint64_t* target) {
    XArgs a;
    for (uint32_t q = 0; q < MAXG; ++q) a.peer[q] = q < x->G ? x->peer[q] : nullptr;
    a.send = x->send;
    a.xrows = x->xrows;
    a.G = x->G;
    a.g = x->g;
    a.nw = xlink_nw(x->G);
    a.fence = x->fence;
    const uint64_t k = x->steps + 1;  // this exchange's number since attach
    a.buf_off = XFLAG_BYTES / sizeof(int64_t) + (k & 1) * (uint64_t)x->G * x->xrows * RW;
    int rc = timed_launch(e, SG_K_EXCHANGE, [&](hipEvent_t ea, hipEvent_t eb) {
        SG_LAUNCH(k_xpush, dim3(x->G * a.nw), dim3(256), 0, e->stream, ea, eb, a);
    });
    if (rc) return rc;
    x->steps = k;
    x->expect += a.nw;
    *recv = x->region + a.buf_off;
    *target = x->expect;
    return SG_OK;
}

static int xlink_ready(sg_engine* e, sg_xlink* x, const char* fn) {
    if (!x || !x->attached || x->e != e) {
        sg_set_error("%s: exchange link not attached to this engine", fn);
        return SG_ERR_STATE;
    }
    if (e->d.xrows != x->xrows) {
        sg_set_error("%s: exchange_cap changed since sg_xlink_create (rows %llu, link %llu)", fn,
                     (unsigned long long)e->d.xrows, (unsigned long long)x->xrows);
        return SG_ERR_STATE;
    }
    return SG_OK;
}

int sg_engine_run_steps_xlink(sg_engine* e, sg_xlink* x, uint64_t n_steps) {
    int rc = need_sharded(e, "sg_engine_run_steps_xlink");
    if (rc || (rc = xlink_ready(e, x, "sg_engine_run_steps_xlink"))) return rc;
    for (uint64_t i = 0; i < n_steps; ++i) {
        const int64_t* recv = nullptr;
        uint64_t target = 0;
        if (x->fuse) {
            // k_proc stores the blocks into the peers' regions, its last
            // workgroup signals each peer once
            const uint64_t k = x->steps + 1;
            const uint64_t buf_off = XFLAG_BYTES / sizeof(int64_t) + (k & 1) * (uint64_t)x->G * x->xrows * RW;
            e->d.xpeer = x->d_peer;
            e->d.xoff = buf_off + (uint64_t)x->g * x->xrows * RW;
            e->d.xfence = x->fence ? 1u : 0u;
            e->d.xskip = x->withhold_step == k ? x->withhold_peer + 1 : 0u;
            rc = sg_engine_step_send(e, x->send);
            e->d.xpeer = nullptr;
            e->d.xskip = 0;
            if (rc) return rc;
            x->steps = k;
            x->expect += 1;
            recv = x->region + buf_off;
            target = x->expect;
        } else {
            if ((rc = sg_engine_step_send(e, x->send))) return rc;
            if ((rc = xlink_push(e, x, &recv, &target))) return rc;
        }
        if (x->shared) {
            hipLaunchKernelGGL(k_xwait, dim3(1), dim3(64), 0, e->stream, (const uint64_t*)x->region, x->G, target,
                               x->err);
            HIPCHK(hipGetLastError());
            if ((rc = sg_engine_step_recv(e, recv))) return rc;
            continue;
        }
        // k_scatter's wave 0 waits for the arrivals before it reads the headers
        e->d.xwait = (const uint64_t*)x->region;
        e->d.xwait_target = target;
        e->d.xwait_err = x->err;
        rc = sg_engine_step_recv(e, recv);
        e->d.xwait = nullptr;
        if (rc) return rc;
    }
    return SG_OK;
}

int sg_xlink_selftest(sg_xlink* x, uint32_t n_steps, uint64_t* bad) {
    if (!bad) return SG_ERR_INVAL;
    *bad = 0;
    int rc = xlink_ready(x ? x->e : nullptr, x, "sg_xlink_selftest");
    if (rc) return rc;
    sg_engine* e = x->e;
    unsigned long long* d_bad = nullptr;
    HIPCHK(hipMalloc(&d_bad, sizeof *d_bad));
    HIPCHK(hipMemsetAsync(d_bad, 0, sizeof *d_bad, e->stream));
    const uint64_t cap = x->xrows - HDR;
    for (uint32_t i = 0; i < n_steps && rc == SG_OK; ++i) {
        const uint64_t k = x->steps + 1;
        // rows this step, the same on every shard; every fourth step a full block
        const uint64_t n = (k & 3) == 3 ? cap : (k * 2654435761ull) % (cap + 1);
        const int64_t* recv = nullptr;
        uint64_t target = 0;
        if (x->fuse) {
            // the fused push real steps take: many workgroups storing into the
            // peers' regions, each releasing and taking a ticket, the last one
            // writing the headers and arriving
            XFArgs a;
            for (uint32_t q = 0; q < MAXG; ++q) a.peer[q] = q < x->G ? x->peer[q] : nullptr;
            a.ticket = x->ticket;
            a.xrows = x->xrows;
            a.buf_off = XFLAG_BYTES / sizeof(int64_t) + (k & 1) * (uint64_t)x->G * x->xrows * RW;
            a.n = n;
            a.step = k;
            a.G = x->G;
            a.g = x->g;
            a.fence = x->fence ? 1u : 0u;
            hipLaunchKernelGGL(k_xfused, dim3(XFW), dim3(256), 0, e->stream, a);
            if (hipGetLastError() != hipSuccess) {
                sg_set_error("sg_xlink_selftest: k_xfused launch failed");
                rc = SG_ERR_HIP;
                break;
            }
            x->steps = k;
            x->expect += 1;
            recv = x->region + a.buf_off;
            target = x->expect;
        } else {
            hipLaunchKernelGGL(k_xfill, dim3(64), dim3(256), 0, e->stream, x->send, x->xrows, x->G, x->g, n, k);
            rc = xlink_push(e, x, &recv, &target);
        }
        if (rc == SG_OK) {
            hipLaunchKernelGGL(k_xwait, dim3(1), dim3(64), 0, e->stream, (const uint64_t*)x->region, x->G, target,
                               x->err);
            hipLaunchKernelGGL(k_xcheck, dim3(64), dim3(256), 0, e->stream, recv, x->xrows, x->G, x->g, n, k, d_bad);
        }
    }
    unsigned long long h_bad = 0;
    uint32_t h_err = 0;
    hipError_t err = hipStreamSynchronize(e->stream);
    if (err == hipSuccess) err = hipMemcpy(&h_bad, d_bad, sizeof h_bad, hipMemcpyDeviceToHost);
    if (err == hipSuccess) err = hipMemcpy(&h_err, x->err, sizeof h_err, hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (rc) return rc;
    HIPCHK(err);
    *bad = h_bad + (h_err ? (1ull << 63) : 0ull);
    x->st_steps = n_steps;
    x->st_fused = x->fuse ? 1u : 0u;
    x->st_bad = *bad;
    return SG_OK;
}

int sg_xlink_status(sg_xlink* x, uint32_t* timed_out) {
    if (!x || !timed_out) return SG_ERR_INVAL;
    HIPCHK(hipStreamSynchronize(x->e->stream));
    HIPCHK(hipMemcpy(timed_out, x->err, sizeof *timed_out, hipMemcpyDeviceToHost));
    return SG_OK;
}

int sg_xlink_info(sg_xlink* x, sg_xlink_desc* out) {
    if (!x || !out) return SG_ERR_INVAL;
    out->fenced = x->fence ? 1u : 0u;
    out->fused = x->fuse ? 1u : 0u;
    out->shared_device = x->shared ? 1u : 0u;
    out->selftest_steps = x->st_steps;
    out->selftest_fused = x->st_fused;
    out->selftest_bad = x->st_bad;
    out->steps = x->steps;
    return SG_OK;
}

int sg_xlink_debug_withhold(sg_xlink* x, uint64_t step, uint32_t peer) {
    if (!x || peer >= x->G) return SG_ERR_INVAL;
    if (!x->fuse) {
        sg_set_error("sg_xlink_debug_withhold: the fused push only (SG_XFUSE=1)");
        return SG_ERR_STATE;
    }
    x->withhold_step = x->steps + step;
    x->withhold_peer = peer;
    return SG_OK;
}

int sg_xlink_destroy(sg_xlink* x) {
    if (!x) return SG_OK;
    int rc = SG_OK;
    if (x->e) {
        (void)hipStreamSynchronize(x->e->stream);
        // the next k_proc stages from the last received blocks: keep them
        const char* lr = (const char*)x->e->last_recv;
        if (x->region && lr >= (const char*)x->region && lr < (const char*)x->region + x->region_bytes)
            rc = hold_last_recv(x->e);
    }
    for (uint32_t q = 0; q < MAXG; ++q)
        if (x->opened[q]) (void)hipIpcCloseMemHandle(x->peer[q]);
    if (x->region) (void)hipFree(x->region);
    if (x->send) (void)hipFree(x->send);
    if (x->err) (void)hipFree(x->err);
    if (x->d_peer) (void)hipFree(x->d_peer);
    if (x->ticket) (void)hipFree(x->ticket);
    delete x;
    return rc;
}

}  // extern "C"
