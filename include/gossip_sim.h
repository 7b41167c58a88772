/*
 * gossip_sim.h -- C ABI of the MI355X batched gossip simulator.
 *
 * A drop-in batched backend for aiocluster's scuttlebutt anti-entropy
 * (aiocluster/state.py) and phi failure detector (aiocluster/failure_detector.py).
 * The reference has no FFI for this path: its hot path is plain Python called
 * in-process by aiocluster/server.py.  Each entry point below replaces, for a
 * whole simulated cluster at once, the reference calls named next to it; the
 * ctypes binding a maintainer would add to the reference is in INTEGRATION.md.
 *
 * Ownership: every device buffer is allocated by the caller (PyTorch in this
 * repo) and bound with gs_bind(); the library never allocates or frees device
 * memory.  Threading: one host thread per handle; all kernels run on the
 * stream given to gs_set_stream() (default: the null stream); only
 * gs_read_counters()/gs_sync() block.  Errors: every function returns 0 on
 * success or a negative GS_E_* code; gs_last_error() describes the last one.
 *
 * Time is simulated in ticks of 1/64 s (15 625 us): whole microseconds, like
 * the reference's datetimes, and dyadic, so the failure detector's
 * interval sums are exact in binary64.
 */
#ifndef GOSSIP_SIM_H
#define GOSSIP_SIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_API_VERSION 20
#define GS_MAX_PHASES 64  /* report bit planes' phases per plane base window of the scheduler (busy bits) */
/* gs_schedule_phases: phases of one round's schedule.  Every selected exchange runs (server.py:476-493): phases
 * past the workload's tick budget are sub-phases, run at one tick (gs_run_phase at the previous phase's tick). */
#define GS_MAX_SCHED_PHASES 65536u
/* DEVICE scratch bytes of gs_schedule_phases for N nodes, fanout F, max_phases P */
#define GS_SCHED_SCRATCH_BYTES(N, F, P) \
    (4ull * (N) * ((F) + 2) + 12ull * (P) + 32ull + 24ull * (N))
#define GS_TICK_US 15625u
#define GS_NONE 0xFFFFFFFFu
#define GS_CAND_CAP 1024u /* GS_R_CAND records per exchange, direction and row half */
#define GS_PLANES 32u     /* GS_R_PEND report bit planes per observer row: phases per plane base */
/* u32 words of gs_phase_overflow's DEVICE list for a phase of n exchanges: 2n slots, ceil(2n / 1024)
 * block counts, the total */
#define GS_OVERFLOW_LIST_LEN(n) (2u * (n) + (2u * (n) + 1023u) / 1024u + 1u)

/* error codes */
#define GS_OK 0
#define GS_E_INVALID (-1)     /* bad argument / config */
#define GS_E_UNBOUND (-2)     /* a required region is not bound */
#define GS_E_HIP (-3)         /* HIP runtime error */
#define GS_E_DEVICE (-4)      /* a device-side check failed (see gs_counters error fields) */
#define GS_E_UNSUPPORTED (-5) /* semantics not implemented by this build (e.g. FD garbage collection) */

/* config flags */
#define GS_CANONICAL 1u   /* every observer knows every node in index order (warm start, no removals) */
#define GS_TOMBSTONES 2u  /* track tombstone receive ticks (needed when deletes/TTL writes occur) */
#define GS_FD_RING 4u     /* keep each sampling window's ring (exact eviction once a window is full) */
#define GS_NO_HELD 8u     /* no GS_R_HELD at all (needs !GS_TOMBSTONES): exact only while every view is a
                             prefix S_j(max_version), i.e. no NodeDelta is ever truncated; a view that would
                             get holes is counted in err_holes.  16 B less per pair at K = 16 (config 4) */
#define GS_HB8 16u        /* 8-bit heartbeat views: GS_R_HB is u8 [N][NP] (mod 2^8, decoded against the owner's
                             own heartbeat like the 16-bit store), exact while every view lags its owner by < 2^8;
                             gs_begin_round and the phases sweep the lags at least every 64 round starts + phases
                             and count a lag >= 128 in err_hb_lag.  Needs GS_CANONICAL, n_keys <= 16 and the record phases
                             (not env GS_FUSED / GS_PACK=fused): half the heartbeat bytes of every exchange */
#define GS_MV8 32u        /* 8-bit max_version views (needs GS_HB8 and !GS_TOMBSTONES): GS_R_MV is u8 [N][NP] =
                             version mod 2^7 | GS_MV_INEXACT >> 8, decoded against the owner's own max_version
                             (GS_R_SELF_MV); exact while every view lags its owner by < 2^7 versions:
                             gs_owner_writes sweeps the lags at least every 64 calls and counts a lag >= 2^6
                             in err_hb_lag */
#define GS_SLICED 64u     /* phases take the sliced path (gs_phase_count / gather / gs_phase_pack, or gs_run_phase
                             over a gs_comm_init communicator) even with one slice (n_shards <= 1): a one-GPU
                             world-1 run of the multi-GPU code (needs GS_CANONICAL) */

/* owner write ops (NodeState.set/delete/set_with_ttl/delete_after_ttl, state.py:137-180) */
#define GS_OP_SET 0u
#define GS_OP_DELETE 1u
#define GS_OP_SET_WITH_TTL 2u
#define GS_OP_DELETE_AFTER_TTL 3u

typedef struct gs_config {
    uint32_t n_nodes;               /* N: simulated cluster size */
    uint32_t n_keys;                /* K <= 64 keys per node */
    uint32_t hist_cap;              /* C <= 255: writes kept per (owner, key), ordinal 0 = absent */
    uint32_t mtu;                   /* Config.max_payload_size (entities.py:105) */
    uint32_t flags;                 /* GS_CANONICAL | GS_TOMBSTONES | GS_FD_RING | GS_NO_HELD | GS_HB8 | GS_MV8 | GS_SLICED */
    uint32_t window;                /* FailureDetectorConfig.sampling_window_size (entities.py:88) */
    uint32_t max_interval_ticks;    /* FailureDetectorConfig.max_interval (entities.py:89) */
    uint32_t tombstone_grace_ticks; /* Config.marked_for_deletion_grace_period (entities.py:101) */
    uint32_t dead_grace_ticks;      /* FailureDetectorConfig.dead_node_grace_period (entities.py:91) */
    uint32_t sched_delay_ticks;     /* smallest d with d*TICK_US >= round_half_even(dead_grace_us/2)
                                       (failure_detector.py:124-126) */
    double phi_threshold;           /* FailureDetectorConfig.phi_threshhold (entities.py:87) */
    double prior_weighted;          /* 5.0 * initial_interval.total_seconds() (failure_detector.py:22-23,51) */
    uint32_t n_shards;              /* G owner-column slices of the cluster (0 or 1 = the whole matrix;
                                       G > 1 needs GS_CANONICAL); one handle per slice, usually one per GPU */
    uint32_t shard;                 /* this handle's slice: columns [shard*B, min(N, (shard+1)*B)),
                                       B = ceil(N/G) rounded up to 64 (every slice must be non-empty) */
    uint32_t ring_rows;             /* sampled rings (not with GS_FD_RING): this many observer rows, chosen by
                                       gs_set_ring_rows, keep every window's interval ring (exact eviction
                                       past W intervals, BoundedArrayStats); the other rows keep compact
                                       windows, exact up to W intervals, and a compact window that would need
                                       an eviction is counted in fd_saturated (not an error) */
    uint32_t esc_cols;              /* GS_MV8 record phases: escape slots for owner columns whose views fall far behind
                                       (<= 4096; 0 = none).  A lag sweep that finds a heartbeat view lagging its owner
                                       by >= 2^7 moves every view of that owner column into a 16-bit slot (GS_R_ESC16,
                                       exact while lags stay < 2^15) instead of counting err_hb_lag, and moves it back
                                       once every view of it lags by < 2^6: the hub columns of the
                                       reference's peer selection (seeds answering every phase) stay exact.  A sweep
                                       that finds no free slot counts the column in err_hb_lag */
} gs_config;

/* device regions (all caller-allocated).  [N][NP] regions hold every observer row o and this
 * handle's owner columns j = col_lo + jl (gs_shard_columns), row stride NP = n_cols rounded up
 * to 64; per-owner regions ([NC]..., NC = n_cols) are indexed by the local column jl.  With one
 * slice col_lo = 0 and n_cols = n_nodes. */
enum gs_region {
    GS_R_HB = 0,      /* u16 [N][NP]   NodeState.heartbeat of owner j as seen by observer o, mod 2^16: decoded
                                        against GS_R_SELF_HB as R - ((R - s) mod 2^16), exact while every view
                                        lags its owner's own heartbeat by less than 2^16.  With escape slots
                                        (gs_config.esc_cols) the bytes of an escaped column (GS_R_ESC_SLOT[j] !=
                                        GS_NONE) are STALE: its views live in GS_R_ESC16 [o][slot] */
    GS_R_MV,          /* u16 [N][NP]   NodeState.max_version (| GS_MV_INEXACT, see below); versions are
                                        bounded by K * (C - 1) <= 16,256, so 15 bits always suffice */
    GS_R_GC,          /* u32 [N][NP]   NodeState.last_gc_version (GS_TOMBSTONES only: without tombstone GC
                                        it is 0 everywhere, and deletes / TTL writes are refused) */
    GS_R_HELD,        /* u8  [N][NP][KP] write ordinal of each key held (0 = absent), KP = K rounded to 4;
                                        kept only for views with GS_MV_INEXACT or with GS_TOMBSTONES;
                                        not allocated with GS_NO_HELD */
    GS_R_FD,          /* u32 [N][NP]   sampling window: _sum in ticks | intervals appended since the last
                                        reset << sum_bits (len = min(cnt, W)); sum_bits = 32 - bits(2W)
                                        (gs_create rejects W * max_interval >= 2^sum_bits) */
    GS_R_FD_STATE,    /* u8  [N][NP]   bits 0-1: 0 = unknown, 1 = live (in _live_nodes), 2 = dead (in
                                        _dead_nodes, time of death in GS_R_FD_TOD); bit 2: the pair has a
                                        sampling window; bit 3: its last report is >= 2^15 ticks old */
    GS_R_TS,          /* u32 [N][NP][KP] tombstone receive tick, GS_NONE for SET entries (GS_TOMBSTONES) */
    GS_R_RING,        /* u16 [N][NP][W] interval ring in ticks (GS_FD_RING); [ring_rows][NP][W] by ring slot
                                        with sampled rings */
    GS_R_POS,         /* u32 [N][NP]   insertion index of owner j in observer o's dict, GS_NONE = absent (general) */
    GS_R_ORD,         /* u32 [N][NP]   owner at insertion index q (general) */
    GS_R_ROW,         /* u32 [N][4]    {dict size, tombstone-present flag, a lower bound of the first tick a
                                        dead target of this slice is scheduled for deletion (exact after a
                                        liveness sweep that found the row due), flags: bit 0 FD-GC due,
                                        bit 1 the current sweep recomputes word 2} */
    GS_R_LAST_W,      /* u8  [NC][KP]  owner's latest write ordinal per key */
    GS_R_HIST,        /* u64 [NC][C][K] write w of (owner, key): version | meta << 32, where
                                        meta = KeyValueUpdatePb size | status << 16 | value bytes << 18 */
    GS_R_HIST_VID,    /* u32 [NC][C][K] interned value id (host string table) */
    GS_R_NID_SIZE,    /* u16 [NP]      NodeIdPb size per owner column (entities.py:62-72) */
    GS_R_KEY_LEN,     /* u8  [KP]      UTF-8 key length per key index */
    GS_R_STAMP,       /* u32 [N rounded to 64] per-node phase stamp (conflict check) */
    GS_R_COUNTERS,    /* u64 [64][48]  sharded gs_counters (summed by gs_read_counters) and census scratch */
    GS_R_SLICE_BITS,  /* u32 [N/2][2][NP/32] stale-owner bitmaps per exchange and direction: between
                                        gs_phase_count and gs_phase_pack (n_shards > 1), and between the two
                                        kernels of a canonical one-slice gs_run_phase */
    GS_R_PEND,        /* u64 [N][GS_PLANES][PW] heartbeat reports of the current round: one bit plane per phase
                                        p (tick = round tick + 1 + p) and observer row, PW = NP rounded up
                                        to 256, / 64; column c at word (c/256)*4 + c%4, bit (c/4)%64;
                                        replayed into GS_R_FD by gs_liveness */
    GS_R_PEND_STAMP,  /* u32 [N][GS_PLANES] tick of the phase that last wrote plane row (o, p): the row is
                                        valid for the current round only if it equals round tick + 1 + p */
    GS_R_LATEST,      /* u32 [NC][KP]  each key's latest write: version | DeltaPb bytes of its KeyValueUpdatePb
                                        field << 16 (no GS_TOMBSTONES only: versions <= 16,256, values < 16 KiB) */
    GS_R_SELF_HB,     /* u32 [NP]      each owner column's own heartbeat (the diagonal of GS_R_HB, full width) */
    GS_R_CAND,        /* u64 [N/2][2][2][GS_CAND_CAP] canonical one-slice phases: each exchange's stale owners
                                        per direction and row half, in column order, as {local column,
                                        sender max_version word | receiver max_version word << 16}, written
                                        by pass 1 for the packer (the first GS_CAND_CAP of each half) */
    GS_R_CAND_N,      /* u32 [N/2][2][2] stale owners found per exchange, direction and row half (may exceed
                                        GS_CAND_CAP: the packer then walks GS_R_SLICE_BITS for that half) */
    GS_R_FD_TOD,      /* u32 [N][NP]   time of death (tick) of a GS_R_FD_STATE = 2 pair; read only for rows
                                        whose word 2 of GS_R_ROW has passed */
    GS_R_FD_LAST,     /* u16 [N][NP]   the window's _last_heartbeat tick mod 2^16 (decoded against the
                                        operation's tick; exact until 2^15 old, then only "old": bit 3 above;
                                        gs_create requires max_interval < 2^14 and
                                        phi_threshold * max(max_interval, prior) < 2^15 ticks) */
    GS_R_SLOT_STAT,   /* u32 [N/2][2][4] sliced canonical handles: per exchange and direction, this slice's
                                        {NodeDeltas, kvs, candidates, needs a pack} of a speculative phase,
                                        between gs_phase_count and gs_phase_pack */
    GS_R_RING_SLOT,   /* u32 [N]       sampled rings: each observer row's ring slot, GS_NONE = compact windows */
    GS_R_SELF_MV,     /* u32 [NP]      each owner column's own max_version (its latest write's version) */
    GS_R_SELF_PK,     /* u32 [NP]      GS_MV8: both, packed for pass 1: own heartbeat mod 2^15 | (heartbeat >= 2^15)
                                        << 15 | own max_version << 16 */
    GS_R_VLOG,        /* u32 [NC][VL]  each owner's writes by version (no GS_TOMBSTONES only: every write is version
                                        max_version + 1), VL = K * (hist_cap - 1) + 1 rounded up to 4: entry v =
                                        DeltaPb bytes of write v's KeyValueUpdatePb field | (version of the
                                        next write of the same key, 0xFFFF = none) << 16 */
    GS_R_P1FLAGS,     /* u32 [NP/16]   GS_MV8: per 16-owner group, bit i = owner 16 g + i's own heartbeat is < 2^8, bit
                                        16 + i = that owner is "hot" (some view of it lagged by >= 64 heartbeats or >= 32
                                        versions at the last lag sweep): pass 1's byte-parallel path skips hot owners */
    GS_R_ESC16,       /* u16 [N][esc_cols] the escaped owner columns' heartbeat views mod 2^16 (observer o, slot s),
                                        decoded against the owner's own heartbeat; GS_R_HB's bytes of those columns
                                        are not used while they are escaped */
    GS_R_ESC_SLOT,    /* u32 [NP]      escape slot of each owner column, GS_NONE = its views are the bytes of GS_R_HB */
    GS_R_ESC_OWNER,   /* u32 [esc_cols] the owner column of each slot, GS_NONE = free */
    GS_R_ESC_REQ,     /* u32 [NP/32 + 16] sweep scratch: columns to escape (bitmap), then the sweep's move list */
    GS_NUM_REGIONS
};

/* Prefix views (no GS_TOMBSTONES: no deletes, no tombstone GC).  Bit 15 of a GS_R_MV word
 * (GS_MV_INEXACT) is set iff the view is NOT S_j(max_version) = owner j's latest write of every
 * key with version <= max_version, i.e. iff it has holes (a truncated NodeDelta, or a delta
 * from a view with holes).  GS_R_HELD is kept only for those views; the others
 * follow from the owner's history (gs_materialize_held writes them out for readers).  With
 * GS_TOMBSTONES bit 15 is always 0 and GS_R_HELD always kept. */
#define GS_MV_INEXACT 0x8000u

typedef struct gs_counters {
    uint64_t exchanges;     /* exchanges executed */
    uint64_t hb_reports;    /* FailureDetector.report_heartbeat calls */
    uint64_t node_deltas;   /* NodeDeltas sent */
    uint64_t kvs_sent;      /* KeyValueUpdates sent */
    uint64_t truncated;     /* NodeDeltas cut by the MTU (sent with a prefix of their kvs) */
    uint64_t delta_bytes;   /* sum of DeltaPb sizes */
    uint64_t alg_bytes;     /* element-granular bytes of HBM-resident regions loaded + stored by the exchange
                               kernels (the L2-resident SELF_HB row they also read is not counted) */
    uint64_t hb_writes;     /* heartbeat entries changed */
    uint64_t candidates;    /* stale owners evaluated by the packers */
    uint64_t live_pairs;    /* (observer, target) pairs swept by the liveness kernel */
    uint64_t tomb_gc;       /* tombstones removed by gc_marked_for_deletion */
    uint64_t err_fd_overflow;  /* compact window full without GS_FD_RING (result inexact) */
    uint64_t err_hist_full;    /* a (owner, key) wrote more than hist_cap - 1 times */
    uint64_t err_bad_index;    /* exchange endpoint out of range or a == b */
    uint64_t err_conflict;     /* a node appeared twice in one phase */
    uint64_t err_fd_gc;        /* a dead target expired in a GS_CANONICAL state (removal needs the general layout) */
    uint64_t err_insert;       /* insertion into a GS_CANONICAL state */
    uint64_t fd_gc;            /* targets removed by FailureDetector.garbage_collect */
    uint64_t q9;               /* garbage_collect calls that raised KeyError */
    uint64_t pack_bytes;       /* the part of alg_bytes moved by delta packing + apply (pass 3) */
    uint64_t err_holes;        /* GS_NO_HELD: a view got holes (a truncated NodeDelta); result inexact */
    uint64_t err_hb_lag;       /* a view lagged its owner's heartbeat by >= 2^15 at a gs_check_heartbeat_lag
                                  sweep: the 16-bit heartbeat store is no longer known to be exact */
    uint64_t plane_flushes;    /* host count: mid-round report replays (phases > GS_PLANES ticks after the plane base) */
    uint64_t fd_saturated;     /* sampled rings: intervals a full compact window could not append (the compact rows'
                                  windows are exact only up to W intervals; the ring rows are exact) */
    uint64_t lite_slots;       /* (exchange, direction) slots whose whole delta k_lite sized and applied (the exact
                                  packer skipped them) */
    uint64_t lag_sweeps;       /* host count: heartbeat / max_version lag sweeps run (gs_check_heartbeat_lag, by
                                  itself or from gs_begin_round / the phases / gs_owner_writes) */
    uint64_t lite_bytes;       /* the part of pack_bytes moved by k_lite (records read, version-log entries, NodeId
                                  sizes, the receivers' max_version stores) */
    uint64_t live_bytes;       /* element bytes the liveness sweeps (k_liveness) loaded and stored: windows, state
                                  bytes, times of death, ring entries, the report planes they replayed */
    uint64_t hb_escapes;       /* owner columns moved to 16-bit escape slots by lag sweeps (gs_config.esc_cols) */
    uint64_t hb_releases;      /* escaped owner columns moved back to 8-bit views */
    uint64_t pack_groups_max;  /* a MAXIMUM, not a sum: the most groups of 64 stale owners one (exchange, direction)
                                  slot's exact packer walked (evaluated or skipped) in one phase since the reset */
    uint64_t pack_steps_max;   /* a MAXIMUM: the longest dependent walk of one slot -- groups evaluated, batches of
                                  groups skipped in first-fit continuation, bitmap windows -- the packer's
                                  critical path */
    uint64_t heavy_slots;      /* (exchange, direction) slots the exact packer handed to its heavy-slot kernel
                                  (k_pack_heavy: more stale owners than the hand-off threshold) */
    uint64_t reserved[7];
} gs_counters;

/* Failure-detector membership census (gs_fd_census): (observer, target) pairs with the observer up and
 * target != observer, split by whether the target is up (BASELINE config 5: false-positive rate =
 * up_dead / up_pairs). */
typedef struct gs_census {
    uint64_t up_pairs;    /* target up */
    uint64_t up_dead;     /* ... and in the observer's dead set (false positive) */
    uint64_t up_live;     /* ... and in the observer's live set */
    uint64_t down_pairs;  /* target down */
    uint64_t down_live;   /* ... but still in the observer's live set (not yet detected) */
} gs_census;

typedef struct gs_write {   /* one owner write */
    uint32_t owner, key, op, value_id, value_len;
} gs_write;

typedef struct gs_handle gs_handle;

int gs_create(const gs_config *cfg, gs_handle **out);
void gs_destroy(gs_handle *h);
const char *gs_last_error(const gs_handle *h);
int gs_api_version(void);

/* bytes the caller must allocate for a region (0 = unused under this config) */
int gs_region_bytes(const gs_handle *h, int region, uint64_t *bytes);
int gs_bind(gs_handle *h, int region, void *device_ptr);
int gs_set_stream(gs_handle *h, void *hip_stream);

/* Fill every bound region with the boot state: each node knows only itself with
 * heartbeat 1 (Cluster.__init__, server.py:90-96).  nid_size/key_len are host arrays. */
int gs_boot(gs_handle *h, const uint16_t *nid_size, const uint8_t *key_len);
/* Warm start: every observer learns every owner's current state, in index order. */
int gs_warm(gs_handle *h);
/* Sampled rings (gs_config.ring_rows > 0): the observer rows (host array, distinct, n <= ring_rows) whose
 * windows keep interval rings, ring slot i = rows[i].  After gs_boot, before the first phase. */
int gs_set_ring_rows(gs_handle *h, const uint32_t *rows, uint32_t n);

/* Fill GS_R_HELD of observer rows [row_lo, row_hi) for the views it is not kept for (see
 * GS_MV_INEXACT).  Readback only; no-op with GS_TOMBSTONES. */
int gs_materialize_held(gs_handle *h, uint32_t row_lo, uint32_t row_hi);

/* Owner writes at `tick` (state.py:137-180).  `ops` is a DEVICE array; owners must be distinct. */
int gs_owner_writes(gs_handle *h, const gs_write *ops, uint32_t n, uint32_t tick);
/* Round start for every node with up[o] != 0 (DEVICE u8 array): inc_heartbeat +
 * gc_marked_for_deletion (server.py:471-474, state.py:253-274, 333-338).  The previous round's
 * phases must have been closed by gs_liveness. */
int gs_begin_round(gs_handle *h, const uint8_t *up, uint32_t tick);
/* One conflict-free phase of exchanges initiators[e] -> responders[e] (DEVICE int32 arrays):
 * Syn/SynAck/Ack = server.py:327-376 + 524, i.e. compute_digest, _report_heartbeat,
 * compute_partial_delta_respecting_mtu and apply_delta on both sides.  At most n_nodes/2 exchanges;
 * the round must still be open (no gs_liveness since the last gs_begin_round) and `tick` must be
 * later than the round start and not earlier than the round's previous phase: a phase at the previous
 * phase's tick is a sub-phase (the exchanges a schedule needs past its tick budget, e.g. the 8 seeds'
 * hundreds of exchanges while every live set is empty: the reference runs every selected exchange,
 * server.py:476-493; its reports at one time append 0-s intervals, failure_detector.py:32-38).  The failure
 * detector's report_heartbeat calls are recorded per phase (GS_R_PEND bit planes, GS_PLANES per row) and
 * applied to the sampling windows, in tick order, by the gs_liveness that closes the round (nothing reads a
 * window in between); a phase past the planes' base's GS_PLANES planes replays the pending planes into the
 * windows first (counted in plane_flushes). */
int gs_run_phase(gs_handle *h, const int32_t *initiators, const int32_t *responders, uint32_t n, uint32_t tick);
/* Owner-column sliced phase (n_shards > 1; gs_run_phase refuses sliced handles).  The slices of one
 * cluster run, per phase, on the same initiators/responders:
 *   1. gs_phase_count: pass 1 of every exchange on this slice's columns (heartbeats, failure-detector
 *      reports, stale-owner bitmaps) and, per exchange and direction, the DeltaPb bytes of all this
 *      slice's stale owners: DEVICE u64 slice_bytes[n][2] (dir 0 = responder -> initiator) =
 *      bytes | (the smallest single-kv NodeDelta among them, GS_TOT_MIN1_NONE if none) << 40;
 *   2. the caller gathers every slice's slice_bytes into slice_bytes_all[G][n][2] (slice order), e.g.
 *      an RCCL all-gather;
 *   3. gs_phase_pack(step 0): packing + apply_delta of this slice's owners, resumed at the DeltaPb
 *      size the earlier slices reach (compute_partial_delta_respecting_mtu walks owners in dict order,
 *      state.py:392-413); its state goes to chain[n][2];
 *   4. only if some exchange's slice totals sum past the mtu: for step = 1 .. G-1, gather every
 *      slice's chain into chain_all[G][n][2], then gs_phase_pack(step).
 * The result equals gs_run_phase on one handle bit for bit. */
int gs_shard_columns(const gs_handle *h, uint32_t *col_lo, uint32_t *n_cols);
int gs_phase_count(gs_handle *h, const int32_t *initiators, const int32_t *responders, uint32_t n, uint32_t tick,
                   uint64_t *slice_bytes);
int gs_phase_pack(gs_handle *h, const int32_t *initiators, const int32_t *responders, uint32_t n, uint32_t tick,
                  uint32_t step, const uint64_t *slice_bytes_all, const uint64_t *chain_all, uint64_t *chain);
#define GS_TOT_BYTES(x) ((x) & ((1ull << 40) - 1ull))
#define GS_TOT_MIN1(x) ((uint32_t)((x) >> 40))
#define GS_TOT_MIN1_NONE 0xFFFFFFu
/* Compacted chain (replaces step 4 above on canonical handles built with candidate records):
 *   gs_phase_overflow (blocking: one 4-byte read): the slots (2e + dir) whose gathered slice totals sum
 *     past the mtu, in slot order, into DEVICE list[GS_OVERFLOW_LIST_LEN(n)] (the tail is scratch), this
 *     slice's chain state of each into DEVICE chainc[2n + 1] and, at chainc[count], how many of them this
 *     slice still has pending; their number into *count (host; NULL: not read back);
 *   then, for step = 1 .. G-1: gather every slice's chainc[0 .. count] into chain_all[G][count + 1]; stop
 *     once every slice's pending entry (chain_all[g][count]) is 0; else gs_phase_chain(step) (one wave per
 *     listed slot; chain, chainc and the pending entry updated).
 * A pending slice resumes from its nearest finished predecessor f when every slice between them is
 * pending and cannot add a NodeDelta: f's delta is complete, or that slice's smallest single-kv
 * NodeDelta (GS_TOT_MIN1 of its total) exceeds the budget f left (first-fit continuation would skip all
 * of its owners) -- so a chain usually resolves in one step instead of G - 1.  Every slice computes the
 * same list from the same gathered totals, so only (count + 1) x 8 bytes per slice travel per step. */
int gs_phase_overflow(gs_handle *h, uint32_t n, const uint64_t *slice_bytes_all, const uint64_t *chain,
                      uint32_t *list, uint64_t *chainc, uint32_t *count);
int gs_phase_chain(gs_handle *h, const int32_t *initiators, const int32_t *responders, uint32_t n, uint32_t tick,
                   uint32_t step, const uint32_t *list, uint32_t count, const uint64_t *chain_all, uint64_t *chain,
                   uint64_t *chainc, const uint64_t *slice_bytes_all);

/* The state after a chain step, read back in one wait (aiocluster_amd/shard.py's driver; the library's own sliced
 * phases do the same): *pending = the listed slots still pending summed over the slices (entry `count` of each
 * slice's row of chain_all, rows of count + 1 entries -- or of GS_CHAIN_CAP + 1 with count = GS_CHAIN_DEVICE, whose
 * count is gs_phase_overflow's device count at the tail of `list`), UINT64_MAX when that device count exceeds
 * GS_CHAIN_CAP (the device step did not run); *count_out = the count.  Replaces shard.py's torch reductions and
 * read (round 5): one small kernel writing a pinned host pair, one stream wait. */
int gs_phase_pending(gs_handle *h, uint32_t n, const uint32_t *list, uint32_t count, const uint64_t *chain_all,
                     uint64_t *pending, uint32_t *count_out);
/* count = GS_CHAIN_DEVICE: the count is not read back -- the kernels take it from `list` (gs_phase_overflow's count
 * entry), every slice gathered GS_CHAIN_CAP + 1 entries of its chainc into chain_all[G][GS_CHAIN_CAP + 1], and a
 * phase whose count exceeds GS_CHAIN_CAP is left to the host path (the step does nothing on any slice).  Lets a
 * driver run step 1 before any host read: a chain usually resolves in that step, so one read of the gathered
 * pending entries (k_sum_pending in the library driver) ends the phase. */
#define GS_CHAIN_DEVICE 0xFFFFFFFFu
#define GS_CHAIN_CAP 1024u

/* ---- Multi-GPU: one handle per device, each holding one owner-column
 * slice; the library drives the sliced phase itself (count, all-gather of the slice totals, packing,
 * the overflow chain) over an RCCL communicator.  Rank 0 calls gs_comm_id and hands the
 * GS_COMM_ID_BYTES bytes to every rank (e.g. a torch.distributed broadcast); each rank then calls
 * gs_comm_init(h, id, n_shards, shard) on its slice (ncclCommInitRank), and gs_run_phase on a sliced
 * handle runs the whole phase (one blocking host read of the overflow count, as gs_phase_overflow).
 * gs_run_phase_group: the same phase for all G slices of one cluster held by this process (one device,
 * one stream; the gathers are device copies; each step one launch for all slices, grid.y = slice) -- the
 * one-GPU rehearsal and test of the same driver.  n_handles = 1 of G > 1 slices: slice 0 held alone, the
 * others' totals and chain states gathered as zeros (a timing rehearsal of one GPU's share; exact for slice 0's
 * columns, whose NodeDeltas start every delta); any other slice alone returns GS_E_UNSUPPORTED (it would pack
 * from a zero predecessor total). */
#define GS_COMM_ID_BYTES 128
int gs_comm_id(void *id);
int gs_comm_init(gs_handle *h, const void *id, uint32_t nranks, uint32_t rank);
int gs_run_phase_group(gs_handle *const *handles, uint32_t n_handles, const int32_t *initiators,
                       const int32_t *responders, uint32_t n, uint32_t tick);

/* Apply the open round's pending failure-detector reports (the GS_R_PEND planes of its phases so far) to
 * the sampling windows now, in tick order, exactly as the closing gs_liveness would (nothing reads a
 * window in between, so the result is the same); the round stays open and its next phase must come after
 * `tick` (>= the last phase's tick).  Lets a checker compare GS_R_FD / GS_R_FD_LAST rows mid-round. */
int gs_flush_reports(gs_handle *h, uint32_t tick);

/* _update_node_liveness for every up node (server.py:606-620; failure_detector.py:89-128),
 * including garbage_collect + remove_node (general layout only). */
int gs_liveness(gs_handle *h, const uint8_t *up, uint32_t tick);

/* SamplingWindow.phi (failure_detector.py:43-53) of every target of `observer` at `tick`
 * into the DEVICE array out[n_cols] (this slice's targets; binary64; NaN where the reference
 * returns None). */
int gs_phi_row(gs_handle *h, uint32_t observer, uint32_t tick, double *out);

/* Heartbeat-lag sweep over every view of this handle (asynchronous): counts in err_hb_lag the views
 * whose heartbeat lags the owner's own by >= 2^15 (GS_R_HB stores heartbeats mod 2^16).  An owner's
 * heartbeat grows by at most one per round start or phase; gs_begin_round runs this sweep by itself
 * whenever 2^14 round starts + phases have passed since the last one, which keeps every decode exact
 * until a sweep reports otherwise. */
int gs_check_heartbeat_lag(gs_handle *h);

/* Batched hook events (Cluster.on_key_change / on_node_join / on_node_leave, server.py:217-257).
 * When enabled, every kernel that changes what a hook reports appends 8 x u32 records
 * {observer, owner, key | kind << 8, old version (0 = none), new version, tick, seq, 0} to the DEVICE
 * array records[capacity][8], counting in the DEVICE u32 *count (records beyond capacity are dropped
 * but counted; the caller resets *count).  kind 0 = on_key_change: a kv stored by apply_delta
 * (state.py:228-231) or an owner set / set_with_ttl (owner deletes mutate the stored value in
 * place and emit nothing, server.py:199-215); 1 = node join, 2 = node leave: the live set of
 * _update_node_liveness against the previous one (server.py:611-616).  Records are appended in no
 * particular order; seq makes the reference's order recoverable:
 *   owner write:  the write's index among all gs_owner_writes ops since gs_set_events (counting every
 *                 op of every call, in call order; a write's index within its call is its row in ops);
 *   apply_delta:  the sender's dict position of the owner (the NodeDelta order of the delta,
 *                 state.py:346-413); a NodeDelta's kvs are applied in version order;
 *   join / leave: 0 (the reference iterates Python sets there: no order to reproduce).
 * So the reference's order (oracle/gen_events_fixture.py) is: by tick; owner writes by seq; in a
 * phase by exchange (its index in the phase), the initiator's apply (SynAck delta) before the
 * responder's (Ack delta), then seq, then new version; liveness by observer, joins before leaves,
 * then owner.  Exchanges between prefix views take the per-key apply path while enabled.
 * records = NULL: off. */
int gs_set_events(gs_handle *h, uint32_t *records, uint32_t capacity, uint32_t *count);

/* select_nodes_for_gossip (server.py:656-717) for every up node at round start (server.py:442-469),
 * from its failure detector's live / dead sets and known peers: `fanout` distinct peers uniformly from
 * the live set (all known peers while it is empty), a dead node with probability dead / (live + 1),
 * a seed (from the DEVICE list seeds[n_seeds], self excluded) when no selected peer is a seed or
 * live < seeds, with probability seeds / (live + dead) (1 when both are 0; always when live = 0).
 * Random numbers: Philox4x32-10 keyed by `seed`, counter (round, node, slot).  Output DEVICE
 * targets[N][fanout + 2] = fanout peers, the dead pick, the seed pick (-1 = none).  DEVICE scratch of
 * 4 * N * (fanout + 6) bytes.  1 <= fanout <= 8; one slice only. */
int gs_select_peers(gs_handle *h, const uint8_t *up, uint32_t fanout, const int32_t *seeds, uint32_t n_seeds,
                    uint64_t seed, uint32_t round, int32_t *targets, void *scratch);
/* The round's exchanges (initiator o, responder targets[o][s], responder up) in <= max_phases
 * (<= GS_MAX_SCHED_PHASES) conflict-free phases: per phase `iters` rounds of a deterministic Luby matching
 * (an exchange whose endpoints are free in that phase takes it if its priority key is the smallest at
 * both).  Writes the exchanges of phase p to DEVICE initiators/responders[phase_offsets[p] ..
 * phase_offsets[p+1]) (order within a phase unspecified: exchanges of one phase commute) and the host
 * array phase_offsets[max_phases + 1]; *unscheduled (host) = valid exchanges (responder up) left
 * after max_phases phases, which are not run (0 unless the round needs more phases).  DEVICE scratch
 * of GS_SCHED_SCRATCH_BYTES(N, fanout, max_phases) bytes.  Blocking. */
int gs_schedule_phases(gs_handle *h, const uint8_t *up, uint32_t fanout, const int32_t *targets, uint64_t seed,
                       uint32_t round, uint32_t iters, uint32_t max_phases, void *scratch, int32_t *initiators,
                       int32_t *responders, uint32_t *phase_offsets, uint32_t *unscheduled);

/* FailureDetector.live_nodes / dead_nodes of every up observer (failure_detector.py:63-67) counted
 * against the DEVICE up mask; blocking.  Sliced handles count their own target columns. */
int gs_fd_census(gs_handle *h, const uint8_t *up, gs_census *out);

/* Wire-format emitter: the protobuf bytes the reference's SerializeToString gives, from device state,
 * so a simulated cluster can talk to real aiocluster nodes (messages.proto:46-74).  String tables are
 * DEVICE arrays owned by the caller: NodeIdPb bytes of every node (entities.py:62-72; node i at
 * node_ids[node_id_off[i] .. node_id_off[i + 1])), the UTF-8 key names (key_off[K + 1]) and the
 * interned values by value id (value_off[n_values + 1]; value ids as passed to gs_owner_writes).
 *   gs_emit_digest: DigestPb of observer's compute_digest at `tick` (state.py:324-331, 56-58; what
 *                   _make_syn_msg sends, server.py:327-332);
 *   gs_emit_delta:  DeltaPb of sender's compute_partial_delta_respecting_mtu(receiver's digest at `tick`,
 *                   mtu, sender's scheduled_for_deletion) (state.py:340-415, 98-99; the SynAck delta,
 *                   server.py:339-346), without applying it.
 * `out` is a DEVICE buffer of `cap` bytes; *len (host) receives the message size.  A size above `cap`
 * returns GS_E_INVALID with *len set and nothing written (out = NULL: size query).  DEVICE scratch of
 * gs_emit_scratch_bytes.  Blocking; one slice only. */
typedef struct gs_wire {
    const uint8_t *node_ids;
    const uint32_t *node_id_off;
    const uint8_t *keys;
    const uint32_t *key_off;
    const uint8_t *values;
    const uint64_t *value_off;
} gs_wire;
int gs_emit_scratch_bytes(const gs_handle *h, uint64_t *bytes);
int gs_emit_digest(gs_handle *h, const gs_wire *w, uint32_t observer, uint32_t tick, uint8_t *out, uint64_t cap,
                   uint64_t *len, void *scratch);
int gs_emit_delta(gs_handle *h, const gs_wire *w, uint32_t sender, uint32_t receiver, uint32_t tick, uint8_t *out,
                  uint64_t cap, uint64_t *len, void *scratch);

/* Measurement (no handle; asynchronous on `stream`): a 16-B-per-lane streaming copy of `bytes`
 * (multiple of 16, 16-B aligned DEVICE buffers) -- the HBM ceiling bench.py reports -- and a
 * read-only stream of `bytes` at `width` = 4, 8 or 16 B per lane (DEVICE u64 *sink keeps the loads), the
 * known byte count that calibrates rocprofv3's FETCH_SIZE for those access widths. */
int gs_stream_copy(void *dst, const void *src, uint64_t bytes, void *stream);
int gs_stream_read(const void *src, uint64_t bytes, uint32_t width, uint64_t *sink, void *stream);
/* a write-only stream of `bytes` at `width` = 4, 8 or 16 B per lane: the known byte count for WRITE_SIZE */
int gs_stream_write(void *dst, uint64_t bytes, uint32_t width, void *stream);
/* a trace marker: which = 0 launches the empty kernel k_mark_begin, 1 k_mark_end, on `stream`.  bench.py brackets
 * its timed rounds with them so that a rocprofv3 kernel trace / PMC pass can select exactly those dispatches
 * (tools/pmc_summary.py). */
int gs_mark(uint32_t which, void *stream);

/* Per-kernel timing (measurement): with timing on, every launch of the kinds below is bracketed by HIP
 * events on the library's stream; gs_kernel_times (blocking) returns the summed milliseconds and launch
 * counts since the previous call and clears them. */
#define GS_KT_PASS1 0     /* pass 1 of a canonical phase (k_pass1; with env GS_PACK=fused, k_pass1 fused with
                             packing), the general-layout k_exchange, pass 1 of gs_phase_count */
#define GS_KT_PACK 1      /* delta packing + apply_delta as their own kernel: k_settle (one-slice phases and
                             gs_phase_pack step 0), k_pack_slice (GS_PACK=split), k_chain_step (gs_phase_chain) */
#define GS_KT_LIVENESS 2  /* k_liveness (report replay + liveness sweep) */
#define GS_KT_COUNT 3     /* the slice byte totals of gs_phase_count (k_settle, count mode) */
#define GS_KT_LITE 4      /* k_lite: the whole-delta fast path of prefix-view record phases (before the exact
                             packer, which then runs only the slots it could not complete) */
#define GS_KT_KINDS 8
typedef struct gs_ktimes {
    double ms[GS_KT_KINDS];
    uint64_t launches[GS_KT_KINDS];
} gs_ktimes;
int gs_set_timing(gs_handle *h, int on);
int gs_kernel_times(gs_handle *h, gs_ktimes *out);

int gs_read_counters(gs_handle *h, gs_counters *out);
int gs_reset_counters(gs_handle *h);
int gs_sync(gs_handle *h);

/* Copy-out (blocking, SURVEY §8(b) gs_read_*): observer rows [row_lo, row_hi) of a region indexed by
 * observer row (GS_R_HB, MV, GC, HELD, FD, FD_LAST, FD_STATE, FD_TOD, TS, RING, POS, ORD, ROW, ESC16) into host memory
 * `out` of `cap` bytes, in the region's layout; *len = the bytes of those rows (set even when they exceed
 * cap, which fails).  GS_R_HELD rows are complete: the prefix views' ordinals are materialized first.
 * GS_R_HB rows are the stored bytes: an escaped owner column's views (GS_R_ESC_SLOT != GS_NONE) are read from
 * GS_R_ESC16 (also a row region here), as GossipSim.decode_heartbeats does. */
int gs_read_rows(gs_handle *h, int region, uint32_t row_lo, uint32_t row_hi, void *out, uint64_t cap, uint64_t *len);

/* The latest tick any operation on h has used: GS_R_FD_LAST rows read with gs_read_rows are decoded against
 * it (tick - ((tick - s) mod 2^16); a window with bit 3 of GS_R_FD_STATE set as tick - 2^15). */
int gs_latest_tick(const gs_handle *h, uint32_t *tick);

#ifdef __cplusplus
}
#endif
#endif
