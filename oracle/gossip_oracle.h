/*
 * gossip_oracle.h -- CPU restatement of aiocluster's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the *checker* for the HIP simulator
 * (aiocluster_amd/csrc), never the product: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  It restates, object by object,
 * the reference's Python semantics:
 *
 *   NodeState / ClusterState  -- aiocluster/state.py:106-415
 *   SamplingWindow / FailureDetector / BoundedArrayStats
 *                             -- aiocluster/failure_detector.py:12-162
 *   exchange + round driver   -- aiocluster/server.py:327-376, 441-495, 523-568, 599-620
 *
 * Time is in microseconds (the reference's datetime resolution).  Values are
 * interned by the host: value_id identifies the string, value_len is its UTF-8
 * byte length (all the hot path needs for protobuf sizes).
 *
 * Pinned against the real reference by tests/golden/scen_*.json.gz (generated
 * by oracle/gen_golden.py) and by ports of the reference's own unit tests.
 */
#ifndef GOSSIP_ORACLE_H
#define GOSSIP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_config {
    int32_t n_nodes;
    int32_t n_keys;
    int32_t mtu;                    /* Config.max_payload_size (entities.py:105) */
    int64_t tombstone_grace_us;     /* Config.marked_for_deletion_grace_period (entities.py:101) */
    double  phi_threshold;          /* FailureDetectorConfig.phi_threshhold (entities.py:87) */
    int32_t window;                 /* sampling_window_size (entities.py:88) */
    int64_t max_interval_us;        /* entities.py:89 */
    int64_t initial_interval_us;    /* entities.py:90 (the prior mean) */
    int64_t dead_grace_us;          /* dead_node_grace_period (entities.py:91) */
} orc_config;

typedef struct orc orc;

typedef struct orc_stats {
    uint64_t exchanges;
    uint64_t node_deltas;
    uint64_t kvs_sent;
    uint64_t delta_bytes;      /* sum of DeltaPb sizes sent */
    uint64_t hb_reports;       /* FailureDetector.report_heartbeat calls */
    uint64_t truncated;        /* NodeDeltas cut by the MTU */
} orc_stats;

orc *orc_create(const orc_config *cfg, const int32_t *nid_size, const int32_t *key_len);
void orc_destroy(orc *o);

/* Cluster.__init__ (server.py:90-100): self view with heartbeat 1. */
void orc_boot(orc *o, int32_t node);
/* Every observer learns every owner in index order (warm start injection). */
void orc_init_warm(orc *o);

/* NodeState.set / delete / set_with_ttl / delete_after_ttl (state.py:137-180). op: 0..3 */
void orc_write(orc *o, int32_t owner, int32_t key, int32_t op, uint32_t value_id, int32_t value_len, int64_t now_us);

/* server.py:471-474: inc_heartbeat + gc_marked_for_deletion. */
void orc_begin_round(orc *o, int32_t node, int64_t now_us);

/* One Syn/SynAck/Ack exchange initiated by a towards b (server.py:327-376, 524). */
void orc_exchange(orc *o, int32_t a, int32_t b, int64_t now_us);

/* _update_node_liveness (server.py:606-620).  Returns -1, or the node index whose
 * missing sampling window raised KeyError in FailureDetector.garbage_collect (Q9). */
int32_t orc_liveness(orc *o, int32_t node, int64_t now_us);

/* The same three operations over a whole phase / all up rows on `threads` host threads (checker speed for
 * the long whole-array tests only).  A phase's exchanges touch disjoint rows and a round start or liveness
 * sweep one row each, so the rows are split over the threads, each with scratch of its own; the result is
 * the sequential one.  Hook events must be off.  q9[node] = orc_liveness's return for each up node (-1 else). */
void orc_run_phase_mt(orc *o, const int32_t *a, const int32_t *b, int32_t n, int64_t now_us, int32_t threads);
void orc_begin_round_mt(orc *o, const uint8_t *up, int64_t now_us, int32_t threads);
void orc_liveness_mt(orc *o, const uint8_t *up, int64_t now_us, int32_t threads, int32_t *q9);

/* ------------------------------------------------------------- readback */
int32_t orc_node_count(const orc *o, int32_t obs);
void    orc_node_order(const orc *o, int32_t obs, int32_t *out);
/* out: heartbeat, max_version, last_gc_version */
void    orc_view(const orc *o, int32_t obs, int32_t owner, uint32_t out[3]);
/* per key: present, version, status, value_id, ts_us */
void    orc_view_kvs(const orc *o, int32_t obs, int32_t owner, int32_t *present, uint32_t *version,
                     int32_t *status, uint32_t *value_id, int64_t *ts_us);
/* failure detector: window (has, last_us, len, sum); live flag; dead tod (or -1) */
int32_t orc_fd_window(const orc *o, int32_t obs, int32_t target, int64_t *last_us, int32_t *len, double *sum);
int32_t orc_fd_phi(const orc *o, int32_t obs, int32_t target, int64_t now_us, double *phi);
int32_t orc_fd_live(const orc *o, int32_t obs, int32_t target);
int64_t orc_fd_dead_since(const orc *o, int32_t obs, int32_t target);
void    orc_get_stats(const orc *o, orc_stats *out);
/* hook events (Cluster.on_key_change / on_node_join / on_node_leave): records of 6 int64
 * {observer, owner, key | kind << 8, old version, new version, now_us}, kind 0/1/2 = key/join/leave */
void    orc_enable_events(orc *o, int32_t on);
int32_t orc_drain_events(orc *o, int64_t *out, int32_t cap);
/* Bulk export of one observer row (arrays sized N, or N*K for per-key fields):
 * present[j] = dict position or -1; per-key version/status/value_id/ts (version 0 = absent);
 * FD: window last (-1 = no window), len, sum; live flag; time of death (-1 = not dead). */
void    orc_export_row(const orc *o, int32_t obs, int32_t *pos, uint32_t *hb, uint32_t *mv, uint32_t *gc,
                       uint32_t *kv_version, int32_t *kv_status, uint32_t *kv_value_id, int64_t *kv_ts,
                       int64_t *fd_last, int32_t *fd_len, double *fd_sum, int32_t *live, int64_t *tod);

/* -------------------------------------------------- state injection (baseline) */
/* Replace observer obs's whole row: order[cnt], heartbeat/max/gc[n], kv ordinals are
 * resolved through the owner write history the caller passes (version, status,
 * value_id, value_len per (owner, key, w)). Used to time the oracle on rows taken
 * from a device snapshot. */
void orc_load_row(orc *o, int32_t obs, int32_t cnt, const int32_t *order,
                  const uint32_t *hb, const uint32_t *mv, const uint32_t *gc,
                  const uint8_t *held_w, int32_t hist_cap,
                  const uint32_t *hist_version, const uint32_t *hist_value_id,
                  const int32_t *hist_value_len, const uint8_t *hist_status,
                  const uint32_t *fd_last_tick, const uint32_t *fd_sum_tick, const uint32_t *fd_len,
                  const uint32_t *fd_state, int64_t tick_us);

/* status_change_ts (state.py:124-131, 222-227) of the tombstones of a row loaded by orc_load_row:
 * ts_tick[N][K] in ticks, 0xFFFFFFFF = none. */
void orc_set_row_ts(orc *o, int32_t obs, const uint32_t *ts_tick, int64_t tick_us);

/* The interval rings of a row loaded by orc_load_row (device rows with sampled rings): ring_tick[N][W]
 * in ticks, cnt[N] = appends since the last reset (< 2W: full once >= W, next slot cnt mod W). */
void orc_set_row_ring(orc *o, int32_t obs, const uint16_t *ring_tick, const uint32_t *cnt, int64_t tick_us);

/* Keep a copy of observer obs's row / put it back (the CPU baseline re-runs the same
 * exchanges on restored rows to accumulate a bounded, repeatable sample). */
void orc_snapshot_row(orc *o, int32_t obs);
void orc_restore_row(orc *o, int32_t obs);

/* ------------------------------------------- method-level hooks (KAT ports)
 * Direct access to single NodeState / ClusterState / FailureDetector methods so the
 * reference's own unit tests (tests/test_state.py, test_node_state.py,
 * test_failure_detector.py) can be replayed against the oracle. */
void    orc_kat_set_view(orc *o, int32_t obs, int32_t owner, uint32_t hb, uint32_t mv, uint32_t gc);
void    orc_kat_set_kv(orc *o, int32_t obs, int32_t owner, int32_t key, uint32_t value_id, int32_t value_len,
                       uint32_t version, int32_t status, int64_t ts_us);
/* NodeState.apply_heartbeat (state.py:280-287) */
int32_t orc_kat_apply_heartbeat(orc *o, int32_t obs, int32_t owner, uint32_t value);
/* NodeState.apply_delta (state.py:190-233) of one NodeDelta (kvs in the given order) */
void    orc_kat_apply_nodedelta(orc *o, int32_t obs, int32_t owner, uint32_t from, uint32_t gc, uint32_t mv,
                                int32_t nkv, const int32_t *keys, const uint32_t *value_ids,
                                const int32_t *value_lens, const uint32_t *versions, const int32_t *statuses,
                                int64_t now_us);
/* NodeState.gc_marked_for_deletion (state.py:253-274) with an explicit grace */
void    orc_kat_gc(orc *o, int32_t obs, int32_t owner, int64_t grace_us, int64_t now_us);
/* compute_partial_delta_respecting_mtu (state.py:340-415) of `sender` for a digest given as
 * (node, last_gc, max_version) triples; returns the NodeDelta count, fills per NodeDelta
 * (node, from, kv count) and the kv versions in order. */
int32_t orc_kat_compute_delta(orc *o, int32_t sender, int32_t n_digest, const int32_t *dg_node,
                              const uint32_t *dg_gc, const uint32_t *dg_mv, int32_t mtu,
                              int32_t *nd_node, uint32_t *nd_from, int32_t *nd_nkv, uint32_t *kv_versions,
                              int32_t max_out);
/* FailureDetector.report_heartbeat / update_node_liveness / garbage_collect /
 * scheduled_for_deletion_nodes (failure_detector.py:79-128) */
void    orc_kat_fd_report(orc *o, int32_t obs, int32_t target, int64_t now_us);
void    orc_kat_fd_update(orc *o, int32_t obs, int32_t target, int64_t now_us);
int32_t orc_kat_fd_gc(orc *o, int32_t obs, int64_t now_us, int32_t *out);
int32_t orc_kat_fd_scheduled(orc *o, int32_t obs, int64_t now_us, int32_t *out);
/* SamplingWindow.reset (failure_detector.py:40-41) */
void    orc_kat_fd_reset(orc *o, int32_t obs, int32_t target);
/* BoundedArrayStats.append / sum / __len__ / clear (failure_detector.py:139-162) on a window */
void    orc_kat_win_append(orc *o, int32_t obs, int32_t target, double x);
double  orc_kat_win_sum(orc *o, int32_t obs, int32_t target);
int32_t orc_kat_win_len(orc *o, int32_t obs, int32_t target);
int32_t orc_kat_win_filled(orc *o, int32_t obs, int32_t target);

#ifdef __cplusplus
}
#endif
#endif
