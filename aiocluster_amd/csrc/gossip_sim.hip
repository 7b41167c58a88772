// gossip_sim.hip -- MI355X (gfx950) batched scuttlebutt + phi-accrual simulator.
//
// Hand-written HIP for CDNA4 (wave64).  The whole simulated cluster lives in HBM
// as dense observer x owner matrices (layout: include/gossip_sim.h).
// One launch of k_exchange runs one conflict-free phase, one 128-thread
// workgroup (2 waves) per exchange (a = initiator, b = responder):
//
//   pass 1 (both waves, both rows streamed with 16-byte loads): responder
//          heartbeat, both heartbeat merges + failure-detector reports,
//          digest membership, stale-owner bitmaps of both directions (LDS);
//   pass 2 (wave 0, general mode only): dict insertions in digest order;
//   pass 3 (wave 0: b -> a, wave 1: a -> b, concurrently): exact
//          protobuf-size MTU packing in the sender's dict order with a
//          wave prefix sum for the part that fits and a ballot-driven
//          first-fit scan once the budget is nearly spent, then apply_delta
//          at the receiver, one lane per NodeDelta.
//
// The two directions touch disjoint owner columns ("why the two
// deltas commute"), so pass 3 needs no synchronisation between the waves.
//
// Reference semantics restated here (aiocluster @ /root/reference):
//   digest            state.py:244-251, 324-331
//   heartbeat merge   server.py:336-337, 356-357, 599-604; state.py:280-287
//   delta             state.py:340-415 (+ staleness_score 425-433)
//   apply             state.py:190-233, 310-322
//   tombstone GC      state.py:253-274, 333-338
//   owner writes      state.py:124-180
//   failure detector  failure_detector.py:12-128

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>
#include <type_traits>

#include "../../include/gossip_sim.h"

namespace {

constexpr uint32_t NONE = GS_NONE;
constexpr int WAVE = 64;
constexpr int XB = 128;  // exchange workgroup: 2 waves
#ifndef XB_WAVES
#define XB_WAVES 4  // waves per SIMD k_exchange is compiled for (VGPR budget 512 / 4 = 128)
#endif
constexpr int LB = 256;  // liveness / elementwise workgroups
#ifndef LIVE_PER
#define LIVE_PER 64  // 1024-column chunks per k_liveness workgroup, at most (r4g/h/k/p at 65,536: 64 -> 10.5-10.8 ms, 32 -> 10.7-11.2, 16 -> 11.0-11.1, 8 -> 11.9, 4 -> 13.6)
#endif
constexpr int NSHARD = 64;
// native vectors: the nontemporal load / store builtins take them (not HIP's uint4 struct)
typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
typedef unsigned int v2u_t __attribute__((ext_vector_type(2)));
constexpr uint32_t WIN = 16 * 64;  // positions per packer window (16 per lane)
// KW of the kernels for K > 16 keys (up to 64).  Those instantiations take most of the build time; a
// development build with -DGS_KW4_ONLY (tools/build_dev.sh) leaves them out and refuses K > 16.
#ifdef GS_KW4_ONLY
constexpr int KWB = 4;
#else
constexpr int KWB = 16;
#endif
constexpr uint32_t NPL = GS_PLANES;  // report bit planes per observer row (phases per plane base)
static_assert(NPL == 16 || NPL == 32, "k_liveness stages 16 or 32 planes");
constexpr double TICK_S = 1.0 / 64.0;
constexpr uint32_t HB_LAG_CHECK_EVERY = 1u << 14;  // round starts + phases between heartbeat-lag sweeps
constexpr uint32_t HB8_LAG_CHECK_EVERY = 1u << 6;  // ... with GS_HB8 (checked before every round start and phase)
constexpr uint32_t MV8_LAG_CHECK_EVERY = 1u << 5;  // GS_MV8: gs_owner_writes calls between max_version lag sweeps

enum Ctr {
    C_EXCH = 0, C_REPORTS, C_ND, C_KVS, C_TRUNC, C_DBYTES, C_ALG, C_HBW, C_CAND, C_LIVE, C_TOMBGC,
    C_E_FDOVF, C_E_HIST, C_E_IDX, C_E_CONFLICT, C_E_FDGC, C_E_INSERT, C_FDGC, C_Q9, C_PACKB, C_E_HOLES,
    C_E_HBLAG, C_FLUSH /* host-side: plane_flushes */, C_FDSAT, C_LITE, C_SWEEPS /* host-side: lag_sweeps */,
    C_LITEB, C_LIVEB, C_ESC, C_ESCREL, C_PGMAX, C_PSMAX, C_HEAVY,
    C_CEN0 = 40, C_NUM = C_CEN0 + 6  // gs_fd_census scratch slots (not part of gs_counters)
};
constexpr int CFIELDS = 40;  // gs_counters fields (the last ones reserved)
constexpr int CROW = 48;     // u64 slots per counter shard row (the gs_counters fields, then the census scratch)
static_assert(C_NUM <= CROW, "counter region");
static_assert(C_HEAVY < CFIELDS, "gs_counters fields");
static_assert(sizeof(gs_counters) == CFIELDS * 8, "gs_counters layout");

struct Dev {
    uint32_t N, NP, K, KP, C, mtu, flags, W;
    // owner-column slice: this handle holds columns [col_lo, col_lo + ncol) of every observer row
    // (NP = ncol rounded to 64 is the row stride); shards = 1: the whole matrix
    uint32_t col_lo, ncol, shards, shard;
    uint32_t max_iv, tomb_grace, dead_grace, sched_delay, lb_min, sum_bits;
    uint32_t ablate;  // profiling only (env GS_ABLATE): 1 = skip packing, 2 = skip pass-1 stores (results invalid);
                      // A/B, results valid: 8 = k_pass1v without its slow-group slots
    double phi_thr, prior5;
    double prior5t;  // prior5 in ticks (x 64): the liveness sweep's division-free phi test
    float phi_thr_f, prior5t_f;  // the same in binary32: the sweep's first, full-rate test (2^-20 margin)
    uint16_t *hb;       // heartbeat mod 2^16 (hb_dec: exact while a view lags its owner by < 2^16)
    uint32_t *self_hb;  // [NP] each owner column's own heartbeat, full width
    uint32_t *gc;
    uint16_t *mv;  // max_version | MV_INEXACT (u16: versions <= K * (C - 1) <= 16,256)
    uint8_t *held;
    uint32_t *fd;       // sampling window: _sum in ticks | intervals appended since the last reset << sum_bits
    uint16_t *fd_last;  // _last_heartbeat tick mod 2^16 (decoded against the operation's tick: fd_get)
    uint8_t *fd_state;  // bits 0-1: 0 unknown, 1 live, 2 dead (_live_nodes / _dead_nodes); FD_WIN, FD_OLD
    uint32_t *tod;      // time of death of a dead pair (read only for rows whose row word 2 has passed)
    uint32_t *ts;
    uint16_t *ring;
    uint32_t *pos, *ord, *row;
    uint8_t *last_w;
    uint64_t *hist;  // version | meta << 32
    uint32_t *lat;   // [NC][KP] each key's latest write: version | DeltaPb bytes of its kv << 16 (prefix views)
    uint32_t *hist_vid;
    uint16_t *nid_size;
    uint8_t *key_len;
    uint32_t *stamp;
    unsigned long long *ctr;
    uint32_t *sbits;  // sharded phases: stale-owner bitmaps of both directions per exchange [e][2][NP/32]
    uint2 *cand;       // split phases: stale-owner records [e][dir][half][GS_CAND_CAP] (GS_R_CAND)
    uint32_t *cand_n;  // [e][dir][half] stale owners found (GS_R_CAND_N)
    // heartbeat reports of the current round not yet applied to the windows: one bit plane per phase
    // p (tick t_round + 1 + p) and observer row, [N][NPL][PW] u64 in quad-interleaved column order
    // (plane_word/plane_bit); a plane row is valid only if pstamp[o][p] holds that phase's tick
    uint64_t *pend;
    uint32_t *pstamp;  // [N][NPL]
    uint32_t PW;       // u64 words per plane row: NP rounded up to 256, / 64
    // plane base: the tick of the last gs_begin_round, or, once a round has run phases more than NPL
    // ticks after it (the planes were replayed into the windows mid-round), the tick before the
    // first phase after that replay; plane p holds the phase at tick t_round + 1 + p
    uint32_t t_round;
    // sub-phases (round 6): several phases at one tick -- every exchange select_nodes_for_gossip chose, however
    // many phases its hubs need (server.py:476-493).  Plane p of the base holds the phase of VIRTUAL tick
    // v_round + 1 + p (pstamp holds virtual ticks, unique over the handle's life) at real tick
    // min(t_round + 1 + p, t_cap) (plane_tick); vt = the virtual tick of the phase being launched (set per phase by
    // the host).  Without sub-phases v_round = t_round, vt = the phase's tick and t_cap = NONE: the round-5 layout.
    uint32_t v_round, vt, t_cap;
    // speculative max-version merge (canonical record phases): pass 1 already wrote
    // max(sender, receiver) into the receiver's max_version word of every recorded candidate whose two
    // views are prefix views; the packers restore the receiver's word of such a candidate when it is not
    // sent, and skip the store when it is sent whole.  Set per phase by the host (gs_run_phase /
    // gs_phase_count), identical in every kernel of the phase.
    uint32_t spec;
    uint4 *slot_stat;  // sliced phases: per (exchange, direction) {NodeDeltas, kvs, candidates, needs a pack}
    // sampled rings (gs_config.ring_rows): ring slot of each observer row (NONE: a compact row), GS_R_RING
    // then holds [ring_rows][NP][W]; nullptr otherwise
    uint32_t *ring_slot;
    // prefix views: each owner's writes by version, [NC][VL] (GS_R_VLOG): DeltaPb bytes of the kv field |
    // version of the next write of the same key (0xFFFF: none) << 16 -- a prefix candidate's NodeDelta
    // size from the entries (mr, ms] alone (pack_lite)
    uint32_t *vlog;
    uint32_t VL;
    uint32_t lite;  // this phase runs k_lite before the exact packer (set per phase by the host)
    uint32_t hb8;   // GS_HB8: hb holds u8 views (mod 2^8), else u16 (mod 2^16)
    uint32_t mv8;   // GS_MV8: mv holds u8 views (version mod 2^7 | inexact << 7), else u16 words
    uint32_t *self_mv;  // [NP] each owner column's own max_version (GS_R_SELF_MV)
    // GS_MV8: [NP] both owner values packed for pass 1 (self_pack): one 16-byte load per 4 columns decodes
    // both 8-bit views -- the heartbeat needs only R mod 2^8 and whether R is 0 (R < 2^15 kept exactly),
    // the max_version word only M (< 2^15)
    uint32_t *self_pk;
    // GS_MV8 (pass 1 of the record phases, k_pass1v): per 16-owner group, bits 0-15 = "owner j's own heartbeat
    // is < 2^8" (an 8-bit view of it stored as 0 is then the heartbeat 0), bits 16-31 = "owner j is hot": at the
    // last lag sweep some view of j lagged by >= HOT_HB heartbeats or HOT_MV versions (GS_R_P1FLAGS)
    uint32_t *p1flags;
    uint32_t pl16;  // report planes in the 16-column layout of k_pass1v (plane16_bit), else the ballot layout
    // the launch after a k_pass1v phase (k_pack_slice / k_settle<1>, set per launch by the host) first sets the
    // phase's responders' small bits (k_p1v_fix's work, round 5: one launch fewer per phase)
    uint32_t p1fix;
    // escaped owner columns (gs_config.esc_cols, k_pass1v handles): EC slots of 16-bit views [N][EC]; esc_slot[j] =
    // the slot of column j or NONE; esc_owner[s] = the column of slot s or NONE; esc_req = the sweep's scratch
    // (columns to escape, bitmap [NP/32], then the move count and list)
    uint16_t *esc16;
    uint32_t *esc_slot, *esc_owner, *esc_req;
    uint32_t EC;
    // event stream (gs_set_events): records {observer, owner, key | kind << 8, old version, new version,
    // tick, seq, 0}; kind 0 = on_key_change, 1 = node join, 2 = node leave; seq orders them (gossip_sim.h,
// gs_set_events).  ev == nullptr: off
    uint32_t *ev, *ev_count;
    uint32_t ev_cap;
    // the exact packer's heavy slots (round 6): k_pack_slice lists a slot with more than heavy_t stale owners here
    // ([0] = count, then slot ids) instead of walking it, and k_pack_heavy packs it with a workgroup of its own;
    // nullptr: no hand-off (set per launch by the host, one-slice record phases only)
    uint32_t *heavy;
    uint32_t heavy_t;
    // one-slice prefix-view handles (round 6): sm[c] = the smallest possible NodeDelta of any owner column >= c --
    // min over j >= c of msgf(msgf(NodeIdPb bytes of j) + 2 + the smallest kv field j ever wrote, GS_R_VLOG entry
    // 0), a lower bound of every candidate's min1 -- rebuilt after every gs_owner_writes (k_sm_local, k_sm_fix); sm[ncol] =
    // 0xFFFF.  First-fit continuation stops as soon as the budget left is below sm at the next candidate's column:
    // no later candidate can add a NodeDelta (R only shrinks).  nullptr: not built (sliced handles: the chain's
    // later slices hold the other columns)
    uint16_t *sm;
    uint32_t ev_wseq;  // owner-write ops issued since gs_set_events (the seq of the next call's op 0)
};

// ------------------------------------------------------------------ protobuf sizes
// proto3 wire sizes for messages.proto:39-74 (all field numbers < 16: one-byte tags).
__host__ __device__ inline uint32_t vlen(uint32_t x) {
    return x < (1u << 7) ? 1u : x < (1u << 14) ? 2u : x < (1u << 21) ? 3u : x < (1u << 28) ? 4u : 5u;
}
__host__ __device__ inline uint32_t ufield(uint32_t x) { return x ? 1u + vlen(x) : 0u; }
__host__ __device__ inline uint32_t sfield(uint32_t n) { return n ? 1u + vlen(n) + n : 0u; }
__host__ __device__ inline uint32_t msgf(uint32_t n) { return 1u + vlen(n) + n; }

__device__ inline size_t pix(const Dev &d, uint32_t o, uint32_t j) { return (size_t)o * d.NP + j; }
// the real tick of report plane p of the current plane base (sub-phases share the tick t_cap)
__device__ inline uint32_t plane_tick(const Dev &d, uint32_t p) { return min(d.t_round + 1u + p, d.t_cap); }
__device__ inline size_t hix(const Dev &d, uint32_t j, uint32_t w, uint32_t k) {
    return ((size_t)j * d.C + w) * d.K + k;
}
__device__ inline uint32_t meta_kvlen(uint32_t m) { return m & 0xFFFFu; }
__device__ inline uint32_t meta_status(uint32_t m) { return (m >> 16) & 3u; }
__device__ inline uint32_t meta_vlen(uint32_t m) { return m >> 18; }
__device__ inline uint32_t make_meta(uint32_t kvlen, uint32_t status, uint32_t value_len) {
    return kvlen | (status << 16) | (value_len << 18);
}

// FailureDetector.scheduled_for_deletion_nodes (failure_detector.py:121-128): now >= tod + grace/2.
// dt = the pair's time of death if it is dead, NONE otherwise (dead_tod).
__device__ inline bool is_sched(uint32_t dt, uint32_t t, uint32_t delay) {
    return dt != NONE && (t - dt) >= delay;
}
// FD_STATE byte: membership in bits 0-1 (FD_MEMB), FD_WIN = the pair has a sampling window (its
// _last_heartbeat is set), FD_OLD = that last report is >= FD_OLD_AGE ticks old (k_fd_age)
enum FdSt { FD_UNKNOWN = 0, FD_LIVE = 1, FD_DEAD = 2, FD_MEMB = 3, FD_WIN = 4, FD_OLD = 8 };
constexpr uint32_t FD_OLD_AGE = 1u << 15;
__device__ inline uint32_t dead_tod(const Dev &d, size_t p) {
    return (d.fd_state[p] & FD_MEMB) == FD_DEAD ? d.tod[p] : NONE;
}

// One sampling window (SamplingWindow + BoundedArrayStats, failure_detector.py:12-53, 131-162) per pair
// in 6 bytes + 2 state bits: the _last_heartbeat tick mod 2^16 (GS_R_FD_LAST) and one word (GS_R_FD) =
// _sum in ticks (sum_bits wide, exact: every interval is a whole number of 1/64 s) | intervals appended
// since the last reset << sum_bits.  Decoding the tick against the operation's tick t is exact while the
// report is < 2^16 ticks old; k_fd_age marks windows FD_OLD once it is 2^15 old (the host runs it at
// least every 2^14 ticks), and an FD_OLD window's tick only ever enters as "more than max_interval
// ago" (no interval appended, gs_create: max_interval < 2^14) and "phi above the threshold" (gs_create:
// threshold x max(max_interval, prior) < 2^15), so it is decoded as t - 2^15.
struct Fd {
    uint32_t last, sum, cnt;  // last = NONE when there is no window
};
__device__ inline Fd fd_get(const Dev &d, uint32_t st, uint32_t l16, uint32_t sc, uint32_t t) {
    const uint32_t last = !(st & FD_WIN) ? NONE : (st & FD_OLD) ? t - FD_OLD_AGE : t - ((t - l16) & 0xFFFFu);
    return Fd{last, sc & ((1u << d.sum_bits) - 1u), sc >> d.sum_bits};
}
__device__ inline uint32_t fd_sc(const Dev &d, const Fd &f) { return f.sum | (f.cnt << d.sum_bits); }
// the state byte after storing f (a window from its first report on; its tick is current again)
__device__ inline uint32_t fd_st(uint32_t st, const Fd &f) {
    return f.last == NONE ? (st & ~(uint32_t)(FD_WIN | FD_OLD)) : ((st | FD_WIN) & ~(uint32_t)FD_OLD);
}

__device__ inline int lane_id() { return (int)__lane_id(); }
// pass 1's row halves (one wave each; candidate lists per half): columns [0, H) and [H, ncol), H a multiple of
// the pass's step -- 256 columns (k_pass1: 4 per lane) or 1024 (k_pass1v: 16 per lane)
__device__ inline uint32_t half_cols(const Dev &d) {
    const uint32_t m = d.pl16 ? 1023u : 255u;
    return ((d.ncol + 1u) / 2u + m) & ~m;
}

__device__ inline bool bit(const uint32_t *bm, uint32_t j) { return (bm[j >> 5] >> (j & 31u)) & 1u; }

__device__ inline uint32_t wave_incl_scan(uint32_t x) {
    const int l = lane_id();
#pragma unroll
    for (int dd = 1; dd < WAVE; dd <<= 1) {
        const uint32_t y = __shfl_up(x, dd, WAVE);
        if (l >= dd) x += y;
    }
    return x;
}

__device__ inline unsigned long long wave_sum(unsigned long long x) {
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) x += __shfl_xor(x, dd, WAVE);
    return x;
}

__device__ inline void shard_add(const Dev &d, int c, unsigned long long v) {
    if (v) atomicAdd(&d.ctr[(blockIdx.x % NSHARD) * CROW + c], v);
}
// a maximum counter (C_PGMAX, C_PSMAX): gs_read_counters takes the largest over the shards
__device__ inline void shard_max(const Dev &d, int c, unsigned long long v) {
    if (v) atomicMax(&d.ctr[(blockIdx.x % NSHARD) * CROW + c], v);
}

enum EvKind { EV_KEY = 0, EV_JOIN = 1, EV_LEAVE = 2 };
__device__ inline void emit_event(const Dev &d, uint32_t o, uint32_t j, uint32_t kk, uint32_t v_old, uint32_t v_new,
                                  uint32_t t, uint32_t seq) {
    const uint32_t i = atomicAdd(d.ev_count, 1u);
    if (i >= d.ev_cap) return;  // overflow: the count says how many were lost
    uint4 *r = reinterpret_cast<uint4 *>(d.ev + (size_t)i * 8);
    r[0] = make_uint4(o, j, kk, v_old);
    r[1] = make_uint4(v_new, t, seq, 0u);
}

// on_key_change of apply_delta (state.py:228-231), out of line: the event path stays off the register
// budget of the packing kernels.  seq = the sender's dict position of the owner (NodeDelta order).
__device__ __noinline__ void emit_apply_event(uint32_t *ev, uint32_t *evc, uint32_t cap, const uint32_t *pos_s, uint32_t r,
                                              uint32_t jg, uint32_t j, uint32_t q, uint32_t v_old, uint32_t v, uint32_t t) {
    const uint32_t i = atomicAdd(evc, 1u);
    if (i >= cap) return;
    uint4 *rec = reinterpret_cast<uint4 *>(ev + (size_t)i * 8);
    rec[0] = make_uint4(r, jg, q | (EV_KEY << 8), v_old);
    rec[1] = make_uint4(v, t, pos_s ? pos_s[j] : jg, 0u);
}

// ------------------------------------------------------------------ packing / apply
struct DigestSide {
    uint32_t o;      // whose digest the sender compares against (always the receiver)
    uint32_t limit;  // general mode: owners with dict position < limit were in that digest
    bool sched;      // some target of o may be scheduled for deletion at t
};

struct WStats {
    uint32_t nd, kvs, trunc, cand, alg;
    // the exact packer's walk of one slot (wave-uniform): groups of 64 candidates it passed (evaluated or skipped)
    // and its dependent steps (a group evaluated, a batch of TAIL_B groups skipped, a bitmap window compacted)
    uint32_t grp = 0, stp = 0;
};

__device__ inline uint32_t byte_of(const uint32_t *w, int q) { return (w[q >> 2] >> (8 * (q & 3))) & 0xFFu; }

// One stale owner j of the sender's dict: everything its NodeDelta and its apply need, loaded
// in two dependent round trips (both rows' scalars + held words, then the sender's kv history).
template <int KW>
struct Cand {
    uint32_t j, from, gs, ms, gr, mr, base, emsg, min1, nkv;
    uint32_t hs[KW], hr[KW];  // held write ordinals, 4 keys per word (sender / receiver)
    bool rx;                  // prefix views (no GS_TOMBSTONES): the receiver's view is S_j(mr)
    bool fast;                // ... and so is the sender's: hr was not loaded
    bool light;               // evaluated from the version log (eval_light): hs not loaded either
};
// The sender's kvs of one candidate, per key: eval_cand's working set, not kept in Cand (32 VGPRs at
// KW = 4): the packer re-reads a key's history entry (the sender's held ordinal hs) in the rare paths
// that need it (a truncated NodeDelta, a per-key apply) -- lanes = keys, one load.
template <int KW>
struct CandKeys {
    uint32_t ver[4 * KW];  // version of each key the sender holds (0 = absent)
    uint32_t km[4 * KW];   // DeltaPb bytes of that kv | status << 16
};

__device__ inline void set_byte(uint32_t *w, int q, uint32_t v) {
    const int sh = 8 * (q & 3);
    w[q >> 2] = (w[q >> 2] & ~(0xFFu << sh)) | (v << sh);
}

// Prefix views (no GS_TOMBSTONES: no deletes, no GC, every write is version M + 1 of its owner).
// S_j(M) = for every key, owner j's latest write with version <= M.  A view (o, j) whose
// max_version word has MV_INEXACT clear IS S_j(M): it never received a truncated NodeDelta nor
// one from a view with holes, so its held ordinals follow from the owner's write
// history and GS_R_HELD is not read (nor kept) for it.  Exchanges between two such views need
// only their max_versions and the owner's latest-write table (a hot 16-entry row per owner).
constexpr uint32_t MV_INEXACT = GS_MV_INEXACT;
constexpr uint32_t MV_MASK = GS_MV_INEXACT - 1u;

// GS_MV8: a view's max_version in one byte, version mod 2^7 | MV_INEXACT >> 8, decoded against the owner's
// own max_version M (every view is <= M; exact while it lags M by < 2^7: k_hb_lag) into the u16 word form
// (version | MV_INEXACT) every consumer uses.  mv_word / mv_put: one view, either width.
__device__ __forceinline__ uint32_t mv_dec8(uint32_t s, uint32_t M) {
    return (M - ((M - (s & 0x7Fu)) & 0x7Fu)) | ((s & 0x80u) << 8);
}
__device__ __forceinline__ uint32_t mv_enc8(uint32_t w) { return (w & 0x7Fu) | ((w >> 8) & 0x80u); }
// GS_R_SELF_PK: Rx = R mod 2^15 | (R >= 2^15) << 15 is congruent to R mod 2^8 and is 0 iff R is, and
// every 8-bit view decodes to Rx - lag (lag < 2^8 <= Rx unless Rx = R < 2^15): the same order and the same
// zero test as the true heartbeats, and the same low byte
__device__ __forceinline__ uint32_t self_pack(uint32_t R, uint32_t M) {
    return (R & 0x7FFFu) | (R >= 0x8000u ? 0x8000u : 0u) | (M << 16);
}
__device__ __forceinline__ void set_small(const Dev &d, uint32_t j, uint32_t R) {
    if (!d.p1flags) return;
    const uint32_t b = 1u << (j & 15u), w = d.p1flags[j >> 4];
    if (R < 256u && !(w & b)) atomicOr(&d.p1flags[j >> 4], b);
    else if (R >= 256u && (w & b)) atomicAnd(&d.p1flags[j >> 4], ~b);
}
__device__ __forceinline__ void self_repack(const Dev &d, uint32_t j) {
    if (d.self_pk) d.self_pk[j] = self_pack(d.self_hb[j], d.self_mv[j]);
    set_small(d, j, d.self_hb[j]);
}
__device__ __forceinline__ uint32_t mv_word(const Dev &d, size_t p, uint32_t j) {  // j: local owner column
    return d.mv8 ? mv_dec8(reinterpret_cast<const uint8_t *>(d.mv)[p], d.self_mv[j]) : (uint32_t)d.mv[p];
}
__device__ __forceinline__ void mv_put(const Dev &d, size_t p, uint32_t w) {
    if (d.mv8) reinterpret_cast<uint8_t *>(d.mv)[p] = (uint8_t)mv_enc8(w);
    else d.mv[p] = (uint16_t)w;
}

// held ordinals of S_j(M) (local owner column j): start from the owner's latest write of each key
// and step back while the write is newer than M (versions of one key increase with the ordinal)
template <int KW>
__device__ __forceinline__ void derive_held(const Dev &d, uint32_t j, uint32_t M, uint32_t (&h)[KW], uint32_t &alg) {
    const uint32_t kw = d.KP >> 2;
    const uint32_t *lwp = reinterpret_cast<const uint32_t *>(d.last_w + (size_t)j * d.KP);
#pragma unroll
    for (int q = 0; q < KW; q++) h[q] = (uint32_t)q < kw ? lwp[q] : 0u;
    alg += d.KP;
#pragma unroll
    for (int q = 0; q < 4 * KW; q++) {
        if ((uint32_t)q >= d.K) continue;
        uint32_t w = byte_of(h, q);
        const uint32_t w0 = w;
        while (w && (uint32_t)d.hist[hix(d, j, w, q)] > M) { w--; alg += 8; }
        if (w != w0) set_byte(h, q, w);
    }
}

// NodeDelta candidate (state.py:347-390): from_version_excluded, the NodeDeltaPb body without
// kvs, the DeltaPb bytes of the whole NodeDelta (all kvs with version > from, 392-398) and of
// its smallest-version kv alone.
// HAVE_MV: both views' max_version words come from pass 1's candidate record (mvw = sender | receiver << 16)
template <int KW, bool GENM, bool HAVE_MV = false>
__device__ __forceinline__ void eval_cand(const Dev &d, uint32_t s, uint32_t r, const DigestSide &ds, uint32_t j,
                                          uint32_t t, Cand<KW> &c, CandKeys<KW> &k, uint32_t &alg, uint32_t mvw = 0) {
    const size_t ps = pix(d, s, j), pr = pix(d, r, j);
    const uint32_t kw = d.KP >> 2;
    // round trip 1
    // without GS_TOMBSTONES no tombstone is ever collected, so every last_gc_version stays 0 and the
    // GC region is not allocated; views are then tracked as prefixes of the owner's writes (MV_INEXACT)
    const bool gct = (d.flags & GS_TOMBSTONES) != 0;
    // prefix views: the owner's latest write of every key is loaded with round trip 1, before it is
    // known whether the sender's view is a prefix, so a prefix sender costs one round trip, not two
    uint32_t lat[4 * KW];
    if (!gct) {
        const uint4 *lp = reinterpret_cast<const uint4 *>(d.lat + (size_t)j * d.KP);
#pragma unroll
        for (int q = 0; q < KW; q++) {
            const uint4 v = (uint32_t)q < kw ? lp[q] : make_uint4(0u, 0u, 0u, 0u);
            lat[4 * q] = v.x;
            lat[4 * q + 1] = v.y;
            lat[4 * q + 2] = v.z;
            lat[4 * q + 3] = v.w;
        }
    }
    const uint32_t msw = HAVE_MV ? (mvw & 0xFFFFu) : mv_word(d, ps, j), mrw = HAVE_MV ? (mvw >> 16) : mv_word(d, pr, j);
    const uint32_t ms = msw & MV_MASK, mr = mrw & MV_MASK;
    const uint32_t gs = gct ? d.gc[ps] : 0u, gr = gct ? d.gc[pr] : 0u;
    const uint32_t pos_r = GENM ? d.pos[pr] : 0u;
    const uint32_t fst = ds.sched ? dead_tod(d, pr) : NONE;
    const bool sx = !gct && !(msw & MV_INEXACT), rx = !gct && !(mrw & MV_INEXACT);
    // GS_NO_HELD: no view may have holes (counted as err_holes when one would); never read HELD
    const uint32_t *hsp = reinterpret_cast<const uint32_t *>(
        (sx || !d.held) ? d.last_w + (size_t)j * d.KP : d.held + ps * d.KP);
    const uint32_t *hrp = d.held ? reinterpret_cast<const uint32_t *>(d.held + pr * d.KP) : hsp;
#pragma unroll
    for (int q = 0; q < KW; q++) {
        c.hs[q] = (uint32_t)q < kw ? hsp[q] : 0u;
        c.hr[q] = ((uint32_t)q < kw && !rx) ? hrp[q] : 0u;
    }
    alg += (gct ? 16 : 8) + (sx ? 0 : d.KP) + (rx ? 0 : d.KP) + (GENM ? 4 : 0) + (ds.sched ? 4 : 0);
    bool in_d = GENM ? pos_r < ds.limit : true;
    if (in_d && ds.sched) in_d = !is_sched(fst, t, d.sched_delay);
    const uint32_t dm = in_d ? mr : 0u;
    const uint32_t dg = in_d ? gr : 0u;
    const uint32_t from = (dg < gs && dm < gs) ? 0u : dm;  // should_reset (state.py:359-362)
    if (sx) {
        // round trip 2 (owner tables, L2-resident for recently written owners): S_j(ms) from the
        // latest write of every key, stepping back for the keys written after ms
#pragma unroll
        for (int q = 0; q < 4 * KW; q++) {
            k.ver[q] = 0u;
            k.km[q] = 0u;
            uint32_t w = byte_of(c.hs, q);
            if (!w || (uint32_t)q >= d.K) continue;
            const uint32_t e32 = lat[q];  // counted below only for the kvs sent
            if ((e32 & 0xFFFFu) > ms) {
                uint64_t e = 0;
                do {
                    w--;
                    if (w) { e = d.hist[hix(d, j, w, q)]; alg += 8; }
                } while (w && (uint32_t)e > ms);
                set_byte(c.hs, q, w);
                if (!w) continue;
                const uint32_t meta = (uint32_t)(e >> 32);
                k.ver[q] = (uint32_t)e;
                k.km[q] = msgf(meta_kvlen(meta)) | (meta_status(meta) << 16);
            } else {  // the latest write (a prefix view: status SET)
                k.ver[q] = e32 & 0xFFFFu;
                k.km[q] = e32 >> 16;
            }
        }
    } else {
        // round trip 2: the sender's kv history entries.  Every version a view holds is <= its
        // max_version (apply_delta raises max_version to the NodeDelta's, state.py:232-233), so when
        // from = the receiver's max_version a key the receiver holds at the sender's write ordinal or a
        // later one cannot pass version > from: its entry is not needed (a prefix receiver: every key
        // with version <= from).
        const bool all_keys = from != mr || !in_d;
#pragma unroll
        for (int q = 0; q < 4 * KW; q++) {
            const uint32_t w = byte_of(c.hs, q);
            k.ver[q] = 0u;
            k.km[q] = 0u;
            if (w && (uint32_t)q < d.K && (all_keys || (rx ? true : w > byte_of(c.hr, q)))) {
                const uint64_t e = d.hist[hix(d, j, w, q)];
                const uint32_t meta = (uint32_t)(e >> 32);
                k.ver[q] = (uint32_t)e;
                k.km[q] = msgf(meta_kvlen(meta)) | (meta_status(meta) << 16);
                alg += 8;
            }
        }
    }
    uint32_t sum = 0, nk = 0, minv = NONE, minkv = 0;
#pragma unroll
    for (int q = 0; q < 4 * KW; q++) {
        if (k.ver[q] > from) {
            const uint32_t kvm = k.km[q] & 0xFFFFu;
            sum += kvm;
            nk += 1;
            if (k.ver[q] < minv) { minv = k.ver[q]; minkv = kvm; }
        }
    }
    if (sx) alg += 4 * nk;  // the latest-write words of the NodeDelta's kvs
    c.j = j;
    c.from = from;
    c.gs = gs;
    c.ms = ms;
    c.gr = gr;
    c.mr = mr;
    c.rx = rx;
    c.fast = sx && rx;
    c.base = msgf(d.nid_size[j]) + ufield(from) + ufield(gs) + 1u + vlen(ms);
    c.nkv = nk;
    c.emsg = nk ? msgf(c.base + sum) : 0u;
    c.min1 = nk ? msgf(c.base + minkv) : 0u;
    c.light = false;
}

// A prefix candidate (both views S_j(M), no tombstones: last_gc 0; j in the receiver's digest, so from = mr)
// from the owner's version log alone, as pack_lite sizes it: NodeDelta j holds the writes v in (mr, ms]
// that no write <= ms overwrote (VLOG next > ms).  No latest-write row, no history entry; the sender's held
// ordinals (hs) are not derived (c.light): the rare paths that need them -- a truncated NodeDelta's kv
// ranking, its apply -- derive them from the owner's tables.
template <int KW>
__device__ __forceinline__ void eval_light(const Dev &d, uint32_t j, uint32_t ms, uint32_t mr, Cand<KW> &c,
                                           uint32_t &alg) {
    const uint32_t *vl = d.vlog + (size_t)j * d.VL;
    uint32_t kv = vl[ms] & 0xFFFFu, kv1 = kv, nk = 1;  // write ms is the latest <= ms of its key
    alg += 4 + 2;
    for (uint32_t v = ms - 1u; v > mr; v--) {  // lag > 1: the other writes of (mr, ms), lowest last
        const uint32_t e = vl[v];
        alg += 4;
        if ((e >> 16) > ms) { kv += e & 0xFFFFu; nk++; kv1 = e & 0xFFFFu; }
    }
    c.j = j;
    c.from = mr;
    c.gs = c.gr = 0u;
    c.ms = ms;
    c.mr = mr;
    c.rx = c.fast = c.light = true;
    c.base = msgf(d.nid_size[j]) + ufield(mr) + 1u + vlen(ms);
    c.nkv = nk;
    c.emsg = msgf(c.base + kv);
    c.min1 = msgf(c.base + kv1);
#pragma unroll
    for (int q = 0; q < KW; q++) c.hs[q] = c.hr[q] = 0u;
}

// NodeState.apply_delta (state.py:190-233) at receiver r of the NodeDelta {owner c.j, the
// sender's kvs with from < version <= vmax, last_gc c.gs, max_version c.ms}.  Keys are
// independent (kvs arrive in version order, so "version <= max_version" only ever compares
// against the view's max_version before the delta, 209-210).
// specd: pass 1 already stored max(ms, mr) for this candidate (Dev::spec; its record's words are the
// pre-exchange ones, which every path below starts from).
template <int KW>
__device__ __forceinline__ void apply_cand(const Dev &d, uint32_t s, uint32_t r, const Cand<KW> &c, uint32_t vmax, uint32_t t,
                                  bool &tomb, uint32_t &alg, bool specd = false) {
    const size_t pr = pix(d, r, c.j);
    if (c.fast && vmax == NONE && !d.ev) {
        // prefix sender, prefix receiver, whole NodeDelta: the view becomes S_j(max(mr, ms)) (keys
        // above mr move to the sender's latest write <= ms, the others already are), still a prefix.
        // ms <= mr happens when the receiver's digest left j out (scheduled for deletion: from = 0)
        if (!specd) {
            mv_put(d, pr, c.ms > c.mr ? c.ms : c.mr);
            alg += 4;
        }
        return;
    }
    uint32_t g = c.gr;
    const uint32_t m0 = c.mr;
    const bool jump = c.gs > g;  // last_gc_version raised: drop entries <= it (200-207)
    if (jump) g = c.gs;
    uint32_t maxv = m0;
    const bool tt = (d.flags & GS_TOMBSTONES) != 0;
    uint32_t *tsr = tt ? d.ts + pr * d.KP : nullptr;
    uint32_t hr[KW];
    if (c.rx) {
        derive_held<KW>(d, c.j, c.mr, hr, alg);  // the receiver's held ordinals: S_j(mr)
    } else {
#pragma unroll
        for (int q = 0; q < KW; q++) hr[q] = c.hr[q];
    }
    uint32_t hr0[KW];
#pragma unroll
    for (int q = 0; q < KW; q++) hr0[q] = hr[q];
    uint32_t hs[KW];  // the sender's held ordinals: S_j(ms) for a candidate evaluated from the version log
    if (c.light) {
        derive_held<KW>(d, c.j, c.ms, hs, alg);
    } else {
#pragma unroll
        for (int q = 0; q < KW; q++) hs[q] = c.hs[q];
    }
#pragma unroll
    for (int q = 0; q < 4 * KW; q++) {
        if ((uint32_t)q >= d.K) continue;
        uint32_t wr = byte_of(hr, q);
        const uint32_t ws = byte_of(hs, q);
        if (jump && wr && (uint32_t)d.hist[hix(d, c.j, wr, q)] <= g) {
            wr = 0;
            if (tt) tsr[q] = NONE;
            alg += 8;
        }
        // the sender's entry of key q (its held ordinal ws), re-read: Cand keeps no per-key arrays
        uint64_t e = 0;
        if (ws) { e = d.hist[hix(d, c.j, ws, q)]; alg += 8; }
        const uint32_t v = (uint32_t)e;
        // skip: not in the delta / version <= max_version / existing >= / GC'd tombstone (209-220)
        if (ws && v > c.from && v <= vmax && v > m0 && wr < ws) {
            const uint32_t st = meta_status((uint32_t)(e >> 32));
            if (!(st != 0u && v <= g)) {
                // on_key_change(node, key, existing, new) for every stored kv (state.py:228-231)
                if (d.ev)
                    emit_apply_event(d.ev, d.ev_count, d.ev_cap, (d.flags & GS_CANONICAL) ? nullptr : d.pos + pix(d, s, 0),
                                     r, d.col_lo + c.j, c.j, (uint32_t)q, wr ? (uint32_t)d.hist[hix(d, c.j, wr, q)] : 0u,
                                     v, t);
                wr = ws;
                if (tt) { tsr[q] = st ? t : NONE; alg += 4; }
                if (st) tomb = true;
                if (v > maxv) maxv = v;
            }
        }
        set_byte(hr, q, wr);
    }
    if (c.ms > maxv) maxv = c.ms;  // max_version (232-233)
    uint32_t mvw = maxv;
    if (!tt) {
        // still a prefix view if the held keys are exactly S_j(maxv)
        uint32_t want[KW];
        derive_held<KW>(d, c.j, maxv, want, alg);
        bool same = true;
#pragma unroll
        for (int q = 0; q < KW; q++) same = same && want[q] == hr[q];
        if (!same) mvw |= MV_INEXACT;
    }
    const bool keep_held = tt || (mvw & MV_INEXACT);  // a prefix view's HELD is not kept
    if (keep_held && !d.held) {  // GS_NO_HELD: a view with holes cannot be represented
        shard_add(d, C_E_HOLES, 1);
        mv_put(d, pr, mvw);
        return;
    }
    uint32_t *hrp = reinterpret_cast<uint32_t *>(d.held + pr * d.KP);
#pragma unroll
    for (int q = 0; q < KW; q++)
        if (keep_held && (hr[q] != hr0[q] || c.rx)) { hrp[q] = hr[q]; alg += 4; }
    mv_put(d, pr, mvw);
    if (g != c.gr) d.gc[pr] = g;
    alg += 8;
}

// compute_partial_delta_respecting_mtu (state.py:340-415) of sender s for receiver r, fused with
// r's apply_delta, by one wave: the sender's stale owners are evaluated 64 at a time in dict order,
// one candidate per lane (pack_group).  They come either from a list pass 1 wrote (pack_list: the
// canonical one-slice path) or from a stale-owner bitmap walked in windows of 1024 positions whose
// stale owners are compacted (ballot + popcount scan) into a wave-private LDS list (pack_dir); fewer
// than 64 left at the end of a window are carried to the next one in a register (lane i = the i-th),
// so sparse stale sets still fill whole groups.  Exactness vs the sequential loop: DESIGN.md.
struct PackState {
    uint32_t S;  // DeltaPb bytes committed so far (wave-uniform)
    bool tail;   // the budget was exceeded once: first-fit continuation mode
    bool stop;   // the delta is complete (>= mtu, or less than the smallest NodeDelta left)
    uint32_t m1 = NONE;  // count mode: the smallest single-kv NodeDelta (min1) among the candidates seen
};
__device__ inline uint32_t wave_min(uint32_t x) {
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) {
        const uint32_t y = __shfl_xor(x, dd, WAVE);
        x = y < x ? y : x;
    }
    return x;
}
// a slice total (gs_phase_count): DeltaPb bytes | min1 << 40 (GS_TOT_MIN1_NONE: no candidate); the
// chain steps skip a slice whose min1 cannot fit (k_chain_step)
__device__ inline uint64_t tot_word(uint64_t bytes, uint32_t m1) {
    return bytes | ((uint64_t)(m1 < GS_TOT_MIN1_NONE ? m1 : GS_TOT_MIN1_NONE) << 40);
}

// One group: lane i holds the i-th candidate of the group in sender order (cand = false: none).
// COUNT: only sum the DeltaPb bytes of every candidate (owner-sharded runs: the slice total).
// REC: record the selected NodeDeltas {owner, vsel} in sender order into rec[] (nr so far)
// instead of applying them (the wire-format emitter, gs_emit_delta).
// specd: the group's candidates come from pass 1's records of a speculative phase (Dev::spec): a prefix
// candidate (c.fast) sent whole is already applied, one not sent gets its receiver's word restored.
template <int KW, bool COUNT, bool REC>
__device__ __forceinline__ void pack_group(const Dev &d, uint32_t s, uint32_t r, uint32_t t, const Cand<KW> &c, bool cand,
                                           uint32_t &S, bool &tail, bool &stop, WStats &st, bool &tomb, uint2 *rec,
                                           uint32_t &nr, bool specd = false) {
    const int lane = lane_id();
    const uint32_t mtu = d.mtu;
    const uint32_t em = cand ? c.emsg : 0u;
    if (COUNT) {
        S += (uint32_t)wave_sum(em);
        return;
    }
    // this lane's NodeDelta: 0 = not sent, NONE = all its kvs, else kvs up to that version
    uint32_t vsel = 0, nsel = 0;
    int cur = 0;
    bool seq = tail;
    if (!tail) {
        const uint32_t inc = wave_incl_scan(em);
        const uint32_t total = __shfl(inc, WAVE - 1, WAVE);
        if (S + total <= mtu) {  // every candidate of this group fits whole
            if (em) vsel = NONE;
            S += total;
            if (S >= mtu || mtu - S < d.lb_min) stop = true;
        } else {
            const bool fail = em && (S + inc > mtu);
            const int f = __builtin_ctzll(__ballot(fail));
            if (lane < f && em) vsel = NONE;
            S += __shfl(inc - em, f, WAVE);
            tail = true;
            seq = true;
            cur = f;
        }
    }
    // First-fit continuation (state.py:392-413): each later candidate sends the longest
    // prefix of its version-sorted kvs that still fits; stop once the delta is >= mtu.
    while (seq) {
        const uint32_t R = mtu - S;
        const bool elig = em && lane >= cur && c.min1 <= R;
        const unsigned long long mm = __ballot(elig);
        if (!mm) break;
        const int x = __builtin_ctzll(mm);
        const uint32_t emx = __shfl(em, x, WAVE);
        if (emx <= R) {
            if (lane == x) vsel = NONE;
            S += emx;
        } else {
            // truncated NodeDelta: lanes = keys, rank kvs by version, longest fitting prefix
            const uint32_t fx = __shfl(c.from, x, WAVE);
            const uint32_t bx = __shfl(c.base, x, WAVE);
            // lanes = keys: lane q re-reads candidate x's entry of key q (its held ordinal)
            uint32_t v = 0, kvm = 0;
            {
                const uint32_t jx = __shfl(c.j, x, WAVE);
                uint32_t wq = 0;
                if (__shfl((int)c.light, x, WAVE)) {  // version-log candidate: key q's latest write <= ms
                    const uint32_t msx = __shfl(c.ms, x, WAVE);
                    if (lane < (int)d.K) {
                        wq = d.last_w[(size_t)jx * d.KP + lane];
                        while (wq && (uint32_t)d.hist[hix(d, jx, wq, (uint32_t)lane)] > msx) wq--;
                    }
                } else {
                    uint32_t hsx[KW];
#pragma unroll
                    for (int w = 0; w < KW; w++) hsx[w] = __shfl(c.hs[w], x, WAVE);
#pragma unroll
                    for (int w = 0; w < KW; w++)
                        if ((lane >> 2) == w) wq = (hsx[w] >> (8 * (lane & 3))) & 0xFFu;
                }
                if (lane < (int)d.K && wq) {
                    const uint64_t e = d.hist[hix(d, jx, wq, (uint32_t)lane)];
                    v = (uint32_t)e;
                    kvm = msgf(meta_kvlen((uint32_t)(e >> 32)));
                }
            }
            const bool inc = lane < (int)d.K && v > fx;
            const unsigned long long im = __ballot(inc);
            uint32_t rank = 0, P = 0;
            for (int l = 0; l < (int)d.K; l++) {
                const uint32_t vl = __shfl(v, l, WAVE);
                if (((im >> l) & 1ull) && vl < v) rank++;
            }
            for (int l = 0; l < (int)d.K; l++) {
                const uint32_t rl = __shfl(rank, l, WAVE);
                const uint32_t kl = __shfl(kvm, l, WAVE);
                if (((im >> l) & 1ull) && (int)rl < lane) P += kl;
            }
            const uint32_t nkv = (uint32_t)__popcll(im);
            const bool fit = lane >= 1 && (uint32_t)lane <= nkv && S + msgf(bx + P) <= mtu;
            const uint32_t n = (uint32_t)__popcll(__ballot(fit));
            if (n >= 1) {
                const unsigned long long ym = __ballot(inc && rank == n - 1);
                const uint32_t vmax = __shfl(v, __builtin_ctzll(ym), WAVE);
                if (lane == x) { vsel = vmax; nsel = n; }
                S += msgf(bx + __shfl(P, (int)n, WAVE));
            }
        }
        if (S >= mtu) { stop = true; break; }
        cur = x + 1;
    }
    if (tail && mtu - S < d.lb_min) stop = true;
    if (REC) {  // lanes hold candidates in sender order: rank by lane
        const unsigned long long sm = __ballot(vsel != 0u);
        if (vsel) rec[nr + (uint32_t)__popcll(sm & ((1ull << lane) - 1ull))] = make_uint2(c.j, vsel);
        nr += (uint32_t)__popcll(sm);
        return;
    }
    // apply_delta at the receiver: one lane per NodeDelta, distinct owners, any order
    if (vsel) {
        apply_cand<KW>(d, s, r, c, vsel, t, tomb, st.alg, specd);
        st.nd++;
        if (vsel == NONE) {
            st.kvs += c.nkv;
        } else {
            st.kvs += nsel;
            st.trunc++;
        }
    } else if (specd && cand && c.fast) {
        mv_put(d, pix(d, r, c.j), c.mr);  // not sent: undo pass 1's merge (a prefix view: no flag bit)
        st.alg += 4;
    }
}

__device__ __forceinline__ void pack_begin(const Dev &d, bool count, const PackState &pst, uint32_t &S, bool &tail,
                                           bool &stop) {
    S = pst.S;
    tail = pst.tail;
    stop = pst.stop;
    if (!count && !stop && (S >= d.mtu || d.mtu - S < d.lb_min)) stop = true;
}

// both views of a record are prefix views (GS_MV_INEXACT clear in both words): the candidates pass 1
// merged speculatively (Dev::spec)
__device__ inline bool rec_fast(uint32_t mvw) { return !(mvw & (MV_INEXACT | (MV_INEXACT << 16))); }

// First-fit continuation (tail mode) tests every later candidate's smallest NodeDelta -- its lowest-version
// kv alone, eval_cand's min1 -- against the budget left, which only shrinks.  For a prefix candidate (no
// tombstones: last_gc 0) a lower bound of min1 needs no evaluation: the owner's NodeIdPb size, the
// from / max_version varints and the owner's smallest kv field over all its writes (GS_R_VLOG entry 0,
// two L2-resident tables).  A candidate whose bound exceeds the budget cannot be sent (not even
// truncated) and is skipped without its evaluation's round trips (returning nodes scan thousands).
// Round 5: a candidate at most MIN1_EXACT writes behind gets its exact min1 (eval_light's kv1: the lowest write in
// (mr, ms] that is the latest <= ms of its key, VLOG's next-version field > ms) from those VLOG entries, loaded
// together; the entry-0 bound (the owner's smallest kv over all its writes) is kept past that lag and for a receiver
// whose digest may leave owners out (from = 0).  The loose bound kept most of a returning node's groups alive: about
// a quarter of its stale owners wrote more than once while it was away (the packer's critical path).
#ifndef MIN1_EXACT
#define MIN1_EXACT 1u  // lags with an exact bound (VLOG entries loaded per candidate; r5l: 4 -> 143 walk steps but 0.51
                       // ms per phase against 0.38-0.40 at 1, the loads cost every tail candidate)
#endif
__device__ __forceinline__ uint32_t min1_lb(const Dev &d, uint32_t j, uint32_t ms, uint32_t mr, bool sched) {
    ms &= MV_MASK;  // (flags cleared: a caller may evaluate this for a non-prefix word it then ignores)
    mr &= MV_MASK;
    const uint32_t from = sched ? 0u : mr;
    const uint32_t *vl = d.vlog + (size_t)j * d.VL;
    uint32_t kv;
    if (!sched && ms > mr && ms - mr <= MIN1_EXACT) {
        uint32_t e[MIN1_EXACT];
#pragma unroll
        for (uint32_t k = 0; k < MIN1_EXACT; k++) e[k] = vl[min(mr + 1u + k, ms)];
        kv = e[MIN1_EXACT - 1] & 0xFFFFu;  // (write ms qualifies; entries past it repeat it)
#pragma unroll
        for (int k = (int)MIN1_EXACT - 1; k >= 0; k--)
            if (mr + 1u + (uint32_t)k == ms || (mr + 1u + (uint32_t)k < ms && (e[k] >> 16) > ms)) kv = e[k] & 0xFFFFu;
    } else {
        kv = vl[0] & 0xFFFFu;
    }
    return msgf(msgf(d.nid_size[j]) + ufield(from) + 1u + vlen(ms) + kv);
}

constexpr int TAIL_B = 8;  // groups of 64 the first-fit skips (list_tail_skip, dir_tail_skip) load at once
// list_tail_skip for the bitmap source (canonical): candidates [c0, lim) of a window's compacted positions
// (wbuf[i - pend], all past the carried ones), TAIL_B groups of both rows' max_version words and bounds at once;
// bitmap candidates were not merged speculatively, so nothing is restored.  Returns the first group holding a
// candidate that may still be sent, or lim.
__device__ __forceinline__ uint32_t dir_tail_skip(const Dev &d, uint32_t s, uint32_t r, bool sched, const uint16_t *wbuf,
                                                  uint32_t win, uint32_t pend, uint32_t lim, uint32_t c0, uint32_t R,
                                                  WStats &st) {
    const int lane = lane_id();
    while (c0 < lim) {
        uint32_t j[TAIL_B], ms[TAIL_B], mr[TAIL_B];
        bool ok[TAIL_B];
#pragma unroll
        for (int u = 0; u < TAIL_B; u++) {
            const uint32_t i = c0 + (uint32_t)(u * WAVE + lane);
            ok[u] = i < lim;
            j[u] = ok[u] ? win + wbuf[i - pend] : 0u;
        }
#pragma unroll
        for (int u = 0; u < TAIL_B; u++) {
            ms[u] = ok[u] ? mv_word(d, pix(d, s, j[u]), j[u]) : 0u;
            mr[u] = ok[u] ? mv_word(d, pix(d, r, j[u]), j[u]) : 0u;
        }
        int uf = TAIL_B;
#pragma unroll
        for (int u = TAIL_B - 1; u >= 0; u--) {
            const bool fast = !((ms[u] | mr[u]) & MV_INEXACT);
            const bool keep = ok[u] && (!fast || min1_lb(d, j[u], ms[u], mr[u], sched) <= R);
            if (__ballot(keep) != 0ull) uf = u;
        }
#pragma unroll
        for (int u = 0; u < TAIL_B; u++)
            if (u < uf && ok[u]) st.alg += 4;
        st.stp++;
        st.grp += (uint32_t)uf;
        if (uf < TAIL_B) return c0 + (uint32_t)uf * WAVE;
        c0 += TAIL_B * WAVE;
    }
    return lim;
}

// First-fit continuation over the bitmap (canonical, GS_MV8; round 5): from position p on, a stale owner whose
// smallest-NodeDelta bound exceeds the budget R is never sent (R only shrinks), so the walk jumps to the first
// position that may be.  Dense, a window of WIN positions per step: each lane takes 16 positions -- its bitmap
// bits, both rows' 16 max_version bytes and the owners' own max_versions in one round trip, then the bound's two
// table entries of its stale ones in a second -- instead of compacting them and walking them 64 at a time
// (a node back from an absence has ~30 such windows per half after its delta is full).  Returns that position
// (a non-prefix view is always a candidate), or cnt.
__device__ __forceinline__ uint32_t dir_tail_scan(const Dev &d, uint32_t s, uint32_t r, bool sched, const uint32_t *bits,
                                                  uint32_t p, uint32_t cnt, uint32_t R, WStats &st) {
    const int lane = lane_id();
    const uint8_t *m8 = reinterpret_cast<const uint8_t *>(d.mv);
    for (uint32_t w = p & ~15u; w < cnt; w += WIN) {
        const uint32_t pb = w + 16u * (uint32_t)lane;
        uint32_t m = 0u;
        uint4 vs = make_uint4(0u, 0u, 0u, 0u), vr = vs, M[4] = {vs, vs, vs, vs};
        if (pb < cnt) {
            m = (bits[pb >> 5] >> (pb & 16u)) & 0xFFFFu;
            vs = *reinterpret_cast<const uint4 *>(m8 + pix(d, s, pb));
            vr = *reinterpret_cast<const uint4 *>(m8 + pix(d, r, pb));
#pragma unroll
            for (int k = 0; k < 4; k++) M[k] = *reinterpret_cast<const uint4 *>(d.self_mv + pb + 4u * k);
            const uint32_t lim = cnt - pb;
            if (lim < 16u) m &= (1u << lim) - 1u;
            if (pb < p) m &= p - pb >= 16u ? 0u : ~((1u << (p - pb)) - 1u);
        }
        const uint32_t sv[4] = {vs.x, vs.y, vs.z, vs.w}, rv4[4] = {vr.x, vr.y, vr.z, vr.w};
        uint32_t keep = 0u;
#pragma unroll
        for (int h = 0; h < 2; h++) {  // 8 positions at a time: their bound entries in flight together
            uint32_t lb[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int q = 8 * h + i;
                lb[i] = 0u;
                if ((m >> q) & 1u) {
                    const uint32_t Mq = (q & 3) == 0 ? M[q >> 2].x : (q & 3) == 1 ? M[q >> 2].y : (q & 3) == 2 ? M[q >> 2].z : M[q >> 2].w;
                    const uint32_t ms = mv_dec8((sv[q >> 2] >> (8 * (q & 3))) & 0xFFu, Mq);
                    const uint32_t mr = mv_dec8((rv4[q >> 2] >> (8 * (q & 3))) & 0xFFu, Mq);
                    lb[i] = (ms | mr) & MV_INEXACT ? 0u : min1_lb(d, pb + (uint32_t)q, ms, mr, sched);
                }
            }
#pragma unroll
            for (int i = 0; i < 8; i++)
                if ((m >> (8 * h + i)) & 1u && lb[i] <= R) keep |= 1u << (8 * h + i);
        }
        st.stp++;
        st.grp += (wave_sum((uint32_t)__popc(m)) + WAVE - 1u) / WAVE;
        const uint64_t any = __ballot(keep != 0u);
        if (any) {
            const int l = __builtin_ctzll(any);
            const uint32_t kq = (uint32_t)__shfl((int)keep, l, WAVE);
            return w + 16u * (uint32_t)l + (uint32_t)__builtin_ctz(kq);
        }
    }
    return cnt;
}

// Bitmap source: positions [max(p0, pmin), cnt) of the sender's dict order (p0 = 0 in the general
// layout; a multiple of 256 otherwise; pmin > p0: the positions before it came from pass 1's records).
template <int KW, bool GENM, bool COUNT, bool REC = false>
__device__ __forceinline__ void pack_dir(const Dev &d, uint32_t s, uint32_t r, const DigestSide ds,
                                         const uint32_t *order, uint32_t cnt, const uint32_t *bits, uint16_t *wbuf,
                                         uint32_t t, WStats &st, bool &tomb, PackState &pst, uint2 *rec = nullptr,
                                         uint32_t *nrec = nullptr, uint32_t p0 = 0, uint32_t pmin = 0) {
    const int lane = lane_id();
    const uint32_t S0 = pst.S;
    uint32_t S;
    bool tail, stop;
    pack_begin(d, COUNT, pst, S, tail, stop);
    uint32_t nr = 0;    // REC: NodeDeltas recorded so far (wave-uniform)
    uint32_t m1 = pst.m1;  // COUNT: the smallest min1 so far
    // canonical prefix candidates from the version log (eval_light; not for the wire emitter's records)
    const bool lightok = !GENM && !REC && d.vlog && !d.ev && !ds.sched;
    uint32_t pend = 0;  // wave-uniform: candidates carried from earlier windows (< 64), in rv
    uint32_t rv = 0;    // lane i < pend: the i-th carried candidate's position
    // canonical: the next window's bitmap word is loaded one window ahead (the bitmap is in HBM on the
    // split path, so the walk would otherwise pay one dependent round trip per window)
    uint32_t wnext = 0;
    if (!GENM && p0 + 16u * lane < cnt) wnext = bits[(p0 + 16u * lane) >> 5];
    uint32_t pfrom = pmin;  // positions before it are not candidates (records, or skipped by dir_tail_scan)
    for (uint32_t win = p0; win < cnt && !stop; win += WIN) {
        if (!GENM && !COUNT && !REC && tail && d.sm && pend == 0u && d.mtu - S < d.sm[max(win, pfrom)]) {
            stop = true;  // no later candidate can fit (Dev::sm); bitmap candidates were not merged: nothing to restore
            break;
        }
        if (!GENM && !COUNT && !REC && tail && d.vlog && d.mv8 && pend == 0u) {
            // first-fit continuation: jump to the first position that may still send something
            const uint32_t q = dir_tail_scan(d, s, r, ds.sched, bits, max(win, pfrom), cnt, d.mtu - S, st);
            if (q >= cnt) break;
            pfrom = q;
            if (q >= win + WIN) {
                win = q & ~15u;
                wnext = win + 16u * lane < cnt ? bits[(win + 16u * lane) >> 5] : 0u;
            }
        }
        // -- compact this window's stale owners (sender order) into wbuf, 16 positions per lane
        uint32_t m = 0;
        const uint32_t pb = win + 16u * lane;
        if (!GENM) {
            const uint32_t wcur = wnext;
            const uint32_t pn = pb + WIN;
            if (pn < cnt) wnext = bits[pn >> 5];
            if (pb < cnt) m = (wcur >> (pb & 16u)) & 0xFFFFu;
        }
        if (pb < cnt) {
            if (GENM) {
                for (uint32_t q = 0; q < 16; q++) {
                    const uint32_t p = pb + q;
                    if (p < cnt && bit(bits, order[p])) m |= 1u << q;
                }
            }
            const uint32_t lim = cnt - pb;
            if (lim < 16) m &= (1u << lim) - 1u;
            if (pb < pfrom) m &= pfrom - pb >= 16u ? 0u : ~((1u << (pfrom - pb)) - 1u);
        }
        const uint32_t cl = (uint32_t)__popc(m);
        const uint32_t incl = wave_incl_scan(cl);
        const uint32_t tot = __shfl(incl, WAVE - 1, WAVE);
        const bool last = win + WIN >= cnt;
        st.stp++;
        if (tot) {
            __builtin_amdgcn_wave_barrier();
            uint32_t wp = incl - cl;
            while (m) {
                const uint32_t b = (uint32_t)__builtin_ctz(m);
                m &= m - 1u;
                wbuf[wp++] = (uint16_t)(16u * lane + b);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        // list = the carried candidates, then this window's; whole groups of 64 are evaluated now,
        // the rest with the next window (all of it at the end)
        const uint32_t total = pend + tot;
        const uint32_t lim = last ? total : (total & ~(uint32_t)(WAVE - 1));
        for (uint32_t c0 = 0; c0 < lim && !stop; c0 += WAVE) {
            if (!GENM && !COUNT && tail && d.vlog && c0 >= pend) {  // first-fit continuation: skip what cannot fit
                c0 = dir_tail_skip(d, s, r, ds.sched, wbuf, win, pend, lim, c0, d.mtu - S, st);
                if (c0 >= lim) break;
            }
            const uint32_t ci = c0 + lane;
            bool cand = ci < lim;
            st.grp++;
            st.stp++;
            Cand<KW> c;
            c.emsg = 0;
            c.min1 = 0;
            uint32_t j = 0;
            bool light = false;
            c.light = false;
            if (cand) {
                const uint32_t p = ci < pend ? rv : win + wbuf[ci - pend];
                j = GENM ? order[p] : p;
                if (!GENM && d.vlog && (lightok || (!COUNT && tail))) {
                    const uint32_t msw = mv_word(d, pix(d, s, j), j), mrw = mv_word(d, pix(d, r, j), j);
                    st.alg += 4;
                    const bool fast = !((msw | mrw) & MV_INEXACT);
                    // tail mode: skip what cannot fit (min1_lb)
                    if (!COUNT && tail && fast && min1_lb(d, j, msw, mrw, ds.sched) > d.mtu - S) cand = false;
                    else if (lightok && fast) {
                        eval_light<KW>(d, j, msw, mrw, c, st.alg);
                        light = true;
                        st.cand++;
                    }
                }
            }
            if (cand && !light) {
                CandKeys<KW> ck;
                eval_cand<KW, GENM>(d, s, r, ds, j, t, c, ck, st.alg);
                st.cand++;
            }
            if (COUNT) m1 = min(m1, wave_min(cand && c.emsg ? c.min1 : NONE));
            pack_group<KW, COUNT, REC>(d, s, r, t, c, cand, S, tail, stop, st, tomb, rec, nr);
        }
        if (!last) {  // carry the rest (< 64): entry lim + i to lane i
            const uint32_t rem = total - lim, idx = lim + lane;
            uint32_t v = 0;
            if ((uint32_t)lane < rem) v = idx < pend ? rv : win + wbuf[idx - pend];  // idx < pend only if lim = 0
            rv = v;
            pend = rem;
        }
        __builtin_amdgcn_wave_barrier();
    }
    pst.S = S;
    pst.tail = tail;
    pst.stop = stop;
    pst.m1 = m1;
    if (REC) {
        if (lane == 0) *nrec = nr;
        return;
    }
    if (!COUNT && lane == 0) shard_add(d, C_DBYTES, S - S0);  // DeltaPb bytes this call added
}


// First-fit continuation (tail mode) over pass 1's records: every later candidate is tested against a budget
// R that only shrinks, so a prefix record whose min1_lb exceeds R now is never sent.  Starting at group c0,
// TAIL_B groups of records and their bounds are loaded at once (one round trip for TAIL_B groups instead of
// one per group: a node back from an absence walks ~150 groups of stale owners past the mtu, and that walk
// was the exact packer's critical path); groups with no possible candidate are skipped, their
// speculatively merged receiver words restored (specd).  Returns the first group that holds a record that
// may still be sent (a non-prefix record is always evaluated), or n.
__device__ __forceinline__ uint32_t list_tail_skip(const Dev &d, uint32_t r, bool sched, const uint2 *L, uint32_t n,
                                                   uint32_t c0, uint32_t R, bool specd, WStats &st) {
    const int lane = lane_id();
    while (c0 < n) {
        uint2 rr[TAIL_B];
        bool ok[TAIL_B];
#pragma unroll
        for (int u = 0; u < TAIL_B; u++) {
            const uint32_t i = c0 + (uint32_t)(u * WAVE + lane);
            ok[u] = i < n;
            rr[u] = ok[u] ? L[i] : make_uint2(0u, 0u);
        }
        uint32_t lb[TAIL_B];
#pragma unroll
        for (int u = 0; u < TAIL_B; u++)
            lb[u] = ok[u] && rec_fast(rr[u].y) ? min1_lb(d, rr[u].x, rr[u].y & 0xFFFFu, rr[u].y >> 16, sched) : 0u;
        int uf = TAIL_B;
#pragma unroll
        for (int u = TAIL_B - 1; u >= 0; u--)
            if (__ballot(ok[u] && (!rec_fast(rr[u].y) || lb[u] <= R)) != 0ull) uf = u;
        if (specd) {
#pragma unroll
            for (int u = 0; u < TAIL_B; u++)
                if (u < uf && ok[u] && rec_fast(rr[u].y)) {  // not sent: undo pass 1's merge
                    mv_put(d, pix(d, r, rr[u].x), rr[u].y >> 16);
                    st.alg += 4;
                }
        }
        st.stp++;
        st.grp += (uint32_t)uf;
        if (uf < TAIL_B) return c0 + (uint32_t)uf * WAVE;
        c0 += TAIL_B * WAVE;
    }
    return n;
}

// List source (canonical records): the n stale owners pass 1 recorded for one row half, in column
// order, each with both views' max_version words (GS_R_CAND), so no row is read again.  The next
// group's records are loaded one group ahead.  Dev::spec: once the delta is complete, the remaining
// prefix candidates' receiver words are restored (pass 1 merged them).
template <int KW, bool COUNT = false>
__device__ __forceinline__ void pack_list(const Dev &d, uint32_t s, uint32_t r, const DigestSide ds, const uint2 *L,
                                          uint32_t n, uint32_t t, WStats &st, bool &tomb, PackState &pst) {
    const int lane = lane_id();
    const uint32_t S0 = pst.S;
    uint32_t S;
    bool tail, stop;
    pack_begin(d, COUNT, pst, S, tail, stop);
    const bool specd = !COUNT && d.spec;
    // prefix candidates from the version log (eval_light): no hook events (their applies take the per-key
    // path), no scheduled-for-deletion test due (a digest may leave owners out: from = 0).  Speculative slots
    // too: eval_light and apply_cand's paths start from the record's pre-exchange words, never the merged row
    const bool lightok = d.vlog && !d.ev && !ds.sched;
    uint32_t nr = 0, m1 = pst.m1;
    uint2 nxt = make_uint2(0u, 0u);
    if ((uint32_t)lane < n) nxt = L[lane];
    for (uint32_t c0 = 0; c0 < n && (specd || !stop); c0 += WAVE) {
        // first-fit continuation: no later candidate can fit once the budget is below their smallest NodeDelta
        if (!COUNT && !stop && tail && d.sm && d.mtu - S < d.sm[L[c0].x]) {
            stop = true;
            if (!specd) break;
        }
        if (stop) {  // specd only: nothing more is sent -- restore every remaining prefix record, TAIL_B groups at once
            for (uint32_t b0 = c0; b0 < n; b0 += TAIL_B * WAVE) {
#pragma unroll
                for (int u = 0; u < TAIL_B; u++) {
                    const uint32_t i = b0 + (uint32_t)(u * WAVE + lane);
                    const uint2 cr = i < n ? L[i] : make_uint2(0u, MV_INEXACT);
                    if (i < n && rec_fast(cr.y)) { mv_put(d, pix(d, r, cr.x), cr.y >> 16); st.alg += 4; }
                }
                st.stp++;
                st.grp += TAIL_B;
            }
            break;
        }
        if (!COUNT && tail && d.vlog) {  // first-fit continuation: skip the groups that cannot send anything
            const uint32_t c1 = list_tail_skip(d, r, ds.sched, L, n, c0, d.mtu - S, specd, st);
            if (c1 >= n) break;
            if (c1 != c0) {
                c0 = c1;
                nxt = c0 + lane < n ? L[c0 + lane] : make_uint2(0u, 0u);
            }
        }
        const uint32_t ci = c0 + lane;
        bool cand = ci < n;
        const uint2 cr = nxt;
        if (ci + WAVE < n) nxt = L[ci + WAVE];
        st.grp++;
        st.stp++;
        if (!COUNT && cand && tail && d.vlog && rec_fast(cr.y)) {  // tail mode: skip what cannot fit (min1_lb)
            const uint32_t mr = cr.y >> 16;
            if (min1_lb(d, cr.x, cr.y & 0xFFFFu, mr, ds.sched) > d.mtu - S) {
                cand = false;
                if (specd) { mv_put(d, pix(d, r, cr.x), mr); st.alg += 4; }  // not sent: undo the merge
            }
        }
        Cand<KW> c;
        c.emsg = 0;
        c.min1 = 0;
        c.light = false;
        if (cand) {
            if (lightok && rec_fast(cr.y)) {
                eval_light<KW>(d, cr.x, cr.y & 0xFFFFu, cr.y >> 16, c, st.alg);
            } else {
                CandKeys<KW> ck;
                eval_cand<KW, false, true>(d, s, r, ds, cr.x, t, c, ck, st.alg, cr.y);
            }
            st.cand++;
        }
        if (COUNT) m1 = min(m1, wave_min(cand && c.emsg ? c.min1 : NONE));
        pack_group<KW, COUNT, false>(d, s, r, t, c, cand, S, tail, stop, st, tomb, nullptr, nr, specd);
    }
    pst.S = S;
    pst.tail = tail;
    pst.stop = stop;
    pst.m1 = m1;
    if (!COUNT && lane == 0) shard_add(d, C_DBYTES, S - S0);
}

// Whole-delta fast path of one direction of a record phase (prefix views, pack_lite): when every stale owner
// pass 1 recorded is a prefix candidate (both views S_j(M), no GS_MV_INEXACT) and the receiver's digest
// holds all of them (no scheduled-for-deletion test due), NodeDelta j is {from = mr, last_gc 0,
// max_version ms, the kvs of S_j(ms) above mr} (state.py:347-390) = the writes v in (mr, ms] that no write
// <= ms overwrote (GS_R_VLOG: next > ms), so its DeltaPb bytes follow from those entries and the owner's
// NodeIdPb size alone -- no latest-write row, no history entry.  If the delta then fits from S0, every
// NodeDelta is sent whole (state.py:392-398) and each apply is apply_cand's fast path, one max_version
// store.  Returns false with nothing stored otherwise; the caller runs the exact packer (pack_records).
// Lane l takes candidates l, l + 64, ... of the two halves' lists in order (sums only: order-free); B
// groups per step, so their record loads, then their log loads, are in flight together.
constexpr int LITE_B = 4;
// The applies of a whole delta of prefix candidates (pack_lite): each receiver view becomes S_j(ms), one
// max_version store per recorded owner (apply_cand's fast path); lanes take records l, l + 64, ...
__device__ __forceinline__ void lite_apply(const Dev &d, uint32_t rcv, size_t slot, WStats &st) {
    if (d.spec) {  // k_pass1v merged every recorded prefix candidate (Dev::spec): only the counts
        const uint32_t nt = d.cand_n[slot * 2] + d.cand_n[slot * 2 + 1];
        if (lane_id() == 0) { st.nd += nt; st.cand += nt; }
        return;
    }
    const int lane = lane_id();
    const uint32_t n0 = d.cand_n[slot * 2], n1 = d.cand_n[slot * 2 + 1], nt = n0 + n1;
    const uint2 *L0 = d.cand + slot * 2 * GS_CAND_CAP, *L1 = L0 + GS_CAND_CAP;
    for (uint32_t c0 = 0; c0 < nt; c0 += WAVE * LITE_B) {
        uint2 rc[LITE_B];
#pragma unroll
        for (int u = 0; u < LITE_B; u++) {
            const uint32_t i = c0 + (uint32_t)(u * WAVE + lane);
            rc[u] = i < nt ? (i < n0 ? L0[i] : L1[i - n0]) : make_uint2(NONE, 0u);
        }
#pragma unroll
        for (int u = 0; u < LITE_B; u++) {
            if (rc[u].x == NONE) continue;
            mv_put(d, pix(d, rcv, rc[u].x), rc[u].y & 0xFFFFu);  // max(ms, mr) = ms
            st.alg += 8 + 4;
            st.nd++;
            st.cand++;
        }
    }
}
// APPLY = false: only the delta's DeltaPb total (a sliced count pass: every candidate, whatever the mtu).
// k_lite's per-slot flags (Dev::slot_stat[slot].w): LITE_FULL = the exact packer must size / pack the slot,
// LITE_DONE = k_lite completed it
constexpr uint32_t LITE_FULL = 1u, LITE_DONE = 2u;
// sched: the receiver's row may hold targets scheduled for deletion (its digest leaves them out, so their
// NodeDeltas start from version 0): any recorded owner that is one sends the slot to the exact packer.
template <bool APPLY = true>
__device__ __forceinline__ bool pack_lite(const Dev &d, uint32_t rcv, size_t slot, uint32_t S0, WStats &st,
                                          uint32_t &Tout, uint32_t *m1out = nullptr, bool sched = false,
                                          uint32_t t = 0u) {
    const int lane = lane_id();
    const uint32_t n0 = d.cand_n[slot * 2], n1 = d.cand_n[slot * 2 + 1];
    if (n0 > GS_CAND_CAP || n1 > GS_CAND_CAP) return false;  // a half continues in its bitmap
    const uint2 *L0 = d.cand + slot * 2 * GS_CAND_CAP, *L1 = L0 + GS_CAND_CAP;
    const uint32_t nt = n0 + n1;
    // every recorded owner is a NodeDelta of >= lb_min bytes (or the slot is not a lite one): past that many the
    // whole delta cannot fit, so the exact packer takes the slot without this pass sizing it
    if (APPLY && (uint64_t)nt * d.lb_min > (uint64_t)(d.mtu - min(S0, d.mtu))) return false;
    uint32_t sum = 0, kvs = 0, alg = 0, m1 = NONE;
    bool bad = false;
    for (uint32_t c0 = 0; c0 < nt; c0 += WAVE * LITE_B) {
        uint2 rc[LITE_B];
#pragma unroll
        for (int u = 0; u < LITE_B; u++) {
            const uint32_t i = c0 + (uint32_t)(u * WAVE + lane);
            rc[u] = i < nt ? (i < n0 ? L0[i] : L1[i - n0]) : make_uint2(NONE, 0u);
        }
        uint32_t ev[LITE_B], ns[LITE_B];
#pragma unroll
        for (int u = 0; u < LITE_B; u++) {
            ev[u] = 0u;
            ns[u] = 0u;
            if (rc[u].x == NONE) continue;
            const uint32_t ms = rc[u].y & 0xFFFFu, mr = rc[u].y >> 16;  // sender / receiver words
            if (!rec_fast(rc[u].y) || ms <= mr) { bad = true; continue; }
            if (sched) {  // owner rc.x left out of the receiver's digest (scheduled for deletion): from = 0
                const size_t p = pix(d, rcv, rc[u].x);
                if ((d.fd_state[p] & FD_MEMB) == FD_DEAD && is_sched(d.tod[p], t, d.sched_delay)) { bad = true; continue; }
                alg += 1;
            }
            ev[u] = d.vlog[(size_t)rc[u].x * d.VL + ms];
            ns[u] = d.nid_size[rc[u].x];
        }
#pragma unroll
        for (int u = 0; u < LITE_B; u++) {
            if (rc[u].x == NONE || !ev[u]) continue;
            const uint32_t j = rc[u].x, ms = rc[u].y & 0xFFFFu, mr = rc[u].y >> 16;
            uint32_t kv = ev[u] & 0xFFFFu, nk = 1;  // write ms is the latest <= ms of its key
            uint32_t kv1 = kv;  // the lowest version's kv (min1: the NodeDelta with only that kv)
            for (uint32_t v = ms - 1u; v > mr; v--) {  // lag > 1 (rare): the other writes of (mr, ms)
                const uint32_t e = d.vlog[(size_t)j * d.VL + v];
                if ((e >> 16) > ms) { kv += e & 0xFFFFu; nk++; kv1 = e & 0xFFFFu; }
                alg += 4;
            }
            const uint32_t base = msgf(ns[u]) + ufield(mr) + 1u + vlen(ms);
            sum += msgf(base + kv);
            m1 = min(m1, msgf(base + kv1));
            kvs += nk;
            alg += 8 + 4 + 2;
        }
    }
    const uint32_t T = (uint32_t)wave_sum(sum);
    if (__ballot(bad) != 0ull) return false;
    if (!APPLY) {
        st.alg += alg;
        st.kvs += kvs;  // (per lane: the caller reduces it)
        Tout = T;
        if (m1out) *m1out = wave_min(m1);
        return true;
    }
    if ((uint64_t)S0 + T > d.mtu) return false;
    lite_apply(d, rcv, slot, st);  // the records are L2-hot from the pass above
    st.kvs += kvs;
    st.alg += alg;
    Tout = T;
    return true;
}

// Candidates of one direction of exchange slot from pass 1's records (row half 0, then half 1); a half
// with more stale owners than GS_CAND_CAP continues in the bitmap after its last record (those owners
// were not merged speculatively: the bitmap walk reads their rows).
template <int KW, bool COUNT>
__device__ __forceinline__ void pack_records(const Dev &d, uint32_t snd, uint32_t rcv, const DigestSide &ds,
                                             size_t slot, uint16_t *wbuf, uint32_t t, WStats &st, bool &tomb,
                                             PackState &pst) {
    const uint32_t H = half_cols(d);
    const uint32_t words = d.NP / 32;
    for (uint32_t hf = 0; hf < 2 && (COUNT || d.spec || !pst.stop); hf++) {
        const uint32_t nh = d.cand_n[slot * 2 + hf];
        const uint2 *L = d.cand + (slot * 2 + hf) * GS_CAND_CAP;
        pack_list<KW, COUNT>(d, snd, rcv, ds, L, min(nh, GS_CAND_CAP), t, st, tomb, pst);
        if (nh > GS_CAND_CAP && (COUNT || !pst.stop)) {
            const uint32_t pmin = L[GS_CAND_CAP - 1].x + 1u;  // wave-uniform load
            pack_dir<KW, false, COUNT>(d, snd, rcv, ds, nullptr, min(H * (hf + 1), d.ncol), d.sbits + (slot * words),
                                       wbuf, t, st, tomb, pst, nullptr, nullptr, pmin & ~15u, pmin);
        }
    }
}

// ------------------------------------------------------------------ exchange kernel
// Pass-1 work of one group of 4 consecutive owners (one 16-byte load per array and row), held
// as scalar arrays so every element stays in a register after unrolling.
struct Grp {
    uint32_t hA[4], hB[4], mA[4], mB[4], pA[4], pB[4];
    uint32_t sA, sB;  // bit i: column c0 + i is scheduled for deletion in that row (only if the row may have one)
};

// Report bit planes (Dev::pend): column c of a plane row sits in word (c / 256) * 4 + c % 4, bit
// (c / 4) % 64 -- the order in which one wave's four ballots over its 64 lanes x 4 consecutive
// columns come out, so pass 1 stores its ballots as they are and never reads a plane.
__device__ inline uint32_t plane_word(uint32_t c) { return (c >> 8) * 4u + (c & 3u); }
__device__ inline uint32_t plane_bit(uint32_t c) { return (c >> 2) & 63u; }

__device__ __forceinline__ void ld4(const uint32_t *p, uint32_t (&v)[4]) {
    const uint4 x = *reinterpret_cast<const uint4 *>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}
// Heartbeats are stored mod 2^16 and decoded against the owner's own heartbeat R (every view of
// owner j is <= R, and views lag R by < 2^16: DESIGN.md §3), so H = R - ((R - s) mod 2^16).
__device__ __forceinline__ uint32_t hb_dec(uint32_t s, uint32_t R) { return R - ((R - s) & 0xFFFFu); }
// GS_HB8: views stored mod 2^8 (exact while they lag their owner by < 2^8: k_hb_lag), same decode
__device__ __forceinline__ uint32_t hb_dec8(uint32_t s, uint32_t R) { return R - ((R - s) & 0xFFu); }
// one view's stored heartbeat, any width (the small kernels; pass 1 is specialised on the width)
__device__ __forceinline__ uint32_t hb_raw(const Dev &d, size_t p) {
    return d.hb8 ? (uint32_t) reinterpret_cast<const uint8_t *>(d.hb)[p] : (uint32_t)d.hb[p];
}
// an escaped owner column (gs_config.esc_cols) keeps its views in 16-bit slots: the slot index of view p, or NONE
__device__ __forceinline__ uint32_t esc_of(const Dev &d, size_t p) { return d.EC ? d.esc_slot[p % d.NP] : NONE; }
__device__ __forceinline__ void hb_put(const Dev &d, size_t p, uint32_t v) {
    const uint32_t es = esc_of(d, p);
    if (es != NONE) d.esc16[(p / d.NP) * d.EC + es] = (uint16_t)v;
    else if (d.hb8) reinterpret_cast<uint8_t *>(d.hb)[p] = (uint8_t)v;
    else d.hb[p] = (uint16_t)v;
}
__device__ __forceinline__ uint32_t hb_view(const Dev &d, size_t p, uint32_t R) {
    const uint32_t es = esc_of(d, p);
    if (es != NONE) return hb_dec(d.esc16[(p / d.NP) * d.EC + es], R);
    return d.hb8 ? hb_dec8(hb_raw(d, p), R) : hb_dec(hb_raw(d, p), R);
}
__device__ __forceinline__ void st4b(uint8_t *p, const uint32_t (&v)[4]) {
    *reinterpret_cast<uint32_t *>(p) = (v[0] & 0xFFu) | ((v[1] & 0xFFu) << 8) | ((v[2] & 0xFFu) << 16) | (v[3] << 24);
}
__device__ __forceinline__ void st4h(uint16_t *p, const uint32_t (&v)[4]) {
    *reinterpret_cast<uint2 *>(p) = make_uint2((v[0] & 0xFFFFu) | (v[1] << 16), (v[2] & 0xFFFFu) | (v[3] << 16));
}
__device__ __forceinline__ void ld4h(const uint16_t *p, uint32_t (&v)[4]) {
    const uint2 x = *reinterpret_cast<const uint2 *>(p);
    v[0] = x.x & 0xFFFFu; v[1] = x.x >> 16; v[2] = x.y & 0xFFFFu; v[3] = x.y >> 16;
}
__device__ __forceinline__ void st4(uint32_t *p, const uint32_t (&v)[4]) {
    *reinterpret_cast<uint4 *>(p) = make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void ld4w(const uint64_t *p, uint64_t (&v)[4]) {
    const ulonglong2 x = reinterpret_cast<const ulonglong2 *>(p)[0], y = reinterpret_cast<const ulonglong2 *>(p)[1];
    v[0] = x.x; v[1] = x.y; v[2] = y.x; v[3] = y.y;
}
__device__ __forceinline__ void st4w(uint64_t *p, const uint64_t (&v)[4]) {
    reinterpret_cast<ulonglong2 *>(p)[0] = make_ulonglong2(v[0], v[1]);
    reinterpret_cast<ulonglong2 *>(p)[1] = make_ulonglong2(v[2], v[3]);
}
// scheduled-for-deletion mask of 4 consecutive pairs (p a multiple of 4): their 4 state bytes, then the
// times of death if any is dead (rows whose earliest scheduled tick has passed only)
__device__ __forceinline__ uint32_t sched4(const Dev &d, size_t p, uint32_t t) {
    const uint32_t s4 = *reinterpret_cast<const uint32_t *>(d.fd_state + p);
    if (!(s4 & 0x02020202u)) return 0u;
    uint32_t td[4];
    ld4(d.tod + p, td);
    uint32_t m = 0u;
#pragma unroll
    for (int i = 0; i < 4; i++)
        m |= (uint32_t)(((s4 >> (8 * i)) & FD_MEMB) == FD_DEAD && is_sched(td[i], t, d.sched_delay)) << i;
    return m;
}
// One group's loads as they arrive (packed u16 pairs, not yet decoded): the loop keeps the next group in
// this form while the current one computes, so nothing waits on the prefetch until it is decoded one
// iteration later (and the packed form holds 12 VGPRs instead of 20).
struct GrpRaw {
    uint4 R;  // the owners' own heartbeats (MV8: GS_R_SELF_PK, both values packed)
    uint2 hA, hB, mA, mB;
    uint4 pA, pB;
    uint32_t sA, sB;
};
template <bool GENM, bool HB8 = false, bool MV8 = false>
__device__ __forceinline__ void load_grp(const Dev &d, size_t ra, size_t rb, uint32_t c0, uint32_t t, bool schA,
                                         bool schB, GrpRaw &g) {
    g.R = *reinterpret_cast<const uint4 *>((MV8 ? d.self_pk : d.self_hb) + c0);
    if (HB8) {  // 4 bytes per lane (4 views)
        const uint8_t *h8 = reinterpret_cast<const uint8_t *>(d.hb);
        g.hA = make_uint2(*reinterpret_cast<const uint32_t *>(h8 + ra + c0), 0u);
        g.hB = make_uint2(*reinterpret_cast<const uint32_t *>(h8 + rb + c0), 0u);
    } else {
        g.hA = *reinterpret_cast<const uint2 *>(d.hb + ra + c0);
        g.hB = *reinterpret_cast<const uint2 *>(d.hb + rb + c0);
    }
    if (MV8) {  // 4 bytes per lane, decoded against the owners' own max_versions
        const uint8_t *m8 = reinterpret_cast<const uint8_t *>(d.mv);
        g.mA = make_uint2(*reinterpret_cast<const uint32_t *>(m8 + ra + c0), 0u);
        g.mB = make_uint2(*reinterpret_cast<const uint32_t *>(m8 + rb + c0), 0u);
    } else {
        g.mA = *reinterpret_cast<const uint2 *>(d.mv + ra + c0);
        g.mB = *reinterpret_cast<const uint2 *>(d.mv + rb + c0);
    }
    g.pA = g.pB = make_uint4(0u, 0u, 0u, 0u);
    g.sA = g.sB = 0u;
    if (GENM) {
        g.pA = *reinterpret_cast<const uint4 *>(d.pos + ra + c0);
        g.pB = *reinterpret_cast<const uint4 *>(d.pos + rb + c0);
    }
    if (schA) g.sA = sched4(d, ra + c0, t);
    if (schB) g.sB = sched4(d, rb + c0, t);
}
// decode: heartbeats against the owners' own (hb_dec); raw max_version words (prefix-view flag included):
// pass 1 masks them where it compares, and the split path hands them to the packer in its records
template <bool HB8 = false, bool MV8 = false>
__device__ __forceinline__ void dec_grp(const GrpRaw &r, Grp &g) {
    const uint32_t R[4] = {r.R.x, r.R.y, r.R.z, r.R.w};
    if (MV8) {  // packed: Rx = the low 16 bits (self_pack), M = the high 16
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t Rx = R[i] & 0xFFFFu, M = R[i] >> 16;
            g.hA[i] = hb_dec8((r.hA.x >> (8 * i)) & 0xFFu, Rx);
            g.hB[i] = hb_dec8((r.hB.x >> (8 * i)) & 0xFFu, Rx);
            g.mA[i] = mv_dec8((r.mA.x >> (8 * i)) & 0xFFu, M);
            g.mB[i] = mv_dec8((r.mB.x >> (8 * i)) & 0xFFu, M);
        }
    } else if (HB8) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            g.hA[i] = hb_dec8((r.hA.x >> (8 * i)) & 0xFFu, R[i]);
            g.hB[i] = hb_dec8((r.hB.x >> (8 * i)) & 0xFFu, R[i]);
        }
    } else {
        const uint32_t hA[4] = {r.hA.x & 0xFFFFu, r.hA.x >> 16, r.hA.y & 0xFFFFu, r.hA.y >> 16};
        const uint32_t hB[4] = {r.hB.x & 0xFFFFu, r.hB.x >> 16, r.hB.y & 0xFFFFu, r.hB.y >> 16};
#pragma unroll
        for (int i = 0; i < 4; i++) { g.hA[i] = hb_dec(hA[i], R[i]); g.hB[i] = hb_dec(hB[i], R[i]); }
    }
    if (!MV8) {
        g.mA[0] = r.mA.x & 0xFFFFu; g.mA[1] = r.mA.x >> 16; g.mA[2] = r.mA.y & 0xFFFFu; g.mA[3] = r.mA.y >> 16;
        g.mB[0] = r.mB.x & 0xFFFFu; g.mB[1] = r.mB.x >> 16; g.mB[2] = r.mB.y & 0xFFFFu; g.mB[3] = r.mB.y >> 16;
    }
    g.pA[0] = r.pA.x; g.pA[1] = r.pA.y; g.pA[2] = r.pA.z; g.pA[3] = r.pA.w;
    g.pB[0] = r.pB.x; g.pB[1] = r.pB.y; g.pB[2] = r.pB.z; g.pB[3] = r.pB.w;
    g.sA = r.sA;
    g.sB = r.sB;
}

// FailureDetector.report_heartbeat -> SamplingWindow.report_heartbeat on one unpacked window
// (failure_detector.py:79-81, 32-38): the first report only records the time; later intervals
// <= max_interval go to BoundedArrayStats (139-150).
// rg: this pair's interval ring (GS_FD_RING, or a sampled ring row), nullptr for a compact window.
__device__ __forceinline__ Fd fd_report_val(const Dev &d, uint16_t *rg, uint32_t t, Fd f, uint32_t &alg, uint32_t &ovf) {
    if (f.last != NONE) {
        const uint32_t iv = t - f.last;
        if (iv <= d.max_iv) {
            if (rg) {
                const uint32_t slot = f.cnt % d.W;
                if (f.cnt >= d.W) { f.sum -= rg[slot]; alg += 2; }  // subtract-then-add (failure_detector.py:140-143)
                rg[slot] = (uint16_t)iv;
                f.sum += iv;
                f.cnt += 1;
                if (f.cnt >= 2u * d.W) f.cnt -= d.W;
                alg += 2;
            } else if (f.cnt >= d.W) {
                ovf += 1;  // eviction needs the ring: flagged, the run is reported inexact
            } else {
                f.sum += iv;
                f.cnt += 1;
            }
        }
    }
    f.last = t;
    return f;
}

// Partial-line writes: HBM3E has no write data mask, so a dirty line that was only partly written costs the
// memory a read-modify-write.  P1_LINE bit 0: a changed heartbeat group stores its whole 64-byte line (the
// 8 lanes covering it store their 8 bytes, changed or not); bit 1: the same for the speculative merge's
// max_version groups (A/B, tools/build_dev.sh -DP1_LINE=n).
#ifndef P1_LINE
#define P1_LINE 0
#endif
// any of the 8 lanes sharing this lane's 64-byte line (8 bytes per lane; lines start at a multiple of 8
// lanes: rows are 128-byte aligned and a wave's groups start at a multiple of 256 columns)
__device__ __forceinline__ bool line_any8(bool w) {
    const uint64_t m = __ballot(w);
    return ((m >> (lane_id() & ~7)) & 0xFFull) != 0ull;
}

// Reports are deferred: the window of (observer, owner) is only read by phi, i.e. by the liveness
// sweep at the end of the round, so pass 1 records each report as one bit in the phase's bit plane
// (rmA/rmB: bit i = column c0 + i) and k_liveness replays them in tick order before computing phi
// (same appends, same order).
// SCH = false: neither row can have a target scheduled for deletion at t (schA = schB = false; the
// per-column predicates drop out).  SELF = false: the caller stores the responder's own new heartbeat.
template <bool GENM, bool SCH = true, bool SELF = true, bool HB8 = false, bool MV8 = false>
__device__ __forceinline__ void pass1_grp(const Dev &d, size_t ra, size_t rb, uint32_t c0, uint32_t a, uint32_t b,
                                          uint32_t t, bool schA, bool schB, Grp &g, uint32_t &nBA, uint32_t &nAB,
                                          uint32_t &nNB, uint32_t &nNA, uint32_t &alg, uint32_t &reports,
                                          uint32_t &hbw, uint32_t &rmA, uint32_t &rmB) {
    bool dA = false, dB = false;
    rmA = rmB = 0u;
    nBA = nAB = nNB = nNA = 0u;
    // HBM-resident elements only: the SELF_HB row (16 B per group, 256 KiB per row, L2-resident) is not counted
    alg += (HB8 ? 8 : 16) + (MV8 ? 8 : 16) + (GENM ? 32 : 0) + (schA ? 4 : 0) + (schB ? 4 : 0);
    // Branch-free (selects, no exec-mask juggling per column): the per-column rules of the reference,
    // restated as predicates.  _report_heartbeat (server.py:599-604, state.py:280-287) of a known view
    // stores the larger heartbeat and reports only if the old one was non-zero; an unknown owner is
    // inserted with the sender's heartbeat (node_state_or_default).
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t j = c0 + i, jg = d.col_lo + j;  // local column, node id
        const bool valid = j < d.ncol;
        const bool pa = GENM ? g.pA[i] != NONE : true;
        const bool pb = GENM ? g.pB[i] != NONE : true;
        const bool sa = SCH && schA && pa && ((g.sA >> i) & 1u);
        const bool sb = SCH && schB && pb && ((g.sB >> i) & 1u);
        const bool inA = pa && !sa;  // j is in a's digest (compute_digest, state.py:324-331)
        uint32_t hA = g.hA[i], hB = g.hB[i];
        // responder inc_heartbeat (server.py:524): b's view of itself
        const bool isb = valid && jg == b;
        hB += isb ? 1u : 0u;
        if (SELF && isb) d.self_hb[j] = hB;
        // b: _report_heartbeat over a's digest (server.py:336-337, 599-604)
        const bool mrgB = valid && inA && jg != b;
        const bool newB = mrgB && !pb;
        const bool upB = mrgB && (newB || hA > hB);
        const bool repB = upB && pb && hB != 0u;
        hB = upB ? hA : hB;
        // a: _report_heartbeat over b's digest, computed after b's merge (server.py:340, 356-357)
        const bool pb2 = pb || newB;
        const bool inB = pb2 && !sb;  // j is in b's digest
        const bool mrgA = valid && inB && jg != a;
        const bool newA = mrgA && !pa;
        const bool upA = mrgA && (newA || hB > hA);
        const bool repA = upA && pa && hA != 0u;
        hA = upA ? hB : hA;
        g.hA[i] = hA;
        g.hB[i] = hB;
        dA = dA || upA;
        dB = dB || upB || isb;
        hbw += (uint32_t)upA + (uint32_t)upB + (uint32_t)isb;
        rmB |= (uint32_t)repB << i;
        rmA |= (uint32_t)repA << i;
        reports += (uint32_t)repA + (uint32_t)repB;
        // stale owners (state.py:347-357): sender's max_version above the digest's
        const uint32_t mA = g.mA[i] & MV_MASK, mB = g.mB[i] & MV_MASK;
        const uint32_t dmA = inA ? mA : 0u;
        const uint32_t dmB = inB ? mB : 0u;
        nBA |= (uint32_t)(valid && pb2 && !sb && mB > dmA) << i;
        nAB |= (uint32_t)(valid && pa && !sa && mA > dmB) << i;
        nNB |= (uint32_t)newB << i;
        nNA |= (uint32_t)newA << i;
    }
    // only changed 16/32-byte groups are written back (writing whole lines measured slower: r1c vs r1b)
    if (d.ablate & 2u) return;
    if (P1_LINE & 1) {
        dA = line_any8(dA);
        dB = line_any8(dB);
    }
    if (HB8) {
        uint8_t *h8 = reinterpret_cast<uint8_t *>(d.hb);
        if (dA) { st4b(h8 + ra + c0, g.hA); alg += 4; }
        if (dB) { st4b(h8 + rb + c0, g.hB); alg += 4; }
    } else {
        if (dA) { st4h(d.hb + ra + c0, g.hA); alg += 8; }
        if (dB) { st4h(d.hb + rb + c0, g.hB); alg += 8; }
    }
}

// The four ballots of one group step are this wave's 32-byte block of the phase's bit plane
// (plane_word/plane_bit): stored whole, zeros included, so a plane row written in this phase never
// needs clearing.  Lane 0 is active whenever any lane of the wave is (it has the lowest column).
__device__ __forceinline__ void store_plane(uint64_t *plane, uint32_t c0, uint32_t rm, uint32_t &alg) {
    const uint64_t b0 = __ballot(rm & 1u), b1 = __ballot(rm & 2u), b2 = __ballot(rm & 4u), b3 = __ballot(rm & 8u);
    if (lane_id() == 0) {
        ulonglong2 *p = reinterpret_cast<ulonglong2 *>(plane + plane_word(c0));
        p[0] = make_ulonglong2(b0, b1);
        p[1] = make_ulonglong2(b2, b3);
        alg += 32;
    }
}

// bit m of an 8-bit value -> bit 4m
__device__ __forceinline__ uint32_t spread8(uint32_t x) {
    x &= 0xFFu;
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return x;
}

// Split path (k_pass1): one wave step's stale owners of one direction (a nibble of 4 consecutive
// columns per lane) go out twice, from the same four ballots (inactive lanes contribute zeros):
//  * as natural-order bitmap words (bit c % 32 of word c / 32), zeros included, so the buffer never
//    needs clearing; the first lane of each 8 stores its word: 32 contiguous bytes per wave -- only from
//    the step whose owners overflow the list on (the packers walk the bitmap past the last record only);
//  * as records {column, sender max_version word | receiver max_version word << 16} appended in
//    column order to the wave's list L (the first GS_CAND_CAP of them; cnt counts all, wave-uniform).
// Returns the lane's recorded columns (bit i: column c0 + i got a record).
__device__ __forceinline__ uint32_t emit_dir(uint32_t *gw, uint2 *L, uint32_t &cnt, uint32_t c0, uint32_t nib,
                                             const uint32_t (&ms)[4], const uint32_t (&mr)[4], uint32_t &alg) {
    const uint64_t b0 = __ballot(nib & 1u), b1 = __ballot(nib & 2u), b2 = __ballot(nib & 4u), b3 = __ballot(nib & 8u);
    const int l = lane_id();
    const bool any = (b0 | b1 | b2 | b3) != 0ull;
    const uint32_t tot = (uint32_t)(__popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3));
    if ((l & 7) == 0 && cnt + tot > GS_CAND_CAP) {
        const uint32_t w = !any ? 0u
                                : spread8((uint32_t)(b0 >> l)) | (spread8((uint32_t)(b1 >> l)) << 1) |
                                      (spread8((uint32_t)(b2 >> l)) << 2) | (spread8((uint32_t)(b3 >> l)) << 3);
        gw[c0 >> 5] = w;
        alg += 4;
    }
    if (!any) return 0u;
    const uint64_t lt = (1ull << l) - 1ull;
    uint32_t off = cnt + (uint32_t)(__popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt));
    uint32_t recm = 0u;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if ((nib >> i) & 1u) {
            if (off < GS_CAND_CAP) {
                L[off] = make_uint2(c0 + i, (ms[i] & 0xFFFFu) | (mr[i] << 16));
                alg += 8;
                recm |= 1u << i;
            }
            off++;
        }
    }
    cnt += tot;
    return recm;
}

// Speculative apply (Dev::spec): every recorded candidate whose two views are prefix views gets
// max(sender, receiver) as the receiver's max_version now, in the row group pass 1 just loaded (an
// 8-byte store into a line still in L2 -- instead of a scattered 2-byte store per NodeDelta later).  A
// delta that fits the mtu sends all of them whole, which is exactly apply_delta's result for a prefix
// view (apply_cand's fast path); the packers restore the receiver's word of the others.
template <bool MV8 = false>
__device__ __forceinline__ void spec_merge(const Dev &d, size_t ra, size_t rb, uint32_t c0, uint32_t recBA,
                                           uint32_t recAB, const uint32_t (&mA)[4], const uint32_t (&mB)[4],
                                           uint32_t &alg) {
    uint32_t nA[4], nB[4];
    bool wA = false, wB = false;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const bool fast = !((mA[i] | mB[i]) & MV_INEXACT);
        const uint32_t mx = mA[i] > mB[i] ? mA[i] : mB[i];
        const bool ba = fast && ((recBA >> i) & 1u), ab = fast && ((recAB >> i) & 1u);
        nA[i] = ba ? mx : mA[i];
        nB[i] = ab ? mx : mB[i];
        wA = wA || ba;
        wB = wB || ab;
    }
    if (P1_LINE & 2) {
        wA = line_any8(wA);
        wB = line_any8(wB);
    }
    if (MV8) {
        uint8_t *m8 = reinterpret_cast<uint8_t *>(d.mv);
        const uint32_t eA[4] = {mv_enc8(nA[0]), mv_enc8(nA[1]), mv_enc8(nA[2]), mv_enc8(nA[3])};
        const uint32_t eB[4] = {mv_enc8(nB[0]), mv_enc8(nB[1]), mv_enc8(nB[2]), mv_enc8(nB[3])};
        if (wA) { st4b(m8 + ra + c0, eA); alg += 4; }
        if (wB) { st4b(m8 + rb + c0, eB); alg += 4; }
    } else {
        if (wA) { st4h(d.mv + ra + c0, nA); alg += 8; }
        if (wB) { st4h(d.mv + rb + c0, nB); alg += 8; }
    }
}

// Owner-column sharded phases ("multi-GPU"): the count pass leaves each exchange's
// stale-owner bitmaps in GS_R_SLICE_BITS and the DeltaPb bytes of all this slice's candidates per
// direction in tot[e][dir]; the pack passes resume the sender-order packing where the previous
// slice left it: chain[e][dir] = S | tail << 32 | stop << 33, or CHAIN_PENDING.
constexpr uint64_t CHAIN_PENDING = ~0ull;
struct SliceIO {
    uint64_t *tot;              // [n][2] count pass output
    const uint64_t *tot_all;    // [shards][n][2] every slice's totals (gathered)
    const uint64_t *chain_all;  // [shards][n][2] every slice's chain state after the previous step
    uint64_t *chain;            // [n][2] this slice's chain state
    uint32_t step;
};
__device__ inline uint64_t chain_pack(const PackState &p) {
    return (uint64_t)p.S | ((uint64_t)p.tail << 32) | ((uint64_t)p.stop << 33);
}
__device__ inline PackState chain_unpack(uint64_t v) {
    return PackState{(uint32_t)v, ((v >> 32) & 1ull) != 0, ((v >> 33) & 1ull) != 0};
}

// In-process slice groups (gs_run_phase_group, round 5): one launch per step runs every slice of the group,
// blockIdx.y = slice.  Each workgroup takes its slice's Dev and scratch pointers from a GroupArgs in device
// memory (uploaded when they change: in a steady run never); the Dev fields that change per phase come by value
// (DevDyn).  A single handle's launch passes ga = nullptr and uses its own arguments.
constexpr uint32_t GRP_MAX = 8;
struct DevDyn {
    uint32_t t_round, spec, lite, p1fix, v_round, vt, t_cap;
};
struct GroupArgs {
    Dev dv[GRP_MAX];
    SliceIO io[GRP_MAX];  // tot (count), tot_all + chain (steps)
    uint32_t *list[GRP_MAX];
    uint64_t *chain_all[GRP_MAX], *chainc[GRP_MAX];
};
__device__ __forceinline__ void group_pick(Dev &d, const GroupArgs *ga, const DevDyn &dyn) {
    d = ga->dv[blockIdx.y];
    d.t_round = dyn.t_round;
    d.v_round = dyn.v_round;
    d.vt = dyn.vt;
    d.t_cap = dyn.t_cap;
    d.spec = dyn.spec;
    d.lite = dyn.lite;
    d.p1fix = dyn.p1fix;
}

// Split canonical phase, kernel 1 of 2 (k_pass1 -> k_pack_slice): pass 1 alone, streaming both rows with
// no LDS at all; the stale-owner bitmaps of both directions go to GS_R_SLICE_BITS ([e][2][NP/32],
// natural bit order) for the packer.  Without LDS the occupancy is set by registers only, and the
// latency-bound packing no longer holds a streaming workgroup's slot.
#ifndef P1_WAVES
#define P1_WAVES 4
#endif
#ifndef P1_AHEAD
#define P1_AHEAD 1  // pass-1 groups loaded ahead of the one being computed (1 or 2: 2 measured slower, r2o)
#endif
// 8-bit views (HB8 + MV8, GS_R_SELF_PK): a group's loads are a third of the 16-bit ones, so the pass is
// bound by groups in flight, not bytes: two groups ahead at 5 waves per SIMD, 96 VGPRs, no spills
// (r3j: 3.11 ms per phase vs 3.42 at one ahead / 4 waves; 6 waves spill, 4.43 ms)
#ifndef P1N_AHEAD
#define P1N_AHEAD 2
#endif
#ifndef P1N_WAVES
#define P1N_WAVES 5
#endif
// FUSE: the same workgroup then packs and applies both directions from the records (wave 0: b -> a,
// wave 1: a -> b) right after streaming the rows, while the receivers' max_version lines are still in L2
// (the applies are one scattered 2-byte store per NodeDelta; tools/membench.hip prices those at 25 G/s
// from HBM).
#ifndef P1S_WAVES
#define P1S_WAVES 4  // waves per SIMD of the pass-1-only kernel (split phases, sliced count pass); 5 spills and measured slower (r2r)
#endif
// SPEC (not with FUSE): the speculative max-version merge of the recorded prefix candidates (spec_merge,
// Dev::spec); k_settle then only settles the deltas that do not fit and the candidates with holes.
// HB8 (not with FUSE): GS_HB8's 8-bit heartbeat views.
template <int KW, bool FUSE, bool SPEC = false, bool HB8 = false, bool MV8 = false>
__global__ __launch_bounds__(XB, (KW == 4 ? (FUSE ? P1_WAVES : MV8 ? P1N_WAVES : P1S_WAVES) : 1)) void k_pass1(Dev d, const int32_t *ini, const int32_t *res,
                                                                       uint32_t n, uint32_t t, uint32_t seq,
                                                                       uint32_t e0) {
    static_assert(!(FUSE && SPEC), "the fused packer applies every NodeDelta itself");
    static_assert(!(FUSE && HB8), "8-bit heartbeats: record phases only");
    const uint32_t e = e0 + blockIdx.x;  // exchanges [e0, e0 + grid) of the phase (one chunk)
    if (e >= n) return;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid >> 6;
    const int32_t ai = ini[e], bi = res[e];
    if (ai < 0 || bi < 0 || (uint32_t)ai >= d.N || (uint32_t)bi >= d.N || ai == bi) {
        if (tid == 0) shard_add(d, C_E_IDX, 1);
        return;
    }
    const uint32_t a = (uint32_t)ai, b = (uint32_t)bi;
    if (tid == 0) {
        const uint32_t oa = atomicMax(&d.stamp[a], seq), ob = atomicMax(&d.stamp[b], seq);
        if (oa == seq || ob == seq) shard_add(d, C_E_CONFLICT, 1);
    }
    const bool schA = t >= d.row[a * 4 + 2];
    const bool schB = t >= d.row[b * 4 + 2];
    const size_t ra = (size_t)a * d.NP, rb = (size_t)b * d.NP;
    const uint32_t words = d.NP / 32;
    uint32_t *gBA = d.sbits + (size_t)e * 2 * words, *gAB = gBA + words;
    // wave w streams row half w (columns [w*H, min((w+1)*H, ncol)), H a multiple of 256), so its candidate
    // lists hold that half in column order and the packer reads half 0's list, then half 1's
    const uint32_t H = half_cols(d);
    const uint32_t lo = (uint32_t)wid * H, hi = min(lo + H, d.ncol);
    uint2 *LBA = d.cand + ((size_t)e * 4 + 0 * 2 + wid) * GS_CAND_CAP;
    uint2 *LAB = d.cand + ((size_t)e * 4 + 1 * 2 + wid) * GS_CAND_CAP;
    uint32_t nBAc = 0, nABc = 0;
    uint32_t alg = 0, reports = 0, hbw = 0;
    bool anynew = false;
    const uint32_t ph = d.vt - d.v_round - 1u;  // this phase's plane (host-checked: < NPL)
    if (ph >= NPL) {  // (never: plane_slot checks it; a guard, so that a host bug cannot write past the planes)
        if (tid == 0) shard_add(d, C_E_IDX, 1);
        return;
    }
    uint64_t *planeA = d.pend + ((size_t)a * NPL + ph) * d.PW;
    uint64_t *planeB = d.pend + ((size_t)b * NPL + ph) * d.PW;
    if (tid == 0) {
        d.pstamp[a * NPL + ph] = d.vt;
        d.pstamp[b * NPL + ph] = d.vt;
    }
    // responder inc_heartbeat (server.py:524): the owner's own heartbeat R is raised once, here; the
    // view hb[b][b] is raised in the loop.  Other exchanges of the phase decode column b against R or
    // R + 1, and both bound every view of b in the rows they touch
    if (tid == 0 && b - d.col_lo < d.ncol) {
        const uint32_t jb = b - d.col_lo, R1 = d.self_hb[jb] + 1u;
        d.self_hb[jb] = R1;
        if (MV8) d.self_pk[jb] = self_pack(R1, d.self_mv[jb]);
    }
    const uint32_t c0s = lo + (uint32_t)lane * 4u;
    auto loop = [&](auto sch) {
        constexpr bool SCH = decltype(sch)::value;
        uint32_t c0 = c0s;
        // AHEAD groups in flight ahead of the one being computed
        constexpr int AHEAD = MV8 ? P1N_AHEAD : P1_AHEAD;
        GrpRaw r0, r1, r2;
        constexpr uint32_t STEP = WAVE * 4u;
        if (c0 < hi) load_grp<false, HB8, MV8>(d, ra, rb, c0, t, SCH && schA, SCH && schB, r0);
        if (AHEAD > 1 && c0 + STEP < hi) load_grp<false, HB8, MV8>(d, ra, rb, c0 + STEP, t, SCH && schA, SCH && schB, r1);
        while (c0 < hi) {
            const uint32_t c1 = c0 + STEP;
            if (AHEAD > 1) {
                if (c1 + STEP < hi) load_grp<false, HB8, MV8>(d, ra, rb, c1 + STEP, t, SCH && schA, SCH && schB, r2);
            } else if (c1 < hi) {
                load_grp<false, HB8, MV8>(d, ra, rb, c1, t, SCH && schA, SCH && schB, r1);
            }
            Grp g0;
            dec_grp<HB8, MV8>(r0, g0);
            uint32_t rmA, rmB, nBA, nAB, nNB, nNA;
            const uint32_t mA[4] = {g0.mA[0], g0.mA[1], g0.mA[2], g0.mA[3]};
            const uint32_t mB[4] = {g0.mB[0], g0.mB[1], g0.mB[2], g0.mB[3]};
            pass1_grp<false, SCH, false, HB8, MV8>(d, ra, rb, c0, a, b, t, schA, schB, g0, nBA, nAB, nNB, nNA, alg, reports, hbw,
                                         rmA, rmB);
            anynew = anynew || (nNB | nNA) != 0u;
            store_plane(planeA, c0, rmA, alg);
            store_plane(planeB, c0, rmB, alg);
            const uint32_t recBA = emit_dir(gBA, LBA, nBAc, c0, nBA, mB, mA, alg);  // b -> a: sender b, receiver a
            const uint32_t recAB = emit_dir(gAB, LAB, nABc, c0, nAB, mA, mB, alg);
            if (SPEC && ((P1_LINE & 2) || (recBA | recAB))) spec_merge<MV8>(d, ra, rb, c0, recBA, recAB, mA, mB, alg);
            r0 = r1;
            if (AHEAD > 1) r1 = r2;
            c0 = c1;
        }
    };
    if (schA || schB) loop(std::true_type{});
    else loop(std::false_type{});
    if (lane == 0) {
        d.cand_n[(size_t)e * 4 + 0 * 2 + wid] = nBAc;
        d.cand_n[(size_t)e * 4 + 1 * 2 + wid] = nABc;
    }
    // canonical: every observer knows every owner, so no owner can be new to a side
    const unsigned long long s_alg = wave_sum(alg), s_rep = wave_sum(reports), s_hbw = wave_sum(hbw);
    const bool wnew = __ballot(anynew) != 0ull;
    if (lane == 0) {
        shard_add(d, C_ALG, s_alg);
        shard_add(d, C_REPORTS, s_rep);
        shard_add(d, C_HBW, s_hbw);
        if (wnew) shard_add(d, C_E_INSERT, 1);
        if (wid == 0 && d.shard == 0) shard_add(d, C_EXCH, 1);  // slices: every slice runs every exchange
    }
    if constexpr (FUSE) {
        __shared__ __attribute__((aligned(16))) uint16_t s_wbuf[2 * WIN];
        __syncthreads();  // both halves' records and counts are written (workgroup scope)
        const size_t slot = (size_t)e * 2 + wid;
        const bool w0 = wid == 0;
        const uint32_t snd = w0 ? b : a, rcv = w0 ? a : b;
        const DigestSide ds{rcv, d.ncol, w0 ? schA : schB};
        WStats st{0, 0, 0, 0, 0};
        bool tomb = false;
        PackState pst{0u, false, false};
        pack_records<KW, false>(d, snd, rcv, ds, slot, s_wbuf + wid * WIN, t, st, tomb, pst);
        if (tomb) d.row[rcv * 4 + 1] = 1u;
        const unsigned long long p_alg = wave_sum(st.alg), p_nd = wave_sum(st.nd), p_kv = wave_sum(st.kvs);
        const unsigned long long p_tr = wave_sum(st.trunc), p_cd = wave_sum(st.cand);
        if (lane == 0) {
            shard_add(d, C_ALG, p_alg);
            shard_add(d, C_PACKB, p_alg);
            shard_add(d, C_ND, p_nd);
            shard_add(d, C_KVS, p_kv);
            shard_add(d, C_TRUNC, p_tr);
            shard_add(d, C_CAND, p_cd);
        }
    }
}

// ---------------------------------------------------------------- k_pass1v (GS_HB8 + GS_MV8, round 4)
// Pass 1 of a canonical record phase on 8-bit views, byte-parallel: each lane takes 16 consecutive owner
// columns per step (one 16-byte load per row and region), and the per-column rules of pass1_grp run on four
// views per 32-bit word.  Two views of one owner compare without the owner's own value: at the last lag sweep
// no view of a column or row that is not hot lagged by HOT_HB heartbeats / HOT_MV versions or more, and since
// then it fell behind by at most 64 / 32 more (k_hb_lag), so two such heartbeat views differ by less than 2^7
// and two max_version views by less than 2^6: the sign of their difference mod 2^8 (mod 2^7) orders them.  A
// stored heartbeat byte 0 is the heartbeat 0 exactly when the owner's own heartbeat is < 2^8 (GS_R_P1FLAGS
// small bits).  Everything else -- the exchange's own columns a and b (the responder's +1), a row that may hold
// targets scheduled for deletion, hot rows and columns, the partial last group -- takes pass1_grp's per-column
// path on the same loads (decoded against the owners' own values: exact for lags < 2^8).
// Report planes: 16-column layout (d.pl16, plane16_bit): one u16 per lane and step, zeros included.
#ifndef P1V_AHEAD
#define P1V_AHEAD 1  // groups of 16 columns loaded ahead of the one being computed
#endif
#ifndef P1V_LINE
#define P1V_LINE 8  // k_pass1v's row stores cover whole 128-byte lines (8 lanes; 4: 64 B; 0: per lane): a partial
                    // line written back costs the memory a read-modify-write (r4m, with the merge: 2.08 vs 2.26 ms)
#endif
// whether any lane of this lane's line (P1V_LINE consecutive lanes) has p set; every lane of the wave calls it
__device__ __forceinline__ bool line_any_v(bool p) {
    const uint64_t m = __ballot(p);
    const uint32_t l = (uint32_t)__lane_id() & ~(uint32_t)(P1V_LINE - 1);
    return ((m >> l) & ((1ull << P1V_LINE) - 1ull)) != 0ull;
}
#ifndef P1V_NT
#define P1V_NT 1  // non-temporal row loads and heartbeat / max_version stores in k_pass1v (r4l: 1.81-1.86 vs 2.14-2.22 ms)
#endif
#ifndef P1V_WAVES
#define P1V_WAVES 5  // waves per SIMD k_pass1v is compiled for (r4i: 5 -> 2.19 ms per phase, 6 -> 2.25)
#endif
constexpr uint32_t B7 = 0x80808080u, L7 = 0x7F7F7F7Fu;
// the 16-column plane layout: plane u16 g holds columns 16 g .. 16 g + 15, column 16 g + 4 q + i at bit 4 i + q
__device__ __forceinline__ uint32_t plane16_bit(uint32_t c) { return 4u * (c & 3u) + ((c >> 2) & 3u); }
// bit 7 of byte i of w[q] -> bit 4 i + q (the plane layout of one lane's 16 columns)
__device__ __forceinline__ uint32_t pack16(const uint32_t (&w)[4]) {
    const uint32_t x = (w[0] >> 7) | (w[1] >> 6) | (w[2] >> 5) | (w[3] >> 4);  // byte i: bit q
    const uint32_t y = (x | (x >> 4)) & 0x00FF00FFu;
    return (y & 0xFFu) | (y >> 8);
}
// bit 7 of byte i of w -> bit i
__device__ __forceinline__ uint32_t nib7(uint32_t w) {
    const uint32_t x = (w >> 7) & 0x01010101u;
    return (x | (x >> 7) | (x >> 14) | (x >> 21)) & 0xFu;
}
// bit i of a nibble -> bit 7 of byte i
__device__ __forceinline__ uint32_t spread7(uint32_t n) { return ((n * 0x204081u) & 0x01010101u) << 7; }
// bit i of a nibble -> bit 4 i
__device__ __forceinline__ uint32_t spread4(uint32_t n) {
    return (n & 1u) | ((n & 2u) << 3) | ((n & 4u) << 6) | ((n & 8u) << 9);
}
// per-byte (x - y) mod 2^8
__device__ __forceinline__ uint32_t bsub(uint32_t x, uint32_t y) { return ((x | B7) - (y & L7)) ^ (~(x ^ y) & B7); }
// wave-wide inclusive prefix sum (DPP: row shifts, then the row broadcasts)
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}

// One direction's stale owners of one step (nm[q]: bit 7 of byte i = column c + 4 q + i) go out as records
// {column, sender max_version byte | receiver max_version byte << 16} appended in column order (lane order,
// then column) to the wave's list L (the first GS_CAND_CAP; cnt counts all), and -- from the step whose owners
// overflow the list on -- as natural-order bitmap bits, 16 per lane (the packers walk the bitmap past the
// last record).  Every lane of the wave calls this (act = false: no columns).  The bytes are decoded into
// the record's word form after the loop (p1v_decode_records): a load of the owner's own max_version here
// would make the wave wait for the loads in flight for the next step.
__device__ __forceinline__ void emit_v(uint16_t *gw16, uint2 *L, uint32_t &cnt, uint32_t c, bool act,
                                       const uint32_t (&nm)[4], const uint4 &sS, const uint4 &sR, uint32_t &alg,
                                       uint32_t (&rec)[4]) {
    const uint32_t my = act ? (uint32_t)(__popc(nm[0]) + __popc(nm[1]) + __popc(nm[2]) + __popc(nm[3])) : 0u;
    const uint32_t incl = wave_scan_dpp(my);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (act && cnt + tot > GS_CAND_CAP) {
        gw16[c >> 4] = (uint16_t)(nib7(nm[0]) | (nib7(nm[1]) << 4) | (nib7(nm[2]) << 8) | (nib7(nm[3]) << 12));
        alg += 2;
    }
    if (tot == 0u) return;
    if (my) {
        uint32_t off = cnt + incl - my;
        const uint32_t s4[4] = {sS.x, sS.y, sS.z, sS.w}, r4[4] = {sR.x, sR.y, sR.z, sR.w};
        // straight-line (at most 16 records): a loop with stores would make the compiler wait for every load
        // in flight before entering it (the loaded views it reads were loaded outside it)
#pragma unroll
        for (int q = 0; q < 4; q++) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                if ((nm[q] >> (8 * i + 7)) & 1u) {
                    if (off < GS_CAND_CAP) {
                        L[off] = make_uint2(c + 4u * q + i, ((s4[q] >> (8 * i)) & 0xFFu) | (((r4[q] >> (8 * i)) & 0xFFu) << 16));
                        rec[q] |= 0x80u << (8 * i);
                        alg += 8;
                    }
                    off++;
                }
            }
        }
    }
    cnt += tot;
}

// k_pass1v's per-column path for one lane's 16 columns (out of line: it runs for a few lanes per exchange, and
// inlined its registers would cost the byte-parallel loop its occupancy): pass1_grp's rules on decoded values
// (exact for lags < 2^8) -- the responder's +1, columns a and b, targets scheduled for deletion, the last
// partial group.  Outputs in k_pass1v's word forms.
struct P1vSlow {
    uint32_t nwA[4], nwB[4], nba[4], nab[4];
    uint32_t gba[4], gab[4];  // bit 7 of byte i: the sender's max_version is the larger (b -> a: mB > mA; a -> b)
    uint32_t pA, pB, upA, upB, hbw, reports;
};
__device__ __noinline__ P1vSlow pass1v_slow(const uint32_t *self_pk, const uint8_t *fd_state, const uint32_t *tod,
                                            uint32_t delay, uint32_t col_lo, uint32_t ncol, size_t ra, size_t rb,
                                            uint32_t c, uint32_t a, uint32_t b, uint32_t t, bool schA, bool schB,
                                            uint4 hA4, uint4 hB4, uint4 mA4, uint4 mB4, const uint32_t *esc_slot,
                                            uint16_t *esc16, uint32_t EC, const uint32_t *self_hb) {
    P1vSlow o{};
    const uint32_t x4[4] = {hA4.x, hA4.y, hA4.z, hA4.w}, y4[4] = {hB4.x, hB4.y, hB4.z, hB4.w};
    const uint32_t ma4[4] = {mA4.x, mA4.y, mA4.z, mA4.w}, mb4[4] = {mB4.x, mB4.y, mB4.z, mB4.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t c0 = c + 4u * q;
        const uint4 pk = *reinterpret_cast<const uint4 *>(self_pk + c0);
        const uint32_t pk4[4] = {pk.x, pk.y, pk.z, pk.w};
        uint32_t es4[4] = {NONE, NONE, NONE, NONE};  // escaped columns: 16-bit views in their slots
        if (EC) {
            const uint4 e = *reinterpret_cast<const uint4 *>(esc_slot + c0);
            es4[0] = e.x; es4[1] = e.y; es4[2] = e.z; es4[3] = e.w;
        }
        uint32_t oA = 0u, oB = 0u, rA = 0u, rB = 0u, bA = 0u, bB = 0u, gA = 0u, gB = 0u;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t j = c0 + i, jg = col_lo + j;
            const bool valid = j < ncol;
            // scheduled for deletion (only in rows whose earliest scheduled tick has passed): not in the digest
            const bool sa = schA && valid && (fd_state[ra + j] & FD_MEMB) == FD_DEAD && is_sched(tod[ra + j], t, delay);
            const bool sb = schB && valid && (fd_state[rb + j] & FD_MEMB) == FD_DEAD && is_sched(tod[rb + j], t, delay);
            const uint32_t Rx = pk4[i] & 0xFFFFu, M = pk4[i] >> 16;
            const uint32_t es = es4[i];
            const size_t eA = (size_t)a * EC + es, eB = (size_t)b * EC + es;
            uint32_t hA, hB;
            if (es != NONE) {  // decoded against the full own heartbeat: the stores below keep its low 16 bits
                const uint32_t R = self_hb[j];
                hA = hb_dec(esc16[eA], R);
                hB = hb_dec(esc16[eB], R);
            } else {
                hA = hb_dec8((x4[q] >> (8 * i)) & 0xFFu, Rx);
                hB = hb_dec8((y4[q] >> (8 * i)) & 0xFFu, Rx);
            }
            const uint32_t mA = mv_dec8((ma4[q] >> (8 * i)) & 0xFFu, M) & MV_MASK;
            const uint32_t mB = mv_dec8((mb4[q] >> (8 * i)) & 0xFFu, M) & MV_MASK;
            const bool isb = valid && jg == b;
            hB += isb ? 1u : 0u;  // responder inc_heartbeat (server.py:524)
            const bool upB = valid && !sa && jg != b && hA > hB;  // b merges a's digest (server.py:336-337)
            const bool repB = upB && hB != 0u;                   // state.py:280-287
            hB = upB ? hA : hB;
            const bool upA = valid && !sb && jg != a && hB > hA;  // then a merges b's (server.py:340, 356-357)
            const bool repA = upA && hA != 0u;
            hA = upA ? hB : hA;
            if (es != NONE) {
                if (upA) esc16[eA] = (uint16_t)hA;
                if (upB || isb) esc16[eB] = (uint16_t)hB;
            }
            oA |= (hA & 0xFFu) << (8 * i);
            oB |= (hB & 0xFFu) << (8 * i);
            o.upA |= (uint32_t)upA;
            o.upB |= (uint32_t)(upB || isb);
            o.hbw += (uint32_t)upA + (uint32_t)upB + (uint32_t)isb;
            rA |= (uint32_t)repA << i;
            rB |= (uint32_t)repB << i;
            o.reports += (uint32_t)repA + (uint32_t)repB;
            // stale owners (state.py:347-357) against each side's digest
            bA |= (uint32_t)(valid && !sb && mB > (sa ? 0u : mA)) << (8 * i + 7);  // b -> a
            bB |= (uint32_t)(valid && !sa && mA > (sb ? 0u : mB)) << (8 * i + 7);  // a -> b
            gA |= (uint32_t)(mB > mA) << (8 * i + 7);
            gB |= (uint32_t)(mA > mB) << (8 * i + 7);
        }
        o.gba[q] = gA;
        o.gab[q] = gB;
        o.nwA[q] = oA;
        o.nwB[q] = oB;
        o.nba[q] = bA;
        o.nab[q] = bB;
        o.pA |= spread4(rA) << q;
        o.pB |= spread4(rB) << q;
    }
    return o;
}

struct V16 {
    uint4 hA, hB, mA, mB;
    uint32_t fl;  // GS_R_P1FLAGS word of the group: small bits | hot bits << 16
};

// Slow groups taken ahead of the loop (one per lane): the loop itself then holds no call.  A call in the loop
// makes the wave spill and reload around it, and the waits for those reloads where the two paths join drain
// the loads in flight for the next step on every step, slow or not.
constexpr uint32_t P1V_K = WAVE;
constexpr uint32_t P1V_SLOT = 17;  // words per slow group: planes (pA | pB << 16), nba[4], nab[4], gba[4], gab[4]
constexpr uint32_t P1V_SCAN = 128; // flag words per lane the scan takes (4 mask words): up to 8192 groups a wave

// The records' max_version bytes -> the word form every consumer reads (emit_v stores the bytes)
__device__ __forceinline__ void p1v_decode_records(const Dev &d, uint2 *L, uint32_t cnt, int lane) {
    const uint32_t m = min(cnt, GS_CAND_CAP);
    for (uint32_t i0 = 0; i0 < m; i0 += 4u * WAVE) {
        uint2 r[4];
        uint32_t M[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + (uint32_t)(u * WAVE + lane);
            r[u] = i < m ? L[i] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < 4; u++) M[u] = i0 + (uint32_t)(u * WAVE + lane) < m ? d.self_mv[r[u].x] : 0u;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + (uint32_t)(u * WAVE + lane);
            if (i < m) L[i].y = mv_dec8(r[u].y & 0xFFu, M[u]) | (mv_dec8((r[u].y >> 16) & 0xFFu, M[u]) << 16);
        }
    }
}

// k_lite's work for one (exchange, direction) slot (also run at the head of k_settle<LITE = true>, the sliced
// phases' fused kernels); returns the slot's flag (slot_stat[slot].w, written here too)
template <int MODE>
__device__ __forceinline__ uint32_t lite_slot(const Dev &d, int32_t ai, int32_t bi, uint32_t n, uint32_t t,
                                              const SliceIO &io, size_t slot, int wid, int lane) {
    const uint32_t rcv = wid == 0 ? (uint32_t)ai : (uint32_t)bi;
    const bool sched = t >= d.row[rcv * 4 + 2];  // the receiver's digest may leave owners out: checked per record
    WStats st{0, 0, 0, 0, 0};
    uint32_t T = 0, flag = LITE_FULL;
    if (MODE == 0) {
        if (pack_lite<true>(d, rcv, slot, 0u, st, T, nullptr, sched, t)) {
            flag = LITE_DONE;
            if (lane == 0) shard_add(d, C_DBYTES, T);
        }
    } else if (MODE == 1) {
        uint32_t m1 = NONE;
        if (pack_lite<false>(d, rcv, slot, 0u, st, T, &m1, sched, t)) {
            flag = 0u;
            const uint32_t kv = (uint32_t)wave_sum(st.kvs);  // for step 0 (MODE 2): it applies without re-sizing
            if (lane == 0) {
                io.tot[slot] = tot_word(T, m1);
                d.slot_stat[slot].y = kv;
            }
            st.kvs = 0u;  // counted when sent (MODE 2 or the exact packer)
        }
    } else {
        unsigned long long P = 0;
        for (uint32_t g = 0; g < d.shard; g++) P += GS_TOT_BYTES(io.tot_all[(size_t)g * n * 2 + slot]);
        const unsigned long long own = GS_TOT_BYTES(io.tot_all[(size_t)d.shard * n * 2 + slot]);
        // the count pass (MODE 1) sized this slot from the version log (slot_stat flag 0): apply only
        const uint4 ss = d.slot_stat[slot];
        if (P + own <= d.mtu && ss.w == 0u) {  // (the count pass checked a scheduled receiver's records)
            lite_apply(d, rcv, slot, st);
            if (lane == 0) st.kvs = ss.y;
            T = (uint32_t)own;
        }
        if (P + own <= d.mtu && (ss.w == 0u || pack_lite<true>(d, rcv, slot, (uint32_t)P, st, T, nullptr, sched, t))) {
            flag = LITE_DONE;
            const uint32_t S = (uint32_t)P + T;  // every NodeDelta whole: pack_group's state after the last one
            const bool stop = S >= d.mtu || d.mtu - S < d.lb_min;
            if (lane == 0) {
                shard_add(d, C_DBYTES, T);
                io.chain[slot] = (uint64_t)S | ((uint64_t)stop << 33);
            }
        }
    }
    if (lane == 0) {
        d.slot_stat[slot].w = flag;
        if (flag == LITE_DONE) shard_add(d, C_LITE, 1);
        // a heavy slot (Dev::heavy): listed for k_pack_heavy, which runs beside k_pack_slice
        if (MODE == 0 && flag == LITE_FULL && d.heavy && d.cand_n[slot * 2] + d.cand_n[slot * 2 + 1] > d.heavy_t) {
            d.heavy[1u + atomicAdd(d.heavy, 1u)] = (uint32_t)slot;
            shard_add(d, C_HEAVY, 1);
        }
    }
    const unsigned long long s_alg = wave_sum(st.alg), s_nd = wave_sum(st.nd), s_kv = wave_sum(st.kvs);
    const unsigned long long s_cd = wave_sum(st.cand);
    if (lane == 0) {
        shard_add(d, C_ALG, s_alg);
        shard_add(d, C_PACKB, s_alg);
        shard_add(d, C_LITEB, s_alg);  // k_lite's share of pack_bytes (its own roofline entry)
        shard_add(d, C_ND, s_nd);
        shard_add(d, C_KVS, s_kv);
        shard_add(d, C_CAND, s_cd);
    }
    return flag;
}

// LM >= 0: k_lite's slot work (lite_slot<LM>: 0 = one slice, 1 = a sliced count pass) runs in the same workgroup
// after the stream, wave w taking direction w -- no k_lite launch (round 5; env GS_P1LITE=0: the launch of its own)
template <int AHEAD, int LM, bool GRP = false>
__global__ __launch_bounds__(XB, P1V_WAVES) void k_pass1v(Dev d, const int32_t *ini, const int32_t *res, uint32_t n,
                                                          uint32_t t, uint32_t seq, SliceIO io, const GroupArgs *ga,
                                                          DevDyn dyn) {
    static_assert(AHEAD == 1, "k_pass1v double-buffers one group ahead (r4g: two ahead at 5 waves per SIMD, no faster)");
    __shared__ uint32_t s_col[XB / WAVE][P1V_K];
    __shared__ uint32_t s_out[XB / WAVE][P1V_K * P1V_SLOT];
    const uint32_t e = blockIdx.x;
    if (e >= n) return;
    if constexpr (GRP) {  // a slice of an in-process group (blockIdx.y; its own instantiation: the Dev copy
        group_pick(d, ga, dyn);  // costs the single-handle kernel nothing)
        io = ga->io[blockIdx.y];
    }
    // wid through readfirstlane: the half bounds, list and plane pointers derived from it stay scalar
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int32_t ai = ini[e], bi = res[e];
    if (ai < 0 || bi < 0 || (uint32_t)ai >= d.N || (uint32_t)bi >= d.N || ai == bi) {
        if (tid == 0) shard_add(d, C_E_IDX, 1);
        if (LM >= 0 && lane == 0) d.slot_stat[(size_t)e * 2 + wid].w = LITE_DONE;  // (as k_lite: counted already)
        return;
    }
    const uint32_t a = (uint32_t)ai, b = (uint32_t)bi;
    if (tid == 0) {
        const uint32_t oa = atomicMax(&d.stamp[a], seq), ob = atomicMax(&d.stamp[b], seq);
        if (oa == seq || ob == seq) shard_add(d, C_E_CONFLICT, 1);
    }
    const uint4 rowA = *reinterpret_cast<const uint4 *>(d.row + (size_t)a * 4);
    const uint4 rowB = *reinterpret_cast<const uint4 *>(d.row + (size_t)b * 4);
    const bool schA = t >= rowA.z, schB = t >= rowB.z;
    // the whole exchange on the per-column path: a row that may hold a target scheduled for deletion, or a hot row
    const bool rslow = schA || schB || ((rowA.w | rowB.w) & 4u);
    const size_t ra = (size_t)a * d.NP, rb = (size_t)b * d.NP;
    const uint32_t words = d.NP / 32;
    uint16_t *gBA = reinterpret_cast<uint16_t *>(d.sbits + (size_t)e * 2 * words), *gAB = gBA + 2 * words;
    // wave w streams row half w (columns [w H, min((w + 1) H, ncol)), H a multiple of 1024): its candidate lists
    // hold that half in column order, and the packer reads half 0's list, then half 1's
    const uint32_t H = half_cols(d);
    const uint32_t lo = (uint32_t)wid * H, hi = min(lo + H, d.ncol);
    uint2 *LBA = d.cand + ((size_t)e * 4 + 0 * 2 + wid) * GS_CAND_CAP;
    uint2 *LAB = d.cand + ((size_t)e * 4 + 1 * 2 + wid) * GS_CAND_CAP;
    uint32_t nBAc = 0, nABc = 0, alg = 0, reports = 0, hbw = 0;
    const uint32_t ph = d.vt - d.v_round - 1u;  // this phase's plane (host-checked: < NPL)
    if (ph >= NPL) {  // (never: plane_slot checks it; a guard, so that a host bug cannot write past the planes)
        if (tid == 0) shard_add(d, C_E_IDX, 1);
        return;
    }
    uint16_t *planeA = reinterpret_cast<uint16_t *>(d.pend + ((size_t)a * NPL + ph) * d.PW);
    uint16_t *planeB = reinterpret_cast<uint16_t *>(d.pend + ((size_t)b * NPL + ph) * d.PW);
    if (tid == 0) {
        d.pstamp[a * NPL + ph] = d.vt;
        d.pstamp[b * NPL + ph] = d.vt;
    }
    const uint32_t ja = a - d.col_lo, jb = b - d.col_lo;  // this slice's columns of a and b (>= ncol: not here)
    // responder inc_heartbeat (server.py:524): the owner's own heartbeat is raised here (the per-column path
    // decodes against it, R or R + 1 alike); the view hb[b][b] in the loop; the small bit after the phase
    if (tid == 0 && jb < d.ncol) {
        const uint32_t R1 = d.self_hb[jb] + 1u;
        d.self_hb[jb] = R1;
        d.self_pk[jb] = self_pack(R1, d.self_mv[jb]);
    }
    const uint8_t *h8 = reinterpret_cast<const uint8_t *>(d.hb), *m8 = reinterpret_cast<const uint8_t *>(d.mv);
    uint8_t *hw8 = reinterpret_cast<uint8_t *>(d.hb), *mw8 = reinterpret_cast<uint8_t *>(d.mv);
    const bool hbst = !(d.ablate & 2u), spec = d.spec != 0u;
    auto load = [&](uint32_t c, V16 &v) {
        if (P1V_NT) {  // (A/B) the rows streamed non-temporally
            const v4u_t x0 = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(h8 + ra + c));
            const v4u_t x1 = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(h8 + rb + c));
            const v4u_t x2 = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(m8 + ra + c));
            const v4u_t x3 = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(m8 + rb + c));
            v.hA = make_uint4(x0.x, x0.y, x0.z, x0.w);
            v.hB = make_uint4(x1.x, x1.y, x1.z, x1.w);
            v.mA = make_uint4(x2.x, x2.y, x2.z, x2.w);
            v.mB = make_uint4(x3.x, x3.y, x3.z, x3.w);
        } else {
            v.hA = *reinterpret_cast<const uint4 *>(h8 + ra + c);
            v.hB = *reinterpret_cast<const uint4 *>(h8 + rb + c);
            v.mA = *reinterpret_cast<const uint4 *>(m8 + ra + c);
            v.mB = *reinterpret_cast<const uint4 *>(m8 + rb + c);
        }
        v.fl = d.p1flags[c >> 4];
    };
    // the per-column path's predicate for the group at column c (c < hi)
    auto slow_at = [&](uint32_t c, uint32_t fl) {
        return rslow || (fl >> 16) || c + 16u > d.ncol || ja - c < 16u || jb - c < 16u;
    };
    auto slow_group = [&](uint32_t c, const V16 &v) {
        const P1vSlow o = pass1v_slow(d.self_pk, d.fd_state, d.tod, d.sched_delay, d.col_lo, d.ncol, ra, rb, c, a, b,
                                      t, schA, schB, v.hA, v.hB, v.mA, v.mB, d.esc_slot, d.esc16, d.EC, d.self_hb);
        if (hbst) {
            if (o.upA) *reinterpret_cast<uint4 *>(hw8 + ra + c) = make_uint4(o.nwA[0], o.nwA[1], o.nwA[2], o.nwA[3]);
            if (o.upB) *reinterpret_cast<uint4 *>(hw8 + rb + c) = make_uint4(o.nwB[0], o.nwB[1], o.nwB[2], o.nwB[3]);
        }
        alg += 64u + (o.upA ? 16u : 0u) + (o.upB ? 16u : 0u);
        hbw += o.hbw;
        reports += o.reports;
        return o;
    };

    // Slow-group scan (not for a whole-slow exchange): lane l reads the flag words of the wave's groups
    // [l CH, (l + 1) CH) (column order = lane order, then group), the slow groups are ranked by a wave scan
    // and, if at most P1V_K, run now, one per lane, their outputs kept in LDS in column order
    const uint32_t G = hi > lo ? (hi - lo + 15u) / 16u : 0u;
    const uint32_t CH = ((G + WAVE - 1u) / WAVE + 3u) & ~3u;
    bool table = false;
    if (!rslow) {
        table = CH <= P1V_SCAN && !(d.ablate & 8u);
        uint32_t msk[P1V_SCAN / 32] = {0u, 0u, 0u, 0u}, cnt = 0u;
        const uint32_t g0 = (uint32_t)lane * CH;
        if (table) {
            // branch-free: the hot groups from the flag words, then the groups of columns a and b and the
            // partial last group by index; bits past the lane's chunk or the half are cleared
            const uint32_t gmax4 = (G - 1u) & ~3u;  // loads past the lane's groups stay inside the wave's words
            const uint32_t nv = G > g0 ? min(CH, G - g0) : 0u;  // the lane's groups
            const uint32_t sp[3] = {ja - lo, jb - lo, (d.ncol & 15u) ? (d.ncol & ~15u) - lo : NONE};
#pragma unroll
            for (int w = 0; w < (int)(P1V_SCAN / 32); w++) {
                if (32u * w >= CH) break;  // wave-uniform
                uint4 f[8];
#pragma unroll
                for (int j = 0; j < 8; j++)
                    f[j] = *reinterpret_cast<const uint4 *>(d.p1flags + (lo >> 4) + min(g0 + 32u * w + 4u * j, gmax4));
                uint32_t m = 0u;
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    m |= (uint32_t)(f[j].x > 0xFFFFu) << (4 * j);
                    m |= (uint32_t)(f[j].y > 0xFFFFu) << (4 * j + 1);
                    m |= (uint32_t)(f[j].z > 0xFFFFu) << (4 * j + 2);
                    m |= (uint32_t)(f[j].w > 0xFFFFu) << (4 * j + 3);
                }
#pragma unroll
                for (int u = 0; u < 3; u++) {  // column offsets from lo -> group index within this block
                    const uint32_t k = (sp[u] >> 4) - g0 - 32u * w;
                    if (sp[u] < hi - lo && k < 32u) m |= 1u << k;
                }
                const uint32_t r = nv > 32u * w ? nv - 32u * w : 0u;
                m &= r >= 32u ? ~0u : (1u << r) - 1u;
                msk[w] = m;
                cnt += (uint32_t)__popc(m);
            }
        }
        const uint32_t incl = wave_scan_dpp(cnt);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        table = table && tot <= P1V_K;
        if (table) {
            uint32_t off = incl - cnt;
#pragma unroll
            for (int w = 0; w < (int)(P1V_SCAN / 32); w++)
                for (uint32_t m = msk[w]; m; m &= m - 1u) s_col[wid][off++] = lo + 16u * (g0 + 32u * w + (uint32_t)__builtin_ctz(m));
        }
        __syncthreads();
        if (table && (uint32_t)lane < tot) {
            const uint32_t c = s_col[wid][lane];
            V16 v;
            load(c, v);
            const P1vSlow o = slow_group(c, v);
            uint32_t *so = &s_out[wid][lane * P1V_SLOT];
            so[0] = o.pA | (o.pB << 16);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                so[1 + q] = o.nba[q];
                so[5 + q] = o.nab[q];
                so[9 + q] = o.gba[q];
                so[13 + q] = o.gab[q];
            }
        }
        __syncthreads();
    }

    // The stream: two buffers, the next group's loads issued before the current group is computed.  TABLE:
    // slow groups read their outputs from the scan's slots (no call in the loop); else they run the per-column
    // path here (a whole-slow exchange, or more slow groups than slots).
    constexpr uint32_t STEP = WAVE * 16u;
    const uint32_t clast = (max(hi, 1u) - 1u) & ~15u;  // the wave's last group (a valid one for an empty half)
    auto stream = [&](auto tag) {
        constexpr bool TABLE = decltype(tag)::value;
        uint32_t sbase = 0u;  // slow groups of the wave before this step (TABLE)
        auto step = [&](uint32_t s0, const V16 &v, V16 &nx) __attribute__((always_inline)) {
            const uint32_t c = s0 + (uint32_t)lane * 16u;
            const bool act = c < hi;
            // unconditional (a lane past the end reloads the last group): a load under a branch would make
            // the wait for the current group's loads count as if the next group's were not in flight
            load(c + STEP < hi ? c + STEP : clast, nx);
            const uint32_t x4[4] = {v.hA.x, v.hA.y, v.hA.z, v.hA.w}, y4[4] = {v.hB.x, v.hB.y, v.hB.z, v.hB.w};
            const uint32_t ma4[4] = {v.mA.x, v.mA.y, v.mA.z, v.mA.w}, mb4[4] = {v.mB.x, v.mB.y, v.mB.z, v.mB.w};
            uint32_t nba[4] = {0u, 0u, 0u, 0u}, nab[4] = {0u, 0u, 0u, 0u};
            uint32_t gba[4], gab[4];    // the sender's view is the larger (Dev::spec; the fast path's stale masks)
            uint32_t pA = 0u, pB = 0u;  // the lane's plane u16s
            const bool slow = act && slow_at(c, v.fl);
            if (act && !slow) {
                uint32_t repA[4], repB[4], nw[4], upAll = 0u, upBll = 0u;
                const uint32_t sm = v.fl & 0xFFFFu;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t x = x4[q], y = y4[q];
                    const uint32_t dd = bsub(x, y);  // (hA - hB) mod 2^8, |hA - hB| < 2^7
                    const uint32_t upA = dd & B7;    // hB > hA: a takes b's heartbeat
                    const uint32_t upB = ((((dd & L7) + L7) | dd) & ~dd) & B7;  // hA > hB: b takes a's
                    const uint32_t mA_ = (upA << 1) - (upA >> 7);
                    nw[q] = (y & mA_) | (x & ~mA_);  // both rows end with the larger heartbeat
                    // _report_heartbeat reports unless the old heartbeat was 0 (state.py:280-287)
                    const uint32_t s7 = sm ? spread7((sm >> (4 * q)) & 0xFu) : 0u;
                    const uint32_t zA = ~(((x & L7) + L7) | x) & B7, zB = ~(((y & L7) + L7) | y) & B7;
                    repA[q] = upA & ~(zA & s7);
                    repB[q] = upB & ~(zB & s7);
                    upAll |= upA;
                    upBll |= upB;
                    hbw += (uint32_t)__popc(upA | upB);
                    // stale owners (state.py:347-357): mB > mA -> b -> a, mA > mB -> a -> b; |mA - mB| < 2^6
                    const uint32_t ev = (((mb4[q] & L7) | B7) - (ma4[q] & L7)) & L7;  // (mB - mA) mod 2^7
                    const uint32_t e6 = (ev << 1) & B7;
                    nba[q] = (ev + L7) & B7 & ~e6;
                    nab[q] = e6;
                }
                if (P1V_LINE) {  // whole lines (the unchanged lanes' bytes are their rows' own)
                    upAll = line_any_v(upAll != 0u) ? 1u : 0u;
                    upBll = line_any_v(upBll != 0u) ? 1u : 0u;
                }
                if (hbst) {
                    if (P1V_NT) {
                        if (upAll) __builtin_nontemporal_store(v4u_t{nw[0], nw[1], nw[2], nw[3]}, reinterpret_cast<v4u_t *>(hw8 + ra + c));
                        if (upBll) __builtin_nontemporal_store(v4u_t{nw[0], nw[1], nw[2], nw[3]}, reinterpret_cast<v4u_t *>(hw8 + rb + c));
                    } else {
                        if (upAll) *reinterpret_cast<uint4 *>(hw8 + ra + c) = make_uint4(nw[0], nw[1], nw[2], nw[3]);
                        if (upBll) *reinterpret_cast<uint4 *>(hw8 + rb + c) = make_uint4(nw[0], nw[1], nw[2], nw[3]);
                    }
                }
                alg += 64u + (upAll ? 16u : 0u) + (upBll ? 16u : 0u);
                pA = pack16(repA);
                pB = pack16(repB);
                reports += (uint32_t)(__popc(pA) + __popc(pB));
            }
            if constexpr (TABLE) {
                const uint64_t sm = __ballot(slow);
                if (slow) {
                    const uint32_t slot = sbase + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                    const uint32_t *so = &s_out[wid][slot * P1V_SLOT];
                    pA = so[0] & 0xFFFFu;
                    pB = so[0] >> 16;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        nba[q] = so[1 + q];
                        nab[q] = so[5 + q];
                        gba[q] = so[9 + q];
                        gab[q] = so[13 + q];
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        gba[q] = nba[q];
                        gab[q] = nab[q];
                    }
                }
                sbase += (uint32_t)__popcll(sm);
            } else if (slow) {
                const P1vSlow o = slow_group(c, v);
                pA = o.pA;
                pB = o.pB;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    nba[q] = o.nba[q];
                    nab[q] = o.nab[q];
                    gba[q] = o.gba[q];
                    gab[q] = o.gab[q];
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    gba[q] = nba[q];
                    gab[q] = nab[q];
                }
            }
            if (act) {
                planeA[c >> 4] = (uint16_t)pA;
                planeB[c >> 4] = (uint16_t)pB;
                alg += 4;
            }
            uint32_t rBA[4] = {0u, 0u, 0u, 0u}, rAB[4] = {0u, 0u, 0u, 0u};  // recorded stale owners
            emit_v(gBA, LBA, nBAc, c, act, nba, v.mB, v.mA, alg, rBA);  // b -> a: sender b, receiver a
            emit_v(gAB, LAB, nABc, c, act, nab, v.mA, v.mB, alg, rAB);
            if (spec && act) {
                // speculative merge (Dev::spec): each recorded stale owner whose two views are prefix views
                // (GS_MV_INEXACT clear: bit 7 of both bytes) gets the sender's view now, in the 16 bytes this
                // step loaded -- a delta that fits sends every such NodeDelta whole, which is exactly that
                // (apply_cand's fast path); the packer restores the receiver byte of the others (pack_list)
                uint32_t nA[4], nB[4], wA = 0u, wB = 0u;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t fm = ~(ma4[q] | mb4[q]) & B7;
                    const uint32_t ba = rBA[q] & fm & gba[q], ab = rAB[q] & fm & gab[q];  // max(ms, mr)
                    const uint32_t sA = (ba << 1) - (ba >> 7), sB = (ab << 1) - (ab >> 7);  // byte masks
                    nA[q] = (mb4[q] & sA) | (ma4[q] & ~sA);
                    nB[q] = (ma4[q] & sB) | (mb4[q] & ~sB);
                    wA |= ba;
                    wB |= ab;
                }
                if (P1V_LINE) {  // whole lines: a partial line costs the memory a read-modify-write
                    wA = line_any_v(wA != 0u);
                    wB = line_any_v(wB != 0u);
                }
                if (wA) {
                    if (P1V_NT) __builtin_nontemporal_store(v4u_t{nA[0], nA[1], nA[2], nA[3]}, reinterpret_cast<v4u_t *>(mw8 + ra + c));
                    else *reinterpret_cast<uint4 *>(mw8 + ra + c) = make_uint4(nA[0], nA[1], nA[2], nA[3]);
                    alg += 16;
                }
                if (wB) {
                    if (P1V_NT) __builtin_nontemporal_store(v4u_t{nB[0], nB[1], nB[2], nB[3]}, reinterpret_cast<v4u_t *>(mw8 + rb + c));
                    else *reinterpret_cast<uint4 *>(mw8 + rb + c) = make_uint4(nB[0], nB[1], nB[2], nB[3]);
                    alg += 16;
                }
            }
        };
        // two buffers in turn (the loop unrolled by two steps: no register moves)
        V16 b0, b1;
        load(min(lo + (uint32_t)lane * 16u, clast), b0);
        for (uint32_t s0 = lo; s0 < hi; s0 += 2u * STEP) {  // wave-uniform trip count (the scans need every lane)
            step(s0, b0, b1);
            if (s0 + STEP < hi) step(s0 + STEP, b1, b0);
        }
    };
    if (table)
        stream(std::true_type{});
    else
        stream(std::false_type{});
    // this wave's records: bytes -> words (its own stores: visible to the wave after the fence)
    __threadfence_block();
    p1v_decode_records(d, LBA, nBAc, lane);
    p1v_decode_records(d, LAB, nABc, lane);
    if (lane == 0) {
        d.cand_n[(size_t)e * 4 + 0 * 2 + wid] = nBAc;
        d.cand_n[(size_t)e * 4 + 1 * 2 + wid] = nABc;
    }
    const unsigned long long s_alg = wave_sum(alg), s_rep = wave_sum(reports), s_hbw = wave_sum(hbw);
    if (lane == 0) {
        shard_add(d, C_ALG, s_alg);
        shard_add(d, C_REPORTS, s_rep);
        shard_add(d, C_HBW, s_hbw);
        if (wid == 0 && d.shard == 0) shard_add(d, C_EXCH, 1);  // slices: every slice runs every exchange
    }
    if constexpr (LM >= 0) {
        // both halves' records (and counts) are final after the barrier (one CU: workgroup-scope visibility);
        // wave w sizes / completes direction w (0: the SynAck delta b -> a, 1: the Ack delta a -> b) as k_lite
        // would, while the other workgroups on the CU stream their rows
        __syncthreads();
        lite_slot<LM>(d, ai, bi, n, t, io, (size_t)e * 2 + wid, wid, lane);
    }
}
// After a k_pass1v phase: the responders' small bits (their own heartbeat rose by one in the phase; pass 1
// read the bits as they were before it, consistently for every exchange of the phase)
__device__ __forceinline__ void p1v_fix_one(const Dev &d, const int32_t *res, uint32_t e) {
    const uint32_t jb = (uint32_t)res[e] - d.col_lo;
    if ((uint32_t)res[e] < d.N && jb < d.ncol) set_small(d, jb, d.self_hb[jb]);
}
__global__ __launch_bounds__(LB) void k_p1v_fix(Dev d, const int32_t *res, uint32_t n) {
    const uint32_t e = blockIdx.x * LB + threadIdx.x;
    if (e >= n) return;
    p1v_fix_one(d, res, e);
}

// MODE 0: the whole exchange (one slice).  MODE 1: sharded count pass (pass 1, then the slice totals).
template <int KW, bool GENM, int MODE>
__global__ __launch_bounds__(XB, (KW == 4 ? XB_WAVES : 1)) void k_exchange(Dev d, const int32_t *ini, const int32_t *res, uint32_t n,
                                                 uint32_t t, uint32_t seq, SliceIO io) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t e = blockIdx.x;
    if (e >= n) return;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid >> 6;
    const int32_t ai = ini[e], bi = res[e];
    if (ai < 0 || bi < 0 || (uint32_t)ai >= d.N || (uint32_t)bi >= d.N || ai == bi) {
        if (tid == 0) shard_add(d, C_E_IDX, 1);
        return;
    }
    const uint32_t a = (uint32_t)ai, b = (uint32_t)bi;
    constexpr bool genm = GENM;
    const uint32_t words = d.NP / 32;
    // LDS: WIN-entry compaction list per wave, then the stale-owner bitmaps (+ insertion bitmaps)
    uint16_t *wbuf = reinterpret_cast<uint16_t *>(lds) + wid * WIN;
    uint32_t *bm = lds + WIN;  // after the two waves' WIN x u16 candidate lists
    uint32_t *bBA = bm, *bAB = bm + words, *bNB = bm + 2 * words, *bNA = bm + 3 * words;
    for (uint32_t i = tid; i < words * (genm ? 4u : 2u); i += XB) bm[i] = 0u;
    // pass 1's "some owner is new to a side" flag: the last word of wave 1's candidate list, which
    // wave 1 only writes in pass 3, after reading the flag (no static LDS: see below)
    uint32_t *s_new = lds + WIN - 1;
    if (tid == 0) {
        *s_new = 0u;
        const uint32_t oa = atomicMax(&d.stamp[a], seq), ob = atomicMax(&d.stamp[b], seq);
        if (oa == seq || ob == seq) shard_add(d, C_E_CONFLICT, 1);
    }
    const uint32_t cntA0 = genm ? d.row[a * 4 + 0] : d.ncol;
    const uint32_t cntB0 = genm ? d.row[b * 4 + 0] : d.ncol;
    const bool schA = t >= d.row[a * 4 + 2];
    const bool schB = t >= d.row[b * 4 + 2];
    __syncthreads();

    // ---- pass 1: Syn at a, heartbeat merge at b, SynAck digest, heartbeat merge at a
    const size_t ra = (size_t)a * d.NP, rb = (size_t)b * d.NP;
    uint32_t alg = 0, reports = 0, hbw = 0;
    bool anynew = false;
    const uint32_t ph = d.vt - d.v_round - 1u;  // phase of this round (host-checked: < NPL)
    if (ph >= NPL) {  // (never: plane_slot checks it; a guard, so that a host bug cannot write past the planes)
        if (tid == 0) shard_add(d, C_E_IDX, 1);
        return;
    }
    uint64_t *planeA = d.pend + ((size_t)a * NPL + ph) * d.PW;
    uint64_t *planeB = d.pend + ((size_t)b * NPL + ph) * d.PW;
    if (tid == 0) {  // both plane rows are rewritten below: valid for this phase
        d.pstamp[a * NPL + ph] = d.vt;
        d.pstamp[b * NPL + ph] = d.vt;
    }
    // software-pipelined: the next group's loads are in flight while this group computes and stores
    // (different owners, so the early loads never read a location this group writes)
    uint32_t c0 = (uint32_t)tid * 4u;
    GrpRaw r0, r1;
    if (c0 < d.ncol) load_grp<GENM>(d, ra, rb, c0, t, schA, schB, r0);
    while (c0 < d.ncol) {
        const uint32_t c1 = c0 + XB * 4u;
        if (c1 < d.ncol) load_grp<GENM>(d, ra, rb, c1, t, schA, schB, r1);
        Grp g0;
        dec_grp(r0, g0);
        uint32_t rmA, rmB, nBA, nAB, nNB, nNA;
        pass1_grp<GENM>(d, ra, rb, c0, a, b, t, schA, schB, g0, nBA, nAB, nNB, nNA, alg, reports, hbw, rmA, rmB);
        // one LDS atomic per lane and bitmap (4 consecutive columns sit in one word); stale owners are sparse
        const uint32_t sh = c0 & 31u;
        if (nBA) atomicOr(&bBA[c0 >> 5], nBA << sh);
        if (nAB) atomicOr(&bAB[c0 >> 5], nAB << sh);
        if (nNB) { atomicOr(&bNB[c0 >> 5], nNB << sh); anynew = true; }
        if (nNA) { atomicOr(&bNA[c0 >> 5], nNA << sh); anynew = true; }
        if (!(d.ablate & 2u)) {
            store_plane(planeA, c0, rmA, alg);
            store_plane(planeB, c0, rmB, alg);
        }
        r0 = r1;
        c0 = c1;
    }
    // no static LDS: the 20 KB of dynamic LDS per workgroup (N = 65,536, canonical) then fits 8
    // workgroups = 4 waves per SIMD
    if (anynew) *s_new = 1u;
    __syncthreads();
    const bool any_new = *s_new != 0u;

    if (MODE == 1) {
        // ---- sharded count pass: publish the bitmaps, total this slice's candidates per direction
        if (any_new && tid == 0) shard_add(d, C_E_INSERT, 1);
        uint32_t *gb = d.sbits + (size_t)e * 2 * words;
        for (uint32_t i = tid; i < 2 * words; i += XB) gb[i] = bm[i];
        const bool w0 = wid == 0;
        const uint32_t snd = w0 ? b : a, rcv = w0 ? a : b;
        const DigestSide ds{rcv, d.ncol, w0 ? schA : schB};
        WStats cs{0, 0, 0, 0, 0};
        bool ctomb = false;
        PackState pst{0u, false, false};
        pack_dir<KW, false, true>(d, snd, rcv, ds, nullptr, d.ncol, w0 ? bBA : bAB, wbuf, t, cs, ctomb, pst);
        if (lane == 0) io.tot[(size_t)e * 2 + wid] = tot_word(pst.S, pst.m1);
        const unsigned long long s_alg = wave_sum(alg), s_rep = wave_sum(reports), s_hbw = wave_sum(hbw);
        if (lane == 0) {
            shard_add(d, C_ALG, s_alg);
            shard_add(d, C_REPORTS, s_rep);
            shard_add(d, C_HBW, s_hbw);
            if (wid == 0 && d.shard == 0) shard_add(d, C_EXCH, 1);
        }
        return;
    }

    // ---- pass 2: dict insertions (node_state_or_default appends in digest order)
    uint32_t cntA = cntA0, cntB = cntB0;
    if (any_new) {
        if (!genm) {
            if (tid == 0) shard_add(d, C_E_INSERT, 1);
        } else if (wid == 0) {
            uint32_t baseB = cntB0;  // b inserts in a's digest order (a's dict order at Syn time)
            for (uint32_t p0 = 0; p0 < cntA0; p0 += WAVE) {
                const uint32_t p = p0 + lane;
                const uint32_t j = p < cntA0 ? d.ord[ra + p] : NONE;
                const bool f = j != NONE && bit(bNB, j);
                const unsigned long long m = __ballot(f);
                const uint32_t rk = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (f) { d.pos[rb + j] = baseB + rk; d.ord[rb + baseB + rk] = j; }
                baseB += (uint32_t)__popcll(m);
            }
            __threadfence_block();
            uint32_t baseA = cntA0;  // a inserts in b's digest order (b's dict after its insertions)
            for (uint32_t p0 = 0; p0 < baseB; p0 += WAVE) {
                const uint32_t p = p0 + lane;
                const uint32_t j = p < baseB ? d.ord[rb + p] : NONE;
                const bool f = j != NONE && bit(bNA, j);
                const unsigned long long m = __ballot(f);
                const uint32_t rk = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                if (f) { d.pos[ra + j] = baseA + rk; d.ord[ra + baseA + rk] = j; }
                baseA += (uint32_t)__popcll(m);
            }
            if (lane == 0) {
                d.row[b * 4 + 0] = baseB;
                d.row[a * 4 + 0] = baseA;
            }
            __threadfence_block();
        }
        __syncthreads();
        if (genm) { cntB = d.row[b * 4 + 0]; cntA = d.row[a * 4 + 0]; }  // wave 0's counts (fenced above)
    }

    // ---- pass 3: SynAck delta b -> a (wave 0) and Ack delta a -> b (wave 1), each applied
    WStats st{0, 0, 0, 0, 0};
    bool tomb = false;
    if (!(d.ablate & 1u)) {
        const bool w0 = wid == 0;  // wave-uniform: one call site, so pack_dir inlines
        const uint32_t snd = w0 ? b : a, rcv = w0 ? a : b;
        const DigestSide ds{rcv, w0 ? cntA0 : cntB, w0 ? schA : schB};
        const uint32_t *ord = genm ? d.ord + (w0 ? rb : ra) : nullptr;
        PackState pst{0u, false, false};
        pack_dir<KW, GENM, false>(d, snd, rcv, ds, ord, w0 ? cntB : cntA, w0 ? bBA : bAB, wbuf, t, st, tomb, pst);
        if (tomb) d.row[rcv * 4 + 1] = 1u;
    }

    // ---- counters: wave-reduced, sharded atomics
    const unsigned long long s_alg = wave_sum((unsigned long long)alg + st.alg), s_pk = wave_sum(st.alg);
    const unsigned long long s_rep = wave_sum(reports), s_hbw = wave_sum(hbw);
    const unsigned long long s_nd = wave_sum(st.nd), s_kv = wave_sum(st.kvs), s_tr = wave_sum(st.trunc);
    const unsigned long long s_cd = wave_sum(st.cand);
    if (lane == 0) {
        shard_add(d, C_ALG, s_alg);
        shard_add(d, C_PACKB, s_pk);
        shard_add(d, C_REPORTS, s_rep);
        shard_add(d, C_HBW, s_hbw);
        shard_add(d, C_ND, s_nd);
        shard_add(d, C_KVS, s_kv);
        shard_add(d, C_TRUNC, s_tr);
        shard_add(d, C_CAND, s_cd);
        shard_max(d, C_PGMAX, st.grp);
        shard_max(d, C_PSMAX, st.stp);
        if (wid == 0) shard_add(d, C_EXCH, 1);
    }
}

// Sharded pack pass, step `io.step` (wave 0: b -> a, wave 1: a -> b).  Step 0: a slice whose
// predecessors' totals fit in the MTU starts at their sum (every one of their candidates is sent
// whole, state.py:392-398); the others wait.  Step k: a waiting slice whose predecessor has
// finished continues from the predecessor's state.  Sequential semantics over the slices in
// column (= canonical dict) order, so the result is the single-slice result bit for bit.
template <int KW>
#ifndef PK_WAVES
#define PK_WAVES 4
#endif
__global__ __launch_bounds__(XB, (KW == 4 ? PK_WAVES : 1)) void k_pack_slice(Dev d, const int32_t *ini, const int32_t *res, uint32_t n,
                                                   uint32_t t, SliceIO io, uint32_t e0) {
    __shared__ __attribute__((aligned(16))) uint16_t s_wbuf[2 * WIN];
    const uint32_t e = e0 + blockIdx.x;
    if (e >= n) return;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid >> 6;
    if (d.p1fix && tid == 0) p1v_fix_one(d, res, e);  // k_p1v_fix's work (Dev::p1fix)
    const int32_t ai = ini[e], bi = res[e];
    if (ai < 0 || bi < 0 || (uint32_t)ai >= d.N || (uint32_t)bi >= d.N || ai == bi) return;  // counted already
    const uint32_t a = (uint32_t)ai, b = (uint32_t)bi;
    const size_t slot = (size_t)e * 2 + wid;
    if (io.step == 0 && d.lite && (d.slot_stat[slot].w & LITE_DONE)) return;  // k_lite completed it
    // a heavy slot: the lite slot work listed it (Dev::heavy) and k_pack_heavy packs it
    if (d.heavy && d.cand_n[slot * 2] + d.cand_n[slot * 2 + 1] > d.heavy_t) return;
    PackState pst;
    if (io.step == 0) {
        uint64_t P = 0;
        for (uint32_t g = 0; g < d.shard; g++) P += GS_TOT_BYTES(io.tot_all[(size_t)g * n * 2 + slot]);
        if (P > d.mtu) {
            if (lane == 0) io.chain[slot] = CHAIN_PENDING;
            return;
        }
        pst = PackState{(uint32_t)P, false, false};
    } else {
        if (io.chain[slot] != CHAIN_PENDING) return;
        const uint64_t prev = io.chain_all[(size_t)(d.shard - 1) * n * 2 + slot];
        if (prev == CHAIN_PENDING) return;
        pst = chain_unpack(prev);
    }
    const bool w0 = wid == 0;
    const uint32_t snd = w0 ? b : a, rcv = w0 ? a : b;
    const DigestSide ds{rcv, d.ncol, t >= d.row[rcv * 4 + 2]};
    const uint32_t words = d.NP / 32;
    WStats st{0, 0, 0, 0, 0};
    bool tomb = false;
    if (d.cand) {
        // pass 1's candidate lists (k_pass1), half 0 then half 1; a half with more stale owners than the
        // list holds is walked in the bitmap instead
        pack_records<KW, false>(d, snd, rcv, ds, slot, s_wbuf + wid * WIN, t, st, tomb, pst);
    } else {
        pack_dir<KW, false, false>(d, snd, rcv, ds, nullptr, d.ncol, d.sbits + (slot * words), s_wbuf + wid * WIN, t,
                                   st, tomb, pst);
    }
    if (tomb) d.row[rcv * 4 + 1] = 1u;
    if (lane == 0 && io.chain) io.chain[slot] = chain_pack(pst);
    const unsigned long long s_alg = wave_sum(st.alg), s_nd = wave_sum(st.nd), s_kv = wave_sum(st.kvs);
    const unsigned long long s_tr = wave_sum(st.trunc), s_cd = wave_sum(st.cand);
    if (lane == 0) {
        shard_add(d, C_ALG, s_alg);
        shard_add(d, C_PACKB, s_alg);
        shard_add(d, C_ND, s_nd);
        shard_add(d, C_KVS, s_kv);
        shard_add(d, C_TRUNC, s_tr);
        shard_add(d, C_CAND, s_cd);
        shard_max(d, C_PGMAX, st.grp);
        shard_max(d, C_PSMAX, st.stp);
    }
}

// ---- the exact packer's heavy slots (round 6).  A slot with thousands of stale owners -- a
// node back from an absence -- kept k_pack_slice's two-wave workgroup walking for ~270 dependent steps (the launch
// lasts as long as its heaviest slot) while the others were long done.  k_pack_slice hands such slots to this
// kernel (Dev::heavy), which packs each with HW_WAVES waves, in sender order:
//  * whole-fit prefix (state.py:392-398): blocks of HT candidates are evaluated in parallel, a block scan of their
//    DeltaPb sizes finds the first one that does not fit whole, and every candidate before it is sent whole
//    (applied in parallel: distinct owners);
//  * first-fit continuation (state.py:392-413): every later candidate is tested against the budget R left, which
//    only shrinks, so one whose smallest NodeDelta (its lowest-version kv alone, min1) exceeds R now is never sent,
//    and once R is below the smallest NodeDelta of any owner (lb_min) nothing is: super-blocks of HT x HTB
//    candidates are filtered in parallel (min1_lb first, the exact min1 for those that pass), and one wave runs
//    pack_group's sequential first-fit over the survivors alone, in sender order;
//  * a speculatively merged record (Dev::spec) that is not sent gets its receiver word restored, as in pack_list.
// Bit-exact with pack_records: the same candidates, the same order, the same decisions.
#ifndef HW_WAVES
#define HW_WAVES 4
#endif
#ifndef HTB
#define HTB 8  // candidates per thread in a first-fit super-block (candidate k * HT + thread)
#endif
#ifndef HPK
#define HPK 4  // consecutive candidates per thread in a whole-fit block
#endif
constexpr int HT = HW_WAVES * WAVE;           // threads per heavy workgroup
constexpr uint32_t HSB = (uint32_t)HT * HTB;  // candidates per first-fit super-block
constexpr uint32_t HPB = (uint32_t)HT * HPK;  // candidates per whole-fit block
constexpr uint32_t HWIN = 16u * HT;           // bitmap positions compacted per window (16 per thread)
struct HeavyLds {
    uint32_t wsum[HW_WAVES];
    uint32_t wcnt[HTB][HW_WAVES];
    uint32_t first, S, stop, tail, steps, groups;
    uint16_t surv[HSB];  // first-fit survivors in sender order (offsets from the super-block's start)
    uint32_t pe[HPB];    // a whole-fit block's candidates: DeltaPb bytes | kv count << 16 | prefix views << 24
    uint16_t wl[HWIN];   // a bitmap window's stale positions (offsets from the window start)
};
// a candidate source: pass 1's records of a row half, or a compacted bitmap window (rows read for the words)
struct HSrc {
    const uint2 *L;  // records, or nullptr: the window wl at column w
    uint32_t w;
};
__device__ __forceinline__ void hsrc_get(const Dev &d, const HSrc &src, const HeavyLds &sh, uint32_t q, uint32_t s,
                                         uint32_t r, uint32_t &j, uint32_t &mvw, uint32_t &alg) {
    if (src.L) {
        const uint2 x = src.L[q];
        j = x.x;
        mvw = x.y;
        alg += 8;
    } else {
        j = src.w + sh.wl[q];
        mvw = mv_word(d, pix(d, s, j), j) | (mv_word(d, pix(d, r, j), j) << 16);
        alg += 2;
    }
}
// block-wide exclusive scan of x (all threads call); returns the exclusive prefix, *total the block's sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, HeavyLds &sh, uint32_t *total) {
    const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
    const uint32_t inc = wave_incl_scan(x);
    if (lane == WAVE - 1) sh.wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < HW_WAVES; w++) {
        const uint32_t v = sh.wsum[w];
        if (w < wv) pre += v;
        tot += v;
    }
    __syncthreads();  // (wsum is reused by the next scan)
    *total = tot;
    return pre + inc - x;
}

template <int KW>
__device__ __forceinline__ void heavy_eval(const Dev &d, uint32_t s, uint32_t r, const DigestSide &ds, uint32_t t,
                                           uint32_t j, uint32_t mvw, bool lightok, Cand<KW> &c, WStats &st) {
    c.emsg = 0;
    c.min1 = 0;
    c.light = false;
    c.fast = false;
    if (lightok && rec_fast(mvw)) {
        eval_light<KW>(d, j, mvw & MV_MASK, (mvw >> 16) & MV_MASK, c, st.alg);
    } else {
        CandKeys<KW> ck;
        eval_cand<KW, false, true>(d, s, r, ds, j, t, c, ck, st.alg, mvw);
    }
    st.cand++;
}

// whole-fit prefix: candidates [pos, pos + HPB) of src (thread i: the HPK consecutive ones from pos + i HPK, those
// < len), none of them in first-fit continuation yet.  Sends whole every candidate before the first that does not
// fit; returns how many candidates it consumed (HPB, or that first one's offset: first-fit continuation, sh.tail,
// resumes there).  Each candidate's size, kv count and prefix flag wait in LDS (sh.pe) through the scan; a sent
// prefix candidate's apply is one max_version store (none if pass 1 merged it), any other is evaluated again
template <int KW>
__device__ __forceinline__ uint32_t heavy_prefix(const Dev &d, uint32_t s, uint32_t r, const DigestSide &ds, uint32_t t,
                                                 const HSrc &src, uint32_t pos, uint32_t len, bool specd, bool lightok,
                                                 HeavyLds &sh, WStats &st, bool &tomb) {
    const int tid = (int)threadIdx.x;
    const uint32_t mtu = d.mtu, S = sh.S;
    const uint32_t q0 = pos + (uint32_t)tid * HPK;
    uint32_t *pe = sh.pe + (uint32_t)tid * HPK;
    uint32_t sum = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < HPK; k++) {
        uint32_t x = 0u;
        if (q0 + k < len) {
            uint32_t j, m;
            hsrc_get(d, src, sh, q0 + k, s, r, j, m, st.alg);
            Cand<KW> c;
            heavy_eval<KW>(d, s, r, ds, t, j, m, lightok, c, st);
            x = c.emsg | (c.nkv << 16) | (c.fast ? 1u << 24 : 0u);
            sum += c.emsg;
        }
        pe[k] = x;
    }
    uint32_t total;
    const uint32_t ex = block_excl_scan(sum, sh, &total);
    uint32_t f = HPB;  // offset (from pos) of the first candidate that does not fit whole
    if (S + total <= mtu) {
        if (tid == 0) {
            const uint32_t S1 = S + total;
            sh.S = S1;
            if (S1 >= mtu || mtu - S1 < d.lb_min) sh.stop = 1u;
        }
    } else {
        if (tid == 0) sh.first = HPB;
        __syncthreads();
        uint32_t run = S + ex;
#pragma unroll 1
        for (uint32_t k = 0; k < HPK; k++) {
            const uint32_t em = pe[k] & 0xFFFFu;
            if (em && run + em > mtu) {
                atomicMin(&sh.first, (uint32_t)tid * HPK + k);
                break;
            }
            run += em;
        }
        __syncthreads();
        f = sh.first;
        if ((uint32_t)tid == f / HPK) {  // the thread holding candidate f: the bytes before it
            uint32_t bb = S + ex;
            for (uint32_t k = 0; k < f % HPK; k++) bb += pe[k] & 0xFFFFu;
            sh.S = bb;
            sh.tail = 1u;
        }
    }
    const bool merged = specd && src.L != nullptr;  // pass 1 merged the records' receiver words (prefix views)
#pragma unroll 1
    for (uint32_t k = 0; k < HPK; k++) {
        if ((uint32_t)tid * HPK + k >= f || q0 + k >= len) break;
        const uint32_t x = pe[k], em = x & 0xFFFFu;
        const bool fast = (x >> 24) & 1u;
        if (!em && !(merged && fast)) continue;
        uint32_t j, m;
        hsrc_get(d, src, sh, q0 + k, s, r, j, m, st.alg);  // (cache-hot)
        if (!em) {  // nothing to send: restore the merge
            mv_put(d, pix(d, r, j), m >> 16);
            st.alg += 4;
            continue;
        }
        st.nd++;
        st.kvs += (x >> 16) & 0xFFu;
        if (fast && !d.ev) {  // apply_cand's fast path: the view becomes S_j(max(ms, mr)), still a prefix
            if (!merged) {
                const uint32_t ms = m & MV_MASK, mr = (m >> 16) & MV_MASK;
                mv_put(d, pix(d, r, j), ms > mr ? ms : mr);
                st.alg += 4;
            }
            continue;
        }
        Cand<KW> c;
        heavy_eval<KW>(d, s, r, ds, t, j, m, lightok, c, st);
        st.cand--;  // (evaluated twice)
        apply_cand<KW>(d, s, r, c, NONE, t, tomb, st.alg, merged);
    }
    __syncthreads();
    return f;
}

// first-fit continuation over candidates [pos, pos + HSB) of src (candidate pos + k * HT + thread, if < len), or, once
// the delta is complete (sh.stop), only the restores of the merged records among them
template <int KW>
__device__ __forceinline__ void heavy_tail(const Dev &d, uint32_t s, uint32_t r, const DigestSide &ds, uint32_t t,
                                           const HSrc &src, uint32_t pos, uint32_t len, bool specd, bool lightok,
                                           HeavyLds &sh, WStats &st, bool &tomb) {
    const int tid = (int)threadIdx.x, lane = lane_id(), wv = tid >> 6;
    uint32_t S = sh.S;
    const uint32_t R = d.mtu - S;
    // nothing fits any more (every NodeDelta is >= lb_min, and every one of owners from the next candidate's
    // column on >= Dev::sm there): the delta is complete (pack_group's rule)
    uint32_t bound = d.lb_min;
    if (d.sm && pos < len) bound = max(bound, (uint32_t)d.sm[src.L ? src.L[pos].x : src.w + sh.wl[pos]]);
    if (!sh.stop && R < bound) {
        __syncthreads();
        if (tid == 0) sh.stop = 1u;
        __syncthreads();
    }
    const bool stopped = sh.stop != 0u;
    const bool merged = specd && src.L != nullptr;
    if (stopped && !merged) return;
    // every candidate's words, and the cheap bound, loads in flight together; a merged record that cannot be sent
    // gets its receiver word back at once
    uint32_t live = 0u;  // bit k: candidate k may still be sent
#pragma unroll
    for (int k = 0; k < HTB; k++) {
        const uint32_t q = pos + (uint32_t)k * HT + (uint32_t)tid;
        if (q >= len) continue;
        uint32_t j, m;
        hsrc_get(d, src, sh, q, s, r, j, m, st.alg);
        const bool fast = rec_fast(m);
        bool can = !stopped;
        if (can && fast && d.vlog && min1_lb(d, j, m & 0xFFFFu, m >> 16, ds.sched) > R) {
            can = false;
            st.alg += 4;
        }
        if (can) live |= 1u << k;
        else if (merged && fast) { mv_put(d, pix(d, r, j), m >> 16); st.alg += 4; }
    }
    if (stopped) return;
    // the exact min1 of those that pass
#pragma unroll 1
    for (uint32_t k = 0; k < HTB; k++) {
        if (!((live >> k) & 1u)) continue;
        uint32_t j, m;
        hsrc_get(d, src, sh, pos + k * HT + (uint32_t)tid, s, r, j, m, st.alg);  // (cache-hot)
        Cand<KW> c;
        heavy_eval<KW>(d, s, r, ds, t, j, m, lightok, c, st);
        if (!(c.emsg != 0u && c.min1 <= R)) {
            live &= ~(1u << k);
            if (merged && rec_fast(m)) { mv_put(d, pix(d, r, j), m >> 16); st.alg += 4; }  // never sent: restore
        }
    }
    // survivors compacted in sender order (k-major, then thread): per (k, wave) ballot counts, one barrier
#pragma unroll
    for (int k = 0; k < HTB; k++) {
        const unsigned long long bl = __ballot((live >> k) & 1u);
        if (lane == 0) sh.wcnt[k][wv] = (uint32_t)__popcll(bl);
    }
    __syncthreads();
    uint32_t base = 0;
    const unsigned long long lm = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < HTB; k++) {
        uint32_t off = base;
#pragma unroll
        for (int w = 0; w < HW_WAVES; w++) {
            const uint32_t v = sh.wcnt[k][w];
            if (w < wv) off += v;
            base += v;
        }
        const bool lv = (live >> k) & 1u;
        const unsigned long long bl = __ballot(lv);
        if (lv) sh.surv[off + (uint32_t)__popcll(bl & lm)] = (uint16_t)((uint32_t)k * HT + (uint32_t)tid);
    }
    const uint32_t nsurv = base;
    __syncthreads();
    if (tid < WAVE && nsurv) {  // one wave: pack_group's sequential first-fit over the survivors, 64 at a time
        bool tl = true, sp = false;
        uint32_t nr = 0, steps = 0;
        for (uint32_t g0 = 0; g0 < nsurv; g0 += WAVE) {
            const bool cand = g0 + (uint32_t)lane < nsurv;
            uint32_t jj = 0u, mm = 0u;
            if (cand) hsrc_get(d, src, sh, pos + sh.surv[g0 + lane], s, r, jj, mm, st.alg);
            if (sp) {  // complete: restore the rest of the merged survivors
                if (cand && merged && rec_fast(mm)) { mv_put(d, pix(d, r, jj), mm >> 16); st.alg += 4; }
                continue;
            }
            Cand<KW> cc;
            cc.emsg = 0;
            cc.min1 = 0;
            cc.light = false;
            cc.fast = false;
            if (cand) heavy_eval<KW>(d, s, r, ds, t, jj, mm, lightok, cc, st);
            pack_group<KW, false, false>(d, s, r, t, cc, cand, S, tl, sp, st, tomb, nullptr, nr, merged);
            steps++;
        }
        if (lane == 0) {
            sh.S = S;
            if (sp) sh.stop = 1u;
            sh.steps += steps;
        }
    }
    __syncthreads();
}

// all candidates of one source in sender order: whole-fit blocks while not in first-fit continuation, then
// first-fit super-blocks (which, once the delta is complete, only restore merged records)
template <int KW>
__device__ __forceinline__ void heavy_source(const Dev &d, uint32_t s, uint32_t r, const DigestSide &ds, uint32_t t,
                                             const HSrc &src, uint32_t len, bool specd, bool lightok, HeavyLds &sh,
                                             WStats &st, bool &tomb) {
    uint32_t pos = 0;
    while (pos < len) {
        if (sh.stop && !(specd && src.L)) break;
        if (!sh.tail && !sh.stop) {
            pos += heavy_prefix<KW>(d, s, r, ds, t, src, pos, len, specd, lightok, sh, st, tomb);  // HPB, or the first
                                                                                                  // that did not fit
        } else {
            heavy_tail<KW>(d, s, r, ds, t, src, pos, len, specd, lightok, sh, st, tomb);
            pos += HSB;
        }
        if (threadIdx.x == 0) { sh.steps++; sh.groups = max(sh.groups, (pos + WAVE - 1) / WAVE); }
    }
}

template <int KW>
#ifndef HW_OCC
#define HW_OCC 4  // waves per SIMD k_pack_heavy is compiled for (one workgroup = one wave per SIMD)
#endif
__global__ __launch_bounds__(HT, HW_OCC) void k_pack_heavy(Dev d, const int32_t *ini, const int32_t *res, uint32_t t,
                                                   const uint32_t *heavy) {
    __shared__ HeavyLds sh;
    const uint32_t count = heavy[0];
    const int tid = (int)threadIdx.x, lane = lane_id();
    const uint32_t H = half_cols(d), words = d.NP / 32;
    WStats st{0, 0, 0, 0, 0};
    for (uint32_t hi = blockIdx.x; hi < count; hi += gridDim.x) {
        const uint32_t slot = heavy[1u + hi], e = slot >> 1;
        const bool w0 = (slot & 1u) == 0u;
        const uint32_t a = (uint32_t)ini[e], b = (uint32_t)res[e];  // (k_pack_slice listed valid exchanges only)
        const uint32_t snd = w0 ? b : a, rcv = w0 ? a : b;
        const DigestSide ds{rcv, d.ncol, t >= d.row[rcv * 4 + 2]};
        const bool specd = d.spec != 0u, lightok = d.vlog && !d.ev && !ds.sched;
        if (tid == 0) { sh.S = 0u; sh.stop = 0u; sh.tail = 0u; sh.steps = 0u; sh.groups = 0u; }
        __syncthreads();
        bool tb = false;
        uint32_t done = 0;  // candidates of earlier sources (pack_groups_max)
        for (uint32_t hf = 0; hf < 2; hf++) {
            const uint32_t nh = d.cand_n[(size_t)slot * 2 + hf];
            const uint2 *L = d.cand + ((size_t)slot * 2 + hf) * GS_CAND_CAP;
            heavy_source<KW>(d, snd, rcv, ds, t, HSrc{L, 0u}, min(nh, GS_CAND_CAP), specd, lightok, sh, st, tb);
            if (nh <= GS_CAND_CAP || sh.stop) continue;
            // past the half's records: its bitmap, compacted window by window (those owners were not merged)
            const uint32_t pmin = L[GS_CAND_CAP - 1].x + 1u, end = min(H * (hf + 1u), d.ncol);
            const uint32_t *bits = d.sbits + (size_t)slot * words;
            for (uint32_t w = pmin & ~15u; w < end && !sh.stop; w += HWIN) {
                const uint32_t pb = w + 16u * (uint32_t)tid;
                uint32_t m = 0u;
                if (pb < end) {
                    m = (bits[pb >> 5] >> (pb & 16u)) & 0xFFFFu;
                    st.alg += 2;
                    if (end - pb < 16u) m &= (1u << (end - pb)) - 1u;
                    if (pb < pmin) m &= pmin - pb >= 16u ? 0u : ~((1u << (pmin - pb)) - 1u);
                }
                uint32_t cnt;
                uint32_t wp = block_excl_scan((uint32_t)__popc(m), sh, &cnt);
                while (m) {
                    const uint32_t bb = (uint32_t)__builtin_ctz(m);
                    m &= m - 1u;
                    sh.wl[wp++] = (uint16_t)(16u * (uint32_t)tid + bb);
                }
                __syncthreads();
                heavy_source<KW>(d, snd, rcv, ds, t, HSrc{nullptr, w}, cnt, specd, lightok, sh, st, tb);
                __syncthreads();  // (wl is rewritten by the next window)
            }
            (void)done;
        }
        const uint32_t S1 = sh.S;
        if (__syncthreads_or(tb) && tid == 0) d.row[rcv * 4 + 1] = 1u;
        if (tid == 0) {
            shard_add(d, C_DBYTES, S1);
            shard_max(d, C_PGMAX, sh.groups);
            shard_max(d, C_PSMAX, sh.steps);
        }
        __syncthreads();  // (sh is reset for the next slot)
    }
    const unsigned long long s_alg = wave_sum(st.alg), s_nd = wave_sum(st.nd), s_kv = wave_sum(st.kvs);
    const unsigned long long s_tr = wave_sum(st.trunc), s_cd = wave_sum(st.cand);
    if (lane == 0) {
        shard_add(d, C_ALG, s_alg);
        shard_add(d, C_PACKB, s_alg);
        shard_add(d, C_ND, s_nd);
        shard_add(d, C_KVS, s_kv);
        shard_add(d, C_TRUNC, s_tr);
        shard_add(d, C_CAND, s_cd);
    }
}

// Overflowing slots of a sliced phase (gs_phase_overflow): every (exchange, direction) slot whose slice
// totals sum past the mtu, in slot order -- the same list on every slice, since all hold the same
// gathered totals -- plus this slice's chain state of each listed slot (chainc[i] = chain[list[i]]).
// Two launches of 1024-thread blocks: per-block counts, then per-block offsets (a sum over the block
// counts: ceil(2n / 1024) of them) and a ballot scan inside the block.  scratch = list + 2n: [blocks]
// counts, then the total -- GS_OVERFLOW_LIST_LEN(n) words in all.
constexpr uint32_t OVB = 1024;
__global__ __launch_bounds__(OVB) void k_ov_count(const uint64_t *tot_all, uint32_t slots, uint32_t G, uint32_t mtu,
                                                  uint32_t *blkcnt, const GroupArgs *ga) {
    if (ga) {  // a slice of an in-process group (blockIdx.y)
        tot_all = ga->io[blockIdx.y].tot_all;
        blkcnt = ga->list[blockIdx.y] + slots;
    }
    const uint32_t sl = blockIdx.x * OVB + threadIdx.x;
    uint64_t sum = 0;
    if (sl < slots)
        for (uint32_t g = 0; g < G; g++) sum += GS_TOT_BYTES(tot_all[(size_t)g * slots + sl]);
    const int c = __syncthreads_count(sl < slots && sum > mtu);
    if (threadIdx.x == 0) blkcnt[blockIdx.x] = (uint32_t)c;
}
__global__ __launch_bounds__(OVB) void k_ov_write(const uint64_t *tot_all, uint32_t slots, uint32_t G, uint32_t mtu,
                                                  const uint64_t *chain, uint32_t *list, uint64_t *chainc,
                                                  const GroupArgs *ga) {
    __shared__ uint32_t s_w[OVB / WAVE];
    __shared__ uint32_t s_off;
    if (ga) {  // a slice of an in-process group (blockIdx.y)
        tot_all = ga->io[blockIdx.y].tot_all;
        chain = ga->io[blockIdx.y].chain;
        list = ga->list[blockIdx.y];
        chainc = ga->chainc[blockIdx.y];
    }
    const uint32_t nb = gridDim.x;
    const uint32_t *blkcnt = list + slots;
    if (threadIdx.x == 0) {
        uint32_t off = 0, all = 0;
        for (uint32_t b = 0; b < nb; b++) {
            if (b < blockIdx.x) off += blkcnt[b];
            all += blkcnt[b];
        }
        s_off = off;
        if (blockIdx.x == nb - 1) list[slots + nb] = all;  // the count (read by the host)
    }
    const uint32_t sl = blockIdx.x * OVB + threadIdx.x;
    uint64_t sum = 0;
    if (sl < slots)
        for (uint32_t g = 0; g < G; g++) sum += GS_TOT_BYTES(tot_all[(size_t)g * slots + sl]);
    const bool f = sl < slots && sum > mtu;
    const unsigned long long m = __ballot(f);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = s_off;
    for (int x = 0; x < w; x++) pre += s_w[x];
    if (f) {
        const uint32_t i = pre + (uint32_t)__popcll(m & ((1ull << l) - 1ull));
        list[i] = sl;
        chainc[i] = chain[sl];
    }
}

// the pending counts of all G slices (entry count of each gathered chainc) summed into *out.  cnt_dev: the count
// is read on the device (GS_CHAIN_DEVICE: gathered rows of GS_CHAIN_CAP + 1 entries); a count above the cap gives
// ~0 (the device step did not run: the host takes over)
// out[1] = the count (gs_phase_pending; out may be host-mapped pinned memory: the host reads it after the wait)
__global__ __launch_bounds__(WAVE) void k_sum_pending(const uint64_t *chain_all, uint32_t G, uint32_t count,
                                                      const uint32_t *cnt_dev, uint64_t *out) {
    const uint32_t c = cnt_dev ? *cnt_dev : count;
    const size_t stride = cnt_dev ? GS_CHAIN_CAP + 1u : (size_t)count + 1u;
    unsigned long long s = 0;
    if (!cnt_dev || c <= GS_CHAIN_CAP)
        for (uint32_t g = threadIdx.x; g < G; g += WAVE) s += chain_all[(size_t)g * stride + c];
    s = wave_sum(s);
    if (threadIdx.x == 0) {
        out[0] = cnt_dev && c > GS_CHAIN_CAP ? ~0ull : s;
        out[1] = c;
    }
}

// chainc[count] = this slice's listed slots still pending (the count itself read from the list's tail when
// cnt_dev is set: gs_phase_overflow's count is not known to the host without a read)
__global__ __launch_bounds__(OVB) void k_pending(const uint32_t *list, const uint32_t *cnt_dev, uint32_t count,
                                                 const uint64_t *chain, uint64_t *chainc, const GroupArgs *ga,
                                                 uint32_t n) {
    if (ga) {  // a slice of an in-process group (blockIdx.y)
        if (cnt_dev) cnt_dev = ga->list[blockIdx.y] + 2u * n + (2u * n + OVB - 1u) / OVB;
        list = ga->list[blockIdx.y];
        chain = ga->io[blockIdx.y].chain;
        chainc = ga->chainc[blockIdx.y];
    }
    const uint32_t c = cnt_dev ? *cnt_dev : count;
    uint32_t p = 0;
    for (uint32_t i = threadIdx.x; i < c; i += OVB) p += chain[list[i]] == CHAIN_PENDING ? 1u : 0u;
    __shared__ uint32_t s[OVB / WAVE];
    const unsigned long long w = wave_sum(p);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = (uint32_t)w;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0;
        for (uint32_t k = 0; k < OVB / WAVE; k++) a += s[k];
        chainc[c] = a;
    }
}

// In-process all-gather (gs_run_phase_group: every slice on one device and stream): dst[i][g * count + k]
// = src[g][k] for every destination slice i (grid.y) -- one launch instead of G^2 copies.
constexpr uint32_t GATHER_MAX = 64;
struct GatherPtrs {
    const uint64_t *src[GATHER_MAX];
    uint64_t *dst[GATHER_MAX];
};
__global__ __launch_bounds__(LB) void k_gather_u64(GatherPtrs p, uint32_t G, uint64_t count) {
    uint64_t *dst = p.dst[blockIdx.y];
    const uint64_t total = (uint64_t)G * count;
    for (uint64_t x = (uint64_t)blockIdx.x * LB + threadIdx.x; x < total; x += (uint64_t)gridDim.x * LB) {
        const uint64_t *s = p.src[x / count];  // (null: a slice held by no one here, gathered as zeros)
        dst[x] = s ? s[x % count] : 0ull;
    }
}

// Chain step `step` >= 1 over the overflowing slots only (gs_phase_chain): one wave per listed slot; a
// slot still pending on this slice continues from its predecessor's gathered state (chain_all =
// [G][count] of every slice's chainc).  State goes to both chain (by slot) and chainc (by list index).
template <int KW, bool GRP = false>
// Resume point (gs_phase_chain): the nearest finished predecessor f; every slice between f and this one is
// pending, and is skipped only if it cannot add a NodeDelta after f (f's delta is complete, or that slice's
// smallest single-kv NodeDelta exceeds the budget f left: first-fit continuation tests each owner's
// smallest prefix against it, state.py:392-413, and the budget only shrinks) -- its own resume then ends in
// f's state too.  Slices before the first to overflow all finished at step 0, so f exists.
__global__ __launch_bounds__(WAVE) void k_chain_step(Dev d, const int32_t *ini, const int32_t *res, uint32_t t,
                                                     const uint32_t *list, uint32_t count, const uint64_t *chain_all,
                                                     uint64_t *chain, uint64_t *chainc, const uint64_t *tot_all,
                                                     uint32_t n, const uint32_t *cnt_dev, const GroupArgs *ga,
                                                     DevDyn dyn) {
    __shared__ __attribute__((aligned(16))) uint16_t s_wbuf[WIN];
    const int lane = lane_id();
    if constexpr (GRP) {  // a slice of an in-process group (blockIdx.y): its own scratch
        group_pick(d, ga, dyn);
        const uint32_t y = blockIdx.y;
        if (cnt_dev) cnt_dev = ga->list[y] + 2u * n + (2u * n + OVB - 1u) / OVB;
        list = ga->list[y];
        chain_all = ga->chain_all[y];
        chain = ga->io[y].chain;
        chainc = ga->chainc[y];
        tot_all = ga->io[y].tot_all;
    }
    // chain_all[g][count + 1]: entry count = g's pending slots; GS_CHAIN_DEVICE (cnt_dev): the count from the
    // device, rows of GS_CHAIN_CAP + 1 entries, nothing done above the cap (every slice sees the same count)
    if (cnt_dev) {
        count = *cnt_dev;
        if (count > GS_CHAIN_CAP) return;
    }
    const size_t stride = cnt_dev ? GS_CHAIN_CAP + 1u : (size_t)count + 1u;
    for (uint32_t i = blockIdx.x; i < count; i += gridDim.x) {
        const uint32_t slot = list[i];
        if (chain[slot] != CHAIN_PENDING) continue;
        int f = (int)d.shard - 1;
        while (f >= 0 && chain_all[(size_t)f * stride + i] == CHAIN_PENDING) f--;
        if (f < 0) continue;
        const uint64_t prev = chain_all[(size_t)f * stride + i];
        PackState pst = chain_unpack(prev);
        bool ok = true;
        for (uint32_t h = (uint32_t)f + 1u; h < d.shard && ok; h++)
            ok = pst.stop || pst.S >= d.mtu ||
                 (pst.tail && GS_TOT_MIN1(tot_all[(size_t)h * n * 2 + slot]) > d.mtu - pst.S);
        if (!ok) continue;
        const uint32_t e = slot >> 1, wid = slot & 1u;
        const uint32_t a = (uint32_t)ini[e], b = (uint32_t)res[e];
        const bool w0 = wid == 0;
        const uint32_t snd = w0 ? b : a, rcv = w0 ? a : b;
        const DigestSide ds{rcv, d.ncol, t >= d.row[rcv * 4 + 2]};
        WStats st{0, 0, 0, 0, 0};
        bool tomb = false;
        pack_records<KW, false>(d, snd, rcv, ds, slot, s_wbuf, t, st, tomb, pst);
        if (tomb) d.row[rcv * 4 + 1] = 1u;
        if (lane == 0) {
            chain[slot] = chain_pack(pst);
            chainc[i] = chain_pack(pst);
        }
        const unsigned long long s_alg = wave_sum(st.alg), s_nd = wave_sum(st.nd), s_kv = wave_sum(st.kvs);
        const unsigned long long s_tr = wave_sum(st.trunc), s_cd = wave_sum(st.cand);
        if (lane == 0) {
            shard_add(d, C_ALG, s_alg);
            shard_add(d, C_PACKB, s_alg);
            shard_add(d, C_ND, s_nd);
            shard_add(d, C_KVS, s_kv);
            shard_add(d, C_TRUNC, s_tr);
            shard_add(d, C_CAND, s_cd);
            shard_max(d, C_PGMAX, st.grp);
            shard_max(d, C_PSMAX, st.stp);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// The settle pass of a speculative phase, per (exchange, direction) slot: every record's NodeDelta is
// evaluated (eval_cand: DeltaPb bytes, kvs), independently -- no sequential budget walk, so the loads of
// a wave's groups overlap -- giving the slot's DeltaPb total T and, if the delta fits, its statistics.
// clean: every candidate was recorded and merged by pass 1 (no candidate with holes, no bitmap tail).
struct SlotSum {
    unsigned long long T;
    uint32_t nd, kvs, cand;
    bool clean;
};
template <int KW>
__device__ __forceinline__ SlotSum settle_sum(const Dev &d, uint32_t snd, uint32_t rcv, const DigestSide &ds,
                                              size_t slot, uint16_t *wbuf, uint32_t t, uint32_t &alg) {
    const int lane = lane_id();
    uint32_t T = 0, nd = 0, kvs = 0, cand = 0;
    bool clean = true;
    unsigned long long tail = 0;
    for (uint32_t hf = 0; hf < 2; hf++) {
        const uint32_t nh = d.cand_n[slot * 2 + hf], m = min(nh, GS_CAND_CAP);
        const uint2 *L = d.cand + (slot * 2 + hf) * GS_CAND_CAP;
#pragma unroll 2
        for (uint32_t c0 = 0; c0 < m; c0 += WAVE) {
            const uint32_t ci = c0 + lane;
            if (ci < m) {
                const uint2 cr = L[ci];
                Cand<KW> c;
                CandKeys<KW> ck;
                eval_cand<KW, false, true>(d, snd, rcv, ds, cr.x, t, c, ck, alg, cr.y);
                T += c.emsg;
                nd += c.emsg ? 1u : 0u;
                kvs += c.nkv;
                cand++;
                clean = clean && c.fast;
            }
        }
        if (nh > GS_CAND_CAP) {  // the bitmap tail: its owners are not merged, the pack walks them
            const uint32_t H = half_cols(d), words = d.NP / 32;
            const uint32_t pmin = L[GS_CAND_CAP - 1].x + 1u;
            WStats cs{0, 0, 0, 0, 0};
            bool ctomb = false;
            PackState pst{0u, false, false};
            pack_dir<KW, false, true>(d, snd, rcv, ds, nullptr, min(H * (hf + 1), d.ncol), d.sbits + (slot * words),
                                      wbuf, t, cs, ctomb, pst, nullptr, nullptr, pmin & ~15u, pmin);
            tail += pst.S;
            alg += cs.alg;
            clean = false;
        }
    }
    SlotSum r;
    r.T = wave_sum(T) + tail;
    r.nd = (uint32_t)wave_sum(nd);
    r.kvs = (uint32_t)wave_sum(kvs);
    r.cand = (uint32_t)wave_sum(cand);
    r.clean = __ballot(!clean) == 0ull;
    return r;
}

// Phase completion after k_pass1 on canonical record handles, one wave per (exchange, direction) slot
// (wave 0: the SynAck delta b -> a, wave 1: the Ack delta a -> b):
//   MODE 0 (one slice, gs_run_phase): a speculative phase whose delta fits (T <= mtu) and is clean is
//          complete -- pass 1 applied it -- and only its statistics are added; any other slot runs the
//          sequential packer (pack_records: exact first-fit, restores of the merged candidates it does
//          not send, applies of the rest); a non-speculative phase always does.
//   MODE 1 (sliced count, gs_phase_count): the slot's DeltaPb total of this slice into io.tot (and, when
//          speculative, its statistics into slot_stat for MODE 2).
//   MODE 2 (sliced pack step 0, gs_phase_pack): the slice resumes the sender-order walk at the bytes
//          its predecessors reach when they all fit whole (pending otherwise: the chain steps); a
//          speculative slot whose whole delta fits over every slice and is clean here is complete.
// Sequential semantics over the slices in column (= canonical dict) order, so the result is the
// single-slice result bit for bit.
// LITE (sliced phases with Dev::lite, MODE 1 and 2): k_lite's slot work first, in the same wave, and the exact
// count / pack only for the slots it leaves (one launch per step instead of two: a slice's kernels are short,
// and their fixed cost per launch is what a sliced phase pays over one handle)
#ifndef SETTLE_LITE_WAVES
#define SETTLE_LITE_WAVES PK_WAVES  // waves per SIMD of the sliced steps' k_settle<LITE>: nearly every slot ends in the
                                    // lite slot work; the exact count / pack below it runs for the few others
#endif
template <int KW, int MODE, bool LITE = false, bool GRP = false>
__global__ __launch_bounds__(XB, (KW == 4 ? (LITE ? SETTLE_LITE_WAVES : PK_WAVES) : 1)) void k_settle(Dev d, const int32_t *ini, const int32_t *res,
                                                                        uint32_t n, uint32_t t, SliceIO io,
                                                                        const GroupArgs *ga, DevDyn dyn) {
    __shared__ __attribute__((aligned(16))) uint16_t s_wbuf[2 * WIN];
    const uint32_t e = blockIdx.x;
    if (e >= n) return;
    if constexpr (GRP) {  // a slice of an in-process group (blockIdx.y); the step comes by value
        group_pick(d, ga, dyn);
        const uint32_t step = io.step;
        io = ga->io[blockIdx.y];
        io.step = step;
    }
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid >> 6;
    if (d.p1fix && tid == 0) p1v_fix_one(d, res, e);  // k_p1v_fix's work (Dev::p1fix)
    const int32_t ai = ini[e], bi = res[e];
    const size_t slot = (size_t)e * 2 + wid;
    if (ai < 0 || bi < 0 || (uint32_t)ai >= d.N || (uint32_t)bi >= d.N || ai == bi) {  // counted already
        if (LITE && lane == 0) d.slot_stat[slot].w = LITE_DONE;
        return;
    }
    uint32_t lflag = 0u;  // LITE: the slot's flag from lite_slot
    if (LITE) {
        static_assert(!LITE || MODE == 1 || MODE == 2, "k_settle<LITE> runs the sliced steps");
        lflag = lite_slot<MODE>(d, ai, bi, n, t, io, slot, wid, lane);
        if (MODE == 1 ? !(lflag & LITE_FULL) : (lflag & LITE_DONE) != 0u) return;
    }
    const uint32_t a = (uint32_t)ai, b = (uint32_t)bi;
    const bool w0 = wid == 0;
    const uint32_t snd = w0 ? b : a, rcv = w0 ? a : b;
    const DigestSide ds{rcv, d.ncol, t >= d.row[rcv * 4 + 2]};
    uint16_t *wbuf = s_wbuf + wid * WIN;
    WStats st{0, 0, 0, 0, 0};
    bool tomb = false;
    PackState pst{0u, false, false};
    uint32_t salg = 0;
    bool done = false;
    // d.spec without d.lite: the speculative A/B path (GS_PACK=spec) sizes and settles from settle_sum; with
    // d.lite (k_pass1v's merge) the lite / exact-packer path below restores what is not sent
    if (MODE == 1) {
        if (d.spec && !d.lite) {
            const SlotSum s = settle_sum<KW>(d, snd, rcv, ds, slot, wbuf, t, salg);
            if (lane == 0) {
                io.tot[slot] = tot_word(s.T, 0u);  // (speculative A/B path: no chain skipping)
                d.slot_stat[slot] = make_uint4(s.nd, s.kvs, s.cand, s.clean ? 0u : 1u);
            }
        } else {
            if (!LITE && d.lite && !(d.slot_stat[slot].w & LITE_FULL)) return;  // k_lite wrote the slice total
            pack_records<KW, true>(d, snd, rcv, ds, slot, wbuf, t, st, tomb, pst);
            if (lane == 0) io.tot[slot] = tot_word(pst.S, pst.m1);
            salg = st.alg;
        }
        const unsigned long long s_alg = wave_sum(salg);
        if (lane == 0) { shard_add(d, C_ALG, s_alg); shard_add(d, C_PACKB, s_alg); }
        return;
    }
    if (MODE == 0) {
        if (d.spec) {
            const SlotSum s = settle_sum<KW>(d, snd, rcv, ds, slot, wbuf, t, salg);
            if (s.clean && s.T <= d.mtu) {
                done = true;
                st.nd = s.nd;  // wave totals: added by lane 0 only (below)
                st.kvs = s.kvs;
                st.cand = s.cand;
                if (lane == 0) shard_add(d, C_DBYTES, s.T);
            }
        }
    } else {  // MODE 2
        if (!LITE && d.lite && (d.slot_stat[slot].w & LITE_DONE)) return;  // k_lite applied it and wrote its chain state
        unsigned long long P = 0, all = 0;
        for (uint32_t g = 0; g < d.shards; g++) {
            const unsigned long long x = GS_TOT_BYTES(io.tot_all[(size_t)g * n * 2 + slot]);
            if (g < d.shard) P += x;
            all += x;
        }
        if (P > d.mtu) {
            if (lane == 0) io.chain[slot] = CHAIN_PENDING;
            return;
        }
        pst = PackState{(uint32_t)P, false, false};
        if (d.spec && !d.lite && all <= d.mtu) {
            const uint4 ss = d.slot_stat[slot];
            if (!ss.w) {
                done = true;
                st.nd = ss.x;
                st.kvs = ss.y;
                st.cand = ss.z;
                if (lane == 0) {
                    const unsigned long long own = GS_TOT_BYTES(io.tot_all[(size_t)d.shard * n * 2 + slot]);
                    shard_add(d, C_DBYTES, own);
                    io.chain[slot] = (uint64_t)(P + own);  // not listed
                }
            }
        }
    }
    if (!done) {
        pack_records<KW, false>(d, snd, rcv, ds, slot, wbuf, t, st, tomb, pst);
        if (tomb) d.row[rcv * 4 + 1] = 1u;
        if (MODE == 2 && lane == 0) io.chain[slot] = chain_pack(pst);
        st.alg += salg;
        st.nd = (uint32_t)wave_sum(st.nd);
        st.kvs = (uint32_t)wave_sum(st.kvs);
        st.trunc = (uint32_t)wave_sum(st.trunc);
        st.cand = (uint32_t)wave_sum(st.cand);
    } else {
        st.alg = salg;
    }
    const unsigned long long s_alg = wave_sum(st.alg);
    if (lane == 0) {
        shard_add(d, C_ALG, s_alg);
        shard_add(d, C_PACKB, s_alg);
        shard_add(d, C_ND, st.nd);
        shard_add(d, C_KVS, st.kvs);
        shard_add(d, C_TRUNC, st.trunc);
        shard_add(d, C_CAND, st.cand);
        shard_max(d, C_PGMAX, st.grp);
        shard_max(d, C_PSMAX, st.stp);
    }
}


// Record phases of prefix-view handles (Dev::lite): the whole-delta fast path of every (exchange,
// direction) slot as a kernel of its own (pack_lite: few registers, 8 waves per SIMD), between k_pass1 and
// the exact packer, which then only runs the slots flagged here (slot_stat[slot].w):
//   MODE 0 (one slice): a delta of prefix candidates that fits is applied here (LITE_DONE);
//   MODE 1 (sliced count): the slice total of a slot whose candidates are all prefix candidates is
//          written here (else LITE_FULL: k_settle counts it);
//   MODE 2 (sliced pack step 0): such a slot whose predecessors' totals and its own fit from their sum
//          is applied here and its chain state written (LITE_DONE); the rest is k_settle's.
#ifndef LITE_WAVES
#define LITE_WAVES 8
#endif
template <int MODE>
__global__ __launch_bounds__(XB, LITE_WAVES) void k_lite(Dev d, const int32_t *ini, const int32_t *res, uint32_t n,
                                                         uint32_t t, SliceIO io) {
    const uint32_t e = blockIdx.x;
    if (e >= n) return;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid >> 6;
    const int32_t ai = ini[e], bi = res[e];
    const size_t slot = (size_t)e * 2 + wid;
    if (ai < 0 || bi < 0 || (uint32_t)ai >= d.N || (uint32_t)bi >= d.N || ai == bi) {  // counted already
        if (lane == 0) d.slot_stat[slot].w = LITE_DONE;
        return;
    }
    lite_slot<MODE>(d, ai, bi, n, t, io, slot, wid, lane);
}

// ------------------------------------------------------------------ round start
// inc_heartbeat + ClusterState.gc_marked_for_deletion (server.py:471-474; state.py:253-274, 333-338)
__global__ __launch_bounds__(LB) void k_begin_round(Dev d, const uint8_t *up, uint32_t t) {
    const uint32_t o = blockIdx.x;
    if (o >= d.N || !up[o]) return;
    if (threadIdx.x == 0 && o - d.col_lo < d.ncol) {
        const uint32_t R = d.self_hb[o - d.col_lo] + 1u;
        d.self_hb[o - d.col_lo] = R;
        self_repack(d, o - d.col_lo);
        hb_put(d, pix(d, o, o - d.col_lo), R);
    }
    if (!(d.flags & GS_TOMBSTONES) || !d.row[o * 4 + 1]) return;
    const bool genm = !(d.flags & GS_CANONICAL);
    bool remaining = false;
    uint32_t gcn = 0;
    for (uint32_t j = threadIdx.x; j < d.ncol; j += LB) {
        const size_t p = pix(d, o, j);
        if (genm && d.pos[p] == NONE) continue;
        uint32_t maxdel = d.gc[p];
        bool changed = false;
        for (uint32_t k = 0; k < d.K; k++) {
            const uint32_t tv = d.ts[p * d.KP + k];
            if (tv == NONE) continue;
            if ((uint64_t)t >= (uint64_t)tv + d.tomb_grace) {
                const uint32_t w = d.held[p * d.KP + k];
                const uint32_t v = (uint32_t)d.hist[hix(d, j, w, k)];
                d.held[p * d.KP + k] = 0;
                d.ts[p * d.KP + k] = NONE;
                if (v > maxdel) maxdel = v;
                changed = true;
                gcn++;
            } else {
                remaining = true;
            }
        }
        if (changed) d.gc[p] = maxdel;
    }
    remaining = __syncthreads_or(remaining);
    if (threadIdx.x == 0) d.row[o * 4 + 1] = remaining ? 1u : 0u;
    const unsigned long long s = wave_sum(gcn);
    if ((threadIdx.x & 63) == 0) shard_add(d, C_TOMBGC, s);
}

// ------------------------------------------------------------------ liveness
// Row word 2 is a lower bound of the row's earliest scheduled-for-deletion tick (tod + grace/2 over its
// dead targets): a new death lowers it, a revival or FD GC leaves it.  Only a row whose bound has passed
// (so that a target may be scheduled, or due for FD GC: grace >= grace/2) is recomputed exactly, by the
// sweep that follows (flag bit 1), which is then the only one to read its times of death.
__global__ __launch_bounds__(LB) void k_reset_sched(Dev d, const uint8_t *up, uint32_t t) {
    const uint32_t o = blockIdx.x * LB + threadIdx.x;
    if (o >= d.N || !up[o]) return;
    uint32_t f = d.row[o * 4 + 3] & ~2u;
    if (t >= d.row[o * 4 + 2]) {
        d.row[o * 4 + 2] = NONE;
        f |= 2u;
    }
    d.row[o * 4 + 3] = f;
}

// First the round's deferred heartbeat reports (pass 1 of k_exchange) are replayed into the
// sampling windows in tick order (FailureDetector.report_heartbeat, failure_detector.py:79-81),
// for every row.  Then, for up observers, Cluster._update_node_liveness ->
// FailureDetector.update_node_liveness for every known node but self (server.py:606-610;
// failure_detector.py:89-106), phi in binary64 exactly as SamplingWindow.phi (43-53).  Also folds
// the earliest "scheduled for deletion" tick per row.
// RING: 0 = compact windows only (no ring pointer at all: k_liveness stays within 64 VGPRs without
// spills), 1 = every row has interval rings (GS_FD_RING), 2 = the sampled ring rows (gs_config.ring_rows).
template <int RING>
// One workgroup sweeps `per` consecutive 1024-column chunks of one row (fewer, longer workgroups:
// the per-workgroup plane staging, stamp check and counter atomics are paid once per `per` chunks).
// decide = false: only replay the pending reports into the windows, for every row (a round with phases
// more than 16 ticks after its plane base: the planes are emptied mid-round)
#ifndef LIVE_F32
#define LIVE_F32 1  // the phi decision's first test in binary32 (A/B: 0 = binary64 with a 2^-30 margin)
#endif
#ifndef LIVE_WAVES
#define LIVE_WAVES 6  // waves per SIMD k_liveness is compiled for (<= 80 VGPRs: two chunks in flight)
#endif
#ifndef LIVE_NT
#define LIVE_NT 1  // non-temporal loads / stores of the windows and state bytes (streamed once per round; r4c: 11.86 vs 12.21 ms)
#endif
__global__ __launch_bounds__(LB, LIVE_WAVES) void k_liveness(Dev d, const uint8_t *up, uint32_t t, uint32_t chunks,
                                                 uint32_t per, bool replay, bool decide) {
    // [wave][phase][the wave's 4 plane words of this chunk]: each wave stages and reads only its own
    // words (lane l: phase l / 2, words 2 (l % 2) + {0, 1}), so the chunks need no workgroup barrier
    __shared__ __attribute__((aligned(16))) uint64_t s_pl[LB / WAVE][NPL][4];
    __shared__ uint32_t s_vm;
    const uint32_t groups = (chunks + per - 1) / per;
    const uint32_t o = blockIdx.x / groups, cb0 = (blockIdx.x % groups) * per;
    const bool upo = decide && up[o] != 0;
    const bool exact = upo && (d.row[o * 4 + 3] & 2u);  // recompute row word 2 (k_reset_sched)
    const bool genm = !(d.flags & GS_CANONICAL);
    // this row's interval rings: every row has them (RING: GS_FD_RING), or this is a sampled ring row
    uint16_t *rrow = nullptr;
    if (RING == 1) {
        rrow = d.ring + (size_t)o * d.NP * d.W;
    } else if (RING == 2) {
        const uint32_t rs = d.ring_slot[o];
        if (rs != NONE) rrow = d.ring + (size_t)rs * d.NP * d.W;
    }
    uint32_t minS = NONE, live = 0, gcdue = 0, ovf = 0, alg = 0;
    // phases of the current round in which row o was in an exchange (its plane rows are valid);
    // replay = false once this round's reports were replayed (the host closes the round)
    if (threadIdx.x < 64) {
        const bool v = replay && threadIdx.x < NPL && d.pstamp[o * NPL + threadIdx.x] == d.v_round + 1u + threadIdx.x;
        const uint32_t m = (uint32_t)__ballot(v);
        if (threadIdx.x == 0) s_vm = m;
    }
    __syncthreads();
    const uint32_t vm = s_vm;
    const uint32_t cb1 = min(chunks, cb0 + per);
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
    // A down row without valid planes (its node was in no exchange) has nothing to replay or decide.  The
    // chunks stream double-buffered: the next chunk's windows, states and plane words are loaded (always, at
    // a clamped or shared address past the end, so that no wait counts them as absent) before the current
    // chunk is computed, and the waits for the current chunk leave them in flight.
    if (upo || vm) {
        struct LW {
            uint4 sc;      // the four windows' sum | cnt words
            uint2 l;       // ... and their last-report ticks, u16 pairs
            uint32_t s;    // the four pairs' state bytes
            ulonglong2 pw; // this lane's 16 B of the chunk's report planes (lane l: phase l / 2, words 2 (l % 2) + {0, 1})
        };
        const uint32_t cmax = (d.ncol - 1u) & ~3u;
        const uint32_t ph = ln >> 1;
        const bool phv = ph < NPL && ((vm >> ph) & 1u);  // NPL = 16: lanes 0-31 only
        const uint64_t *prow = d.pend + ((size_t)o * NPL + (phv ? ph : 0u)) * d.PW;
        auto ldw = [&](uint32_t cb, bool real, LW &w) {
            const uint32_t c0 = real ? min((cb * LB + threadIdx.x) * 4u, cmax) : 0u;
            const size_t p = pix(d, o, c0);
            if (LIVE_NT) {  // streamed once per round: non-temporal
                const v4u_t x = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(d.fd + p));
                const v2u_t y = __builtin_nontemporal_load(reinterpret_cast<const v2u_t *>(d.fd_last + p));
                w.sc = make_uint4(x.x, x.y, x.z, x.w);
                w.l = make_uint2(y.x, y.y);
                w.s = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(d.fd_state + p));
            } else {
                w.sc = *reinterpret_cast<const uint4 *>(d.fd + p);
                w.l = *reinterpret_cast<const uint2 *>(d.fd_last + p);
                w.s = *reinterpret_cast<const uint32_t *>(d.fd_state + p);
            }
            // PW is a multiple of 4 and each wave's 4 words start on a multiple of 4
            const uint32_t wi = cb * 16u + wv * 4u + (ln & 1u) * 2u;
            w.pw = *reinterpret_cast<const ulonglong2 *>(prow + (real && phv && wi < d.PW ? wi : 0u));
        };
        auto chunk = [&](uint32_t cb, const LW &cur, LW &nxt) __attribute__((always_inline)) {
            const uint32_t c0 = (cb * LB + threadIdx.x) * 4u;
            // the general layout's dict positions: loaded before the prefetch (and always, from a shared word
            // of this row otherwise) so that their wait leaves the prefetch in flight
            uint32_t ps[4];
            {
                const bool pl = upo && genm && c0 < d.ncol;
                const uint4 pv = *reinterpret_cast<const uint4 *>(pl ? d.pos + pix(d, o, c0) : d.fd + pix(d, o, 0u));
                ps[0] = pv.x; ps[1] = pv.y; ps[2] = pv.z; ps[3] = pv.w;
            }
            ldw(cb + 1u, cb + 1u < cb1, nxt);
            const uint4 sc4 = cur.sc;
            const uint2 l4 = cur.l;
            const uint32_t s4 = cur.s;
            if (vm) {
                __builtin_amdgcn_wave_barrier();  // this wave is done with the previous chunk's words
                const uint32_t wi = cb * 16u + wv * 4u + (ln & 1u) * 2u;
                if (phv) *reinterpret_cast<ulonglong2 *>(&s_pl[wv][ph][(ln & 1u) * 2u]) = wi < d.PW ? cur.pw : make_ulonglong2(0ull, 0ull);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
            if (c0 < d.ncol) {
                const size_t p = pix(d, o, c0);
                // this thread's four columns: bit ph of q[i] = a report in phase ph
                uint32_t q[4] = {0u, 0u, 0u, 0u};
                if (d.pl16) {  // k_pass1v's layout: column 16 g + 4 q + i at bit 4 i + q of u16 g
                    const uint32_t ui = (c0 & 255u) >> 4, qs = (c0 >> 2) & 3u;
                    for (uint32_t m = vm; m; m &= m - 1u) {
                        const uint32_t ph = (uint32_t)__builtin_ctz(m);
                        const uint32_t u = (uint32_t)reinterpret_cast<const uint16_t *>(s_pl[wv][ph])[ui] >> qs;
        #pragma unroll
                        for (int i = 0; i < 4; i++) q[i] |= ((u >> (4 * i)) & 1u) << ph;
                    }
                } else {
                    const uint32_t lb = plane_bit(c0);
                    for (uint32_t m = vm; m; m &= m - 1u) {
                        const uint32_t ph = (uint32_t)__builtin_ctz(m);
        #pragma unroll
                        for (int i = 0; i < 4; i++) q[i] |= (uint32_t)((s_pl[wv][ph][i] >> lb) & 1ull) << ph;
                    }
                }
                uint32_t sc[4] = {sc4.x, sc4.y, sc4.z, sc4.w};
                uint32_t lt[4] = {l4.x & 0xFFFFu, l4.x >> 16, l4.y & 0xFFFFu, l4.y >> 16};
                bool dw = false;
                uint32_t td[4] = {NONE, NONE, NONE, NONE};
                if (exact && (s4 & 0x02020202u)) { ld4(d.tod + p, td); alg += 16; }
                uint32_t s4n = s4;
        #pragma unroll
                for (int i = 0; i < 4; i++) {
                    uint32_t st = (s4 >> (8 * i)) & 0xFFu;
                    Fd f = fd_get(d, st, lt[i], sc[i], t);  // t is at or after every report tick of this round
                    uint32_t m = q[i];  // only if vm != 0: then the window was loaded
                    if (m) {
                        // report_heartbeat at ticks plane_tick(p) for the phases p of m (failure_detector.py:32-38):
                        // non-decreasing, and less than NPL ticks apart within a base, so with max_interval >= NPL - 1
                        // all but the first are appended (sub-phases at one tick append 0 s, as the reference does
                        // for two reports at one time) and they telescope: (k - 1) intervals summing to
                        // tick(p_last) - tick(p_first), plus the first one if it is <= max_interval; a compact window
                        // that would fill up, and the rings (their intervals one by one), replay report by report
                        bool loop = (RING && rrow) || d.max_iv < NPL - 1u;
                        if (!loop) {
                            const uint32_t p1 = (uint32_t)__builtin_ctz(m), pk = 31u - (uint32_t)__builtin_clz(m);
                            const uint32_t t1 = plane_tick(d, p1), tk = plane_tick(d, pk);
                            uint32_t app = (uint32_t)__popc(m) - 1u, add = tk - t1;
                            if (f.last != NONE) {
                                const uint32_t iv = t1 - f.last;
                                if (iv <= d.max_iv) { app++; add += iv; }
                            }
                            if (f.cnt + app <= d.W) {
                                f.cnt += app;
                                f.sum += add;
                                f.last = tk;
                            } else {
                                loop = true;
                            }
                        }
                        if (loop) {
                            while (m) {
                                const uint32_t bb = (uint32_t)__builtin_ctz(m);
                                m &= m - 1u;
                                f = fd_report_val(d, RING && rrow ? rrow + (size_t)(c0 + i) * d.W : nullptr, plane_tick(d, bb),
                                                  f, alg, ovf);
                            }
                        }
                        dw = true;
                    }
                    const uint32_t j = c0 + i;
                    if (upo && j < d.ncol && d.col_lo + j != o && !(genm && ps[i] == NONE)) {
                        live++;
                        const bool has = f.last != NONE;
                        const uint32_t len = RING && rrow ? (f.cnt < d.W ? f.cnt : d.W) : f.cnt;
                        bool alive = false;
                        if (has && len) {
                            // phi <= threshold (failure_detector.py:43-53, 97-98) decided without the two binary64
                            // divisions when it is clear by a margin: phi ~ elapsed (len + 5) / (sum + 5 prior) in
                            // ticks.  First in binary32 (full rate: elapsed < 2^24 ticks, len + 5 and sum < 2^24 are
                            // exact, the three roundings and the two constants' add < 2^-21 relative) with a 2^-20
                            // margin, then in binary64 with 2^-30 (far above its rounding), the exact expression
                            // otherwise
        #if LIVE_F32
                            const float lf = (float)(t - f.last) * (float)(len + 5u);
                            const float rf = d.phi_thr_f * ((float)f.sum + d.prior5t_f);
                            if (lf < rf * (1.0f - 0x1p-20f)) {
                                alive = true;
                            } else if (!(lf > rf * (1.0f + 0x1p-20f))) {  // too close: the exact expression
        #else
                            const double lhs = (double)(t - f.last) * (double)(len + 5u);  // exact: < 2^43
                            const double rhs = d.phi_thr * ((double)f.sum + d.prior5t);
                            if (lhs < rhs * (1.0 - 0x1p-30)) {
                                alive = true;
                            } else if (!(lhs > rhs * (1.0 + 0x1p-30))) {
        #endif
                                const double mean = ((double)f.sum * TICK_S + d.prior5) / ((double)len + 5.0);
                                alive = ((double)(t - f.last) * TICK_S) / mean <= d.phi_thr;
                            }
                        }
                        const uint32_t mb = st & FD_MEMB;
                        // node join / leave: the live set against the previous call's (server.py:611-616)
                        if (d.ev && alive != (mb == FD_LIVE))
                            emit_event(d, o, d.col_lo + j, (alive ? EV_JOIN : EV_LEAVE) << 8, 0u, 0u, t, 0u);
                        uint32_t sn = FD_LIVE;
                        if (!alive) {
                            sn = FD_DEAD;
                            uint32_t tod = td[i];  // loaded for the dead pairs of a row being recomputed
                            if (mb != FD_DEAD) { tod = t; d.tod[p + i] = t; alg += 4; }  // time_of_death recorded once
                            if (has && (f.sum | f.cnt)) { f.sum = f.cnt = 0u; dw = true; }  // reset
                            if (mb != FD_DEAD || exact) {
                                const uint32_t sat = tod + d.sched_delay;
                                if (sat < minS) minS = sat;
                            }
                            if (exact && (uint64_t)t >= (uint64_t)tod + d.dead_grace) gcdue++;
                        }
                        st = (st & ~(uint32_t)FD_MEMB) | sn;
                    }
                    // a window whose last report is >= FD_OLD_AGE old keeps only that fact (fd_get)
                    if ((st & (FD_WIN | FD_OLD)) == FD_WIN && t - f.last >= FD_OLD_AGE) st |= FD_OLD;
                    if (q[i]) st = fd_st(st, f);
                    sc[i] = fd_sc(d, f);
                    lt[i] = f.last & 0xFFFFu;
                    s4n = (s4n & ~(0xFFu << (8 * i))) | (st << (8 * i));
                }
                if (dw) {
                    if (LIVE_NT) {
                        __builtin_nontemporal_store(v4u_t{sc[0], sc[1], sc[2], sc[3]}, reinterpret_cast<v4u_t *>(d.fd + p));
                        __builtin_nontemporal_store(v2u_t{lt[0] | (lt[1] << 16), lt[2] | (lt[3] << 16)},
                                                    reinterpret_cast<v2u_t *>(d.fd_last + p));
                    } else {
                        *reinterpret_cast<uint4 *>(d.fd + p) = make_uint4(sc[0], sc[1], sc[2], sc[3]);
                        *reinterpret_cast<uint2 *>(d.fd_last + p) = make_uint2(lt[0] | (lt[1] << 16), lt[2] | (lt[3] << 16));
                    }
                    alg += 24;
                }
                if (s4n != s4) {
                    if (LIVE_NT) __builtin_nontemporal_store(s4n, reinterpret_cast<uint32_t *>(d.fd_state + p));
                    else *reinterpret_cast<uint32_t *>(d.fd_state + p) = s4n;
                    alg += 4;
                }
                if (upo || vm) alg += 28;  // the four windows (sum | cnt, last tick) and state bytes read
            }
        };
        LW w0, w1;
        ldw(cb0, true, w0);
        for (uint32_t cb = cb0; cb < cb1; cb += 2u) {
            chunk(cb, w0, w1);
            if (cb + 1u < cb1) chunk(cb + 1u, w1, w0);
        }
    }
    // earliest scheduled-for-deletion tick of this row
    for (int dd = 32; dd >= 1; dd >>= 1) {
        const uint32_t y = __shfl_xor(minS, dd, WAVE);
        if (y < minS) minS = y;
    }
    // in-kernel algorithmic bytes (C_LIVEB): windows, states, times of death and ring entries read and
    // written (fd_report_val's per-report 16 B estimate is replaced by these element counts), and the
    // report planes staged (32 B per valid phase per wave and chunk)
    const unsigned long long sl = wave_sum(live), sg = wave_sum(gcdue), so = wave_sum(ovf), sa = wave_sum(alg);
    if ((threadIdx.x & 63) == 0) {
        if (minS != NONE) atomicMin(&d.row[o * 4 + 2], minS);
        if (sl) shard_add(d, C_LIVE, sl);
        shard_add(d, C_LIVEB, sa + (unsigned long long)__popc(vm) * 32u * (cb1 - cb0));
        // a full compact window that needed an eviction: an error, except with sampled rings, where the
        // compact rows are documented as exact only up to W intervals (fd_saturated)
        if (so) shard_add(d, d.ring_slot ? C_FDSAT : C_E_FDOVF, so);
        if (sg) {
            if (genm) atomicOr(&d.row[o * 4 + 3], 1u);  // k_fd_gc collects this row
            else shard_add(d, C_E_FDGC, sg);  // removal would break the canonical layout
        }
    }
}

// FailureDetector.garbage_collect + ClusterState.remove_node, the tail of _update_node_liveness
// (failure_detector.py:108-119, server.py:618-620), for rows k_liveness flagged.  The reference walks
// _dead_nodes in insertion order = (time of death, dict position) and deletes the dead entry, then
// the sampling window, of each expired target; a target without a window raises KeyError there
// (SURVEY Q9): earlier targets lose dead entry + window, the failing one its dead entry, later ones
// nothing, and no node leaves the dict.  Otherwise every expired target leaves the dict (the
// insertion order of the others is kept: stable compaction of ORD/POS).
__global__ __launch_bounds__(LB) void k_fd_gc(Dev d, const uint8_t *up, uint32_t t) {
    __shared__ unsigned long long s_key[LB / WAVE];
    __shared__ uint32_t s_wsum[LB / WAVE];
    extern __shared__ __attribute__((aligned(16))) uint32_t rmv[];  // removal bitmap, NP bits
    const uint32_t o = blockIdx.x;
    if (!up[o] || !(d.row[o * 4 + 3] & 1u)) return;
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid >> 6;
    const size_t ro = (size_t)o * d.NP;
    const uint32_t cnt = d.row[o * 4 + 0];
    // 1. earliest expired target (in dead-dict order) that has no window
    unsigned long long fkey = ~0ull;
    for (uint32_t j = tid; j < d.ncol; j += LB) {
        const uint32_t tod = dead_tod(d, ro + j), pos = d.pos[ro + j];
        if (tod != NONE && pos != NONE && (uint64_t)t >= (uint64_t)tod + d.dead_grace && !(d.fd_state[ro + j] & FD_WIN)) {
            const unsigned long long key = ((unsigned long long)tod << 32) | pos;
            if (key < fkey) fkey = key;
        }
    }
    for (int dd = 32; dd >= 1; dd >>= 1) {
        const unsigned long long y = __shfl_xor(fkey, dd, WAVE);
        if (y < fkey) fkey = y;
    }
    if (lane == 0) s_key[wid] = fkey;
    for (uint32_t i = tid; i < d.NP / 32; i += LB) rmv[i] = 0u;
    __syncthreads();
    fkey = ~0ull;
    for (int w = 0; w < LB / WAVE; w++) fkey = s_key[w] < fkey ? s_key[w] : fkey;
    const bool q9 = fkey != ~0ull;
    // 2. drop dead entries / windows; mark dict removals
    uint32_t gcn = 0;
    for (uint32_t j = tid; j < d.ncol; j += LB) {
        const uint32_t tod = dead_tod(d, ro + j), pos = d.pos[ro + j];
        if (!(tod != NONE && pos != NONE && (uint64_t)t >= (uint64_t)tod + d.dead_grace)) continue;
        const unsigned long long key = ((unsigned long long)tod << 32) | pos;
        if (q9 && key > fkey) continue;
        if (q9 && key == fkey) {
            d.fd_state[ro + j] &= (uint8_t)~FD_MEMB;  // del self._dead_nodes[gossip_id]
            continue;
        }
        d.fd_state[ro + j] = 0u;  // ... and del self._node_samples[gossip_id]
        d.fd[ro + j] = 0u;
        gcn++;
        if (!q9) atomicOr(&rmv[j >> 5], 1u << (j & 31u));
    }
    __syncthreads();
    if (!q9) {
        // 3. remove_node: stable compaction of the dict order, clear the removed views
        uint32_t base = 0;
        for (uint32_t p0 = 0; p0 < cnt; p0 += LB) {
            const uint32_t p = p0 + tid;
            const uint32_t j = p < cnt ? d.ord[ro + p] : NONE;
            const bool keep = j != NONE && !bit(rmv, j);
            const unsigned long long m = __ballot(keep);
            const uint32_t rk = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (lane == 0) s_wsum[wid] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t off = base, tot = 0;
            for (int w = 0; w < LB / WAVE; w++) {
                if (w < wid) off += s_wsum[w];
                tot += s_wsum[w];
            }
            if (keep) {
                d.ord[ro + off + rk] = j;
                d.pos[ro + j] = off + rk;
            }
            base += tot;
            __syncthreads();
        }
        for (uint32_t j = tid; j < d.ncol; j += LB) {
            if (!bit(rmv, j)) continue;
            const size_t p = ro + j;
            d.pos[p] = NONE;
            hb_put(d, p, 0u);
            mv_put(d, p, 0u);
            if (d.flags & GS_TOMBSTONES) d.gc[p] = 0u;
            if (d.held)
                for (uint32_t k = 0; k < d.KP; k += 4) *reinterpret_cast<uint32_t *>(d.held + p * d.KP + k) = 0u;
            if (d.flags & GS_TOMBSTONES)
                for (uint32_t k = 0; k < d.KP; k++) d.ts[p * d.KP + k] = NONE;
        }
        if (tid == 0) d.row[o * 4 + 0] = base;
    }
    if (tid == 0) {
        d.row[o * 4 + 3] &= ~1u;
        if (q9) shard_add(d, C_Q9, 1);
    }
    const unsigned long long sg = wave_sum(gcn);
    if (lane == 0) shard_add(d, C_FDGC, sg);
}

// Membership census over (observer, target) pairs, observer up and target != observer, from the
// failure detector's live / dead sets (failure_detector.py:60-67): by whether the target is up
// {up pairs, up and dead-marked (false positives), up and live, down pairs, down and live}.
__global__ __launch_bounds__(LB) void k_fd_census(Dev d, const uint8_t *up) {
    const uint32_t o = blockIdx.y;
    const uint32_t j = blockIdx.x * LB + threadIdx.x;
    uint32_t c[5] = {0u, 0u, 0u, 0u, 0u};
    if (up[o] && j < d.ncol && d.col_lo + j != o) {
        const uint32_t st = d.fd_state[pix(d, o, j)] & FD_MEMB;
        if (up[d.col_lo + j]) {
            c[0] = 1u;
            c[1] = st >= 2u;
            c[2] = st == 1u;
        } else {
            c[3] = 1u;
            c[4] = st == 1u;
        }
    }
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const unsigned long long v = wave_sum(c[i]);
        if ((threadIdx.x & 63) == 0) shard_add(d, C_CEN0 + i, v);
    }
}

__global__ void k_zero_slots(Dev d, uint32_t lo, uint32_t n) {
    const uint32_t i = threadIdx.x;
    if (i < NSHARD * n) d.ctr[(i / n) * CROW + lo + i % n] = 0ull;
}

// SamplingWindow.phi (failure_detector.py:43-53) of every target of observer o; NaN for None.
__global__ __launch_bounds__(LB) void k_phi_row(Dev d, uint32_t o, uint32_t t, double *out) {
    const uint32_t j = blockIdx.x * LB + threadIdx.x;
    if (j >= d.ncol) return;
    const size_t p = pix(d, o, j);
    const uint32_t st = d.fd_state[p];
    const Fd f = fd_get(d, st, d.fd_last[p], d.fd[p], t);
    if ((st & FD_OLD) && f.cnt) shard_add(d, C_E_FDOVF, 1);  // phi of a window silent for >= 2^15 ticks: inexact
    // ring windows count up to 2W (len = min(cnt, W)); a compact window never holds more than W
    const uint32_t len = f.cnt < d.W ? f.cnt : d.W;
    double phi = __builtin_nan("");
    if (f.last != NONE && len) {
        const double mean = ((double)f.sum * TICK_S + d.prior5) / ((double)len + 5.0);
        phi = ((double)(t - f.last) * TICK_S) / mean;
    }
    out[j] = phi;
}

// Marks every window whose last report is >= FD_OLD_AGE ticks before t FD_OLD (all rows; the host runs
// it at least every 2^14 ticks, so an unmarked window is < 2^15 + 2^14 ticks old and decodes exactly).
__global__ __launch_bounds__(LB) void k_fd_age(Dev d, uint32_t t) {
    const uint64_t total = (uint64_t)d.N * d.NP / 4;
    for (uint64_t x = (uint64_t)blockIdx.x * LB + threadIdx.x; x < total; x += (uint64_t)gridDim.x * LB) {
        const size_t p = x * 4;
        const uint32_t s4 = *reinterpret_cast<const uint32_t *>(d.fd_state + p);
        if (!(s4 & 0x04040404u)) continue;
        const uint2 l4 = *reinterpret_cast<const uint2 *>(d.fd_last + p);
        const uint32_t lt[4] = {l4.x & 0xFFFFu, l4.x >> 16, l4.y & 0xFFFFu, l4.y >> 16};
        uint32_t s4n = s4;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t st = (s4 >> (8 * i)) & 0xFFu;
            if ((st & (FD_WIN | FD_OLD)) == FD_WIN && ((t - lt[i]) & 0xFFFFu) >= FD_OLD_AGE) s4n |= (uint32_t)FD_OLD << (8 * i);
        }
        if (s4n != s4) *reinterpret_cast<uint32_t *>(d.fd_state + p) = s4n;
    }
}

// 16-bit heartbeats (hb_dec) are exact while every view lags its owner's own heartbeat by < 2^16.  An
// owner's heartbeat grows by at most one per round start or phase, and the host runs this sweep at
// least every 2^14 of those: if every decoded lag was < 2^15 at the previous sweep (and so exact), every
// lag is < 2^15 + 2^14 < 2^16 until this one, so every decode in between was exact and this sweep's
// decoded lags are the true ones -- a view at >= 2^15 is counted in err_hb_lag (the run is reported
// inexact) before any decode can go wrong.
// GS_HB8 (views mod 2^8): the same argument with a sweep at least every 64 round starts + phases (checked
// before every round start and every phase, so at most 64 increments apart) and lags >= 2^7 counted:
// < 2^7 + 2^6 < 2^8.
// GS_MV8 (max_version views mod 2^7): a view only falls behind when its owner writes (one version per
// gs_owner_writes call at most), gs_owner_writes sweeps at least every 32 calls, and lags >= 2^6 are
// counted: < 2^6 + 2^5 < 2^7 between sweeps.
// The same sweep marks the views k_pass1v's byte-parallel path may not take (GS_R_P1FLAGS, ROW word 3 bit 2):
// a view lagging by >= HOT_HB heartbeats or HOT_MV versions makes its owner column "hot", or, when a chunk
// of the row holds HOT_ROW_MIN such views (a node back from a long absence), its observer row.  Between two
// sweeps a view falls behind by at most 64 heartbeats (HB8_LAG_CHECK_EVERY) and 32 versions
// (MV8_LAG_CHECK_EVERY), so every view of a row and column that are not hot lags by < 128 heartbeats and
// < 64 versions: the bounds under which pass 1 compares two 8-bit views without their owner's value.
// One workgroup per (row, chunk of LB x 16 columns); each thread reads 16 views (u8) or 8 (u16).
constexpr uint32_t HOT_HB = 64, HOT_MV = 32, HOT_ROW_MIN = 16;
// One workgroup per (LAG_ROWS consecutive observer rows, 4,096-column chunk): a row's chunk is 16 bytes per
// region and thread, too little for a workgroup of its own (one per row: 1 M workgroups at 65,536 nodes, 4.1 ms
// per sweep, 2.1 TB/s); the next row's views are loaded while this row's are checked.
constexpr uint32_t LAG_ROWS = 16;
__global__ __launch_bounds__(LB) void k_hb_lag(Dev d, uint32_t chunks) {
    __shared__ uint32_t s_hot[LAG_ROWS];
    __shared__ uint16_t s_hm[LAG_ROWS][LB];  // each row's hot views of this thread's 16 columns
    const bool genm = !(d.flags & GS_CANONICAL);
    const uint32_t rb = blockIdx.x / chunks, cb = blockIdx.x % chunks;
    const uint32_t per = d.hb8 ? 16u : 8u;
    const uint32_t j0 = (cb * LB + threadIdx.x) * per;
    const uint32_t o0 = rb * LAG_ROWS, nrow = min(LAG_ROWS, d.N - o0);
    uint32_t bad = 0;
    uint32_t hotc = 0;  // views of escaped columns: always mark the column (k_esc_plan's release test)
    if (d.p1flags) {
        if (threadIdx.x < LAG_ROWS) s_hot[threadIdx.x] = 0u;
        __syncthreads();
    }
    // one 16-byte load per region and row: the thread's heartbeat views (and GS_MV8 max_version views)
    // (8-bit views: streamed once per sweep, non-temporal), one row ahead
    auto ldv = [&](uint32_t o, uint4 &hr, uint4 &mr) {
        const size_t p0 = pix(d, o, j0 < d.ncol ? j0 : 0u);
        mr = make_uint4(0u, 0u, 0u, 0u);
        if (d.hb8) {
            const v4u_t x = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(reinterpret_cast<const uint8_t *>(d.hb) + p0));
            hr = make_uint4(x.x, x.y, x.z, x.w);
        } else {
            hr = *reinterpret_cast<const uint4 *>(d.hb + p0);
        }
        if (d.mv8) {
            const v4u_t x = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(reinterpret_cast<const uint8_t *>(d.mv) + p0));
            mr = make_uint4(x.x, x.y, x.z, x.w);
        }
    };
    uint4 nh, nm;
    ldv(o0, nh, nm);
    // the headline's layout (canonical, GS_HB8 + GS_MV8): four views per 32-bit word against the owners'
    // packed own values (SELF_PK: heartbeat mod 2^8 in byte 0, max_version in the high half), per-byte
    // lags with borrow-isolated subtracts; only escaped columns and escape requests go column by column.
    // The owners' values and escape slots are the same for every row: loaded once (L2 reads 4x the rows' bytes)
    const bool swar = !genm && d.hb8 && d.mv8 && d.self_pk;
    uint32_t own8v[4] = {0u, 0u, 0u, 0u}, owm7v[4] = {0u, 0u, 0u, 0u}, vm7v[4] = {0u, 0u, 0u, 0u}, esc7v[4] = {0u, 0u, 0u, 0u};
    uint32_t esv[4][4];
#pragma unroll
    for (uint32_t q = 0; q < 4u; q++) {
        const uint32_t jq = j0 + 4u * q;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) esv[q][i] = NONE;
        if (!swar || jq >= d.ncol) continue;  // (vm7v[q] = 0: the step's bits all clear)
        const uint4 pk = *reinterpret_cast<const uint4 *>(d.self_pk + jq);
        own8v[q] = (pk.x & 0xFFu) | ((pk.y & 0xFFu) << 8) | ((pk.z & 0xFFu) << 16) | (pk.w << 24);
        owm7v[q] = ((pk.x >> 16) & 0x7Fu) | (((pk.y >> 16) & 0x7Fu) << 8) | (((pk.z >> 16) & 0x7Fu) << 16) |
                   (((pk.w >> 16) & 0x7Fu) << 24);
        const uint32_t nv = min(d.ncol - jq, 4u);
        vm7v[q] = nv >= 4u ? B7 : B7 & ((1u << (8u * nv)) - 1u);  // bit 7 of the valid columns
        if (d.EC) {
            ld4(d.esc_slot + jq, esv[q]);
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) esc7v[q] |= (uint32_t)(esv[q][i] != NONE) << (8 * i + 7);
        }
    }
    for (uint32_t r = 0; r < nrow; r++) {
    const uint32_t o = o0 + r;
    const uint4 hr = nh, mr = nm;
    ldv(o0 + min(r + 1u, nrow - 1u), nh, nm);  // (the last row reloads itself: no wait counts a load as absent)
    uint32_t hot = 0;  // bit k = view k of this thread's (at most 16)
    if (j0 < d.ncol) {
        const size_t p0 = pix(d, o, j0);
        const uint32_t hw[4] = {hr.x, hr.y, hr.z, hr.w}, mw[4] = {mr.x, mr.y, mr.z, mr.w};
        if (swar) {
#pragma unroll
            for (uint32_t q = 0; q < 4u; q++) {
                const uint32_t jq = j0 + 4u * q;
                const uint32_t own8 = own8v[q], owm7 = owm7v[q], vm7 = vm7v[q], esc7 = esc7v[q];
                const uint32_t *es = esv[q];
                const uint32_t lagH = bsub(own8, hw[q]);                            // (own - view) mod 2^8
                const uint32_t lagM = ((owm7 | B7) - (mw[q] & L7)) & L7;           // (own - view) mod 2^7
                const uint32_t hb7 = lagH & B7 & ~esc7 & vm7;                       // heartbeat lag >= 2^7
                const uint32_t hh7 = (lagH | (lagH << 1)) & B7 & ~esc7 & vm7;       // >= HOT_HB (64)
                const uint32_t mb7 = (lagM << 1) & B7 & vm7;                        // max_version lag >= 2^6
                const uint32_t mh7 = ((lagM << 1) | (lagM << 2)) & B7 & vm7;        // >= HOT_MV (32)
                hot |= nib7(hh7 | mh7) << (4u * q);
                bad += (uint32_t)__popc(mb7);
                if (hb7) {
                    if (d.EC) {
                        for (uint32_t m = hb7; m; m &= m - 1u) {
                            const uint32_t j = jq + ((uint32_t)__builtin_ctz(m) >> 3);
                            atomicOr(&d.esc_req[j >> 5], 1u << (j & 31u));
                        }
                    } else {
                        bad += (uint32_t)__popc(hb7);
                    }
                }
                for (uint32_t m = esc7 & vm7; m; m &= m - 1u) {  // escaped columns: 16-bit views, exact while < 2^15
                    const uint32_t i = (uint32_t)__builtin_ctz(m) >> 3;
                    const uint32_t R = d.self_hb[jq + i];
                    const uint32_t lag = (R - d.esc16[(size_t)o * d.EC + es[i]]) & 0xFFFFu;
                    if (lag >= 0x8000u) bad++;
                    hotc |= (uint32_t)(lag >= HOT_HB) << (4u * q + i);
                }
            }
        }
        for (uint32_t q = 0; !swar && q < per / 4u && j0 + 4u * q < d.ncol; q++) {
            const uint32_t jq = j0 + 4u * q;
            // the owners' own values, 4 columns per 16-byte load (L2)
            const uint4 ow = *reinterpret_cast<const uint4 *>(d.self_hb + jq);
            const uint4 om = d.mv8 ? *reinterpret_cast<const uint4 *>(d.self_mv + jq) : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t own[4] = {ow.x, ow.y, ow.z, ow.w}, owm[4] = {om.x, om.y, om.z, om.w};
            uint32_t ps[4] = {0u, 0u, 0u, 0u};
            if (genm) ld4(d.pos + p0 + 4u * q, ps);
            uint32_t es[4] = {NONE, NONE, NONE, NONE};  // escape slots (gs_config.esc_cols)
            if (d.EC) ld4(d.esc_slot + jq, es);
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                if (jq + i >= d.ncol || (genm && ps[i] == NONE)) continue;
                const uint32_t k = 4u * q + i;  // view index within the thread's loads
                bool h;
                if (es[i] != NONE) {  // an escaped column: 16-bit views, exact while they lag by < 2^15
                    const uint32_t lag = (own[i] - d.esc16[(size_t)o * d.EC + es[i]]) & 0xFFFFu;
                    if (lag >= 0x8000u) bad++;
                    hotc |= (uint32_t)(lag >= HOT_HB) << k;  // no view hot at this sweep: k_esc_plan moves it back
                    h = false;
                } else {
                    const uint32_t s = d.hb8 ? (hw[k >> 2] >> (8 * (k & 3))) & 0xFFu : (hw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                    const uint32_t lag = d.hb8 ? (own[i] - s) & 0xFFu : (own[i] - s) & 0xFFFFu;
                    if (lag >= (d.hb8 ? 0x80u : 0x8000u)) {
                        // 8-bit views: escape the column (k_esc_plan; its views lag by < 2^7 + 2^6 now, exact), or,
                        // without escape slots, count the view
                        if (d.EC) atomicOr(&d.esc_req[(jq + i) >> 5], 1u << ((jq + i) & 31u));
                        else bad++;
                    }
                    h = d.hb8 && lag >= HOT_HB;
                }
                if (d.mv8) {  // GS_MV8: max_version views lag their owner by < 2^6 at every sweep
                    const uint32_t sm = (mw[k >> 2] >> (8 * (k & 3))) & 0x7Fu;
                    const uint32_t ml = (owm[i] - sm) & 0x7Fu;
                    if (ml >= 0x40u) bad++;
                    h = h || ml >= HOT_MV;
                }
                hot |= (uint32_t)h << k;
            }
        }
    }
    if (d.p1flags) {  // this row's hot views in its chunk (counted for the row's hot test below)
        const unsigned long long wn = wave_sum((uint32_t)__popc(hot));
        if ((threadIdx.x & 63) == 0 && wn) atomicAdd(&s_hot[r], (uint32_t)wn);
        s_hm[r][threadIdx.x] = (uint16_t)hot;
    }
    }
    if (d.p1flags) {  // k_pass1v's hot rows and columns (cleared by k_hot_clear before the sweep)
        __syncthreads();
        uint32_t col = hotc;
        for (uint32_t r = 0; r < nrow; r++) {
            if (s_hot[r] >= HOT_ROW_MIN) {  // a hot row: its views take the per-column path, not its columns
                if (threadIdx.x == 0) atomicOr(&d.row[(o0 + r) * 4 + 3], 4u);
            } else {
                col |= s_hm[r][threadIdx.x];
            }
        }
        if (col && j0 < d.ncol) atomicOr(&d.p1flags[j0 >> 4], col << 16);  // 16 views: one 16-column group
    }
    const unsigned long long sb = wave_sum(bad);
    if ((threadIdx.x & 63) == 0) shard_add(d, C_E_HBLAG, sb);
}
// k_hb_lag's hot marks start from nothing at every sweep
__global__ __launch_bounds__(LB) void k_hot_clear(Dev d) {
    const uint32_t i = blockIdx.x * LB + threadIdx.x;
    if (i < d.N) d.row[i * 4 + 3] &= ~4u;
    if (i < d.NP / 16u) d.p1flags[i] &= 0xFFFFu;
}

// Escaped owner columns (gs_config.esc_cols), after a lag sweep: one workgroup decides the moves -- an escaped
// column none of whose views is hot any more (every lag < HOT_HB) goes back to 8-bit views, a column the sweep
// flagged (a view lagging by >= 2^7) takes a free slot (none free: counted in err_hb_lag) -- and marks every
// escaped column hot (pass 1 takes them on its per-column path); k_esc_move then copies the columns.  A slot
// released here is not reused before the next sweep (the copy out reads it).
constexpr uint32_t ESC_MAX = 4096;
__device__ inline uint32_t *esc_moves(const Dev &d) { return d.esc_req + d.NP / 32; }  // [0] count, then pairs
__global__ __launch_bounds__(1024) void k_esc_plan(Dev d) {
    __shared__ uint32_t s_free[ESC_MAX];
    __shared__ uint32_t s_nfree, s_next, s_nmove, s_esc, s_rel, s_err;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) { s_nfree = 0; s_next = 0; s_nmove = 0; s_esc = 0; s_rel = 0; s_err = 0; }
    __syncthreads();
    uint32_t *mv = esc_moves(d);
    // releases, and the slots free before this sweep
    for (uint32_t sl = tid; sl < d.EC; sl += 1024) {
        const uint32_t j = d.esc_owner[sl];
        if (j == NONE) {
            s_free[atomicAdd(&s_nfree, 1u)] = sl;
        } else if (!((d.p1flags[j >> 4] >> (16u + (j & 15u))) & 1u)) {
            const uint32_t m = atomicAdd(&s_nmove, 1u);
            mv[1 + 2 * m] = j | 0x80000000u;  // out
            mv[2 + 2 * m] = sl;
            d.esc_slot[j] = NONE;
            d.esc_owner[sl] = NONE;
            atomicAdd(&s_rel, 1u);
        }
    }
    __syncthreads();
    // escapes
    for (uint32_t w = tid; w < d.NP / 32; w += 1024) {
        uint32_t bits = d.esc_req[w];
        if (!bits) continue;
        d.esc_req[w] = 0u;
        for (; bits; bits &= bits - 1u) {
            const uint32_t j = w * 32u + (uint32_t)__builtin_ctz(bits);
            if (d.esc_slot[j] != NONE) continue;  // (already escaped: the sweep flags bytes only)
            const uint32_t k = atomicAdd(&s_next, 1u);
            if (k >= s_nfree) { atomicAdd(&s_err, 1u); continue; }
            const uint32_t sl = s_free[k];
            d.esc_owner[sl] = j;
            d.esc_slot[j] = sl;
            const uint32_t m = atomicAdd(&s_nmove, 1u);
            mv[1 + 2 * m] = j;  // in
            mv[2 + 2 * m] = sl;
            atomicAdd(&s_esc, 1u);
        }
    }
    __syncthreads();
    // every escaped column is hot until it is moved back
    for (uint32_t sl = tid; sl < d.EC; sl += 1024) {
        const uint32_t j = d.esc_owner[sl];
        if (j != NONE) atomicOr(&d.p1flags[j >> 4], 1u << (16u + (j & 15u)));
    }
    if (tid == 0) {
        mv[0] = s_nmove;
        shard_add(d, C_ESC, s_esc);
        shard_add(d, C_ESCREL, s_rel);
        shard_add(d, C_E_HBLAG, s_err);  // no free slot: the column stays in bytes, the run is reported inexact
    }
}
// The moves of k_esc_plan for every observer row (one thread per row): in = the 8-bit view decoded against the
// owner's own heartbeat (its lag < 2^7 + 2^6: exact) into the slot, out = the slot's view back to its byte (lag
// < HOT_HB: exact)
__global__ __launch_bounds__(LB) void k_esc_move(Dev d) {
    const uint32_t o = blockIdx.x * LB + threadIdx.x;
    if (o >= d.N) return;
    const uint32_t *mv = esc_moves(d);
    const uint32_t nm = mv[0];
    uint8_t *h8 = reinterpret_cast<uint8_t *>(d.hb);
    for (uint32_t m = 0; m < nm; m++) {
        const uint32_t jw = mv[1 + 2 * m], sl = mv[2 + 2 * m], j = jw & 0x7FFFFFFFu;
        const uint32_t R = d.self_hb[j];
        const size_t p = pix(d, o, j), e = (size_t)o * d.EC + sl;
        if (jw & 0x80000000u) h8[p] = (uint8_t)hb_dec(d.esc16[e], R);
        else d.esc16[e] = (uint16_t)hb_dec8(h8[p], R);
    }
}

// ------------------------------------------------------------------ owner writes
// NodeState.set / delete / set_with_ttl / delete_after_ttl on the owner's own view (state.py:124-180).
// Dev::sm (round 6), in two launches over blocks of 1,024 columns: k_sm_local -- one column per thread, the
// block's suffix minima (LDS scan) and the block's minimum into sm_blk; k_sm_fix -- each column's value min the
// minima of the later blocks
__device__ __forceinline__ uint32_t lb0_col(const Dev &d, uint32_t c) {
    return min(msgf(msgf(d.nid_size[c]) + 2u + (d.vlog[(size_t)c * d.VL] & 0xFFFFu)), 0xFFFFu);
}
__global__ __launch_bounds__(1024) void k_sm_local(Dev d, uint32_t *sm_blk) {
    __shared__ uint32_t s_m[1024];
    const uint32_t t = threadIdx.x, c = blockIdx.x * 1024u + t;
    s_m[t] = c < d.ncol ? lb0_col(d, c) : 0xFFFFu;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {
        const uint32_t v = t + off < 1024u ? s_m[t + off] : 0xFFFFu;
        __syncthreads();
        s_m[t] = min(s_m[t], v);
        __syncthreads();
    }
    if (c < d.ncol) d.sm[c] = (uint16_t)s_m[t];
    if (t == 0) sm_blk[blockIdx.x] = s_m[0];
}
__global__ __launch_bounds__(1024) void k_sm_fix(Dev d, const uint32_t *sm_blk, uint32_t nblk) {
    __shared__ uint32_t s_after;
    const uint32_t t = threadIdx.x, c = blockIdx.x * 1024u + t;
    if (t == 0) {
        uint32_t m = 0xFFFFu;
        for (uint32_t b2 = blockIdx.x + 1u; b2 < nblk; b2++) m = min(m, sm_blk[b2]);
        s_after = m;
    }
    __syncthreads();
    if (c < d.ncol) d.sm[c] = (uint16_t)min((uint32_t)d.sm[c], s_after);
    if (c == 0) d.sm[d.ncol] = 0xFFFFu;
}

__global__ __launch_bounds__(LB) void k_owner_writes(Dev d, const gs_write *ops, uint32_t n, uint32_t t) {
    const uint32_t i = blockIdx.x * LB + threadIdx.x;
    if (i >= n) return;
    const gs_write op = ops[i];
    // deletes and TTL writes leave tombstones, which need GS_TOMBSTONES (receive ticks + GC)
    if (op.owner >= d.N || op.key >= d.K || op.op > 3u || (op.op != GS_OP_SET && !(d.flags & GS_TOMBSTONES))) {
        shard_add(d, C_E_IDX, 1);
        return;
    }
    const uint32_t j = op.owner - d.col_lo, k = op.key;  // local column of the owner
    if (j >= d.ncol) return;  // another slice's owner
    const size_t pj = pix(d, op.owner, j);
    // the owner's own view holds every latest write (no GC of its own keys without tombstones);
    // with GS_NO_HELD its held ordinals are the latest-write table
    uint8_t *held = d.held ? d.held + pj * d.KP + k : d.last_w + (size_t)j * d.KP + k;
    const uint32_t w = *held;
    const uint32_t M = mv_word(d, pj, j);
    uint32_t st, vid, vl;
    if (op.op == GS_OP_SET || op.op == GS_OP_SET_WITH_TTL) {
        st = op.op == GS_OP_SET ? 0u : 2u;
        if (w) {  // same value with the same status: no-op (state.py:140-141, 146-151)
            const size_t h = hix(d, j, w, k);
            if (d.hist_vid[h] == op.value_id && meta_status((uint32_t)(d.hist[h] >> 32)) == st) return;
        }
        vid = op.value_id;
        vl = op.value_len;
    } else {
        if (!w) return;  // delete of an absent key is a no-op (state.py:163-164, 175-176)
        const size_t h = hix(d, j, w, k);
        st = op.op == GS_OP_DELETE ? 1u : 2u;
        vid = op.op == GS_OP_DELETE ? 0u : d.hist_vid[h];        // delete clears the value (171)
        vl = op.op == GS_OP_DELETE ? 0u : meta_vlen((uint32_t)(d.hist[h] >> 32));
    }
    const uint32_t nw = (uint32_t)d.last_w[(size_t)j * d.KP + k] + 1u;
    if (nw >= d.C || vl >= (1u << 14)) { shard_add(d, C_E_HIST, 1); return; }
    const uint32_t ver = M + 1u;
    if (ver > MV_MASK) { shard_add(d, C_E_HIST, 1); return; }
    const size_t h = hix(d, j, nw, k);
    d.hist[h] = (uint64_t)ver |
                ((uint64_t)make_meta(sfield(d.key_len[k]) + sfield(vl) + ufield(ver) + ufield(st), st, vl) << 32);
    d.hist_vid[h] = vid;
    if (d.lat) {
        const uint32_t kvb = msgf(meta_kvlen((uint32_t)(d.hist[h] >> 32)));
        uint32_t *lk = d.lat + (size_t)j * d.KP + k;
        if (d.vlog) {  // the key's previous write (if any) now has a next write at ver
            uint32_t *vl = d.vlog + (size_t)j * d.VL;
            const uint32_t prev = *lk & 0xFFFFu;
            if (prev) vl[prev] = (vl[prev] & 0xFFFFu) | (ver << 16);
            vl[ver] = kvb | 0xFFFF0000u;
            const uint32_t kmin = vl[0];  // entry 0: the owner's smallest kv field over all its writes (min1_lb)
            if (!kmin || kvb < kmin) vl[0] = kvb;
        }
        *lk = ver | (kvb << 16);
    }
    d.last_w[(size_t)j * d.KP + k] = (uint8_t)nw;
    *held = (uint8_t)nw;
    mv_put(d, pj, ver);
    d.self_mv[j] = ver;
    self_repack(d, j);
    // Cluster.set / set_with_ttl emit on_key_change (server.py:193-215, 238-252); delete and
    // delete_after_ttl mutate the stored VersionedValue in place, so old and new are the same
    // object and nothing is emitted (server.py:199-203, 211-215)
    if (d.ev && (op.op == GS_OP_SET || op.op == GS_OP_SET_WITH_TTL))
        emit_event(d, op.owner, op.owner, k | (EV_KEY << 8), w ? (uint32_t)d.hist[hix(d, j, w, k)] : 0u, ver, t,
                   d.ev_wseq + i);
    if (d.flags & GS_TOMBSTONES) {
        d.ts[pj * d.KP + k] = st ? t : NONE;
        if (st) d.row[op.owner * 4 + 1] = 1u;
    }
}

// ------------------------------------------------------------------ boot / warm
__global__ __launch_bounds__(LB) void k_boot_self(Dev d) {
    const uint32_t o = blockIdx.x * LB + threadIdx.x;
    if (o >= d.N) return;
    d.row[o * 4 + 0] = 1u;
    d.row[o * 4 + 1] = 0u;
    d.row[o * 4 + 2] = NONE;
    d.row[o * 4 + 3] = 0u;
    if (o - d.col_lo >= d.ncol) return;
    const size_t p = pix(d, o, o - d.col_lo);
    hb_put(d, p, 1u);  // Cluster.__init__: inc_heartbeat (server.py:95-96)
    d.self_hb[o - d.col_lo] = 1u;
    self_repack(d, o - d.col_lo);
    if (!(d.flags & GS_CANONICAL)) {
        d.pos[p] = 0u;
        d.ord[(size_t)o * d.NP] = o;
    }
}

__global__ __launch_bounds__(LB) void k_warm(Dev d) {
    // grid-stride over (observer, owner) pairs: N^2 exceeds one launch's 2^32 work-items at N = 65,536
    const uint64_t total = (uint64_t)d.N * d.ncol;
    for (uint64_t x = (uint64_t)blockIdx.x * LB + threadIdx.x; x < total; x += (uint64_t)gridDim.x * LB) {
        const uint32_t o = (uint32_t)(x / d.ncol), j = (uint32_t)(x % d.ncol), jg = d.col_lo + j;
        const size_t p = pix(d, o, j);
        if (!(d.flags & GS_CANONICAL)) {
            d.pos[p] = j;
            d.ord[p] = j;
            if (j == 0) d.row[o * 4 + 0] = d.N;
        }
        if (jg == o) continue;
        const size_t q = pix(d, jg, j);  // the owner's own view
        hb_put(d, p, hb_raw(d, q));
        if (d.mv8) reinterpret_cast<uint8_t *>(d.mv)[p] = reinterpret_cast<const uint8_t *>(d.mv)[q];
        else d.mv[p] = d.mv[q];
        if (d.flags & GS_TOMBSTONES) d.gc[p] = d.gc[q];
        if (d.held)
            for (uint32_t k = 0; k < d.KP; k += 4)
                *reinterpret_cast<uint32_t *>(d.held + p * d.KP + k) =
                    *reinterpret_cast<const uint32_t *>(d.held + q * d.KP + k);
        if (d.flags & GS_TOMBSTONES) {
            bool tb = false;
            for (uint32_t k = 0; k < d.KP; k++) {
                const uint32_t v = d.ts[q * d.KP + k];
                d.ts[p * d.KP + k] = v;
                tb |= v != NONE;
            }
            if (tb) d.row[o * 4 + 1] = 1u;
        }
    }
}

// Fill GS_R_HELD for the prefix views of rows [r0, r1) (MV_INEXACT clear: HELD not kept by the
// exchange kernel), so a reader sees every view's held ordinals.  Readback only.
__global__ __launch_bounds__(LB) void k_materialize(Dev d, uint32_t r0, uint32_t r1) {
    const uint64_t total = (uint64_t)(r1 - r0) * d.ncol;
    for (uint64_t x = (uint64_t)blockIdx.x * LB + threadIdx.x; x < total; x += (uint64_t)gridDim.x * LB) {
        const uint32_t o = r0 + (uint32_t)(x / d.ncol), j = (uint32_t)(x % d.ncol);
        const size_t p = pix(d, o, j);
        const uint32_t mv = mv_word(d, p, j);
        if (mv & MV_INEXACT) continue;
        uint32_t h[16], alg = 0;
        derive_held<16>(d, j, mv, h, alg);
        for (uint32_t q = 0; q < d.KP / 4; q++) reinterpret_cast<uint32_t *>(d.held + p * d.KP)[q] = h[q];
    }
}

// ------------------------------------------------------------------ wire-format emitter
// The bytes the reference's SerializeToString gives for DigestPb / DeltaPb (messages.proto:46-74,
// built at state.py:56-58, 74-81, 98-99 and entities.py:62-72, 125-131): fields in field-number
// order, proto3 scalars only when non-zero, NodeDeltaPb.max_version always (it is `optional`).
// String tables (NodeIdPb bytes per node, key names, interned values) are caller-owned device arrays.
struct Wire {
    const uint8_t *nid;
    const uint32_t *nid_off;  // [n_nodes + 1]
    const uint8_t *key;
    const uint32_t *key_off;  // [K + 1]
    const uint8_t *val;
    const uint64_t *val_off;  // [values + 1], indexed by value id
};
__device__ inline uint8_t *put_var(uint8_t *p, uint32_t x) {
    while (x >= 0x80u) { *p++ = (uint8_t)(x | 0x80u); x >>= 7; }
    *p++ = (uint8_t)x;
    return p;
}
__device__ inline uint8_t *put_bytes(uint8_t *p, const uint8_t *src, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) p[i] = src[i];
    return p + n;
}
__device__ inline uint8_t *put_u(uint8_t *p, uint32_t tag, uint32_t x) {
    if (x) { *p++ = (uint8_t)tag; p = put_var(p, x); }
    return p;
}

// Entry q of observer o's digest (compute_digest, state.py:324-331: dict order minus the targets
// scheduled for deletion): the owner's local column, or NONE.
__device__ inline uint32_t digest_owner(const Dev &d, uint32_t o, uint32_t q, uint32_t t, bool sch) {
    const uint32_t j = (d.flags & GS_CANONICAL) ? q : d.ord[(size_t)o * d.NP + q];
    if (j == NONE) return NONE;
    if (sch && is_sched(dead_tod(d, pix(d, o, j)), t, d.sched_delay)) return NONE;
    return j;
}
__device__ inline void view_hgm(const Dev &d, uint32_t o, uint32_t j, uint32_t &H, uint32_t &G, uint32_t &M) {
    const size_t p = pix(d, o, j);
    H = hb_view(d, p, d.self_hb[j]);
    G = (d.flags & GS_TOMBSTONES) ? d.gc[p] : 0u;
    M = mv_word(d, p, j) & MV_MASK;
}
__global__ __launch_bounds__(LB) void k_digest_size(Dev d, Wire w, uint32_t o, uint32_t t, bool sch, uint32_t cnt,
                                                    uint64_t *sz) {
    const uint32_t q = blockIdx.x * LB + threadIdx.x;
    if (q >= cnt) return;
    const uint32_t j = digest_owner(d, o, q, t, sch);
    uint64_t n = 0;
    if (j != NONE) {
        uint32_t H, G, M;
        view_hgm(d, o, j, H, G, M);
        const uint32_t jg = d.col_lo + j, nl = w.nid_off[jg + 1] - w.nid_off[jg];
        n = msgf(msgf(nl) + ufield(H) + ufield(G) + ufield(M));
    }
    sz[q] = n;
}
__global__ __launch_bounds__(LB) void k_digest_write(Dev d, Wire w, uint32_t o, uint32_t t, bool sch, uint32_t cnt,
                                                     const uint64_t *off, uint8_t *out) {
    const uint32_t q = blockIdx.x * LB + threadIdx.x;
    if (q >= cnt) return;
    const uint32_t j = digest_owner(d, o, q, t, sch);
    if (j == NONE) return;
    uint32_t H, G, M;
    view_hgm(d, o, j, H, G, M);
    const uint32_t jg = d.col_lo + j, nl = w.nid_off[jg + 1] - w.nid_off[jg];
    uint8_t *p = out + off[q];
    *p++ = 0x0Au;  // DigestPb.node_digests (1)
    p = put_var(p, msgf(nl) + ufield(H) + ufield(G) + ufield(M));
    *p++ = 0x0Au;  // NodeDigestPb.node_id (1)
    p = put_var(p, nl);
    p = put_bytes(p, w.nid + w.nid_off[jg], nl);
    p = put_u(p, 0x10u, H);  // heartbeat (2)
    p = put_u(p, 0x18u, G);  // last_gc_version (3)
    put_u(p, 0x20u, M);      // max_version (4)
}

// exclusive prefix sum of n u64 sizes into off[0..n] (one workgroup; the emitter's n <= n_cols)
__global__ __launch_bounds__(1024) void k_scan_sizes(const uint64_t *in, uint32_t n, uint64_t *off) {
    __shared__ uint64_t part[1024];
    const uint32_t tid = threadIdx.x, per = (n + 1023u) / 1024u;
    const uint32_t lo = min(n, tid * per), hi = min(n, lo + per);
    uint64_t acc = 0;
    for (uint32_t i = lo; i < hi; i++) acc += in[i];
    part[tid] = acc;
    __syncthreads();
    for (uint32_t k = 1; k < 1024u; k <<= 1) {
        const uint64_t v = tid >= k ? part[tid - k] : 0ull;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint64_t base = tid ? part[tid - 1] : 0ull;
    for (uint32_t i = lo; i < hi; i++) { off[i] = base; base += in[i]; }
    if (tid == 1023u) off[n] = part[1023];
}

// compute_partial_delta_respecting_mtu(r's digest, mtu, s's scheduled_for_deletion) of sender s
// (state.py:340-415), without applying it: one wave builds the stale-owner bitmap of the direction
// s -> r (as pass 1 does) and runs the packer in record mode: rec[] = {owner, vsel} in s's dict order.
template <int KW, bool GENM>
__global__ __launch_bounds__(WAVE) void k_delta_plan(Dev d, uint32_t s, uint32_t r, uint32_t t, uint2 *rec,
                                                     uint32_t *nrec) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint16_t *wbuf = reinterpret_cast<uint16_t *>(lds);
    uint32_t *bits = lds + WIN / 2;
    const int lane = lane_id();
    const bool schS = t >= d.row[s * 4 + 2], schR = t >= d.row[r * 4 + 2];
    const uint32_t cntS = GENM ? d.row[s * 4 + 0] : d.ncol, cntR = GENM ? d.row[r * 4 + 0] : d.ncol;
    for (uint32_t j0 = 0; j0 < d.NP; j0 += WAVE) {
        const uint32_t j = j0 + (uint32_t)lane;
        bool stale = false;
        if (j < d.ncol) {
            const size_t ps = pix(d, s, j), pr = pix(d, r, j);
            const bool has = GENM ? d.pos[ps] != NONE : true;
            if (has && !(schS && is_sched(dead_tod(d, ps), t, d.sched_delay))) {
                bool in_d = GENM ? d.pos[pr] < cntR : true;
                if (in_d && schR && is_sched(dead_tod(d, pr), t, d.sched_delay)) in_d = false;
                const uint32_t dm = in_d ? (mv_word(d, pr, j) & MV_MASK) : 0u;
                stale = (mv_word(d, ps, j) & MV_MASK) > dm;  // state.py:347-357
            }
        }
        const unsigned long long m = __ballot(stale);
        if (lane == 0) { bits[j0 >> 5] = (uint32_t)m; bits[(j0 >> 5) + 1] = (uint32_t)(m >> 32); }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const DigestSide ds{r, cntR, schR};
    WStats st{0, 0, 0, 0, 0};
    bool tomb = false;
    PackState pst{0u, false, false};
    pack_dir<KW, GENM, false, true>(d, s, r, ds, GENM ? d.ord + (size_t)s * d.NP : nullptr, cntS, bits, wbuf, t, st,
                                    tomb, pst, rec, nrec);
}

// one recorded NodeDelta: the sender's candidate (eval_cand) and its NodeDeltaPb body size
template <int KW, bool GENM>
__device__ inline uint32_t nd_eval(const Dev &d, uint32_t s, uint32_t r, uint32_t t, uint2 rc, Cand<KW> &c,
                                   CandKeys<KW> &k) {
    const bool schR = t >= d.row[r * 4 + 2];
    const DigestSide ds{r, GENM ? d.row[r * 4 + 0] : d.ncol, schR};
    uint32_t alg = 0;
    eval_cand<KW, GENM>(d, s, r, ds, rc.x, t, c, k, alg);
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < 4 * KW; q++)
        if (k.ver[q] > c.from && k.ver[q] <= rc.y) sum += k.km[q] & 0xFFFFu;
    return c.base + sum;
}
template <int KW, bool GENM>
__global__ __launch_bounds__(LB) void k_delta_size(Dev d, uint32_t s, uint32_t r, uint32_t t, const uint2 *rec,
                                                   uint32_t n, uint64_t *sz) {
    const uint32_t i = blockIdx.x * LB + threadIdx.x;
    if (i >= n) return;
    Cand<KW> c;
    CandKeys<KW> k;
    sz[i] = msgf(nd_eval<KW, GENM>(d, s, r, t, rec[i], c, k));
}
template <int KW, bool GENM>
__global__ __launch_bounds__(LB) void k_delta_write(Dev d, Wire w, uint32_t s, uint32_t r, uint32_t t,
                                                    const uint2 *rec, uint32_t n, const uint64_t *off, uint8_t *out) {
    const uint32_t i = blockIdx.x * LB + threadIdx.x;
    if (i >= n) return;
    Cand<KW> c;
    CandKeys<KW> k;
    const uint2 rc = rec[i];
    const uint32_t body = nd_eval<KW, GENM>(d, s, r, t, rc, c, k);
    const uint32_t j = rc.x, jg = d.col_lo + j, nl = w.nid_off[jg + 1] - w.nid_off[jg];
    uint8_t *p = out + off[i];
    *p++ = 0x0Au;  // DeltaPb.node_deltas (1)
    p = put_var(p, body);
    *p++ = 0x0Au;  // NodeDeltaPb.node_id (1)
    p = put_var(p, nl);
    p = put_bytes(p, w.nid + w.nid_off[jg], nl);
    p = put_u(p, 0x10u, c.from);  // from_version_excluded (2)
    p = put_u(p, 0x18u, c.gs);    // last_gc_version (3)
    // key_values (4), increasing version (state.py:373-374); versions of one owner are distinct
    uint32_t last = c.from;
    for (;;) {
        int qm = -1;
        uint32_t vm = NONE;
        for (int q = 0; q < 4 * KW; q++)
            if (k.ver[q] > last && k.ver[q] <= rc.y && k.ver[q] < vm) { vm = k.ver[q]; qm = q; }
        if (qm < 0) break;
        last = vm;
        const size_t hx = hix(d, j, byte_of(c.hs, qm), (uint32_t)qm);
        const uint32_t meta = (uint32_t)(d.hist[hx] >> 32), vl = meta_vlen(meta), st = meta_status(meta);
        const uint32_t kl = w.key_off[qm + 1] - w.key_off[qm];
        *p++ = 0x22u;
        p = put_var(p, meta_kvlen(meta));
        if (kl) { *p++ = 0x0Au; p = put_var(p, kl); p = put_bytes(p, w.key + w.key_off[qm], kl); }  // key (1)
        if (vl) {  // value (2)
            *p++ = 0x12u;
            p = put_var(p, vl);
            p = put_bytes(p, w.val + w.val_off[d.hist_vid[hx]], vl);
        }
        p = put_u(p, 0x18u, vm);  // version (3)
        p = put_u(p, 0x20u, st);  // status (4)
    }
    *p++ = 0x28u;  // max_version (5), explicit presence
    put_var(p, c.ms);
}

// ------------------------------------------------------------------ peer selection
// select_nodes_for_gossip (server.py:656-717) for every up node from its failure detector's
// live / dead sets and its known peers, as _gossip_multiple uses them at round start
// (server.py:442-469): F distinct peers sampled uniformly from the live set (from all known
// peers while the live set is empty), one dead node with probability dead / (live + 1), and one
// seed when no selected peer is a seed or live < seeds, with probability seeds / (live + dead)
// (1 if both are empty; always when live = 0).  Random numbers: Philox4x32-10 keyed by the run
// seed, counter (round, node, slot) -- reproducible, where the reference's Random() over set
// iteration order is not.  Slots 0..F-1 feed Floyd's sample, SEL_DEAD and SEL_SEED
// the two probes.  Restated on the CPU by oracle/peer_select.py.
constexpr uint32_t SEL_DEAD = 14, SEL_SEED = 15;

__host__ __device__ inline void philox4x32(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c[0] = hi1 ^ c[1] ^ k0;
        c[1] = lo1;
        c[2] = hi0 ^ c[3] ^ k1;
        c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}
__host__ __device__ inline void sel_rand(uint64_t seed, uint32_t round, uint32_t node, uint32_t slot, uint32_t (&c)[4]) {
    c[0] = round; c[1] = node; c[2] = slot; c[3] = 0u;
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}
__host__ __device__ inline uint32_t below(uint32_t x, uint32_t n) { return (uint32_t)(((uint64_t)x * n) >> 32); }
__host__ __device__ inline double unit53(uint32_t a, uint32_t b) {
    return (double)(((uint64_t)a << 21) ^ (uint64_t)(b >> 11)) * (1.0 / 9007199254740992.0);
}

// per row: live / dead / known-peer counts (observer up); SCNT[o] = {live, dead, peers, 0}
__global__ __launch_bounds__(LB) void k_sel_count(Dev d, const uint8_t *up, uint32_t *scnt) {
    const uint32_t o = blockIdx.x;
    if (!up[o]) return;
    const bool genm = !(d.flags & GS_CANONICAL);
    uint32_t L = 0, D = 0, P = 0;
    for (uint32_t j = threadIdx.x; j < d.ncol; j += LB) {
        const size_t p = pix(d, o, j);
        if (j == o || (genm && d.pos[p] == NONE)) continue;
        const uint32_t st = d.fd_state[p] & FD_MEMB;
        P++;
        L += st == 1u;
        D += st >= 2u;
    }
    __shared__ uint32_t s3[3][LB / WAVE];
    const uint32_t w = threadIdx.x >> 6;
    const unsigned long long l = wave_sum(L), dd = wave_sum(D), pp = wave_sum(P);
    if ((threadIdx.x & 63) == 0) { s3[0][w] = (uint32_t)l; s3[1][w] = (uint32_t)dd; s3[2][w] = (uint32_t)pp; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0, c = 0;
        for (int i = 0; i < LB / WAVE; i++) { a += s3[0][i]; b += s3[1][i]; c += s3[2][i]; }
        scnt[o * 4 + 0] = a; scnt[o * 4 + 1] = b; scnt[o * 4 + 2] = c;
    }
}

// The seed probe (server.py:700-717) of row o and the resolved picks out: thread 0 of the resolve kernels.
__device__ void sel_seed_probe(const Dev &d, uint32_t o, uint32_t L, uint32_t D, uint32_t F, uint64_t seed,
                               uint32_t round, const int32_t *seeds, uint32_t n_seeds, const uint32_t *s_hit,
                               int32_t *oo, const uint32_t *pre = nullptr) {
    bool has_seed = false;
    uint32_t S = 0;
    for (uint32_t q = 0; q < n_seeds; q++) {
        if ((uint32_t)seeds[q] == o) continue;
        S++;
        for (uint32_t i = 0; i < F; i++) has_seed |= s_hit[i] == (uint32_t)seeds[q];
    }
    uint32_t pick = NONE;
    if (S && (!has_seed || L < S)) {
        uint32_t c[4];
        if (pre) {  // (drawn earlier by another lane: the same counter, the same values)
            for (int q = 0; q < 4; q++) c[q] = pre[q];
        } else {
            sel_rand(seed, round, o, SEL_SEED, c);
        }
        const double ps = (L + D) == 0u ? 1.0 : (double)S / (double)(L + D);
        if (L == 0u || unit53(c[0], c[1]) <= ps) {
            uint32_t k = below(c[2], S);
            for (uint32_t q = 0; q < n_seeds; q++) {
                if ((uint32_t)seeds[q] == o) continue;
                if (k-- == 0) { pick = (uint32_t)seeds[q]; break; }
            }
        }
    }
    for (uint32_t i = 0; i < F + 1; i++) oo[i] = s_hit[i] == NONE ? -1 : (int32_t)(d.col_lo + s_hit[i]);
    oo[F + 1] = pick == NONE ? -1 : (int32_t)pick;
}

// Canonical layout (every observer knows every owner, no dict positions): the same counts from 16 state
// bytes per thread and load -- live = membership 1, dead = membership 2 (bit 1), known = every column but
// the observer's own (whose state stays unknown: liveness skips it).
__device__ __forceinline__ uint32_t memb_live4(uint32_t w) {  // bytes whose membership bits are 01
    const uint32_t m = w & 0x03030303u;
    return m & ~(m >> 1) & 0x01010101u;
}
__device__ __forceinline__ uint32_t memb_dead4(uint32_t w) { return (w >> 1) & 0x01010101u; }
__global__ __launch_bounds__(LB) void k_sel_count16(Dev d, const uint8_t *up, uint32_t *scnt) {
    const uint32_t o = blockIdx.x;
    if (!up[o]) return;
    uint32_t L = 0, D = 0;
    const uint8_t *row = d.fd_state + (size_t)o * d.NP;
    for (uint32_t j0 = threadIdx.x * 16u; j0 < d.ncol; j0 += LB * 16u) {
        const uint4 v = *reinterpret_cast<const uint4 *>(row + j0);  // NP is a multiple of 64: in the row
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t jq = j0 + 4u * q;
            uint32_t keep = 0x01010101u;  // columns < ncol (the padding's state bytes are never written: 0)
            if (jq + 4u > d.ncol) keep = jq >= d.ncol ? 0u : (0x01010101u >> (8u * (jq + 4u - d.ncol)));
            const uint32_t js = o - d.col_lo - jq;  // the observer's own column is not a peer
            if (js < 4u) keep &= ~(0x01u << (8u * js));
            L += (uint32_t)__popc(memb_live4(w[q]) & keep);
            D += (uint32_t)__popc(memb_dead4(w[q]) & keep);
        }
    }
    __shared__ uint32_t s2[2][LB / WAVE];
    const uint32_t wv = threadIdx.x >> 6;
    const unsigned long long l = wave_sum(L), dd = wave_sum(D);
    if ((threadIdx.x & 63) == 0) { s2[0][wv] = (uint32_t)l; s2[1][wv] = (uint32_t)dd; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0;
        for (int i = 0; i < LB / WAVE; i++) { a += s2[0][i]; b += s2[1][i]; }
        scnt[o * 4 + 0] = a;
        scnt[o * 4 + 1] = b;
        scnt[o * 4 + 2] = d.ncol - (o - d.col_lo < d.ncol ? 1u : 0u);  // known: every column but o's own
    }
}

// Floyd's sample of k distinct ranks of [0, n) (n = L live, or P known when none is live) and the dead probe,
// by rank, into so[0..F] (NONE where absent: so[] starts all NONE)
// pre (optional): the draws of counters (round, o, slot) already made, pre[4 i + q] for slot i < F, then SEL_DEAD
__device__ inline void sel_ranks(uint32_t o, uint32_t L, uint32_t D, uint32_t P, uint32_t F, uint64_t seed,
                                 uint32_t round, uint32_t *so, const uint32_t *pre = nullptr) {
    const uint32_t n = L ? L : P, k = F < n ? F : n;
    uint32_t c[4];
    for (uint32_t i = 0; i < k; i++) {
        const uint32_t t = n - k + i;
        if (pre) c[0] = pre[4 * i];
        else sel_rand(seed, round, o, i, c);
        uint32_t r = below(c[0], t + 1);
        for (uint32_t q = 0; q < i; q++)
            if (so[q] == r) { r = t; break; }
        so[i] = r;
    }
    if (D) {
        if (pre) {
            for (int q = 0; q < 4; q++) c[q] = pre[4 * F + q];
        } else {
            sel_rand(seed, round, o, SEL_DEAD, c);
        }
        const double pd = (double)D / (double)(L + 1u);
        if (pd > unit53(c[0], c[1])) so[F] = below(c[2], D);
    }
}
// Floyd's sample of k distinct ranks of [0, n) and the dead probe, by rank; targets resolved next.
// sel[o][0..F) = live (or peer) ranks, sel[o][F] = dead rank, NONE where absent.
__global__ __launch_bounds__(LB) void k_sel_pick(Dev d, const uint8_t *up, const uint32_t *scnt, uint32_t F,
                                                 uint64_t seed, uint32_t round, uint32_t *sel) {
    const uint32_t o = blockIdx.x * LB + threadIdx.x;
    if (o >= d.N) return;
    uint32_t *so = sel + (size_t)o * (F + 2);
    for (uint32_t i = 0; i < F + 2; i++) so[i] = NONE;
    if (!up[o]) return;
    sel_ranks(o, scnt[o * 4 + 0], scnt[o * 4 + 1], scnt[o * 4 + 2], F, seed, round, so);
}

// k-th set bit (k < popc(m)) of a 16-bit mask
__device__ __forceinline__ uint32_t nth_bit16(uint32_t m, uint32_t k) {
    for (uint32_t i = 0; i < k; i++) m &= m - 1u;
    return (uint32_t)__builtin_ctz(m);
}
// Canonical layout: k_sel_resolve with 16 columns per thread and step (one 16-byte state load); the pool
// (live, or every known node when none is live) and dead masks are ranked by a block scan of their
// popcounts, so a row takes ncol / 4096 steps instead of ncol / 256.
__global__ __launch_bounds__(LB) void k_sel_resolve16(Dev d, const uint8_t *up, const uint32_t *scnt, uint32_t F,
                                                      uint64_t seed, uint32_t round, const int32_t *seeds,
                                                      uint32_t n_seeds, const uint32_t *sel, int32_t *out) {
    __shared__ uint32_t s_w[LB / WAVE][2];
    __shared__ uint32_t s_rank[10], s_hit[10];
    const uint32_t o = blockIdx.x;
    int32_t *oo = out + (size_t)o * (F + 2);
    if (!up[o]) {
        for (uint32_t i = threadIdx.x; i < F + 2; i += LB) oo[i] = -1;
        return;
    }
    const uint32_t L = scnt[o * 4 + 0];
    const bool from_live = L != 0;
    if (threadIdx.x < F + 1) {
        s_rank[threadIdx.x] = sel[(size_t)o * (F + 2) + threadIdx.x];
        s_hit[threadIdx.x] = NONE;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint8_t *row = d.fd_state + (size_t)o * d.NP;
    uint32_t base_pool = 0, base_dead = 0;
    for (uint32_t b0 = 0; b0 < d.ncol; b0 += LB * 16u) {
        const uint32_t j0 = b0 + threadIdx.x * 16u;
        uint32_t mp = 0, md = 0;  // bit i: column j0 + i is in the pool / dead
        if (j0 < d.ncol) {
            const uint4 v = *reinterpret_cast<const uint4 *>(row + j0);
            const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint32_t j = j0 + 4u * q + b;
                    const uint32_t st = (wd[q] >> (8 * b)) & FD_MEMB;
                    const bool valid = j < d.ncol && d.col_lo + j != o;
                    const bool live = valid && st == 1u, dead = valid && st >= 2u;
                    mp |= (uint32_t)(from_live ? live : valid) << (4 * q + b);
                    md |= (uint32_t)dead << (4 * q + b);
                }
            }
        }
        const uint32_t cp = (uint32_t)__popc(mp), cd = (uint32_t)__popc(md);
        const uint32_t ip = wave_incl_scan(cp), id = wave_incl_scan(cd);
        if (lane == 63) { s_w[w][0] = ip; s_w[w][1] = id; }
        __syncthreads();
        uint32_t op = base_pool + ip - cp, od = base_dead + id - cd, tp = 0, td = 0;
        for (uint32_t i = 0; i < LB / WAVE; i++) {
            if (i < w) { op += s_w[i][0]; od += s_w[i][1]; }
            tp += s_w[i][0];
            td += s_w[i][1];
        }
        for (uint32_t i = 0; i < F; i++) {
            const uint32_t r = s_rank[i];
            if (r != NONE && r >= op && r < op + cp) s_hit[i] = j0 + nth_bit16(mp, r - op);
        }
        {
            const uint32_t r = s_rank[F];
            if (r != NONE && r >= od && r < od + cd) s_hit[F] = j0 + nth_bit16(md, r - od);
        }
        base_pool += tp;
        base_dead += td;
        __syncthreads();
    }
    if (threadIdx.x == 0) sel_seed_probe(d, o, L, scnt[o * 4 + 1], F, seed, round, seeds, n_seeds, s_hit, oo);
}

// Canonical layout, ncol <= SEL_ROW_IT * 4096: k_sel_count16 + k_sel_pick + k_sel_resolve16 in one workgroup per
// row that reads the row's state bytes once -- each thread keeps its 16-column live / dead masks of every
// 4,096-column step in registers: the counts, the ranks (thread 0), then one block scan of all steps at once
// (one barrier instead of two per step)
constexpr uint32_t SEL_ROW_IT = 16;
__global__ __launch_bounds__(LB, 4) void k_sel_row16(Dev d, const uint8_t *up, uint32_t F, uint64_t seed, uint32_t round,
                                                  const int32_t *seeds, uint32_t n_seeds, uint32_t *scnt, int32_t *out) {
    // the live / dead masks of every step in LDS (16 KB: registers would hold the occupancy to 2 waves per SIMD)
    __shared__ uint16_t s_m[SEL_ROW_IT][2][LB];
    __shared__ uint32_t s_w[SEL_ROW_IT][LB / WAVE][2];
    __shared__ uint32_t s_rank[10], s_hit[10], s_cnt[2], s_rnd[10 * 4];
    const uint32_t o = blockIdx.x;
    int32_t *oo = out + (size_t)o * (F + 2);
    if (!up[o]) {
        for (uint32_t i = threadIdx.x; i < F + 2; i += LB) oo[i] = -1;
        return;
    }
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    if (threadIdx.x < F + 2) {  // the row's Philox draws, one lane each (thread 0 only does the arithmetic)
        uint32_t c[4];
        sel_rand(seed, round, o, threadIdx.x < F ? threadIdx.x : threadIdx.x == F ? SEL_DEAD : SEL_SEED, c);
        for (int q = 0; q < 4; q++) s_rnd[4 * threadIdx.x + q] = c[q];
    }
    const uint8_t *row = d.fd_state + (size_t)o * d.NP;
    const uint32_t nit = (d.ncol + LB * 16u - 1u) / (LB * 16u);
    uint32_t L = 0, D = 0;
#pragma unroll
    for (uint32_t h = 0; h < SEL_ROW_IT; h += 8) {  // eight steps' loads in flight at a time
        uint4 v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            // unconditional (a clamped address, masked below): loads under a branch would be waited for one by one
            const uint32_t j0 = (h + u) * LB * 16u + threadIdx.x * 16u;
            v[u] = *reinterpret_cast<const uint4 *>(row + min(j0, d.NP - 16u));
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            const uint32_t it = h + u, j0 = it * LB * 16u + threadIdx.x * 16u;
            const bool inrow = it < nit && j0 < d.ncol;
            const uint32_t wd[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            uint32_t a = 0u, b = 0u;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t jq = j0 + 4u * q;
                uint32_t keep = inrow ? 0x01010101u : 0u;  // (k_sel_count16's column mask: in range, not o's own)
                if (jq + 4u > d.ncol) keep = jq >= d.ncol ? 0u : (keep >> (8u * (jq + 4u - d.ncol)));
                const uint32_t js = o - d.col_lo - jq;
                if (js < 4u) keep &= ~(0x01u << (8u * js));
                // bit 0 of each byte -> 4 adjacent bits: bytes 0..3 times 2^21, 2^14, 2^7, 1 land on bits 21..24
                a |= (((memb_live4(wd[q]) & keep) * 0x204081u) >> 21 & 0xFu) << (4 * q);
                b |= (((memb_dead4(wd[q]) & keep) * 0x204081u) >> 21 & 0xFu) << (4 * q);
            }
            s_m[it][0][threadIdx.x] = (uint16_t)a;
            s_m[it][1][threadIdx.x] = (uint16_t)b;
            L += (uint32_t)__popc(a);
            D += (uint32_t)__popc(b);
        }
    }
    {
        const unsigned long long l = wave_sum(L), dd = wave_sum(D);
        if (lane == 0) { s_w[0][w][0] = (uint32_t)l; s_w[0][w][1] = (uint32_t)dd; }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t a = 0, b = 0;
            for (uint32_t i = 0; i < LB / WAVE; i++) { a += s_w[0][i][0]; b += s_w[0][i][1]; }
            const uint32_t P = d.ncol - (o - d.col_lo < d.ncol ? 1u : 0u);  // known: every column but o's own
            scnt[o * 4 + 0] = a;
            scnt[o * 4 + 1] = b;
            scnt[o * 4 + 2] = P;
            s_cnt[0] = a;
            s_cnt[1] = b;
            uint32_t so[10];
            for (uint32_t i = 0; i < F + 2; i++) so[i] = NONE;
            sel_ranks(o, a, b, P, F, seed, round, so, s_rnd);
            for (uint32_t i = 0; i < F + 1; i++) {
                s_rank[i] = so[i];
                s_hit[i] = NONE;
            }
        }
        __syncthreads();
    }
    L = s_cnt[0];
    const bool from_live = L != 0;
    // the pool (live, or every known column when none is live) and dead ranks of every step, one block scan
    auto pool = [&](uint32_t it) {
        if (from_live) return (uint32_t)s_m[it][0][threadIdx.x];
        const uint32_t j0 = it * LB * 16u + threadIdx.x * 16u;  // every valid column
        uint32_t m = j0 >= d.ncol ? 0u : d.ncol - j0 >= 16u ? 0xFFFFu : (1u << (d.ncol - j0)) - 1u;
        const uint32_t js = o - d.col_lo - j0;
        if (js < 16u) m &= ~(1u << js);
        return m;
    };
    uint32_t ex[SEL_ROW_IT];  // the wave-exclusive scans: pool | dead << 16 (each < 2^10)
#pragma unroll
    for (uint32_t it = 0; it < SEL_ROW_IT; it++) {
        const uint32_t c2 = (uint32_t)__popc(pool(it)) | ((uint32_t)__popc((uint32_t)s_m[it][1][threadIdx.x]) << 16);
        const uint32_t i2 = wave_scan_dpp(c2);  // (both halves at once: no carry out of the low one)
        ex[it] = i2 - c2;
        if (lane == 63) { s_w[it][w][0] = i2 & 0xFFFFu; s_w[it][w][1] = i2 >> 16; }
    }
    __syncthreads();
    uint32_t bp = 0, bd = 0;  // ranks before this step
#pragma unroll
    for (uint32_t it = 0; it < SEL_ROW_IT; it++) {  // (unrolled: ex[] stays in registers)
        uint32_t op = bp + (ex[it] & 0xFFFFu), od = bd + (ex[it] >> 16);
#pragma unroll
        for (uint32_t i = 0; i < LB / WAVE; i++) {
            const uint32_t xp = s_w[it][i][0], xd = s_w[it][i][1];
            if (i < w) { op += xp; od += xd; }
            bp += xp;
            bd += xd;
        }
        const uint32_t j0 = it * LB * 16u + threadIdx.x * 16u;
        const uint32_t mp = pool(it), md = s_m[it][1][threadIdx.x];
        const uint32_t cp = (uint32_t)__popc(mp), cd = (uint32_t)__popc(md);
        if (cp) {
            for (uint32_t i = 0; i < F; i++) {
                const uint32_t r = s_rank[i];
                if (r != NONE && r >= op && r < op + cp) s_hit[i] = j0 + nth_bit16(mp, r - op);
            }
        }
        const uint32_t r = s_rank[F];
        if (cd && r != NONE && r >= od && r < od + cd) s_hit[F] = j0 + nth_bit16(md, r - od);
    }
    __syncthreads();
    if (threadIdx.x == 0) sel_seed_probe(d, o, L, s_cnt[1], F, seed, round, seeds, n_seeds, s_hit, oo, s_rnd + 4 * (F + 1));
}

// Resolve ranks to node ids in column order (one workgroup per row), then the seed probe.
// out[o][0..F) live picks, out[o][F] dead pick, out[o][F+1] seed pick (NONE = none).
__global__ __launch_bounds__(LB) void k_sel_resolve(Dev d, const uint8_t *up, const uint32_t *scnt, uint32_t F,
                                                    uint64_t seed, uint32_t round, const int32_t *seeds,
                                                    uint32_t n_seeds, const uint32_t *sel, int32_t *out) {
    __shared__ uint32_t s_w[LB / WAVE][2];
    __shared__ uint32_t s_rank[10], s_hit[10];
    const uint32_t o = blockIdx.x;
    int32_t *oo = out + (size_t)o * (F + 2);
    if (!up[o]) {
        for (uint32_t i = threadIdx.x; i < F + 2; i += LB) oo[i] = -1;
        return;
    }
    const bool genm = !(d.flags & GS_CANONICAL);
    const uint32_t L = scnt[o * 4 + 0];
    const bool from_live = L != 0;
    if (threadIdx.x < F + 1) {
        s_rank[threadIdx.x] = sel[(size_t)o * (F + 2) + threadIdx.x];
        s_hit[threadIdx.x] = NONE;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t base_pool = 0, base_dead = 0;
    for (uint32_t j0 = 0; j0 < d.ncol; j0 += LB) {
        const uint32_t j = j0 + threadIdx.x;
        bool known = false, live = false, dead = false;
        if (j < d.ncol && j != o) {
            const size_t p = pix(d, o, j);
            known = !genm || d.pos[p] != NONE;
            if (known) {
                const uint32_t st = d.fd_state[p] & FD_MEMB;
                live = st == 1u;
                dead = st >= 2u;
            }
        }
        const bool inpool = from_live ? live : known;
        const unsigned long long mp = __ballot(inpool), md = __ballot(dead);
        if (lane == 0) { s_w[w][0] = (uint32_t)__popcll(mp); s_w[w][1] = (uint32_t)__popcll(md); }
        __syncthreads();
        uint32_t op = base_pool, od = base_dead, tp = 0, td = 0;
        for (uint32_t i = 0; i < LB / WAVE; i++) {
            if (i < w) { op += s_w[i][0]; od += s_w[i][1]; }
            tp += s_w[i][0];
            td += s_w[i][1];
        }
        const uint64_t lm = (1ull << lane) - 1ull;
        const uint32_t rp = op + (uint32_t)__popcll(mp & lm), rd = od + (uint32_t)__popcll(md & lm);
        for (uint32_t i = 0; i < F; i++)
            if (inpool && s_rank[i] == rp) s_hit[i] = j;
        if (dead && s_rank[F] == rd) s_hit[F] = j;
        base_pool += tp;
        base_dead += td;
        __syncthreads();
    }
    if (threadIdx.x == 0) sel_seed_probe(d, o, L, scnt[o * 4 + 1], F, seed, round, seeds, n_seeds, s_hit, oo);
}

// Conflict-free phases for the round's exchanges e = o * (F + 2) + slot (initiator o, responder
// out[e]; exchanges whose responder is down fail before any state change, as a refused
// connection does, and are not scheduled).  Per phase p, IT rounds of a deterministic Luby
// matching: an unscheduled exchange whose two endpoints are free in p takes p if its priority
// key is the smallest at both endpoints.  busy = one bit per phase and node for 64 phases at a time (bit p mod 64;
// the host clears it every 64 phases: a phase's bits are read only while it is being filled).  Up to
// GS_MAX_SCHED_PHASES phases (round 6: the hubs of the reference's selection -- every node picks a seed while its
// live set is empty -- need as many phases as their degree); exchanges left after the last are counted, not run.
__device__ inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
__device__ inline bool luby_valid(const int32_t *out, const uint8_t *up, uint32_t e, uint32_t F, uint32_t &a,
                                  uint32_t &b) {
    const int32_t t = out[e];
    if (t < 0 || !up[t]) return false;
    a = e / (F + 2);
    b = (uint32_t)t;
    return true;
}
__device__ inline bool luby_active(const int32_t *out, const uint8_t *up, const uint32_t *eph,
                                   const unsigned long long *busy, uint32_t e, uint32_t F, uint32_t p, uint32_t &a,
                                   uint32_t &b) {
    if (eph[e] != NONE) return false;
    if (!luby_valid(out, up, e, F, a, b)) return false;
    return !((busy[a] >> (p & 63u)) & 1ull) && !((busy[b] >> (p & 63u)) & 1ull);
}
__device__ inline unsigned long long luby_key(uint64_t seed, uint32_t round, uint32_t e, uint32_t p, uint32_t it) {
    const uint32_t h = fmix32(e ^ fmix32((uint32_t)seed ^ fmix32(round * 0x9E3779B9u + p * 0x632BE5ABu + it)));
    return ((unsigned long long)h << 32) | e;
}
__global__ __launch_bounds__(LB) void k_luby_min(const int32_t *out, const uint8_t *up, const uint32_t *eph,
                                                 const unsigned long long *busy, unsigned long long *best, uint32_t E,
                                                 uint32_t F, uint64_t seed, uint32_t round, uint32_t p, uint32_t it) {
    const uint32_t e = blockIdx.x * LB + threadIdx.x;
    uint32_t a, b;
    if (e >= E || !luby_active(out, up, eph, busy, e, F, p, a, b)) return;
    const unsigned long long k = luby_key(seed, round, e, p, it);
    atomicMin(&best[a], k);
    atomicMin(&best[b], k);
}
__global__ __launch_bounds__(LB) void k_luby_pick(const int32_t *out, const uint8_t *up, uint32_t *eph,
                                                  unsigned long long *busy, const unsigned long long *best,
                                                  unsigned long long *best_next, uint32_t E, uint32_t N, uint32_t F,
                                                  uint64_t seed, uint32_t round, uint32_t p, uint32_t it,
                                                  uint32_t *pcount) {
    const uint32_t x = blockIdx.x * LB + threadIdx.x;
    if (x < N) best_next[x] = ~0ull;
    uint32_t a, b;
    if (x >= E || !luby_active(out, up, eph, busy, x, F, p, a, b)) return;
    const unsigned long long k = luby_key(seed, round, x, p, it);
    if (best[a] == k && best[b] == k) {
        eph[x] = p;
        atomicOr(&busy[a], 1ull << (p & 63u));
        atomicOr(&busy[b], 1ull << (p & 63u));
        atomicAdd(&pcount[p], 1u);
    }
}
// valid exchanges not scheduled yet
__global__ __launch_bounds__(LB) void k_luby_left(const int32_t *out, const uint8_t *up, const uint32_t *eph,
                                                  uint32_t E, uint32_t F, uint32_t *left) {
    const uint32_t e = blockIdx.x * LB + threadIdx.x;
    uint32_t a, b;
    const bool l = e < E && eph[e] == NONE && luby_valid(out, up, e, F, a, b);
    const unsigned long long m = __ballot(l);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(left, (uint32_t)__popcll(m));
}
// scatter the scheduled exchanges into per-phase (initiator, responder) arrays: each workgroup ranks its
// SCAT_PER x LB exchanges per phase in LDS and takes one range per phase with a single global atomic (a
// returning atomic per exchange, or per wave and phase, serialises on the 16 or so phase counters: 0.59 ms).
// Phases past the first 64 (hub exchanges only, a few per phase) take a global atomic each.
constexpr uint32_t SCAT_PER = 4;
__global__ __launch_bounds__(LB) void k_luby_scatter(const int32_t *out, const uint32_t *eph, uint32_t E, uint32_t F,
                                                     const uint32_t *poff, uint32_t *pfill, int32_t *ini,
                                                     int32_t *res) {
    __shared__ uint32_t s_cnt[GS_MAX_PHASES], s_base[GS_MAX_PHASES];
    if (threadIdx.x < GS_MAX_PHASES) s_cnt[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t p[SCAT_PER], loc[SCAT_PER];
#pragma unroll
    for (uint32_t k = 0; k < SCAT_PER; k++) {
        const uint32_t e = (blockIdx.x * SCAT_PER + k) * LB + threadIdx.x;
        p[k] = e < E ? eph[e] : NONE;
        loc[k] = p[k] < GS_MAX_PHASES ? atomicAdd(&s_cnt[p[k]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < GS_MAX_PHASES && s_cnt[threadIdx.x])
        s_base[threadIdx.x] = atomicAdd(&pfill[threadIdx.x], s_cnt[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < SCAT_PER; k++) {
        if (p[k] == NONE) continue;
        const uint32_t e = (blockIdx.x * SCAT_PER + k) * LB + threadIdx.x;
        const uint32_t slot = poff[p[k]] + (p[k] < GS_MAX_PHASES ? s_base[p[k]] + loc[k] : atomicAdd(&pfill[p[k]], 1u));
        ini[slot] = (int32_t)(e / (F + 2));
        res[slot] = out[e];
    }
}

// ------------------------------------------------------------------ measurement kernels
// Streaming copy: the measured HBM ceiling bench.py reports beside the 8 TB/s peak.  And read-only / write-only
// streams at 4, 8 or 16 B per lane whose known byte counts calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE.
// measurement kernels (gs_stream_copy / _read / _write).  The copy: each wave moves contiguous 16 KiB chunks
// (64 lanes x 16 B x 16 loads in flight per lane, non-temporal loads and stores), chunks dealt grid-stride
// over 65,536 workgroups -- the fastest copy shape of tools/membench8.hip on the box (5.99 TB/s vs 5.30 for
// round 3's grid-stride 8-deep copy, r4b)
__global__ __launch_bounds__(256) void k_copy16(v4u_t *__restrict__ dst, const v4u_t *__restrict__ src, uint64_t n16) {
    const uint64_t waves = (uint64_t)gridDim.x * 4u, wid = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t chunks = n16 / 1024u;
    for (uint64_t c = wid; c < chunks; c += waves) {
        const uint64_t b = c * 1024u + lane;
        v4u_t v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = __builtin_nontemporal_load(src + b + u * 64);
#pragma unroll
        for (int u = 0; u < 16; u++) __builtin_nontemporal_store(v[u], dst + b + u * 64);
    }
    // the tail (< 16 KiB): grid-stride
    for (uint64_t i = chunks * 1024u + (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n16; i += waves * 64u) dst[i] = src[i];
}
template <typename V>
__global__ __launch_bounds__(256) void k_write(V *__restrict__ dst, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    V v;
    memset(&v, 0x5A, sizeof v);
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += stride) dst[i] = v;
}
__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y; }
template <typename V>
__global__ __launch_bounds__(256) void k_read(const V *__restrict__ src, uint64_t n, unsigned long long *sink) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint32_t acc = 0;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const V a = src[i], b = src[i + stride], c = src[i + 2 * stride], e = src[i + 3 * stride];
        acc ^= fold(a) ^ fold(b) ^ fold(c) ^ fold(e);
    }
    for (; i < n; i += stride) acc ^= fold(src[i]);
    if (acc == 0x9E3779B9u) atomicAdd(sink, 1ull);  // keeps the loads; practically never taken
}

// gs_mark: empty one-wave dispatches whose names bracket a region of a kernel trace (bench.py's timed rounds), so
// tools/pmc_summary.py averages exactly the dispatches between them
__global__ __launch_bounds__(WAVE) void k_mark_begin() {}
__global__ __launch_bounds__(WAVE) void k_mark_end() {}

}  // namespace

// ====================================================================== C ABI
struct gs_handle {
    gs_config cfg;
    Dev d;
    uint32_t N, NP, K, KP, C, W;
    uint32_t G, shard, col_lo, ncol;  // owner-column slice
    bool sliced;                      // phases take the sliced path (G > 1, or GS_SLICED with one slice)
    bool reports_pending;             // phases ran since the last gs_liveness
    bool round_open;                  // gs_begin_round ran and gs_liveness has not closed the round yet
    uint32_t last_phase_tick;
    // sub-phases (Dev::v_round): the last phase's virtual tick (monotonic over the handle's life); a phase has run
    // at last_phase_tick since the last round start / flush (a further phase at that tick is then a sub-phase);
    // the plane base still needs its virtual base (set by the base's first phase)
    uint32_t last_vt = 0;
    bool sub_ok = false;
    bool base_fresh = true;
    uint64_t plane_flushes;           // mid-round report replays (rounds with phases > 16 ticks after the base)
    uint64_t lag_sweeps = 0;          // k_hb_lag sweeps run (gs_counters.lag_sweeps)
    uint32_t hb_incs;                 // rounds + phases since the last heartbeat-lag check (gs_check_heartbeat_lag)
    uint32_t mv_incs = 0;             // GS_MV8: gs_owner_writes calls since the last lag check
    uint32_t age_tick = 0;            // tick of the last window-age sweep (k_fd_age)
    uint32_t max_tick = 0;            // latest tick of any operation (gs_latest_tick: decodes GS_R_FD_LAST)
    void *reg[GS_NUM_REGIONS];
    uint64_t bytes[GS_NUM_REGIONS];
    hipStream_t stream;
    uint32_t seq;
    bool booted;
    bool started = false;             // a round has begun (gs_set_ring_rows refuses from then on)
    // canonical unsliced handles run a phase on candidate records (k_pass1 + k_settle); env GS_FUSED=1
    // selects the single fused k_exchange (and, on sliced handles, the fused count pass) for A/B runs
    bool split;
    // record phases (env GS_PACK, A/B runs): 0 = k_pass1 with the speculative merge + k_settle (default),
    // 1 = "fused": k_pass1 packing in the same workgroup, 2 = "split": k_pass1 + k_pack_slice
    int pack_mode = 2;
    bool age_init = false;            // age_tick holds the first operation's tick (fd_age)
    // gs_set_timing: HIP events around each kernel launch of a kind (gs_ktimes), on the library's stream
    bool timing;
    uint32_t *heavy_buf = nullptr;  // k_pack_heavy's slot list (Dev::heavy): [0] = count, then up to N slot ids
    uint16_t *sm_buf = nullptr;     // Dev::sm (one-slice prefix-view handles)
    hipStream_t hside = nullptr;    // k_pack_heavy's stream (forked after the lite slot work, joined after the packer)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> tev[GS_KT_KINDS];
    std::vector<hipEvent_t> evpool;
    std::string err;
    // sliced phases driven by the library (gs_comm_init: RCCL across processes; gs_run_phase_group:
    // the slices of one process): device scratch for the gathered totals and chain states
    ncclComm_t comm = nullptr;
    struct {
        uint64_t *tot = nullptr, *tot_all = nullptr, *chain = nullptr, *chainc = nullptr, *chain_all = nullptr;
        uint64_t *pend = nullptr;  // device: the pending slots summed over the slices (sliced_phase's one read per step)
        uint64_t *pin = nullptr, *pin_dev = nullptr;  // pinned host pair {pending, count} the kernel writes directly
        uint32_t *list = nullptr;
        uint32_t cap = 0;  // exchanges the buffers hold
    } sc;
    // gs_run_phase_group: each slice's kernels of a step run on a stream of its own (forked from and joined
    // back into the group's stream around the step), so the slices' short launches overlap on the GPU
    hipStream_t side = nullptr, home = nullptr;
    hipEvent_t fj_fork = nullptr, fj_join = nullptr;
    // gs_run_phase_group's batched launches: the group's GroupArgs in device memory and its host image as last
    // uploaded (held by the group's first handle)
    GroupArgs *grp = nullptr;
    std::vector<uint8_t> grp_img;
};

namespace {

int fail(gs_handle *h, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf;
    return code;
}

#define HIPCHK(h, x)                                                                         \
    do {                                                                                     \
        hipError_t _e = (x);                                                                 \
        if (_e != hipSuccess) return fail((h), GS_E_HIP, "%s: %s", #x, hipGetErrorString(_e)); \
    } while (0)

uint32_t round_up(uint32_t x, uint32_t m) { return (x + m - 1) / m * m; }

// gs_set_timing: an event pair around each timed launch, recorded on the library's stream
int time_begin(gs_handle *h, hipEvent_t &e0) {
    if (!h->timing) return GS_OK;
    if (h->evpool.empty()) {
        HIPCHK(h, hipEventCreate(&e0));
    } else {
        e0 = h->evpool.back();
        h->evpool.pop_back();
    }
    HIPCHK(h, hipEventRecord(e0, h->stream));
    return GS_OK;
}
int time_end(gs_handle *h, int kind, hipEvent_t e0) {
    if (!h->timing) return GS_OK;
    hipEvent_t e1;
    int rc = time_begin(h, e1);
    if (rc) return rc;
    h->tev[kind].push_back({e0, e1});
    return GS_OK;
}

// k_fd_age at least every 2^14 ticks of the operations that decode 16-bit report ticks (phases: the
// mid-round replay; liveness; phi), so every unmarked window is < 2^15 + 2^14 ticks old when decoded
int fd_age(gs_handle *h, uint32_t tick);

int check_bound(gs_handle *h) {
    for (int r = 0; r < GS_NUM_REGIONS; r++)
        if (h->bytes[r] && !h->reg[r]) return fail(h, GS_E_UNBOUND, "region %d not bound", r);
    Dev &d = h->d;
    d.hb = (uint16_t *)h->reg[GS_R_HB];
    d.self_hb = (uint32_t *)h->reg[GS_R_SELF_HB];
    d.mv = (uint16_t *)h->reg[GS_R_MV];
    d.gc = (uint32_t *)h->reg[GS_R_GC];
    d.held = (uint8_t *)h->reg[GS_R_HELD];
    d.fd = (uint32_t *)h->reg[GS_R_FD];
    d.fd_last = (uint16_t *)h->reg[GS_R_FD_LAST];
    d.fd_state = (uint8_t *)h->reg[GS_R_FD_STATE];
    d.tod = (uint32_t *)h->reg[GS_R_FD_TOD];
    d.ts = (uint32_t *)h->reg[GS_R_TS];
    d.ring = (uint16_t *)h->reg[GS_R_RING];
    d.pos = (uint32_t *)h->reg[GS_R_POS];
    d.ord = (uint32_t *)h->reg[GS_R_ORD];
    d.row = (uint32_t *)h->reg[GS_R_ROW];
    d.last_w = (uint8_t *)h->reg[GS_R_LAST_W];
    d.hist = (uint64_t *)h->reg[GS_R_HIST];
    d.lat = (uint32_t *)h->reg[GS_R_LATEST];
    d.hist_vid = (uint32_t *)h->reg[GS_R_HIST_VID];
    d.nid_size = (uint16_t *)h->reg[GS_R_NID_SIZE];
    d.key_len = (uint8_t *)h->reg[GS_R_KEY_LEN];
    d.stamp = (uint32_t *)h->reg[GS_R_STAMP];
    d.ctr = (unsigned long long *)h->reg[GS_R_COUNTERS];
    d.sbits = (uint32_t *)h->reg[GS_R_SLICE_BITS];
    d.cand = (uint2 *)h->reg[GS_R_CAND];
    d.cand_n = (uint32_t *)h->reg[GS_R_CAND_N];
    d.pend = (uint64_t *)h->reg[GS_R_PEND];
    d.pstamp = (uint32_t *)h->reg[GS_R_PEND_STAMP];
    d.slot_stat = (uint4 *)h->reg[GS_R_SLOT_STAT];
    d.ring_slot = (uint32_t *)h->reg[GS_R_RING_SLOT];
    d.vlog = (uint32_t *)h->reg[GS_R_VLOG];
    d.self_mv = (uint32_t *)h->reg[GS_R_SELF_MV];
    d.self_pk = (uint32_t *)h->reg[GS_R_SELF_PK];
    d.p1flags = (uint32_t *)h->reg[GS_R_P1FLAGS];
    d.esc16 = (uint16_t *)h->reg[GS_R_ESC16];
    d.esc_slot = (uint32_t *)h->reg[GS_R_ESC_SLOT];
    d.esc_owner = (uint32_t *)h->reg[GS_R_ESC_OWNER];
    d.esc_req = (uint32_t *)h->reg[GS_R_ESC_REQ];
    return GS_OK;
}

// A record phase may merge its prefix candidates speculatively in pass 1 (Dev::spec): canonical prefix
// views (no tombstones), records on, no hook events (they need the per-key applies), packing not ablated.
bool spec_ok(const gs_handle *h) {
    return h->pack_mode == 0 && (h->cfg.flags & GS_CANONICAL) && !(h->cfg.flags & GS_TOMBSTONES) && h->d.cand &&
           !h->d.ev && !(h->d.ablate & 1u);
}

// k_lite before the exact packer (Dev::lite): canonical prefix views (no tombstones) with records and the
// version log, no hook events, the default packing mode, packing not ablated.
bool lite_ok(const gs_handle *h) {
    return h->pack_mode == 2 && (h->cfg.flags & GS_CANONICAL) && !(h->cfg.flags & GS_TOMBSTONES) && h->d.cand &&
           h->d.vlog && h->d.slot_stat && !h->d.ev && !(h->d.ablate & 1u);
}
// The same speculative merge in k_pass1v (GS_MV8 record phases, before k_lite): k_lite then only sizes the
// deltas, and the exact packer restores what it does not send (a slot a chain step finds stopped restores
// every record: pack_list).  With whole-line row stores (P1V_LINE) the merge costs k_pass1v 0.27 ms and saves
// k_lite 0.42 (r4m: 36.8 vs 38.0 ms per round); per-lane 16-byte stores made it cost as much as it saved (r4i).
// In sliced phases it halves the step-0 kernel (r4i: 0.23 vs 0.43 ms at 2 slices).  Env GS_P1SPEC=0: off (A/B).
bool spec_v_ok(const gs_handle *h) {
    static const bool on = [] {
        const char *e = getenv("GS_P1SPEC");
        return !(e && e[0] == '0');
    }();
    return on && h->d.pl16 && lite_ok(h);
}
template <int MODE>
int launch_lite(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick, const SliceIO &io) {
    hipEvent_t e0 = nullptr;
    int rc = time_begin(h, e0);
    if (rc) return rc;
    k_lite<MODE><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io);
    HIPCHK(h, hipGetLastError());
    return time_end(h, GS_KT_LITE, e0);
}

template <int KW, bool GENM, int MODE>
int launch_exchange(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick, size_t lds,
                    const SliceIO &io) {
    auto *k = k_exchange<KW, GENM, MODE>;
    if (lds > 64 * 1024)
        HIPCHK(h, hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    k<<<n, XB, lds, h->stream>>>(h->d, ini, res, n, tick, h->seq, io);
    HIPCHK(h, hipGetLastError());
    return GS_OK;
}

// LDS of k_exchange: two packer windows, then the stale-owner (+ insertion) bitmaps of this slice
size_t exchange_lds(const gs_handle *h) {
    const bool genm = !(h->cfg.flags & GS_CANONICAL);
    return WIN * 2 * 2 + (size_t)(h->NP / 32) * (genm ? 4 : 2) * 4;
}

int launch_liveness(gs_handle *h, const uint8_t *up, uint32_t tick, bool replay, bool decide) {
    const uint32_t chunks = (h->ncol + 4 * LB - 1) / (4 * LB);
    static const uint32_t live_per = [] {  // env GS_LIVE_PER: chunks per workgroup (tuning sweeps)
        const char *e = getenv("GS_LIVE_PER");
        const int v = e ? atoi(e) : 0;
        return v >= 1 && v <= 64 ? (uint32_t)v : (uint32_t)LIVE_PER;
    }();
    const uint32_t per = live_per, groups = (chunks + per - 1) / per;
    hipEvent_t e0 = nullptr;
    int rc = time_begin(h, e0);
    if (rc) return rc;
    if (h->cfg.flags & GS_FD_RING)
        k_liveness<1><<<groups * h->N, LB, 0, h->stream>>>(h->d, up, tick, chunks, per, replay, decide);
    else if (h->d.ring_slot)
        k_liveness<2><<<groups * h->N, LB, 0, h->stream>>>(h->d, up, tick, chunks, per, replay, decide);
    else
        k_liveness<0><<<groups * h->N, LB, 0, h->stream>>>(h->d, up, tick, chunks, per, replay, decide);
    HIPCHK(h, hipGetLastError());
    return time_end(h, GS_KT_LIVENESS, e0);
}

// The report plane of a new phase at `tick` (sets Dev::vt).  A phase at a later tick takes plane tick - t_round - 1
// of the base, as before; a sub-phase (a further phase at the previous phase's tick) takes the next plane, at the
// same real tick (Dev::t_cap).  A phase past the base's NPL planes -- or at a later tick after sub-phases, whose
// planes clamp to t_cap -- first replays the pending report planes into the sampling windows (nothing reads a
// window before the round's liveness sweep, and the replay applies the same reports in the same tick order), then
// starts a new plane base just before this phase.
uint32_t plane_tick_host(const Dev &d, uint32_t p) { return std::min(d.t_round + 1u + p, d.t_cap); }
int plane_slot(gs_handle *h, uint32_t tick, bool sub) {
    Dev &d = h->d;
    if (h->base_fresh) {  // the base's first phase: every plane's virtual tick is above every earlier phase's
        d.v_round = std::max(d.t_round, h->last_vt);
        d.t_cap = NONE;
        h->base_fresh = false;
    }
    uint32_t vt = sub ? h->last_vt + 1u : tick + (d.v_round - d.t_round);
    const bool full = vt - d.v_round > NPL || (!sub && d.t_cap != NONE && tick > d.t_cap);
    if (full) {
        if (h->reports_pending) {
            int rc = launch_liveness(h, nullptr, tick, true, false);
            if (rc) return rc;
            h->plane_flushes++;
        }
        d.t_round = tick - 1u;
        vt = std::max(tick, h->last_vt + 1u);
        d.v_round = vt - 1u;
        d.t_cap = NONE;
    }
    if (sub) d.t_cap = tick;  // this plane and every later one of the base: the shared tick
    if (vt - d.v_round - 1u >= NPL || plane_tick_host(d, vt - d.v_round - 1u) != tick)
        return fail(h, GS_E_INVALID, "plane_slot: tick %u (virtual %u) does not map to a plane of the base (%u, %u, %u)",
                    tick, vt, d.t_round, d.v_round, d.t_cap);
    d.vt = vt;
    h->last_vt = vt;
    return GS_OK;
}

// pack = true: gs_phase_pack, which completes the phase gs_phase_count started at the same tick
int check_phase(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick, bool pack = false) {
    if (!h || !h->booted) return GS_E_INVALID;
    if (!h->round_open)
        return fail(h, GS_E_INVALID, "phases run between gs_begin_round and gs_liveness (the round is closed)");
    // a phase runs after the round start (or flush) at a tick >= the previous phase's: an equal tick is a sub-phase
    if (pack ? tick != h->last_phase_tick : (tick < h->last_phase_tick || (tick == h->last_phase_tick && !h->sub_ok)))
        return fail(h, GS_E_INVALID, "phase tick %u %s (tick %u)", tick,
                    pack ? "is not the tick of the last gs_phase_count" : "not after the round start / previous phase",
                    h->last_phase_tick);
    if (n && (!ini || !res)) return GS_E_INVALID;
    if (n > h->N / 2) return fail(h, GS_E_INVALID, "a phase has at most n_nodes/2 exchanges (got %u)", n);
    if (exchange_lds(h) > 160 * 1024)
        return fail(h, GS_E_UNSUPPORTED, "slice too wide for the LDS bitmaps (%zu B)", exchange_lds(h));
    // 8-bit heartbeat views: the lag sweep also runs mid-round, so however many phases a round has, no two
    // sweeps are more than HB8_LAG_CHECK_EVERY owner increments apart (the sweep only reads: safe between
    // phases, and gs_phase_pack continues the phase its gs_phase_count started)
    if (!pack && h->d.hb8 && h->hb_incs >= HB8_LAG_CHECK_EVERY) return gs_check_heartbeat_lag(h);
    return GS_OK;
}

// k_lite's slot work at the end of k_pass1v (a record phase with Dev::lite on the byte-parallel pass 1); env
// GS_P1LITE=0: k_lite (or k_settle<1, LITE>) as a launch of its own (A/B)
// mode 0 (one slice): on by default (r5e: 2.27 ms per phase vs 2.10 + 0.235 in two launches); mode 1 (a sliced
// count pass): off by default -- a slice's stream is short, and k_settle<1, LITE> at 8 waves per SIMD did the slot
// work sooner (r5e, 8 slices: 0.304 + 0.061 vs 0.348 + 0.030 ms per phase); GS_P1LITE=0 / 1 / 2: off / mode 0 /
// both (A/B)
bool p1lite(const gs_handle *h, int mode = 0) {
    static const int lvl = [] {
        const char *e = getenv("GS_P1LITE");
        return e ? atoi(e) : 1;
    }();
    return lvl > mode && h->d.pl16 && h->d.lite;
}

// pass 1 of a record phase (k_pass1 without packing), speculative per Dev::spec; lm >= 0 (k_pass1v only): the
// slot work of k_lite<lm> in the same launch (io: the sliced count's totals)
// a launch for every slice of an in-process group at once (grid.y = slices; gs_run_phase_group), or none
struct GroupCtx {
    const GroupArgs *ga = nullptr;
    uint32_t nh = 1;
    DevDyn dyn{};
};
int launch_pass1(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick, int lm = -1,
                 const SliceIO &io = SliceIO{}, bool defer_fix = false, const GroupCtx &gx = GroupCtx{}) {
    hipEvent_t e0 = nullptr;
    int rc = time_begin(h, e0);
    if (rc) return rc;
    if (h->d.pl16) {  // GS_MV8 record phases: the byte-parallel pass 1
        const dim3 grid(n, gx.nh);
        if (gx.ga && lm == 1) k_pass1v<P1V_AHEAD, 1, true><<<grid, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, io, gx.ga, gx.dyn);
        else if (gx.ga) k_pass1v<P1V_AHEAD, -1, true><<<grid, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, io, gx.ga, gx.dyn);
        else if (lm == 0) k_pass1v<P1V_AHEAD, 0><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, io, nullptr, DevDyn{});
        else if (lm == 1) k_pass1v<P1V_AHEAD, 1><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, io, nullptr, DevDyn{});
        else k_pass1v<P1V_AHEAD, -1><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, io, nullptr, DevDyn{});
        HIPCHK(h, hipGetLastError());
        rc = time_end(h, GS_KT_PASS1, e0);
        if (rc) return rc;
        if (defer_fix) return GS_OK;  // the caller's next launch does it (Dev::p1fix)
        k_p1v_fix<<<(n + LB - 1) / LB, LB, 0, h->stream>>>(h->d, res, n);
        HIPCHK(h, hipGetLastError());
        return GS_OK;
    }
    if (h->d.mv8) {  // GS_MV8 implies GS_HB8
        if (h->d.spec) k_pass1<4, false, true, true, true><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
        else k_pass1<4, false, false, true, true><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
    } else if (h->d.hb8) {
        if (h->d.spec) k_pass1<4, false, true, true><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
        else k_pass1<4, false, false, true><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
    } else {
        if (h->d.spec) k_pass1<4, false, true><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
        else k_pass1<4, false, false><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
    }
    HIPCHK(h, hipGetLastError());
    return time_end(h, GS_KT_PASS1, e0);
}
template <int MODE, bool LITE = false>
int launch_settle(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick, const SliceIO &io,
                  int kind, const GroupCtx &gx = GroupCtx{}) {
    hipEvent_t e0 = nullptr;
    int rc = time_begin(h, e0);
    if (rc) return rc;
    const dim3 grid(n, gx.nh);
    if (gx.ga) k_settle<4, MODE, LITE, true><<<grid, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io, gx.ga, gx.dyn);
    else if (h->KP <= 16) k_settle<4, MODE, LITE><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io, nullptr, DevDyn{});
    else k_settle<KWB, MODE, LITE><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io, nullptr, DevDyn{});
    HIPCHK(h, hipGetLastError());
    return time_end(h, kind, e0);
}
// the sliced steps' lite + settle as one kernel (k_settle<LITE>); env GS_LITE_FUSE=0: two launches (A/B)
bool lite_fuse() {
    static const bool on = [] {
        const char *e = getenv("GS_LITE_FUSE");
        return !(e && e[0] == '0');
    }();
    return on;
}

// k_pack_heavy (round 6): on unless env GS_HEAVY=0 (A/B); a slot goes there past GS_HEAVY_T stale owners (default
// HEAVY_T); a grid of at most HEAVY_GRID workgroups loops over the listed slots
#ifndef HEAVY_T
#define HEAVY_T 2048u
#endif
constexpr uint32_t HEAVY_GRID = 4096u;
bool sm_on() {
    static const bool on = [] {
        const char *e = getenv("GS_SM");
        return !(e && e[0] == '0');
    }();
    return on;
}
bool heavy_on() {
    static const bool on = [] {
        const char *e = getenv("GS_HEAVY");
        return !(e && e[0] == '0');
    }();
    return on;
}
uint32_t heavy_t() {
    static const uint32_t v = [] {
        const char *e = getenv("GS_HEAVY_T");
        const long x = e ? atol(e) : 0;
        return x > 0 ? (uint32_t)x : (uint32_t)HEAVY_T;
    }();
    return v;
}

// One canonical one-slice phase on the caller's stream (GS_PACK, A/B runs): default k_pass1 with the
// speculative merge, then k_settle; "fused": k_pass1<FUSE = true> (pass 1, then packing and apply in the
// same workgroup); "split": k_pass1, then k_pack_slice.
int run_split_phase(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick) {
    hipEvent_t e0 = nullptr;
    int rc;
    h->d.spec = spec_ok(h) || spec_v_ok(h) ? 1u : 0u;
    h->d.lite = lite_ok(h) ? 1u : 0u;
    if (h->pack_mode == 1) {
        if ((rc = time_begin(h, e0))) return rc;
        if (h->KP <= 16) k_pass1<4, true><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
        else k_pass1<KWB, true><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, h->seq, 0u);
        HIPCHK(h, hipGetLastError());
        return time_end(h, GS_KT_PASS1, e0);
    }
    const bool fl = p1lite(h), defer = fl && !(h->d.ablate & 1u);  // defer: the packer sets the small bits
    const SliceIO io{};
    // slots with more than heavy_t stale owners: the lite slot work (in pass 1's epilogue or k_lite) lists them
    // and k_pack_heavy packs them on a side stream while k_pack_slice packs the others (K <= 16, prefix views)
    const bool hv = heavy_on() && h->pack_mode == 2 && h->KP <= 16 && h->d.lite && h->d.vlog && !h->d.ev && h->d.cand;
    if (hv) {
        if (!h->heavy_buf) HIPCHK(h, hipMalloc(&h->heavy_buf, ((size_t)h->N + 4) * 4));
        if (!h->hside) {
            HIPCHK(h, hipStreamCreateWithFlags(&h->hside, hipStreamNonBlocking));
            HIPCHK(h, hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
            HIPCHK(h, hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
        }
        HIPCHK(h, hipMemsetAsync(h->heavy_buf, 0, 4, h->stream));
        h->d.heavy = h->heavy_buf;
        h->d.heavy_t = heavy_t();
    }
    if ((rc = launch_pass1(h, ini, res, n, tick, fl ? 0 : -1, io, defer))) return rc;
    if (h->d.ablate & 1u) { h->d.heavy = nullptr; return GS_OK; }  // profiling only: no packing (results invalid)
    if (h->pack_mode == 0) return launch_settle<0>(h, ini, res, n, tick, io, GS_KT_PACK);
    if (h->d.lite && !fl && (rc = launch_lite<0>(h, ini, res, n, tick, io))) return rc;
    if (hv) {  // fork: the heavy slots on the side stream
        HIPCHK(h, hipEventRecord(h->ev_fork, h->stream));
        HIPCHK(h, hipStreamWaitEvent(h->hside, h->ev_fork, 0));
        k_pack_heavy<4><<<std::min(2u * n, HEAVY_GRID), HT, 0, h->hside>>>(h->d, ini, res, tick, h->heavy_buf);
        HIPCHK(h, hipGetLastError());
    }
    if ((rc = time_begin(h, e0))) return rc;
    h->d.p1fix = defer ? 1u : 0u;
    if (h->KP <= 16) k_pack_slice<4><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io, 0u);
    else k_pack_slice<KWB><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io, 0u);
    h->d.p1fix = 0u;
    h->d.heavy = nullptr;
    HIPCHK(h, hipGetLastError());
    if (hv) {  // k_pack_heavy ran on the side stream meanwhile (forked after the lite slot work): join
        HIPCHK(h, hipEventRecord(h->ev_join, h->hside));
        HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_join, 0));
    }
    return time_end(h, GS_KT_PACK, e0);
}

}  // namespace

extern "C" {

int gs_api_version(void) { return GS_API_VERSION; }

const char *gs_last_error(const gs_handle *h) { return h ? h->err.c_str() : "null handle"; }

int gs_create(const gs_config *cfg, gs_handle **out) {
    if (!cfg || !out) return GS_E_INVALID;
    *out = nullptr;
    const gs_config &c = *cfg;
    if (c.n_nodes < 2 || c.n_nodes > (1u << 20)) return GS_E_INVALID;
    // owner-column slices: blocks of round_up(ceil(N / G), 64) columns, none empty, canonical only
    const uint32_t G = c.n_shards ? c.n_shards : 1u;
    if (G > 64 || c.shard >= G) return GS_E_INVALID;
    const uint32_t blk = round_up((c.n_nodes + G - 1) / G, 64);
    const uint64_t col_lo = (uint64_t)c.shard * blk;
    if (G > 1 && (!(c.flags & GS_CANONICAL) || (uint64_t)(G - 1) * blk >= c.n_nodes)) return GS_E_INVALID;
    const uint32_t ncol = G > 1 ? (uint32_t)std::min<uint64_t>(blk, c.n_nodes - col_lo) : c.n_nodes;
    if (c.n_keys < 1 || c.n_keys > 64) return GS_E_INVALID;
    if (c.n_keys > 4u * KWB) return GS_E_UNSUPPORTED;  // a -DGS_KW4_ONLY development build
    if ((c.flags & GS_NO_HELD) && (c.flags & GS_TOMBSTONES)) return GS_E_INVALID;  // prefix views need no GC
    if (c.hist_cap < 2 || c.hist_cap > 255) return GS_E_INVALID;
    if (c.mtu < 1 || c.window < 1) return GS_E_INVALID;
    if ((c.flags & GS_FD_RING) && c.ring_rows) return GS_E_INVALID;  // every row has a ring, or a sample does
    if (c.ring_rows > c.n_nodes) return GS_E_INVALID;
    if (((c.flags & GS_FD_RING) || c.ring_rows) && (c.window > (1u << 20) || c.max_interval_ticks > 0xFFFFu))
        return GS_E_INVALID;
    // packed window: cnt < 2W needs cnt_bits, the sum of <= W intervals <= max_interval the rest of 32
    uint32_t cnt_bits = 1;
    while ((1ull << cnt_bits) <= 2ull * c.window) cnt_bits++;
    const uint32_t sum_bits = 32 - cnt_bits;
    if (cnt_bits > 31 || (uint64_t)c.window * c.max_interval_ticks >= (1ull << sum_bits)) return GS_E_INVALID;
    // 16-bit last-report ticks (GS_R_FD_LAST): a window silent for >= 2^15 ticks must be past max_interval
    // and past the phi threshold whatever its exact age (fd_get)
    const double prior_ticks = c.prior_weighted / 5.0 * 64.0;
    if (c.max_interval_ticks >= (1u << 14) ||
        c.phi_threshold * std::max((double)c.max_interval_ticks, prior_ticks) >= (double)(1u << 15))
        return GS_E_INVALID;
    gs_handle *h = new gs_handle();
    h->cfg = c;
    h->d.t_cap = NONE;  // no sub-phases yet (plane_tick)
    h->N = c.n_nodes;
    h->G = G;
    h->sliced = G > 1 || (c.flags & GS_SLICED);
    h->shard = c.shard;
    h->col_lo = G > 1 ? (uint32_t)col_lo : 0u;
    h->ncol = ncol;
    h->NP = round_up(ncol, 64);
    h->K = c.n_keys;
    h->KP = round_up(c.n_keys, 4);
    h->C = c.hist_cap;
    h->W = c.window;
    h->stream = nullptr;
    h->seq = 0;
    h->booted = false;
    const uint64_t N = h->N, NP = h->NP, KP = h->KP, K = h->K, C = h->C, W = h->W, NC = h->ncol;
    const uint64_t NR = round_up(h->N, 64);
    const uint64_t pairs = N * NP;
    const bool genm = !(c.flags & GS_CANONICAL);
    uint64_t *b = h->bytes;
    b[GS_R_HB] = pairs * ((c.flags & GS_HB8) ? 1 : 2);
    b[GS_R_SELF_HB] = NP * 4;
    b[GS_R_MV] = pairs * ((c.flags & GS_MV8) ? 1 : 2);
    b[GS_R_SELF_MV] = NP * 4;
    b[GS_R_SELF_PK] = (c.flags & GS_MV8) ? NP * 4 : 0;
    b[GS_R_P1FLAGS] = (c.flags & GS_MV8) ? NP / 16 * 4 : 0;  // k_pass1v's small / hot bits
    if (c.esc_cols > ESC_MAX || (c.esc_cols && !(c.flags & GS_MV8))) {
        delete h;
        return GS_E_INVALID;
    }
    // escape slots only where k_pass1v runs (its per-column path reads them): set below with d.pl16
    const uint64_t EC = c.esc_cols;
    b[GS_R_ESC16] = N * EC * 2;
    b[GS_R_ESC_SLOT] = EC ? NP * 4 : 0;
    b[GS_R_ESC_OWNER] = EC * 4;
    b[GS_R_ESC_REQ] = EC ? (NP / 32 + 1 + 4 * EC) * 4 : 0;
    b[GS_R_GC] = (c.flags & GS_TOMBSTONES) ? pairs * 4 : 0;  // last_gc_version stays 0 without tombstone GC
    b[GS_R_HELD] = (c.flags & GS_NO_HELD) ? 0 : pairs * KP;
    b[GS_R_FD] = pairs * 4;
    b[GS_R_FD_LAST] = pairs * 2;
    b[GS_R_FD_STATE] = pairs;
    b[GS_R_FD_TOD] = pairs * 4;
    b[GS_R_TS] = (c.flags & GS_TOMBSTONES) ? pairs * KP * 4 : 0;
    b[GS_R_RING] = (c.flags & GS_FD_RING) ? pairs * W * 2 : (uint64_t)c.ring_rows * NP * W * 2;
    b[GS_R_RING_SLOT] = c.ring_rows ? N * 4 : 0;
    b[GS_R_POS] = b[GS_R_ORD] = genm ? pairs * 4 : 0;
    b[GS_R_ROW] = N * 16;
    b[GS_R_LAST_W] = NC * KP;
    b[GS_R_HIST] = NC * C * K * 8;
    b[GS_R_HIST_VID] = NC * C * K * 4;
    b[GS_R_LATEST] = (c.flags & GS_TOMBSTONES) ? 0 : NC * KP * 4;
    const uint32_t VL = round_up(h->K * (h->C - 1) + 1, 4);  // versions 1 .. K (C - 1) (ordinals < C per key)
    b[GS_R_VLOG] = (c.flags & GS_TOMBSTONES) ? 0 : NC * VL * 4;
    b[GS_R_NID_SIZE] = NP * 2;
    b[GS_R_KEY_LEN] = KP;
    b[GS_R_STAMP] = NR * 4;
    b[GS_R_COUNTERS] = (uint64_t)NSHARD * CROW * 8;
    const bool fused = getenv("GS_FUSED") && atoi(getenv("GS_FUSED"));
    if ((c.flags & GS_SLICED) && !(c.flags & GS_CANONICAL)) {
        delete h;
        return GS_E_INVALID;  // sliced phases walk owners in column order
    }
    h->split = !h->sliced && (c.flags & GS_CANONICAL) && !fused;
    b[GS_R_SLICE_BITS] = (h->sliced || h->split) ? (N / 2) * 2 * (NP / 32) * 4 : 0;
    // candidate records: canonical handles (one slice: k_pass1 fused with packing; sliced: k_pass1 + k_count,
    // gather, k_pack_slice)
    const bool recs = (c.flags & GS_CANONICAL) && !fused;
    b[GS_R_CAND] = recs ? (N / 2) * 4 * GS_CAND_CAP * 8 : 0;
    b[GS_R_CAND_N] = recs ? (N / 2) * 4 * 4 : 0;
    b[GS_R_SLOT_STAT] = recs ? (N / 2) * 2 * 16 : 0;  // sliced spec phases; k_lite's per-slot flags
    if (const char *m = getenv("GS_PACK")) h->pack_mode = !strcmp(m, "fused") ? 1 : !strcmp(m, "spec") ? 0 : 2;
    // 8-bit heartbeats: only the record phases' pass 1 (k_pass1<HB8>) reads them in bulk
    if (((c.flags & GS_HB8) && (!(c.flags & GS_CANONICAL) || c.n_keys > 16 || fused || h->pack_mode == 1)) ||
        ((c.flags & GS_MV8) && (!(c.flags & GS_HB8) || (c.flags & GS_TOMBSTONES)))) {
        delete h;
        return GS_E_UNSUPPORTED;
    }
    const uint64_t PW = round_up(h->NP, 256) / 64;
    b[GS_R_PEND] = N * NPL * PW * 8;  // one phase bit plane per observer row and phase slot
    b[GS_R_PEND_STAMP] = N * NPL * 4;
    Dev &d = h->d;
    memset(&d, 0, sizeof d);
    d.N = h->N;
    d.col_lo = h->col_lo;
    d.ncol = h->ncol;
    d.shards = G;
    d.shard = c.shard;
    d.NP = h->NP;
    d.PW = (uint32_t)PW;
    d.K = h->K;
    d.KP = h->KP;
    d.C = h->C;
    d.mtu = c.mtu;
    d.flags = c.flags;
    d.W = c.window;
    d.max_iv = c.max_interval_ticks;
    d.tomb_grace = c.tombstone_grace_ticks;
    d.dead_grace = c.dead_grace_ticks;
    d.sched_delay = c.sched_delay_ticks;
    d.sum_bits = sum_bits;
    d.VL = VL;
    d.hb8 = (c.flags & GS_HB8) ? 1u : 0u;
    d.mv8 = (c.flags & GS_MV8) ? 1u : 0u;
    // GS_MV8 record phases run k_pass1v (its 16-column report planes) unless env GS_P1=old (round 3's k_pass1, A/B
    // runs) or the speculative-merge mode asks for k_pass1's merge
    {
        const char *p1 = getenv("GS_P1");
        d.pl16 = d.mv8 && h->pack_mode == 2 && !(p1 && !strcmp(p1, "old")) ? 1u : 0u;
    }
    if (!d.pl16)
        for (int r : {GS_R_ESC16, GS_R_ESC_SLOT, GS_R_ESC_OWNER, GS_R_ESC_REQ}) b[r] = 0;
    d.EC = d.pl16 ? c.esc_cols : 0u;
    if (const char *ab = getenv("GS_ABLATE")) d.ablate = (uint32_t)atoi(ab);
    d.phi_thr = c.phi_threshold;
    d.prior5 = c.prior_weighted;
    d.prior5t = c.prior_weighted * 64.0;
    d.phi_thr_f = (float)c.phi_threshold;
    d.prior5t_f = (float)d.prior5t;
    *out = h;
    return GS_OK;
}

void gs_destroy(gs_handle *h) {
    if (!h) return;
    for (auto &v : h->tev)
        for (auto &pr : v) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
    for (hipEvent_t e : h->evpool) (void)hipEventDestroy(e);
    for (void *p : {(void *)h->sc.tot, (void *)h->sc.tot_all, (void *)h->sc.chain, (void *)h->sc.chainc,
                    (void *)h->sc.chain_all, (void *)h->sc.list, (void *)h->sc.pend})
        if (p) (void)hipFree(p);
    if (h->sc.pin) (void)hipHostFree(h->sc.pin);
    if (h->grp) (void)hipFree(h->grp);
    if (h->heavy_buf) (void)hipFree(h->heavy_buf);
    if (h->sm_buf) (void)hipFree(h->sm_buf);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_join) (void)hipEventDestroy(h->ev_join);
    if (h->hside) (void)hipStreamDestroy(h->hside);
    if (h->comm) (void)ncclCommDestroy(h->comm);
    if (h->side) (void)hipStreamDestroy(h->side);
    for (hipEvent_t e : {h->fj_fork, h->fj_join})
        if (e) (void)hipEventDestroy(e);
    delete h;
}

int gs_region_bytes(const gs_handle *h, int region, uint64_t *bytes) {
    if (!h || !bytes || region < 0 || region >= GS_NUM_REGIONS) return GS_E_INVALID;
    *bytes = h->bytes[region];
    return GS_OK;
}

int gs_bind(gs_handle *h, int region, void *ptr) {
    if (!h || region < 0 || region >= GS_NUM_REGIONS) return GS_E_INVALID;
    if (ptr && (reinterpret_cast<uintptr_t>(ptr) & 15u))
        return fail(h, GS_E_INVALID, "region %d: device pointer must be 16-byte aligned", region);
    h->reg[region] = ptr;
    return GS_OK;
}

int gs_set_stream(gs_handle *h, void *stream) {
    if (!h) return GS_E_INVALID;
    h->stream = (hipStream_t)stream;
    return GS_OK;
}

int gs_boot(gs_handle *h, const uint16_t *nid_size, const uint8_t *key_len) {
    if (!h || !nid_size || !key_len) return GS_E_INVALID;
    int rc = check_bound(h);
    if (rc) return rc;
    hipStream_t s = h->stream;
    // regions that start at zero
    const int zero[] = {GS_R_HB, GS_R_SELF_HB, GS_R_MV, GS_R_GC, GS_R_HELD, GS_R_FD, GS_R_FD_LAST, GS_R_FD_STATE, GS_R_FD_TOD,
                        GS_R_RING, GS_R_ROW, GS_R_LAST_W, GS_R_HIST, GS_R_HIST_VID,
                        GS_R_STAMP, GS_R_COUNTERS, GS_R_SLICE_BITS, GS_R_PEND, GS_R_PEND_STAMP, GS_R_LATEST,
                        GS_R_SLOT_STAT, GS_R_VLOG, GS_R_SELF_MV, GS_R_SELF_PK, GS_R_P1FLAGS, GS_R_ESC16, GS_R_ESC_REQ};
    for (int r : zero)
        if (h->bytes[r]) HIPCHK(h, hipMemsetAsync(h->reg[r], 0, h->bytes[r], s));
    if (h->bytes[GS_R_TS]) HIPCHK(h, hipMemsetAsync(h->reg[GS_R_TS], 0xFF, h->bytes[GS_R_TS], s));
    if (h->bytes[GS_R_POS]) HIPCHK(h, hipMemsetAsync(h->reg[GS_R_POS], 0xFF, h->bytes[GS_R_POS], s));
    if (h->bytes[GS_R_ORD]) HIPCHK(h, hipMemsetAsync(h->reg[GS_R_ORD], 0xFF, h->bytes[GS_R_ORD], s));
    if (h->bytes[GS_R_RING_SLOT]) HIPCHK(h, hipMemsetAsync(h->reg[GS_R_RING_SLOT], 0xFF, h->bytes[GS_R_RING_SLOT], s));
    for (int r : {GS_R_ESC_SLOT, GS_R_ESC_OWNER})  // no escaped columns
        if (h->bytes[r]) HIPCHK(h, hipMemsetAsync(h->reg[r], 0xFF, h->bytes[r], s));
    // tables
    // nid_size covers all n_nodes (the packer's stop bound must hold across slices); keep this slice's
    std::vector<uint16_t> ns(h->NP, 0);
    uint32_t min_nid = 0xFFFFFFFFu, min_key = 0xFFFFFFFFu;
    for (uint32_t j = 0; j < h->N; j++) {
        if (j - h->col_lo < h->ncol) ns[j - h->col_lo] = nid_size[j];
        if (nid_size[j] < min_nid) min_nid = nid_size[j];
    }
    std::vector<uint8_t> kl(h->KP, 0);
    for (uint32_t k = 0; k < h->K; k++) {
        kl[k] = key_len[k];
        if (key_len[k] < min_key) min_key = key_len[k];
    }
    HIPCHK(h, hipMemcpyAsync(h->reg[GS_R_NID_SIZE], ns.data(), h->NP * 2, hipMemcpyHostToDevice, s));
    HIPCHK(h, hipMemcpyAsync(h->reg[GS_R_KEY_LEN], kl.data(), h->KP, hipMemcpyHostToDevice, s));
    // smallest possible single-kv NodeDelta: no NodeDelta can fit once fewer bytes remain
    const uint32_t kv_min = msgf(sfield(min_key) + 2u);
    h->d.lb_min = msgf(msgf(min_nid) + 2u + kv_min);
    k_boot_self<<<(h->N + LB - 1) / LB, LB, 0, s>>>(h->d);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(s));
    h->booted = true;
    return GS_OK;
}

int gs_set_ring_rows(gs_handle *h, const uint32_t *rows, uint32_t n) {
    if (!h || !h->booted || (n && !rows)) return GS_E_INVALID;
    if (n > h->cfg.ring_rows)
        return fail(h, GS_E_INVALID, "gs_set_ring_rows: %u rows for %u ring slots (gs_config.ring_rows)", n, h->cfg.ring_rows);
    // a row switched between a compact window and a ring slot later would read a stale or empty ring
    if (h->started) return fail(h, GS_E_INVALID, "gs_set_ring_rows: after gs_boot, before the first round only");
    std::vector<uint32_t> slot(h->N, NONE);
    for (uint32_t i = 0; i < n; i++) {
        if (rows[i] >= h->N || slot[rows[i]] != NONE)
            return fail(h, GS_E_INVALID, "gs_set_ring_rows: row %u out of range or repeated", rows[i]);
        slot[rows[i]] = i;
    }
    HIPCHK(h, hipMemcpyAsync(h->reg[GS_R_RING_SLOT], slot.data(), (size_t)h->N * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return GS_OK;
}

int gs_warm(gs_handle *h) {
    if (!h || !h->booted) return GS_E_INVALID;
    const uint64_t pairs = (uint64_t)h->N * h->ncol;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((pairs + LB - 1) / LB, 1u << 20);
    k_warm<<<blocks, LB, 0, h->stream>>>(h->d);
    HIPCHK(h, hipGetLastError());
    return GS_OK;
}

int gs_materialize_held(gs_handle *h, uint32_t row_lo, uint32_t row_hi) {
    if (!h || !h->booted || row_lo > row_hi || row_hi > h->N) return GS_E_INVALID;
    if ((h->cfg.flags & (GS_TOMBSTONES | GS_NO_HELD)) || row_lo == row_hi) return GS_OK;  // kept / not stored
    const uint64_t pairs = (uint64_t)(row_hi - row_lo) * h->ncol;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((pairs + LB - 1) / LB, 1u << 16);
    k_materialize<<<blocks, LB, 0, h->stream>>>(h->d, row_lo, row_hi);
    HIPCHK(h, hipGetLastError());
    return GS_OK;
}

int gs_owner_writes(gs_handle *h, const gs_write *ops, uint32_t n, uint32_t tick) {
    if (!h || !h->booted) return GS_E_INVALID;
    if (!n) return GS_OK;
    if (h->d.mv8 && h->mv_incs >= MV8_LAG_CHECK_EVERY) {  // 8-bit max_version views: <= 32 owner versions between sweeps
        int rc = gs_check_heartbeat_lag(h);
        if (rc) return rc;
    }
    h->mv_incs++;
    k_owner_writes<<<(n + LB - 1) / LB, LB, 0, h->stream>>>(h->d, ops, n, tick);
    HIPCHK(h, hipGetLastError());
    if (h->d.ev) h->d.ev_wseq += n;
    // the first-fit stop bound (Dev::sm): one-slice canonical prefix-view handles, env GS_SM=0: off (A/B)
    if (sm_on() && h->G == 1 && !h->sliced && h->d.vlog && (h->cfg.flags & GS_CANONICAL)) {
        const uint32_t nblk = (h->ncol + 1023u) / 1024u;
        if (!h->sm_buf) {  // sm [NP + 1] u16, then the block minima [nblk] u32
            HIPCHK(h, hipMalloc(&h->sm_buf, ((size_t)h->NP + 2) * 2 + (size_t)nblk * 4 + 16));
        }
        uint32_t *blk = reinterpret_cast<uint32_t *>(
            (reinterpret_cast<uintptr_t>(h->sm_buf + h->NP + 2) + 15) & ~(uintptr_t)15);
        h->d.sm = h->sm_buf;
        k_sm_local<<<nblk, 1024, 0, h->stream>>>(h->d, blk);
        HIPCHK(h, hipGetLastError());
        k_sm_fix<<<nblk, 1024, 0, h->stream>>>(h->d, blk, nblk);
        HIPCHK(h, hipGetLastError());
    }
    return GS_OK;
}

int gs_begin_round(gs_handle *h, const uint8_t *up, uint32_t tick) {
    if (!h || !h->booted || !up) return GS_E_INVALID;
    if (h->reports_pending)
        return fail(h, GS_E_INVALID, "gs_begin_round: the previous round's phases were not closed by gs_liveness");
    if (h->hb_incs >= (h->d.hb8 ? HB8_LAG_CHECK_EVERY : HB_LAG_CHECK_EVERY)) {
        int rc = gs_check_heartbeat_lag(h);
        if (rc) return rc;
    }
    if (int rc = fd_age(h, tick)) return rc;  // the tick axis of the 16-bit report ticks (and gs_latest_tick)
    h->d.t_round = tick;
    h->base_fresh = true;
    h->sub_ok = false;
    h->last_phase_tick = tick;
    k_begin_round<<<h->N, LB, 0, h->stream>>>(h->d, up, tick);
    HIPCHK(h, hipGetLastError());
    h->round_open = true;
    h->started = true;
    h->hb_incs++;
    return GS_OK;
}

int gs_check_heartbeat_lag(gs_handle *h) {
    if (!h || !h->booted) return GS_E_INVALID;
    const uint32_t per = h->d.hb8 ? 16u : 8u, chunks = (h->ncol + LB * per - 1) / (LB * per);
    if (h->d.p1flags) {
        k_hot_clear<<<(std::max(h->N, h->NP / 16u) + LB - 1) / LB, LB, 0, h->stream>>>(h->d);
        HIPCHK(h, hipGetLastError());
    }
    k_hb_lag<<<(h->N + LAG_ROWS - 1) / LAG_ROWS * chunks, LB, 0, h->stream>>>(h->d, chunks);
    HIPCHK(h, hipGetLastError());
    if (h->d.EC) {  // escaped owner columns: moves decided, then copied (one pass over the rows)
        k_esc_plan<<<1, 1024, 0, h->stream>>>(h->d);
        HIPCHK(h, hipGetLastError());
        k_esc_move<<<(h->N + LB - 1) / LB, LB, 0, h->stream>>>(h->d);
        HIPCHK(h, hipGetLastError());
    }
    h->lag_sweeps++;
    h->hb_incs = 0;
    h->mv_incs = 0;
    return GS_OK;
}

extern "C++" {
namespace {
int sliced_phase(gs_handle *const *hs, uint32_t nh, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick);
}
}

int gs_run_phase(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick) {
    int rc = check_phase(h, ini, res, n, tick);
    if (rc) return rc;
    if (h->sliced) {
        if (!h->comm)
            return fail(h, GS_E_UNSUPPORTED, "sliced handle without gs_comm_init: use gs_run_phase_group or gs_phase_*");
        return n ? sliced_phase(&h, 1, ini, res, n, tick) : GS_OK;
    }
    if (!n) return GS_OK;
    if ((rc = fd_age(h, tick)) || (rc = plane_slot(h, tick, h->sub_ok && tick == h->last_phase_tick))) return rc;
    h->sub_ok = true;
    const bool genm = !(h->cfg.flags & GS_CANONICAL);
    const size_t lds = exchange_lds(h);
    const SliceIO io{};
    h->seq += 1;
    h->reports_pending = true;
    h->last_phase_tick = tick;
    h->hb_incs++;
    if (h->split) return run_split_phase(h, ini, res, n, tick);
    h->d.spec = 0u;
    h->d.lite = 0u;
    hipEvent_t e0 = nullptr;
    if ((rc = time_begin(h, e0))) return rc;
    if (h->KP <= 16) rc = genm ? launch_exchange<4, true, 0>(h, ini, res, n, tick, lds, io)
                               : launch_exchange<4, false, 0>(h, ini, res, n, tick, lds, io);
    else rc = genm ? launch_exchange<KWB, true, 0>(h, ini, res, n, tick, lds, io)
                   : launch_exchange<KWB, false, 0>(h, ini, res, n, tick, lds, io);
    return rc ? rc : time_end(h, GS_KT_PASS1, e0);
}

int gs_shard_columns(const gs_handle *h, uint32_t *col_lo, uint32_t *n_cols) {
    if (!h || !col_lo || !n_cols) return GS_E_INVALID;
    *col_lo = h->col_lo;
    *n_cols = h->ncol;
    return GS_OK;
}

int gs_phase_count(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick,
                   uint64_t *slice_bytes) {
    int rc = check_phase(h, ini, res, n, tick);
    if (rc) return rc;
    if (!h->sliced) return fail(h, GS_E_UNSUPPORTED, "gs_phase_count needs a sliced handle (n_shards > 1 or GS_SLICED)");
    if (!n) return GS_OK;
    if (!slice_bytes) return GS_E_INVALID;
    if ((rc = fd_age(h, tick)) || (rc = plane_slot(h, tick, h->sub_ok && tick == h->last_phase_tick))) return rc;
    h->sub_ok = true;
    const size_t lds = exchange_lds(h);
    SliceIO io{};
    io.tot = slice_bytes;
    h->seq += 1;
    h->reports_pending = true;
    h->last_phase_tick = tick;
    h->hb_incs++;
    if (!h->d.cand) {  // GS_FUSED: the fused count pass (LDS bitmaps)
        h->d.spec = 0u;
        h->d.lite = 0u;
        hipEvent_t e0 = nullptr;
        if ((rc = time_begin(h, e0))) return rc;
        rc = h->KP <= 16 ? launch_exchange<4, false, 1>(h, ini, res, n, tick, lds, io)
                         : launch_exchange<KWB, false, 1>(h, ini, res, n, tick, lds, io);
        return rc ? rc : time_end(h, GS_KT_PASS1, e0);
    }
    // the speculative merge is decided here for the whole phase (gs_phase_pack / gs_phase_chain use it)
    h->d.spec = spec_ok(h) || spec_v_ok(h) ? 1u : 0u;
    h->d.lite = lite_ok(h) ? 1u : 0u;
    if (p1lite(h, 1)) {  // the lite slot work ran in k_pass1v: the exact count of the slots it left (LITE_FULL) only
        if ((rc = launch_pass1(h, ini, res, n, tick, 1, io, true))) return rc;
        h->d.p1fix = 1u;  // and the responders' small bits (k_p1v_fix)
        rc = launch_settle<1>(h, ini, res, n, tick, io, GS_KT_COUNT);
        h->d.p1fix = 0u;
        return rc;
    }
    if (h->d.lite && lite_fuse() && h->d.pl16) {  // lite + count in one launch, which also sets the small bits
        if ((rc = launch_pass1(h, ini, res, n, tick, -1, io, true))) return rc;
        h->d.p1fix = 1u;
        rc = launch_settle<1, true>(h, ini, res, n, tick, io, GS_KT_COUNT);
        h->d.p1fix = 0u;
        return rc;
    }
    if ((rc = launch_pass1(h, ini, res, n, tick))) return rc;
    if (h->d.lite && lite_fuse()) return launch_settle<1, true>(h, ini, res, n, tick, io, GS_KT_COUNT);
    if (h->d.lite && (rc = launch_lite<1>(h, ini, res, n, tick, io))) return rc;
    return launch_settle<1>(h, ini, res, n, tick, io, GS_KT_COUNT);
}

int gs_phase_pack(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick, uint32_t step,
                  const uint64_t *slice_bytes_all, const uint64_t *chain_all, uint64_t *chain) {
    if (h && !n) return GS_OK;
    int rc = check_phase(h, ini, res, n, tick, true);
    if (rc) return rc;
    if (!h->sliced) return fail(h, GS_E_UNSUPPORTED, "gs_phase_pack needs a sliced handle (n_shards > 1 or GS_SLICED)");
    if (!n) return GS_OK;
    if (!slice_bytes_all || !chain || step >= h->G || (step && !chain_all)) return GS_E_INVALID;
    SliceIO io{};
    io.tot_all = slice_bytes_all;
    io.chain_all = chain_all;
    io.chain = chain;
    io.step = step;
    if (step && h->shard == 0) return GS_OK;  // slice 0 always finishes at step 0
    if (step == 0 && h->d.cand) {
        if (h->d.lite && lite_fuse()) return launch_settle<2, true>(h, ini, res, n, tick, io, GS_KT_PACK);
        if (h->d.lite && (rc = launch_lite<2>(h, ini, res, n, tick, io))) return rc;
        return launch_settle<2>(h, ini, res, n, tick, io, GS_KT_PACK);
    }
    hipEvent_t e0 = nullptr;
    if ((rc = time_begin(h, e0))) return rc;
    if (h->KP <= 16) k_pack_slice<4><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io, 0u);
    else k_pack_slice<KWB><<<n, XB, 0, h->stream>>>(h->d, ini, res, n, tick, io, 0u);
    HIPCHK(h, hipGetLastError());
    return time_end(h, GS_KT_PACK, e0);
}

int gs_phase_overflow(gs_handle *h, uint32_t n, const uint64_t *slice_bytes_all, const uint64_t *chain,
                      uint32_t *list, uint64_t *chainc, uint32_t *count) {
    if (!h || !h->booted) return GS_E_INVALID;
    if (count) *count = 0;
    if (!n) return GS_OK;
    if (!h->sliced || !h->d.cand) return fail(h, GS_E_UNSUPPORTED, "gs_phase_overflow needs a sliced canonical handle");
    if (!slice_bytes_all || !chain || !list || !chainc) return GS_E_INVALID;
    const uint32_t slots = 2 * n, nb = (slots + OVB - 1) / OVB;
    k_ov_count<<<nb, OVB, 0, h->stream>>>(slice_bytes_all, slots, h->G, h->cfg.mtu, list + slots, nullptr);
    HIPCHK(h, hipGetLastError());
    k_ov_write<<<nb, OVB, 0, h->stream>>>(slice_bytes_all, slots, h->G, h->cfg.mtu, chain, list, chainc, nullptr);
    HIPCHK(h, hipGetLastError());
    k_pending<<<1, OVB, 0, h->stream>>>(list, list + slots + nb, 0u, chain, chainc, nullptr, n);  // chainc[count]
    HIPCHK(h, hipGetLastError());
    if (count) {  // count = NULL: no read back (another slice in this process reads the same count)
        HIPCHK(h, hipMemcpyAsync(count, list + slots + nb, 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    return GS_OK;
}

int gs_phase_chain(gs_handle *h, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick, uint32_t step,
                   const uint32_t *list, uint32_t count, const uint64_t *chain_all, uint64_t *chain, uint64_t *chainc,
                   const uint64_t *slice_bytes_all) {
    const bool dev = count == GS_CHAIN_DEVICE;  // the count stays on the device (gs_phase_overflow's list tail)
    if (h && (!n || !count)) return GS_OK;
    int rc = check_phase(h, ini, res, n, tick, true);
    if (rc) return rc;
    if (!h->sliced || !h->d.cand) return fail(h, GS_E_UNSUPPORTED, "gs_phase_chain needs a sliced canonical handle");
    if (!list || !chain_all || !chain || !chainc || !slice_bytes_all || step < 1 || step >= h->G ||
        (!dev && count > 2 * n))
        return GS_E_INVALID;
    if (h->shard == 0) return GS_OK;  // slice 0 always finishes at step 0 (its pending entry stays 0)
    hipEvent_t e0 = nullptr;
    if ((rc = time_begin(h, e0))) return rc;
    const uint32_t *cnt_dev = dev ? list + 2u * n + (2u * n + OVB - 1u) / OVB : nullptr;
    const uint32_t grid = std::min<uint32_t>(dev ? GS_CHAIN_CAP : count, 2048u), c = dev ? 0u : count;
    if (h->KP <= 16)
        k_chain_step<4><<<grid, WAVE, 0, h->stream>>>(h->d, ini, res, tick, list, c, chain_all, chain, chainc,
                                                       slice_bytes_all, n, cnt_dev, nullptr, DevDyn{});
    else
        k_chain_step<KWB><<<grid, WAVE, 0, h->stream>>>(h->d, ini, res, tick, list, c, chain_all, chain, chainc,
                                                         slice_bytes_all, n, cnt_dev, nullptr, DevDyn{});
    HIPCHK(h, hipGetLastError());
    k_pending<<<1, OVB, 0, h->stream>>>(list, cnt_dev, c, chain, chainc, nullptr, n);  // chainc[count]
    HIPCHK(h, hipGetLastError());
    return time_end(h, GS_KT_PACK, e0);
}

// ---- sliced phases driven by the library
extern "C++" {
namespace {
int ensure_scratch(gs_handle *h, uint32_t n) {
    if (h->sc.cap >= n) return GS_OK;
    for (void *p : {(void *)h->sc.tot, (void *)h->sc.tot_all, (void *)h->sc.chain, (void *)h->sc.chainc,
                    (void *)h->sc.chain_all, (void *)h->sc.list, (void *)h->sc.pend})
        if (p) HIPCHK(h, hipFree(p));
    const uint32_t cap = std::max(n, 1024u);
    const size_t s2 = (size_t)2 * cap * 8, G = h->G;
    HIPCHK(h, hipMalloc(&h->sc.tot, s2));
    HIPCHK(h, hipMalloc(&h->sc.chain, s2));
    HIPCHK(h, hipMalloc(&h->sc.chainc, s2 + 8));                 // [2 cap + 1]: the pending entry last
    HIPCHK(h, hipMalloc(&h->sc.tot_all, G * s2));
    HIPCHK(h, hipMalloc(&h->sc.chain_all, G * (s2 + 8)));      // [G][count + 1]
    HIPCHK(h, hipMalloc(&h->sc.pend, 16));
    HIPCHK(h, hipMalloc(&h->sc.list, (size_t)GS_OVERFLOW_LIST_LEN(cap) * 4));
    h->sc.cap = cap;
    return GS_OK;
}

// k_sum_pending into the handle's pinned host pair (written by the kernel itself: no copy), then one wait
int read_pending(gs_handle *h, uint32_t G, uint32_t count, const uint32_t *cnt_dev, const uint64_t *chain_all,
                 uint64_t &pend, uint32_t &cnt) {
    if (!h->sc.pin) {
        HIPCHK(h, hipHostMalloc((void **)&h->sc.pin, 16, hipHostMallocMapped));
        HIPCHK(h, hipHostGetDevicePointer((void **)&h->sc.pin_dev, h->sc.pin, 0));
    }
    k_sum_pending<<<1, WAVE, 0, h->stream>>>(chain_all, G, count, cnt_dev, h->sc.pin_dev);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    pend = reinterpret_cast<volatile uint64_t *>(h->sc.pin)[0];
    cnt = (uint32_t)reinterpret_cast<volatile uint64_t *>(h->sc.pin)[1];
    return GS_OK;
}

// all-gather of `count` u64 per slice (src of slice g -> dst[g * count ..], on every slice): one RCCL
// all-gather when this process drives one slice of a communicator, one gather kernel (k_gather_u64)
// when it drives them all
int gather_u64(gs_handle *const *hs, uint32_t nh, uint64_t *(*src)(gs_handle *), uint64_t *(*dst)(gs_handle *),
               size_t count) {
    if (!count) return GS_OK;
    if (nh == 1) {
        gs_handle *h = hs[0];
        if (!h->comm) {  // one slice held alone (gs_run_phase_group): GS_SLICED's one slice, or a rehearsal of one
            // GPU's share of a G-slice cluster, whose other slices gather as zeros (as shard.py's SoloComm)
            // (one k_gather_u64 launch with null sources for the others: zeros and the copy together)
            if (h->G > GATHER_MAX) return fail(h, GS_E_INVALID, "gather over %u slices (at most %u)", h->G, GATHER_MAX);
            GatherPtrs p{};
            p.src[h->shard] = src(h);
            p.dst[0] = dst(h);
            const uint64_t total = (uint64_t)h->G * count;
            const uint32_t bx = (uint32_t)std::min<uint64_t>((total + LB - 1) / LB, 4096u);
            k_gather_u64<<<dim3(bx, 1), LB, 0, h->stream>>>(p, h->G, count);
            HIPCHK(h, hipGetLastError());
            return GS_OK;
        }
        const ncclResult_t r = ncclAllGather(src(h), dst(h), count, ncclUint64, h->comm, h->stream);
        if (r != ncclSuccess) return fail(h, GS_E_HIP, "ncclAllGather: %s", ncclGetErrorString(r));
        return GS_OK;
    }
    if (nh > GATHER_MAX) return fail(hs[0], GS_E_INVALID, "gather over %u slices (at most %u)", nh, GATHER_MAX);
    GatherPtrs p{};
    for (uint32_t g = 0; g < nh; g++) {
        p.src[g] = src(hs[g]);
        p.dst[g] = dst(hs[g]);
    }
    const uint64_t total = (uint64_t)nh * count;
    const uint32_t bx = (uint32_t)std::min<uint64_t>((total + LB - 1) / LB, 4096u);
    k_gather_u64<<<dim3(bx, nh), LB, 0, hs[0]->stream>>>(p, nh, count);
    HIPCHK(hs[0], hipGetLastError());
    return GS_OK;
}

// One phase of a sliced cluster: pass 1 + slice totals on every slice, all-gather of the
// totals (16 B per exchange and slice), packing step 0, then -- only for the (exchange, direction) slots
// whose totals sum past the MTU, listed on the device, one host read -- G - 1 chain steps, each an
// all-gather of those slots' chain states (8 B per slot and slice) and a resume on the next slice.
// In-process slices (gs_run_phase_group): fork every slice onto its own stream after the work queued so far on
// the group's stream, and join them back before a step that reads all slices (the gathers).  One RCCL slice per
// process (nh = 1) runs on its own stream as it is.
int fork_slices(gs_handle *const *hs, uint32_t nh) {
    gs_handle *h0 = hs[0];
    if (nh < 2) return GS_OK;
    if (!h0->fj_fork) HIPCHK(h0, hipEventCreateWithFlags(&h0->fj_fork, hipEventDisableTiming));
    // every stream, event and wait first; the handles switch streams only once nothing can fail (a
    // failure half-way left the earlier handles on their side streams)
    for (uint32_t i = 0; i < nh; i++) {
        gs_handle *h = hs[i];
        if (!h->side) HIPCHK(h, hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
        if (!h->fj_join) HIPCHK(h, hipEventCreateWithFlags(&h->fj_join, hipEventDisableTiming));
    }
    HIPCHK(h0, hipEventRecord(h0->fj_fork, h0->stream));
    for (uint32_t i = 0; i < nh; i++) HIPCHK(hs[i], hipStreamWaitEvent(hs[i]->side, h0->fj_fork, 0));
    for (uint32_t i = 0; i < nh; i++) {
        hs[i]->home = hs[i]->stream;
        hs[i]->stream = hs[i]->side;
    }
    return GS_OK;
}
int join_slices(gs_handle *const *hs, uint32_t nh, int rc = GS_OK) {
    if (nh < 2) return rc;
    for (uint32_t i = 0; i < nh; i++) {  // streams restored first, whatever failed
        gs_handle *h = hs[i];
        const hipError_t e = hipEventRecord(h->fj_join, h->side);
        h->stream = h->home;
        if (e != hipSuccess && rc == GS_OK) rc = fail(h, GS_E_HIP, "hipEventRecord: %s", hipGetErrorString(e));
    }
    for (uint32_t i = 0; i < nh && rc == GS_OK; i++) HIPCHK(hs[0], hipStreamWaitEvent(hs[0]->stream, hs[i]->fj_join, 0));
    return rc;
}
// gs_run_phase_group's batched steps (round 5): the slices of one process run each step as ONE launch (grid.y =
// slice) instead of one launch per slice -- the in-process rehearsal of a G-GPU run otherwise paid G launches
// (and their gaps) per step (1.67x one handle at 8 slices).  The default layout (GS_MV8 record phases
// with the lite path, K <= 16), 2..GRP_MAX slices on one stream; env GS_GROUP_BATCH=0: a launch per slice (A/B).
bool group_batch_ok(gs_handle *const *hs, uint32_t nh) {
    static const bool on = [] {
        const char *e = getenv("GS_GROUP_BATCH");
        return !(e && e[0] == '0');
    }();
    if (!on || nh < 2 || nh > GRP_MAX || hs[0]->comm) return false;
    for (uint32_t i = 0; i < nh; i++) {
        const gs_handle *h = hs[i];
        if (!h->d.cand || !h->d.pl16 || !lite_ok(h) || h->KP > 16 || !lite_fuse() || p1lite(h, 1)) return false;
    }
    return true;
}
// the group's GroupArgs: every slice's Dev (its per-phase fields zero: they come by value) and scratch pointers,
// uploaded only when the image differs from the last one
int group_upload(gs_handle *const *hs, uint32_t nh) {
    gs_handle *h0 = hs[0];
    std::vector<uint8_t> buf(sizeof(GroupArgs), 0u);
    GroupArgs &img = *reinterpret_cast<GroupArgs *>(buf.data());
    for (uint32_t i = 0; i < nh; i++) {
        const gs_handle *h = hs[i];
        memcpy(&img.dv[i], &h->d, sizeof(Dev));
        img.dv[i].t_round = img.dv[i].spec = img.dv[i].lite = img.dv[i].p1fix = 0u;
        img.dv[i].v_round = img.dv[i].vt = img.dv[i].t_cap = 0u;
        img.io[i].tot = h->sc.tot;
        img.io[i].tot_all = h->sc.tot_all;
        img.io[i].chain_all = h->sc.chain_all;
        img.io[i].chain = h->sc.chain;
        img.list[i] = h->sc.list;
        img.chain_all[i] = h->sc.chain_all;
        img.chainc[i] = h->sc.chainc;
    }
    if (!h0->grp) HIPCHK(h0, hipMalloc(&h0->grp, sizeof(GroupArgs)));
    if (h0->grp_img != buf) {
        HIPCHK(h0, hipMemcpyAsync(h0->grp, buf.data(), buf.size(), hipMemcpyHostToDevice, h0->stream));
        HIPCHK(h0, hipStreamSynchronize(h0->stream));  // (the source is this function's buffer)
        h0->grp_img.swap(buf);
    }
    return GS_OK;
}
// count, gather, step 0, the overflow lists and chain step 1 of a sliced phase, batched over the group
int group_steps(gs_handle *const *hs, uint32_t nh, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick) {
    int rc;
    gs_handle *h0 = hs[0];
    // per slice: gs_phase_count's checks and bookkeeping (a lag sweep or a window-age sweep may launch here)
    for (uint32_t i = 0; i < nh; i++) {
        gs_handle *h = hs[i];
        if ((rc = check_phase(h, ini, res, n, tick))) return rc;
        if ((rc = fd_age(h, tick)) || (rc = plane_slot(h, tick, h->sub_ok && tick == h->last_phase_tick))) return rc;
        h->sub_ok = true;
        h->seq += 1;
        h->reports_pending = true;
        h->last_phase_tick = tick;
        h->hb_incs++;
        h->d.spec = spec_ok(h) || spec_v_ok(h) ? 1u : 0u;
        h->d.lite = lite_ok(h) ? 1u : 0u;
        if (h->seq != h0->seq || h->d.t_round != h0->d.t_round || h->d.spec != h0->d.spec || h->d.lite != h0->d.lite ||
            h->d.v_round != h0->d.v_round || h->d.vt != h0->d.vt || h->d.t_cap != h0->d.t_cap)
            return fail(h0, GS_E_INVALID, "gs_run_phase_group: slice %u is not in step with slice 0", i);
    }
    if ((rc = group_upload(hs, nh))) return rc;
    GroupCtx gx;
    gx.ga = h0->grp;
    gx.nh = nh;
    gx.dyn = DevDyn{h0->d.t_round, h0->d.spec, h0->d.lite, 0u, h0->d.v_round, h0->d.vt, h0->d.t_cap};
    SliceIO io{};  // (each slice's from GroupArgs; the step by value)
    // count: pass 1, then lite + the slice totals in one launch, which also sets the responders' small bits; env
    // GS_GRP_P1LITE=1: the lite slot work in pass 1's epilogue instead, the count launch only for LITE_FULL slots
    static const bool glite = [] {
        const char *e = getenv("GS_GRP_P1LITE");
        return e && e[0] == '1';
    }();
    if ((rc = launch_pass1(h0, ini, res, n, tick, glite ? 1 : -1, io, true, gx))) return rc;
    gx.dyn.p1fix = 1u;
    rc = glite ? launch_settle<1>(h0, ini, res, n, tick, io, GS_KT_COUNT, gx)
               : launch_settle<1, true>(h0, ini, res, n, tick, io, GS_KT_COUNT, gx);
    if (rc) return rc;
    gx.dyn.p1fix = 0u;
    if ((rc = gather_u64(hs, nh, [](gs_handle *h) { return h->sc.tot; }, [](gs_handle *h) { return h->sc.tot_all; },
                         (size_t)2 * n)))
        return rc;
    // step 0, then the overflowing slots listed on the device (the same list on every slice)
    if ((rc = launch_settle<2, true>(h0, ini, res, n, tick, io, GS_KT_PACK, gx))) return rc;
    const uint32_t slots = 2 * n, nb = (slots + OVB - 1) / OVB, G = h0->G;
    const uint32_t *cnt0 = h0->sc.list + slots + nb;  // (each slice's own list tail, from GroupArgs)
    k_ov_count<<<dim3(nb, nh), OVB, 0, h0->stream>>>(nullptr, slots, G, h0->cfg.mtu, nullptr, h0->grp);
    HIPCHK(h0, hipGetLastError());
    k_ov_write<<<dim3(nb, nh), OVB, 0, h0->stream>>>(nullptr, slots, G, h0->cfg.mtu, nullptr, nullptr, nullptr, h0->grp);
    HIPCHK(h0, hipGetLastError());
    k_pending<<<dim3(1, nh), OVB, 0, h0->stream>>>(nullptr, cnt0, 0u, nullptr, nullptr, h0->grp, n);
    HIPCHK(h0, hipGetLastError());
    // chain step 1 on the device count
    if ((rc = gather_u64(hs, nh, [](gs_handle *h) { return h->sc.chainc; }, [](gs_handle *h) { return h->sc.chain_all; },
                         GS_CHAIN_CAP + 1u)))
        return rc;
    hipEvent_t e0 = nullptr;
    if ((rc = time_begin(h0, e0))) return rc;
    k_chain_step<4, true><<<dim3(std::min<uint32_t>(GS_CHAIN_CAP, 2048u), nh), WAVE, 0, h0->stream>>>(
        h0->d, ini, res, tick, nullptr, 0u, nullptr, nullptr, nullptr, nullptr, n, cnt0, h0->grp, gx.dyn);
    HIPCHK(h0, hipGetLastError());
    k_pending<<<dim3(1, nh), OVB, 0, h0->stream>>>(nullptr, cnt0, 0u, nullptr, nullptr, h0->grp, n);
    HIPCHK(h0, hipGetLastError());
    return time_end(h0, GS_KT_PACK, e0);
}

int sliced_phase(gs_handle *const *hs, uint32_t nh, const int32_t *ini, const int32_t *res, uint32_t n, uint32_t tick) {
    int rc;
    for (uint32_t i = 0; i < nh; i++) {
        if (!hs[i]->d.cand) return fail(hs[i], GS_E_UNSUPPORTED, "library-driven sliced phases need candidate records");
        if ((rc = ensure_scratch(hs[i], n))) return rc;
    }
    const uint32_t G = hs[0]->G;
    gs_handle *h0 = hs[0];
    const uint32_t *cnt0 = h0->sc.list + 2u * n + (2u * n + OVB - 1u) / OVB;  // gs_phase_overflow's count entry
    auto gather_chain = [&](size_t entries) {
        return gather_u64(hs, nh, [](gs_handle *h) { return h->sc.chainc; }, [](gs_handle *h) { return h->sc.chain_all; },
                          entries);
    };
    auto pending = [&](uint32_t count, const uint32_t *cnt_dev, uint64_t &pend) {
        uint32_t c = 0;
        return read_pending(h0, G, count, cnt_dev, h0->sc.chain_all, pend, c);
    };
    uint64_t pend = 0;
    if (group_batch_ok(hs, nh) && G == nh) {
        if ((rc = group_steps(hs, nh, ini, res, n, tick))) return rc;
    } else {
        if ((rc = fork_slices(hs, nh))) return rc;
        for (uint32_t i = 0; i < nh && !rc; i++) rc = gs_phase_count(hs[i], ini, res, n, tick, hs[i]->sc.tot);
        if ((rc = join_slices(hs, nh, rc))) return rc;
        if ((rc = gather_u64(hs, nh, [](gs_handle *h) { return h->sc.tot; }, [](gs_handle *h) { return h->sc.tot_all; },
                             (size_t)2 * n)))
            return rc;
        if ((rc = fork_slices(hs, nh))) return rc;
        for (uint32_t i = 0; i < nh && !rc; i++) {
            rc = gs_phase_pack(hs[i], ini, res, n, tick, 0, hs[i]->sc.tot_all, nullptr, hs[i]->sc.chain);
            // the overflowing slots, listed on the device (the same list on every slice)
            if (!rc) rc = gs_phase_overflow(hs[i], n, hs[i]->sc.tot_all, hs[i]->sc.chain, hs[i]->sc.list, hs[i]->sc.chainc, nullptr);
        }
        if ((rc = join_slices(hs, nh, rc))) return rc;
        if (G < 2) return GS_OK;  // one slice: step 0 finished every slot
        // step 1 before any host read, on the device count (a chain usually resolves in it: one read ends the phase)
        if ((rc = gather_chain(GS_CHAIN_CAP + 1u)) || (rc = fork_slices(hs, nh))) return rc;
        for (uint32_t i = 0; i < nh && !rc; i++)
            rc = gs_phase_chain(hs[i], ini, res, n, tick, 1, hs[i]->sc.list, GS_CHAIN_DEVICE, hs[i]->sc.chain_all,
                                hs[i]->sc.chain, hs[i]->sc.chainc, hs[i]->sc.tot_all);
        if ((rc = join_slices(hs, nh, rc))) return rc;
    }
    if ((rc = gather_chain(GS_CHAIN_CAP + 1u)) || (rc = pending(0u, cnt0, pend))) return rc;
    if (!pend) return GS_OK;
    // still pending (or more slots than the device step takes): the count to the host, the remaining steps
    uint32_t count = 0;
    HIPCHK(h0, hipMemcpyAsync(&count, cnt0, 4, hipMemcpyDeviceToHost, h0->stream));
    HIPCHK(h0, hipStreamSynchronize(h0->stream));
    for (uint32_t step = count > GS_CHAIN_CAP ? 1u : 2u; step < G; step++) {
        // every slice's chain states and pending count (entry count); the same data on every slice, so each
        // reads the same sum and all stop together
        if ((rc = gather_chain((size_t)count + 1)) || (rc = pending(count, nullptr, pend))) return rc;
        if (!pend) break;
        if ((rc = fork_slices(hs, nh))) return rc;
        for (uint32_t i = 0; i < nh && !rc; i++)
            rc = gs_phase_chain(hs[i], ini, res, n, tick, step, hs[i]->sc.list, count, hs[i]->sc.chain_all,
                                hs[i]->sc.chain, hs[i]->sc.chainc, hs[i]->sc.tot_all);
        if ((rc = join_slices(hs, nh, rc))) return rc;
    }
    return GS_OK;
}
}  // namespace
}

int gs_phase_pending(gs_handle *h, uint32_t n, const uint32_t *list, uint32_t count, const uint64_t *chain_all,
                     uint64_t *pending, uint32_t *count_out) {
    if (!h || !h->booted || !chain_all || !pending || !count_out) return GS_E_INVALID;
    if (!h->sliced) return fail(h, GS_E_UNSUPPORTED, "gs_phase_pending needs a sliced handle");
    const bool dev = count == GS_CHAIN_DEVICE;
    if (dev && (!list || !n)) return GS_E_INVALID;
    const uint32_t *cnt_dev = dev ? list + 2u * n + (2u * n + OVB - 1u) / OVB : nullptr;  // gs_phase_overflow's count
    return read_pending(h, h->G, dev ? 0u : count, cnt_dev, chain_all, *pending, *count_out);
}

int gs_comm_id(void *id) {
    if (!id) return GS_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return GS_E_HIP;
    static_assert(sizeof u == GS_COMM_ID_BYTES, "ncclUniqueId size");
    memcpy(id, &u, sizeof u);
    return GS_OK;
}

int gs_comm_init(gs_handle *h, const void *id, uint32_t nranks, uint32_t rank) {
    if (!h || !id) return GS_E_INVALID;
    if (h->comm) return fail(h, GS_E_INVALID, "gs_comm_init: this handle already has a communicator");
    if (nranks != h->G || rank != h->shard)
        return fail(h, GS_E_INVALID, "gs_comm_init: %u ranks / rank %u for slice %u of %u", nranks, rank, h->shard, h->G);
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    const ncclResult_t r = ncclCommInitRank(&h->comm, (int)nranks, u, (int)rank);
    if (r != ncclSuccess) {
        h->comm = nullptr;
        return fail(h, GS_E_HIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    return GS_OK;
}

int gs_run_phase_group(gs_handle *const *hs, uint32_t n_handles, const int32_t *ini, const int32_t *res, uint32_t n,
                       uint32_t tick) {
    if (!hs || !n_handles || !hs[0]) return GS_E_INVALID;
    gs_handle *h0 = hs[0];
    // every slice of the cluster, or slice 0 held alone (a rehearsal of one GPU's share: the others gather as
    // zeros).  Slice 0 is exact alone whatever the mtu: the packer walks owners in slice order, so slice 0's
    // NodeDeltas start every delta and never depend on the other slices' totals.  Any other slice held alone would
    // pack from a zero predecessor total, silently wrong once the mtu binds, so it is refused.
    if (n_handles != h0->G && n_handles != 1)
        return fail(h0, GS_E_INVALID, "gs_run_phase_group: %u handles for %u slices", n_handles, h0->G);
    if (n_handles == 1 && h0->comm) return gs_run_phase(h0, ini, res, n, tick);
    if (n_handles == 1 && h0->G > 1 && h0->shard != 0)
        return fail(h0, GS_E_UNSUPPORTED, "gs_run_phase_group: slice %u held alone packs from its predecessors' "
                    "totals, which only a communicator or the whole group provides (slice 0 alone is exact)", h0->shard);
    for (uint32_t i = 0; i < n_handles && n_handles > 1; i++) {
        if (!hs[i] || hs[i]->shard != i || hs[i]->G != h0->G || hs[i]->N != h0->N || hs[i]->stream != h0->stream)
            return fail(h0, GS_E_INVALID, "gs_run_phase_group: handle %u is not slice %u of this cluster on one stream", i, i);
    }
    if (!h0->sliced) return gs_run_phase(h0, ini, res, n, tick);
    if (!n) return check_phase(h0, ini, res, n, tick);
    return sliced_phase(hs, n_handles, ini, res, n, tick);
}

extern "C++" {
namespace {
// Invariant: after a sweep at tick A every unmarked window's report is less than 2^15 ticks older than A,
// so decodes are exact at every tick below A + 2^15.  An operation at t sweeps once t - A reaches 2^14;
// when t - A is 2^15 or more it first sweeps at the previous operation's tick (less than 2^14 after A, so
// exact there), which leaves t - A = the step from that operation.  Only a step of 2^15 or more between
// two consecutive operations is refused, and a refused tick changes nothing (a later, smaller step works).
int age_sweep(gs_handle *h, uint32_t tick) {
    const uint64_t quads = (uint64_t)h->N * h->NP / 4;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((quads + LB - 1) / LB, 1u << 16);
    k_fd_age<<<blocks, LB, 0, h->stream>>>(h->d, tick);
    HIPCHK(h, hipGetLastError());
    h->age_tick = tick;
    return GS_OK;
}
int fd_age(gs_handle *h, uint32_t tick) {
    if (!h->age_init) {  // no window exists before the first operation: start the clock there
        h->age_init = true;
        h->age_tick = h->max_tick = tick;
        return GS_OK;
    }
    if ((int32_t)(tick - h->max_tick) < 0) return GS_OK;  // an earlier tick (phi of the past): nothing aged
    const uint32_t step = tick - h->max_tick;
    if (step >= FD_OLD_AGE)
        return fail(h, GS_E_INVALID, "tick %u is %u ticks after the previous operation (at most 2^15 - 1 between "
                    "operations: 16-bit report ticks)", tick, step);
    if (tick - h->age_tick >= FD_OLD_AGE) {
        if (int rc = age_sweep(h, h->max_tick)) return rc;
    }
    h->max_tick = tick;
    if (tick - h->age_tick >= (FD_OLD_AGE >> 1)) return age_sweep(h, tick);
    return GS_OK;
}
}  // namespace
}

int gs_liveness(gs_handle *h, const uint8_t *up, uint32_t tick) {
    if (!h || !h->booted || !up) return GS_E_INVALID;
    if (int rc = fd_age(h, tick)) return rc;
    if (h->reports_pending && tick < h->last_phase_tick)
        return fail(h, GS_E_INVALID, "gs_liveness at tick %u precedes a phase at tick %u", tick, h->last_phase_tick);
    k_reset_sched<<<(h->N + LB - 1) / LB, LB, 0, h->stream>>>(h->d, up, tick);
    HIPCHK(h, hipGetLastError());
    int rc = launch_liveness(h, up, tick, h->reports_pending, true);
    if (rc) return rc;
    h->reports_pending = false;  // replayed
    h->round_open = false;
    if (!(h->cfg.flags & GS_CANONICAL)) {
        k_fd_gc<<<h->N, LB, (h->NP / 32) * 4, h->stream>>>(h->d, up, tick);
        HIPCHK(h, hipGetLastError());
    }
    return GS_OK;
}

int gs_flush_reports(gs_handle *h, uint32_t tick) {
    if (!h || !h->booted) return GS_E_INVALID;
    if (!h->round_open) return fail(h, GS_E_INVALID, "gs_flush_reports: no open round");
    if (tick < h->last_phase_tick)
        return fail(h, GS_E_INVALID, "gs_flush_reports at tick %u precedes a phase at tick %u", tick, h->last_phase_tick);
    if (int rc = fd_age(h, tick)) return rc;
    if (h->reports_pending) {
        if (int rc = launch_liveness(h, nullptr, tick, true, false)) return rc;
        h->reports_pending = false;
    }
    h->d.t_round = tick;  // the next phase (after tick) starts a new plane base
    h->base_fresh = true;
    h->sub_ok = false;
    h->last_phase_tick = tick;
    return GS_OK;
}

int gs_read_rows(gs_handle *h, int region, uint32_t row_lo, uint32_t row_hi, void *out, uint64_t cap, uint64_t *len) {
    static const int rows_major[] = {GS_R_HB, GS_R_MV, GS_R_GC, GS_R_HELD, GS_R_FD, GS_R_FD_LAST, GS_R_FD_STATE,
                                     GS_R_FD_TOD, GS_R_TS, GS_R_RING, GS_R_POS, GS_R_ORD, GS_R_ROW, GS_R_ESC16};
    if (!h || !h->booted || !out || !len || row_lo > row_hi || row_hi > h->N) return GS_E_INVALID;
    if (std::find(std::begin(rows_major), std::end(rows_major), region) == std::end(rows_major))
        return fail(h, GS_E_INVALID, "gs_read_rows: region %d is not indexed by observer row", region);
    if (!h->bytes[region]) return fail(h, GS_E_UNSUPPORTED, "gs_read_rows: region %d is not allocated", region);
    if (region == GS_R_RING && h->cfg.ring_rows)
        return fail(h, GS_E_UNSUPPORTED, "gs_read_rows: sampled rings are indexed by ring slot, not observer row");
    const uint64_t rb = h->bytes[region] / h->N, nb = rb * (row_hi - row_lo);
    *len = nb;
    if (nb > cap) return fail(h, GS_E_INVALID, "gs_read_rows: %llu bytes > capacity %llu", (unsigned long long)nb,
                              (unsigned long long)cap);
    if (region == GS_R_HELD) {  // prefix views do not keep their held ordinals: derive them first
        int rc = gs_materialize_held(h, row_lo, row_hi);
        if (rc) return rc;
    }
    HIPCHK(h, hipMemcpyAsync(out, (const uint8_t *)h->reg[region] + rb * row_lo, nb, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return GS_OK;
}

int gs_latest_tick(const gs_handle *h, uint32_t *tick) {
    if (!h || !tick) return GS_E_INVALID;
    *tick = h->max_tick;
    return GS_OK;
}

int gs_phi_row(gs_handle *h, uint32_t observer, uint32_t tick, double *out) {
    if (!h || !h->booted || !out || observer >= h->N) return GS_E_INVALID;
    if (int rc = fd_age(h, tick)) return rc;
    k_phi_row<<<(h->ncol + LB - 1) / LB, LB, 0, h->stream>>>(h->d, observer, tick, out);
    HIPCHK(h, hipGetLastError());
    return GS_OK;
}

// ---- wire-format emitter (blocking)
extern "C++" {
namespace {
struct EmitScratch {
    uint64_t *sz, *off;
    uint2 *rec;
    uint32_t *nrec;
};
EmitScratch emit_scratch(const gs_handle *h, void *scratch) {
    uint8_t *b = (uint8_t *)scratch;
    const uint64_t NP = h->NP;
    EmitScratch e;
    e.sz = (uint64_t *)b;
    e.off = (uint64_t *)(b + NP * 8);
    e.rec = (uint2 *)(b + NP * 16 + 64);
    e.nrec = (uint32_t *)(b + NP * 24 + 64);
    return e;
}
Wire to_wire(const gs_wire *w) {
    return Wire{w->node_ids, w->node_id_off, w->keys, w->key_off, w->values, w->value_off};
}
int emit_check(gs_handle *h, const gs_wire *w, uint8_t *out, uint64_t *len, void *scratch) {
    if (!h || !h->booted || !w || !len || !scratch || !w->node_ids || !w->node_id_off || !w->keys || !w->key_off)
        return GS_E_INVALID;
    if (h->G > 1) return fail(h, GS_E_UNSUPPORTED, "the wire emitter needs the whole matrix (one slice)");
    (void)out;
    return GS_OK;
}
// copy the total back, check the capacity, then write
int emit_finish(gs_handle *h, const uint64_t *off_total, uint64_t cap, uint64_t *len, uint8_t *out, bool &go) {
    uint64_t total = 0;
    HIPCHK(h, hipMemcpyAsync(&total, off_total, 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    *len = total;
    go = total > 0 && total <= cap && out != nullptr;
    if (total > cap) return fail(h, GS_E_INVALID, "output buffer of %llu bytes < %llu needed",
                                 (unsigned long long)cap, (unsigned long long)total);
    return GS_OK;
}
template <int KW, bool GENM>
int emit_delta(gs_handle *h, const Wire &w, uint32_t s, uint32_t r, uint32_t t, uint8_t *out, uint64_t cap,
               uint64_t *len, const EmitScratch &e) {
    hipStream_t st = h->stream;
    const size_t lds = WIN * 2 + (size_t)(h->NP / 32) * 4;
    HIPCHK(h, hipMemsetAsync(e.nrec, 0, 4, st));
    k_delta_plan<KW, GENM><<<1, WAVE, lds, st>>>(h->d, s, r, t, e.rec, e.nrec);
    HIPCHK(h, hipGetLastError());
    uint32_t n = 0;
    HIPCHK(h, hipMemcpyAsync(&n, e.nrec, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (n > h->ncol) return fail(h, GS_E_DEVICE, "delta plan recorded %u NodeDeltas", n);
    if (n == 0) { *len = 0; return GS_OK; }
    const uint32_t nb = (n + LB - 1) / LB;
    k_delta_size<KW, GENM><<<nb, LB, 0, st>>>(h->d, s, r, t, e.rec, n, e.sz);
    k_scan_sizes<<<1, 1024, 0, st>>>(e.sz, n, e.off);
    HIPCHK(h, hipGetLastError());
    bool go = false;
    int rc = emit_finish(h, e.off + n, cap, len, out, go);
    if (rc || !go) return rc;
    k_delta_write<KW, GENM><<<nb, LB, 0, st>>>(h->d, w, s, r, t, e.rec, n, e.off, out);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(st));
    return GS_OK;
}
}  // namespace
}  // extern "C++"

int gs_emit_scratch_bytes(const gs_handle *h, uint64_t *bytes) {
    if (!h || !bytes) return GS_E_INVALID;
    *bytes = (uint64_t)h->NP * 24 + 128;
    return GS_OK;
}

int gs_emit_digest(gs_handle *h, const gs_wire *w, uint32_t observer, uint32_t tick, uint8_t *out, uint64_t cap,
                   uint64_t *len, void *scratch) {
    int rc = emit_check(h, w, out, len, scratch);
    if (rc) return rc;
    if (observer >= h->N) return GS_E_INVALID;
    const EmitScratch e = emit_scratch(h, scratch);
    const Wire wr = to_wire(w);
    uint32_t row[4];
    HIPCHK(h, hipMemcpyAsync(row, h->d.row + observer * 4, 16, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const uint32_t cnt = (h->cfg.flags & GS_CANONICAL) ? h->ncol : row[0];
    const bool sch = tick >= row[2];
    if (cnt == 0) { *len = 0; return GS_OK; }
    const uint32_t nb = (cnt + LB - 1) / LB;
    k_digest_size<<<nb, LB, 0, h->stream>>>(h->d, wr, observer, tick, sch, cnt, e.sz);
    k_scan_sizes<<<1, 1024, 0, h->stream>>>(e.sz, cnt, e.off);
    HIPCHK(h, hipGetLastError());
    bool go = false;
    rc = emit_finish(h, e.off + cnt, cap, len, out, go);
    if (rc || !go) return rc;
    k_digest_write<<<nb, LB, 0, h->stream>>>(h->d, wr, observer, tick, sch, cnt, e.off, out);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return GS_OK;
}

int gs_emit_delta(gs_handle *h, const gs_wire *w, uint32_t sender, uint32_t receiver, uint32_t tick, uint8_t *out,
                  uint64_t cap, uint64_t *len, void *scratch) {
    int rc = emit_check(h, w, out, len, scratch);
    if (rc) return rc;
    if (sender >= h->N || receiver >= h->N || sender == receiver) return GS_E_INVALID;
    if (!w->values || !w->value_off) return GS_E_INVALID;
    const EmitScratch e = emit_scratch(h, scratch);
    const Wire wr = to_wire(w);
    const bool genm = !(h->cfg.flags & GS_CANONICAL);
    if (h->KP <= 16)
        return genm ? emit_delta<4, true>(h, wr, sender, receiver, tick, out, cap, len, e)
                    : emit_delta<4, false>(h, wr, sender, receiver, tick, out, cap, len, e);
    return genm ? emit_delta<KWB, true>(h, wr, sender, receiver, tick, out, cap, len, e)
                : emit_delta<KWB, false>(h, wr, sender, receiver, tick, out, cap, len, e);
}

int gs_read_counters(gs_handle *h, gs_counters *out) {
    if (!h || !out || !h->reg[GS_R_COUNTERS]) return GS_E_INVALID;
    std::vector<unsigned long long> buf((size_t)NSHARD * CROW);
    HIPCHK(h, hipMemcpyAsync(buf.data(), h->reg[GS_R_COUNTERS], buf.size() * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    uint64_t acc[CFIELDS] = {0};  // the gs_counters fields (the census scratch follows them in each row)
    for (int s = 0; s < NSHARD; s++)
        for (int c = 0; c < CFIELDS; c++) {
            const uint64_t v = buf[(size_t)s * CROW + c];
            if (c == C_PGMAX || c == C_PSMAX) acc[c] = std::max<uint64_t>(acc[c], v);  // maxima, not sums
            else acc[c] += v;
        }
    acc[C_FLUSH] = h->plane_flushes;
    acc[C_SWEEPS] = h->lag_sweeps;
    memcpy(out, acc, sizeof acc);
    return GS_OK;
}

int gs_set_timing(gs_handle *h, int on) {
    if (!h) return GS_E_INVALID;
    h->timing = on != 0;
    return GS_OK;
}

int gs_kernel_times(gs_handle *h, gs_ktimes *out) {
    if (!h || !out) return GS_E_INVALID;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    memset(out, 0, sizeof *out);
    for (int k = 0; k < GS_KT_KINDS; k++) {
        for (auto &pr : h->tev[k]) {
            float ms = 0.f;
            HIPCHK(h, hipEventElapsedTime(&ms, pr.first, pr.second));
            out->ms[k] += ms;
            out->launches[k]++;
            h->evpool.push_back(pr.first);
            h->evpool.push_back(pr.second);
        }
        h->tev[k].clear();
    }
    return GS_OK;
}

int gs_reset_counters(gs_handle *h) {
    if (!h || !h->reg[GS_R_COUNTERS]) return GS_E_INVALID;
    HIPCHK(h, hipMemsetAsync(h->reg[GS_R_COUNTERS], 0, h->bytes[GS_R_COUNTERS], h->stream));
    h->plane_flushes = 0;
    h->lag_sweeps = 0;
    return GS_OK;
}

int gs_set_events(gs_handle *h, uint32_t *records, uint32_t capacity, uint32_t *count) {
    if (!h || (records && !count)) return GS_E_INVALID;
    h->d.ev = records;
    h->d.ev_count = records ? count : nullptr;
    h->d.ev_cap = records ? capacity : 0u;
    h->d.ev_wseq = 0u;
    return GS_OK;
}

int gs_select_peers(gs_handle *h, const uint8_t *up, uint32_t fanout, const int32_t *seeds, uint32_t n_seeds,
                    uint64_t seed, uint32_t round, int32_t *targets, void *scratch) {
    if (!h || !h->booted || !up || !targets || !scratch || fanout < 1 || fanout > 8 || (n_seeds && !seeds))
        return GS_E_INVALID;
    if (h->G > 1) return fail(h, GS_E_UNSUPPORTED, "gs_select_peers needs the whole matrix (one slice)");
    uint32_t *scnt = (uint32_t *)scratch;
    uint32_t *sel = scnt + (size_t)h->N * 4;
    const bool canon = (h->cfg.flags & GS_CANONICAL) != 0;
    if (canon && h->ncol <= SEL_ROW_IT * LB * 16u && !getenv("GS_SEL_SPLIT")) {  // one read of each row
        k_sel_row16<<<h->N, LB, 0, h->stream>>>(h->d, up, fanout, seed, round, seeds, n_seeds, scnt, targets);
        HIPCHK(h, hipGetLastError());
        return GS_OK;
    }
    if (canon) k_sel_count16<<<h->N, LB, 0, h->stream>>>(h->d, up, scnt);
    else k_sel_count<<<h->N, LB, 0, h->stream>>>(h->d, up, scnt);
    HIPCHK(h, hipGetLastError());
    k_sel_pick<<<(h->N + LB - 1) / LB, LB, 0, h->stream>>>(h->d, up, scnt, fanout, seed, round, sel);
    HIPCHK(h, hipGetLastError());
    if (canon) k_sel_resolve16<<<h->N, LB, 0, h->stream>>>(h->d, up, scnt, fanout, seed, round, seeds, n_seeds, sel, targets);
    else k_sel_resolve<<<h->N, LB, 0, h->stream>>>(h->d, up, scnt, fanout, seed, round, seeds, n_seeds, sel, targets);
    HIPCHK(h, hipGetLastError());
    return GS_OK;
}

int gs_schedule_phases(gs_handle *h, const uint8_t *up, uint32_t fanout, const int32_t *targets, uint64_t seed,
                       uint32_t round, uint32_t iters, uint32_t max_phases, void *scratch, int32_t *initiators,
                       int32_t *responders, uint32_t *phase_offsets, uint32_t *unscheduled) {
    if (!h || !up || !targets || !scratch || !initiators || !responders || !phase_offsets || !unscheduled ||
        fanout < 1 || fanout > 8 || iters < 1 || max_phases < 1 || max_phases > GS_MAX_SCHED_PHASES)
        return GS_E_INVALID;
    const uint32_t N = h->N, E = N * (fanout + 2);
    // scratch (GS_SCHED_SCRATCH_BYTES): eph[E] | pcount[P] | pfill[P] | poff[P] | left[4] | busy[N] (u64) |
    // best[2][N] (u64)
    const uint32_t P = max_phases;
    uint32_t *eph = (uint32_t *)scratch;
    uint32_t *pcount = eph + E;
    uint32_t *pfill = pcount + P;
    uint32_t *poff = pfill + P;
    uint32_t *left = poff + P;
    unsigned long long *busy = (unsigned long long *)(((uintptr_t)(left + 4) + 15) & ~(uintptr_t)15);
    unsigned long long *best = busy + N;
    hipStream_t s = h->stream;
    HIPCHK(h, hipMemsetAsync(eph, 0xFF, (size_t)E * 4, s));
    HIPCHK(h, hipMemsetAsync(pcount, 0, ((size_t)3 * P + 4) * 4, s));
    HIPCHK(h, hipMemsetAsync(busy, 0, (size_t)N * 8, s));
    HIPCHK(h, hipMemsetAsync(best, 0xFF, (size_t)N * 16, s));
    const uint32_t gE = (std::max(E, N) + LB - 1) / LB;
    // the two minimum buffers alternate by the GLOBAL iteration index, so each pick resets exactly
    // the buffer the next iteration (of this phase or the next) reduces into, whatever iters is
    uint32_t g = 0, nleft = 0;
    // phases in blocks: 16 first (a round's schedule needs about 15-17 at fanout 3), then 4 at a time (the last few
    // exchanges), each block followed by one count of the exchanges still without a phase
    for (uint32_t p0 = 0, p1; p0 < max_phases; p0 = p1) {
        p1 = std::min(max_phases, p0 + (p0 ? 4u : 16u));
        // busy holds bit p mod 64: a block starting a new window of 64 phases starts from clear bits (blocks are
        // 16 then 4 phases, so windows start at block boundaries)
        if (p0 && (p0 & 63u) == 0) HIPCHK(h, hipMemsetAsync(busy, 0, (size_t)N * 8, s));
        for (uint32_t p = p0; p < p1; p++)
            for (uint32_t it = 0; it < iters; it++, g++) {
                unsigned long long *b0 = best + (size_t)(g & 1) * N, *b1 = best + (size_t)((g + 1) & 1) * N;
                k_luby_min<<<(E + LB - 1) / LB, LB, 0, s>>>(targets, up, eph, busy, b0, E, fanout, seed, round, p,
                                                            it);
                k_luby_pick<<<gE, LB, 0, s>>>(targets, up, eph, busy, b0, b1, E, N, fanout, seed, round, p, it,
                                              pcount);
            }
        // stop once every valid exchange has a phase
        HIPCHK(h, hipMemsetAsync(left, 0, 4, s));
        k_luby_left<<<(E + LB - 1) / LB, LB, 0, s>>>(targets, up, eph, E, fanout, left);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipMemcpyAsync(&nleft, left, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(h, hipStreamSynchronize(s));
        if (!nleft) break;
    }
    std::vector<uint32_t> cnt(max_phases);
    HIPCHK(h, hipMemcpyAsync(cnt.data(), pcount, (size_t)max_phases * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(h, hipStreamSynchronize(s));
    std::vector<uint32_t> off(max_phases + 1);
    off[0] = 0;
    for (uint32_t p = 0; p < max_phases; p++) off[p + 1] = off[p] + cnt[p];
    HIPCHK(h, hipMemcpyAsync(poff, off.data(), max_phases * 4, hipMemcpyHostToDevice, s));
    k_luby_scatter<<<(E + SCAT_PER * LB - 1) / (SCAT_PER * LB), LB, 0, s>>>(targets, eph, E, fanout, poff, pfill,
                                                                        initiators, responders);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(s));
    memcpy(phase_offsets, off.data(), (max_phases + 1) * 4);
    *unscheduled = nleft;
    return GS_OK;
}

int gs_fd_census(gs_handle *h, const uint8_t *up, gs_census *out) {
    if (!h || !h->booted || !up || !out) return GS_E_INVALID;
    k_zero_slots<<<1, NSHARD * 8, 0, h->stream>>>(h->d, C_CEN0, 5);
    HIPCHK(h, hipGetLastError());
    dim3 grid((h->ncol + LB - 1) / LB, h->N);
    k_fd_census<<<grid, LB, 0, h->stream>>>(h->d, up);
    HIPCHK(h, hipGetLastError());
    std::vector<unsigned long long> buf((size_t)NSHARD * CROW);
    HIPCHK(h, hipMemcpyAsync(buf.data(), h->reg[GS_R_COUNTERS], buf.size() * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    uint64_t acc[5] = {0, 0, 0, 0, 0};
    for (int sh = 0; sh < NSHARD; sh++)
        for (int i = 0; i < 5; i++) acc[i] += buf[(size_t)sh * CROW + C_CEN0 + i];
    out->up_pairs = acc[0];
    out->up_dead = acc[1];
    out->up_live = acc[2];
    out->down_pairs = acc[3];
    out->down_live = acc[4];
    return GS_OK;
}

int gs_stream_copy(void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!dst || !src || (bytes & 15u) || ((uintptr_t)dst & 15u) || ((uintptr_t)src & 15u)) return GS_E_INVALID;
    k_copy16<<<65536, 256, 0, (hipStream_t)stream>>>((v4u_t *)dst, (const v4u_t *)src, bytes / 16);
    return hipGetLastError() == hipSuccess ? GS_OK : GS_E_HIP;
}

int gs_stream_write(void *dst, uint64_t bytes, uint32_t width, void *stream) {
    if (!dst || (width != 4 && width != 8 && width != 16) || (bytes % width) || ((uintptr_t)dst & 15u))
        return GS_E_INVALID;
    if (width == 4)
        k_write<uint32_t><<<32768, 256, 0, (hipStream_t)stream>>>((uint32_t *)dst, bytes / 4);
    else if (width == 8)
        k_write<uint2><<<32768, 256, 0, (hipStream_t)stream>>>((uint2 *)dst, bytes / 8);
    else
        k_write<uint4><<<32768, 256, 0, (hipStream_t)stream>>>((uint4 *)dst, bytes / 16);
    return hipGetLastError() == hipSuccess ? GS_OK : GS_E_HIP;
}

int gs_stream_read(const void *src, uint64_t bytes, uint32_t width, uint64_t *sink, void *stream) {
    if (!src || !sink || (width != 4 && width != 8 && width != 16) || (bytes % width) || ((uintptr_t)src & 15u))
        return GS_E_INVALID;
    if (width == 4)
        k_read<uint32_t><<<32768, 256, 0, (hipStream_t)stream>>>((const uint32_t *)src, bytes / 4,
                                                                 (unsigned long long *)sink);
    else if (width == 8)
        k_read<uint2><<<32768, 256, 0, (hipStream_t)stream>>>((const uint2 *)src, bytes / 8,
                                                              (unsigned long long *)sink);
    else
        k_read<uint4><<<32768, 256, 0, (hipStream_t)stream>>>((const uint4 *)src, bytes / 16,
                                                              (unsigned long long *)sink);
    return hipGetLastError() == hipSuccess ? GS_OK : GS_E_HIP;
}

int gs_mark(uint32_t which, void *stream) {
    if (which > 1) return GS_E_INVALID;
    if (which == 0)
        k_mark_begin<<<1, WAVE, 0, (hipStream_t)stream>>>();
    else
        k_mark_end<<<1, WAVE, 0, (hipStream_t)stream>>>();
    return hipGetLastError() == hipSuccess ? GS_OK : GS_E_HIP;
}

int gs_sync(gs_handle *h) {
    if (!h) return GS_E_INVALID;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return GS_OK;
}

}  // extern "C"
