/*
 * gossip_oracle.c -- CPU restatement of aiocluster's anti-entropy + phi failure
 * detector.  TEST INFRASTRUCTURE (see gossip_oracle.h): the checker, never the
 * product.  Every function cites the reference lines it restates.
 *
 * Data structures deliberately mirror the Python objects rather than the
 * device layout: each observer owns an insertion-ordered "dict" of views
 * (order[]/pos[]), each view a per-key slot table of VersionedValue, and a
 * FailureDetector with per-target SamplingWindow rings of doubles.
 */
#include "gossip_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { ST_SET = 0, ST_DELETED = 1, ST_DELETE_AFTER_TTL = 2 };

typedef struct okv {          /* VersionedValue (entities.py:38-43) */
    uint8_t present;
    uint8_t status;
    int32_t value_len;
    uint32_t value_id;
    uint32_t version;
    int64_t ts;               /* status_change_ts, us */
} okv;

typedef struct oview {        /* NodeState (state.py:106-113) */
    uint32_t hb, mv, gc;
} oview;

typedef struct owin {         /* SamplingWindow (failure_detector.py:12-53) */
    int32_t has;              /* present in FailureDetector._node_samples */
    int32_t has_last;
    int64_t last;             /* _last_heartbeat, us */
    /* BoundedArrayStats (failure_detector.py:131-162) */
    double sum;
    int32_t idx;
    int32_t filled;
    int32_t cap_alloc;
    double *vals;
} owin;

typedef struct oobs {
    int32_t alloc;
    /* ClusterState._node_states: insertion-ordered dict */
    int32_t *order;
    int32_t cnt;
    int32_t *pos;             /* -1 when absent */
    oview *v;
    okv *kv;                  /* [N * K] */
    /* FailureDetector */
    owin *w;
    uint8_t *live;            /* _live_nodes (a set: membership only) */
    int32_t *dead_order;      /* _dead_nodes: insertion-ordered dict */
    int32_t ndead;
    int64_t *tod;             /* time of death, valid when dead_pos >= 0 */
    int32_t *dead_pos;
    struct oobs *snap;        /* orc_snapshot_row copy */
} oobs;

typedef struct ond {          /* NodeDelta (state.py:66-72) */
    int32_t node;
    uint32_t from, gc, mv;
    int32_t kv0, nkv;
} ond;

typedef struct okvu {         /* KeyValueUpdate (state.py:22-27) */
    int32_t key;
    uint32_t value_id;
    int32_t value_len;
    uint32_t version;
    int32_t status;
} okvu;

typedef struct odelta {
    ond *nd;
    int32_t nnd, cap_nd;
    okvu *kv;
    int32_t nkv, cap_kv;
} odelta;

typedef struct odigest {      /* Digest (state.py:42-63): dict keyed by node */
    uint8_t *has;
    uint32_t *hb, *gc, *mv;
    int32_t *list;            /* iteration order */
    int32_t n;
} odigest;

struct orc {
    orc_config c;
    int32_t N, K;
    int32_t *nid_size;
    int32_t *key_len;
    oobs *obs;
    double prior_s;
    odigest dg[2];
    odelta dl[2];
    uint8_t *sched[2];
    int32_t *tmp_stale;
    uint32_t *tmp_from;
    int32_t *tmp_keys;
    orc_stats st;
    /* hook events (server.py:217-257): {observer, owner, key | kind << 8, old version, new version, now} */
    int32_t ev_on, ev_n, ev_cap;
    int64_t *ev;
};

static void emit(orc *o, int32_t obs, int32_t owner, int32_t kk, uint32_t v_old, uint32_t v_new, int64_t now) {
    if (!o->ev_on) return;
    if (o->ev_n == o->ev_cap) {
        o->ev_cap = o->ev_cap ? 2 * o->ev_cap : 1024;
        o->ev = realloc(o->ev, sizeof(int64_t) * 6 * (size_t)o->ev_cap);
        if (!o->ev) abort();
    }
    int64_t *r = o->ev + (size_t)o->ev_n * 6;
    r[0] = obs; r[1] = owner; r[2] = kk; r[3] = v_old; r[4] = v_new; r[5] = now;
    o->ev_n++;
}

void orc_enable_events(orc *o, int32_t on) { o->ev_on = on; o->ev_n = 0; }
int32_t orc_drain_events(orc *o, int64_t *out, int32_t cap) {
    int32_t n = o->ev_n;
    if (out) memcpy(out, o->ev, sizeof(int64_t) * 6 * (size_t)(n < cap ? n : cap));
    o->ev_n = 0;
    return n;
}

/* ------------------------------------------------------------ pb sizes */
static int vlen(uint64_t x) { int n = 1; while (x >= 0x80) { x >>= 7; n++; } return n; }
static int s_field(int64_t nbytes) { return nbytes == 0 ? 0 : 1 + vlen((uint64_t)nbytes) + (int)nbytes; }
static int u_field(uint64_t x) { return x == 0 ? 0 : 1 + vlen(x); }
static int msg_field(int64_t len) { return 1 + vlen((uint64_t)len) + (int)len; }

/* KeyValueUpdatePb body (messages.proto:53-58) */
static int kv_size(const orc *o, int key, int value_len, uint32_t version, int status) {
    return s_field(o->key_len[key]) + s_field(value_len) + u_field(version) + u_field((uint64_t)status);
}

/* -------------------------------------------------------------- helpers */
static void *xcalloc(size_t n, size_t s) {
    void *p = calloc(n ? n : 1, s ? s : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}

static oobs *row(orc *o, int32_t i) {
    oobs *b = &o->obs[i];
    if (!b->alloc) {
        int32_t N = o->N;
        b->alloc = 1;
        b->order = xcalloc(N, sizeof(int32_t));
        b->pos = xcalloc(N, sizeof(int32_t));
        b->v = xcalloc(N, sizeof(oview));
        b->kv = xcalloc((size_t)N * o->K, sizeof(okv));
        b->w = xcalloc(N, sizeof(owin));
        b->live = xcalloc(N, 1);
        b->dead_order = xcalloc(N, sizeof(int32_t));
        b->tod = xcalloc(N, sizeof(int64_t));
        b->dead_pos = xcalloc(N, sizeof(int32_t));
        for (int32_t j = 0; j < N; j++) { b->pos[j] = -1; b->dead_pos[j] = -1; }
    }
    return b;
}

static okv *kvp(orc *o, oobs *b, int32_t j) { return &b->kv[(size_t)j * o->K]; }

/* ClusterState.node_state_or_default (state.py:298-299) */
static void insert_node(orc *o, oobs *b, int32_t j) {
    if (b->pos[j] >= 0) return;
    b->pos[j] = b->cnt;
    b->order[b->cnt++] = j;
    b->v[j].hb = b->v[j].mv = b->v[j].gc = 0;
    memset(kvp(o, b, j), 0, sizeof(okv) * o->K);
}

/* ClusterState.remove_node (state.py:307-308) */
static void remove_node(orc *o, oobs *b, int32_t j) {
    int32_t p = b->pos[j];
    if (p < 0) return;
    memmove(&b->order[p], &b->order[p + 1], sizeof(int32_t) * (b->cnt - p - 1));
    b->cnt--;
    for (int32_t q = p; q < b->cnt; q++) b->pos[b->order[q]] = q;
    b->pos[j] = -1;
    b->v[j].hb = b->v[j].mv = b->v[j].gc = 0;
    memset(kvp(o, b, j), 0, sizeof(okv) * o->K);
}

/* --------------------------------------------------------- public: setup */
orc *orc_create(const orc_config *cfg, const int32_t *nid_size, const int32_t *key_len) {
    orc *o = xcalloc(1, sizeof(orc));
    o->c = *cfg;
    o->N = cfg->n_nodes;
    o->K = cfg->n_keys;
    o->nid_size = xcalloc(o->N, sizeof(int32_t));
    memcpy(o->nid_size, nid_size, sizeof(int32_t) * o->N);
    o->key_len = xcalloc(o->K, sizeof(int32_t));
    memcpy(o->key_len, key_len, sizeof(int32_t) * o->K);
    o->obs = xcalloc(o->N, sizeof(oobs));
    /* SamplingWindow._prev_mean = prior_interval.total_seconds() (failure_detector.py:22) */
    o->prior_s = (double)cfg->initial_interval_us / 1e6;
    for (int d = 0; d < 2; d++) {
        o->dg[d].has = xcalloc(o->N, 1);
        o->dg[d].hb = xcalloc(o->N, sizeof(uint32_t));
        o->dg[d].gc = xcalloc(o->N, sizeof(uint32_t));
        o->dg[d].mv = xcalloc(o->N, sizeof(uint32_t));
        o->dg[d].list = xcalloc(o->N, sizeof(int32_t));
        o->sched[d] = xcalloc(o->N, 1);
        o->dl[d].cap_nd = 64;
        o->dl[d].nd = xcalloc(64, sizeof(ond));
        o->dl[d].cap_kv = 256;
        o->dl[d].kv = xcalloc(256, sizeof(okvu));
    }
    o->tmp_stale = xcalloc(o->N, sizeof(int32_t));
    o->tmp_from = xcalloc(o->N, sizeof(uint32_t));
    o->tmp_keys = xcalloc(o->K, sizeof(int32_t));
    return o;
}

void orc_destroy(orc *o) {
    if (!o) return;
    for (int32_t i = 0; i < o->N; i++) {
        oobs *b = &o->obs[i];
        if (!b->alloc) continue;
        for (int32_t j = 0; j < o->N; j++) free(b->w[j].vals);
        free(b->order); free(b->pos); free(b->v); free(b->kv); free(b->w); free(b->live);
        free(b->dead_order); free(b->tod); free(b->dead_pos);
        if (b->snap) {
            oobs *c = b->snap;
            free(c->order); free(c->pos); free(c->v); free(c->kv); free(c->w); free(c->live);
            free(c->dead_order); free(c->tod); free(c->dead_pos); free(c);
        }
    }
    for (int d = 0; d < 2; d++) {
        free(o->dg[d].has); free(o->dg[d].hb); free(o->dg[d].gc); free(o->dg[d].mv); free(o->dg[d].list);
        free(o->sched[d]); free(o->dl[d].nd); free(o->dl[d].kv);
    }
    free(o->tmp_stale); free(o->tmp_from); free(o->tmp_keys);
    free(o->obs); free(o->nid_size); free(o->key_len); free(o);
}

/* Cluster.__init__: self_node_state() + inc_heartbeat() (server.py:95-96) */
void orc_boot(orc *o, int32_t node) {
    oobs *b = row(o, node);
    insert_node(o, b, node);
    b->v[node].hb += 1;
}

void orc_init_warm(orc *o) {
    /* every row rebuilt in index order from the owners' own states */
    for (int32_t i = 0; i < o->N; i++) {
        oobs *b = row(o, i);
        for (int32_t j = 0; j < o->N; j++) {
            if (j == i) continue;
            oobs *own = row(o, j);
            if (b->pos[j] < 0) {
                b->pos[j] = 0; /* placeholder, rebuilt below */
            }
            b->v[j] = own->v[j];
            memcpy(kvp(o, b, j), kvp(o, own, j), sizeof(okv) * o->K);
        }
        b->cnt = o->N;
        for (int32_t j = 0; j < o->N; j++) { b->order[j] = j; b->pos[j] = j; }
    }
}

/* ---------------------------------------------------------- owner writes */
/* NodeState.set_versioned (state.py:124-131) */
static void set_versioned(okv *slot, uint32_t *mv, const okv *nv) {
    if (nv->version > *mv) *mv = nv->version;
    if (slot->present && slot->version >= nv->version) return;
    *slot = *nv;
}

void orc_write(orc *o, int32_t owner, int32_t key, int32_t op, uint32_t value_id, int32_t value_len, int64_t now) {
    oobs *b = row(o, owner);
    oview *v = &b->v[owner];
    okv *slot = &kvp(o, b, owner)[key];
    okv nv;
    memset(&nv, 0, sizeof nv);
    nv.present = 1;
    switch (op) {
    case 0: /* set (state.py:137-142) */
        if (slot->present && slot->value_id == value_id && slot->status == ST_SET) return;
        nv.value_id = value_id; nv.value_len = value_len; nv.version = v->mv + 1; nv.status = ST_SET; nv.ts = now;
        emit(o, owner, owner, key, slot->present ? slot->version : 0u, nv.version, now); /* server.py:193-197 */
        set_versioned(slot, &v->mv, &nv);
        return;
    case 2: /* set_with_ttl (state.py:144-159) */
        if (slot->present && slot->value_id == value_id && slot->status == ST_DELETE_AFTER_TTL) return;
        nv.value_id = value_id; nv.value_len = value_len; nv.version = v->mv + 1;
        nv.status = ST_DELETE_AFTER_TTL; nv.ts = now;
        emit(o, owner, owner, key, slot->present ? slot->version : 0u, nv.version, now); /* server.py:205-209 */
        set_versioned(slot, &v->mv, &nv);
        return;
    case 1: /* delete (state.py:161-171): in-place mutation, value cleared */
        if (!slot->present) return;
        v->mv += 1;
        slot->status = ST_DELETED; slot->version = v->mv; slot->ts = now;
        slot->value_id = 0; slot->value_len = 0;
        return;
    case 3: /* delete_after_ttl (state.py:173-180): value kept */
        if (!slot->present) return;
        v->mv += 1;
        slot->status = ST_DELETE_AFTER_TTL; slot->version = v->mv; slot->ts = now;
        return;
    default:
        fprintf(stderr, "oracle: bad op %d\n", op);
        abort();
    }
}

/* -------------------------------------------------------- failure detector */
static void win_append(owin *w, int32_t cap, double x) { /* BoundedArrayStats.append (139-150) */
    if (w->idx >= w->cap_alloc) {
        int32_t nc = w->cap_alloc ? w->cap_alloc * 2 : 8;
        while (nc <= w->idx) nc *= 2;
        if (nc > cap) nc = cap;
        w->vals = realloc(w->vals, sizeof(double) * nc);
        if (!w->vals) abort();
        w->cap_alloc = nc;
    }
    if (w->filled) w->sum -= w->vals[w->idx];
    w->vals[w->idx] = x;
    w->sum += x;
    if (w->idx == cap - 1) { w->filled = 1; w->idx = 0; }
    else w->idx++;
}

static int32_t win_len(const owin *w, int32_t cap) { return w->filled ? cap : w->idx; } /* 160-162 */

/* FailureDetector.report_heartbeat -> SamplingWindow.report_heartbeat (79-81, 32-38) */
static void fd_report(orc *o, oobs *b, int32_t j, int64_t now) {
    owin *w = &b->w[j];
    if (!w->has) { w->has = 1; w->has_last = 0; w->sum = 0.0; w->idx = 0; w->filled = 0; }
    if (w->has_last) {
        int64_t iv = now - w->last;
        if (iv <= o->c.max_interval_us) win_append(w, o->c.window, (double)iv / 1e6);
    }
    w->last = now;
    w->has_last = 1;
    o->st.hb_reports++;
}

/* SamplingWindow.phi (43-53); returns 0 when None */
static int win_phi(const orc *o, const owin *w, int64_t now, double *phi) {
    if (!w->has || !w->has_last) return 0;
    int32_t len = win_len(w, o->c.window);
    if (len == 0) return 0;
    double mean = (w->sum + 5.0 * o->prior_s) / ((double)len + 5.0);
    double elapsed = (double)(now - w->last) / 1e6;
    *phi = elapsed / mean;
    return 1;
}

static void dead_pop(oobs *b, int32_t j) {
    int32_t p = b->dead_pos[j];
    if (p < 0) return;
    memmove(&b->dead_order[p], &b->dead_order[p + 1], sizeof(int32_t) * (b->ndead - p - 1));
    b->ndead--;
    for (int32_t q = p; q < b->ndead; q++) b->dead_pos[b->dead_order[q]] = q;
    b->dead_pos[j] = -1;
}

/* FailureDetector.update_node_liveness (89-106) */
static void fd_update(orc *o, oobs *b, int32_t j, int64_t now) {
    double phi = 0.0;
    int has = win_phi(o, &b->w[j], now, &phi);
    int alive = has ? (phi <= o->c.phi_threshold) : 0;
    if (alive) {
        b->live[j] = 1;
        dead_pop(b, j);
    } else {
        b->live[j] = 0;
        if (b->dead_pos[j] < 0) {
            b->dead_pos[j] = b->ndead;
            b->dead_order[b->ndead++] = j;
            b->tod[j] = now;
        }
        if (b->w[j].has) { b->w[j].sum = 0.0; b->w[j].idx = 0; b->w[j].filled = 0; } /* reset (40-41) */
    }
}

/* FailureDetector.scheduled_for_deletion_nodes (121-128): now >= tod + grace/2.0 */
static void fd_scheduled(const orc *o, const oobs *b, int64_t now, uint8_t *out) {
    memset(out, 0, o->N);
    /* timedelta / 2.0 rounds half-to-even to whole microseconds */
    int64_t g = o->c.dead_grace_us, half = g / 2;
    if ((g & 1) && (half & 1)) half += 1;
    for (int32_t q = 0; q < b->ndead; q++) {
        int32_t j = b->dead_order[q];
        if (now >= b->tod[j] + half) out[j] = 1;
    }
}

/* ---------------------------------------------------------- state ops */
/* NodeState.gc_marked_for_deletion (state.py:253-274) */
static void gc_view(orc *o, oobs *b, int32_t j, int64_t now) {
    oview *v = &b->v[j];
    okv *kv = kvp(o, b, j);
    uint32_t max_del = v->gc;
    for (int32_t k = 0; k < o->K; k++) {
        if (!kv[k].present) continue;
        if (kv[k].status == ST_SET || now < kv[k].ts + o->c.tombstone_grace_us) continue;
        kv[k].present = 0;
        if (kv[k].version > max_del) max_del = kv[k].version;
    }
    v->gc = max_del;
}

void orc_begin_round(orc *o, int32_t node, int64_t now) {
    oobs *b = row(o, node);
    insert_node(o, b, node);          /* self_node_state() is node_state_or_default */
    b->v[node].hb += 1;               /* server.py:471-472 */
    for (int32_t q = 0; q < b->cnt; q++) gc_view(o, b, b->order[q], now); /* 473-474, state.py:333-338 */
}

/* ClusterState.compute_digest (state.py:324-331) */
static void compute_digest(orc *o, oobs *b, const uint8_t *sched, odigest *d) {
    memset(d->has, 0, o->N);
    d->n = 0;
    for (int32_t q = 0; q < b->cnt; q++) {
        int32_t j = b->order[q];
        if (sched[j]) continue;
        d->has[j] = 1;
        d->hb[j] = b->v[j].hb;
        d->gc[j] = b->v[j].gc;
        d->mv[j] = b->v[j].mv;
        d->list[d->n++] = j;
    }
}

/* Cluster._report_heartbeat (server.py:599-604) over a received digest */
static void merge_heartbeats(orc *o, int32_t self, const odigest *d, int64_t now) {
    oobs *b = row(o, self);
    for (int32_t q = 0; q < d->n; q++) {
        int32_t j = d->list[q];
        if (j == self) continue;
        insert_node(o, b, j);
        oview *v = &b->v[j];
        /* NodeState.apply_heartbeat (state.py:280-287) */
        uint32_t h = d->hb[j];
        if (v->hb == 0) { v->hb = h; continue; }
        if (h > v->hb) { v->hb = h; fd_report(o, b, j, now); }
    }
}

static void delta_reset(odelta *dl) { dl->nnd = 0; dl->nkv = 0; }

static okvu *delta_push_kv(odelta *dl) {
    if (dl->nkv == dl->cap_kv) {
        dl->cap_kv *= 2;
        dl->kv = realloc(dl->kv, sizeof(okvu) * dl->cap_kv);
        if (!dl->kv) abort();
    }
    return &dl->kv[dl->nkv++];
}

static ond *delta_push_nd(odelta *dl) {
    if (dl->nnd == dl->cap_nd) {
        dl->cap_nd *= 2;
        dl->nd = realloc(dl->nd, sizeof(ond) * dl->cap_nd);
        if (!dl->nd) abort();
    }
    return &dl->nd[dl->nnd++];
}

/* ClusterState.compute_partial_delta_respecting_mtu (state.py:340-415) */
static void compute_delta(orc *o, int32_t self, const odigest *d, const uint8_t *sched, odelta *out) {
    oobs *b = row(o, self);
    const int64_t mtu = o->c.mtu;
    int32_t nstale = 0;
    delta_reset(out);
    for (int32_t q = 0; q < b->cnt; q++) {                          /* 347-365 */
        int32_t j = b->order[q];
        if (sched[j]) continue;
        uint32_t dg = 0, dm = 0;
        if (d->has[j]) { dg = d->gc[j]; dm = d->mv[j]; }
        oview *v = &b->v[j];
        if (v->mv <= dm) continue;
        int reset = (dg < v->gc) && (dm < v->gc);
        uint32_t from = reset ? 0 : dm;
        if (v->mv > from) {                                          /* staleness_score (425-427) */
            o->tmp_stale[nstale] = j;
            o->tmp_from[nstale] = from;
            nstale++;
        }
    }
    int64_t committed = 0;                                           /* delta_pb.ByteSize() */
    for (int32_t s = 0; s < nstale; s++) {                           /* 372-413 */
        int32_t j = o->tmp_stale[s];
        uint32_t from = o->tmp_from[s];
        oview *v = &b->v[j];
        okv *kv = kvp(o, b, j);
        int32_t nk = 0;
        for (int32_t k = 0; k < o->K; k++)
            if (kv[k].present && kv[k].version > from) o->tmp_keys[nk++] = k;
        if (nk == 0) continue;                                       /* 378-379 */
        for (int32_t x = 1; x < nk; x++) {                           /* sort by version (382) */
            int32_t key = o->tmp_keys[x], y = x - 1;
            while (y >= 0 && kv[o->tmp_keys[y]].version > kv[key].version) {
                o->tmp_keys[y + 1] = o->tmp_keys[y];
                y--;
            }
            o->tmp_keys[y + 1] = key;
        }
        /* NodeDeltaPb without key_values (385-390) */
        int64_t nd_len = msg_field(o->nid_size[j]) + u_field(from) + u_field(v->gc) + 1 + vlen(v->mv);
        int32_t sel = 0;
        for (int32_t x = 0; x < nk; x++) {                           /* 392-398 */
            okv *e = &kv[o->tmp_keys[x]];
            int64_t l2 = nd_len + msg_field(kv_size(o, o->tmp_keys[x], e->value_len, e->version, e->status));
            if (committed + msg_field(l2) > mtu) break;
            nd_len = l2;
            sel++;
        }
        if (sel > 0) {                                               /* 400-410 */
            ond *nd = delta_push_nd(out);
            nd->node = j; nd->from = from; nd->gc = v->gc; nd->mv = v->mv;
            nd->kv0 = out->nkv; nd->nkv = sel;
            for (int32_t x = 0; x < sel; x++) {
                okv *e = &kv[o->tmp_keys[x]];
                okvu *u = delta_push_kv(out);
                u->key = o->tmp_keys[x]; u->value_id = e->value_id; u->value_len = e->value_len;
                u->version = e->version; u->status = e->status;
            }
            committed += msg_field(nd_len);
            if (sel < nk) o->st.truncated++;
        }
        if (committed >= mtu) break;                                 /* 412-413 */
    }
    o->st.node_deltas += out->nnd;
    o->st.kvs_sent += out->nkv;
    o->st.delta_bytes += committed;
}

/* ClusterState.apply_delta -> NodeState.apply_delta (state.py:310-322, 190-233) */
static void apply_delta(orc *o, int32_t self, const odelta *dl, int64_t now) {
    oobs *b = row(o, self);
    for (int32_t q = 0; q < dl->nnd; q++) {
        const ond *nd = &dl->nd[q];
        insert_node(o, b, nd->node);                                 /* setdefault (321) */
        oview *v = &b->v[nd->node];
        okv *kv = kvp(o, b, nd->node);
        if (nd->gc > v->gc) {                                        /* 200-207 */
            v->gc = nd->gc;
            for (int32_t k = 0; k < o->K; k++)
                if (kv[k].present && kv[k].version <= v->gc) kv[k].present = 0;
        }
        for (int32_t x = 0; x < nd->nkv; x++) {                      /* 208-231 */
            const okvu *u = &dl->kv[nd->kv0 + x];
            if (u->version <= v->mv) continue;
            okv *e = &kv[u->key];
            if (e->present && e->version >= u->version) continue;
            if ((u->status == ST_DELETE_AFTER_TTL || u->status == ST_DELETED) && u->version <= v->gc) continue;
            okv nv;
            nv.present = 1; nv.status = (uint8_t)u->status; nv.value_len = u->value_len;
            nv.value_id = u->value_id; nv.version = u->version; nv.ts = now;
            emit(o, self, nd->node, u->key, e->present ? e->version : 0u, u->version, now); /* 228-231 */
            set_versioned(e, &v->mv, &nv);
        }
        if (nd->mv > v->mv) v->mv = nd->mv;                          /* 232-233 */
    }
}

void orc_exchange(orc *o, int32_t a, int32_t b, int64_t now) {
    oobs *A = row(o, a), *B = row(o, b);
    insert_node(o, A, a);
    insert_node(o, B, b);
    /* a: _make_syn_msg (327-332) */
    fd_scheduled(o, A, now, o->sched[0]);
    compute_digest(o, A, o->sched[0], &o->dg[0]);
    /* b: _handle_message: inc_heartbeat (524) then _handle_syn_msg (334-348) */
    B->v[b].hb += 1;
    merge_heartbeats(o, b, &o->dg[0], now);
    fd_scheduled(o, B, now, o->sched[1]);
    compute_digest(o, B, o->sched[1], &o->dg[1]);
    compute_delta(o, b, &o->dg[0], o->sched[1], &o->dl[0]);
    /* a: _handle_synac_msg (350-370) */
    fd_scheduled(o, A, now, o->sched[0]);
    merge_heartbeats(o, a, &o->dg[1], now);
    apply_delta(o, a, &o->dl[0], now);
    compute_delta(o, a, &o->dg[1], o->sched[0], &o->dl[1]);
    /* b: _handle_ack (372-376) */
    apply_delta(o, b, &o->dl[1], now);
    o->st.exchanges++;
}

/* Cluster._update_node_liveness (server.py:606-620) */
int32_t orc_liveness(orc *o, int32_t node, int64_t now) {
    oobs *b = row(o, node);
    int32_t cnt = b->cnt;
    int32_t *snap = xcalloc(cnt, sizeof(int32_t));
    memcpy(snap, b->order, sizeof(int32_t) * cnt);                   /* nodes() is a tuple */
    /* live-set changes, emitted joins first, then leaves (server.py:611-616); the reference iterates
     * Python sets there (hash order), so each group goes out in node-index order */
    uint8_t *chg = o->ev_on ? xcalloc(o->N, 1) : NULL;
    for (int32_t q = 0; q < cnt; q++)
        if (snap[q] != node) {
            const int32_t j = snap[q];
            const int was = b->live[j];
            fd_update(o, b, j, now);
            if (chg && b->live[j] != was) chg[j] = b->live[j] ? 1 : 2;
        }
    if (chg) {
        for (int kind = 1; kind <= 2; kind++)
            for (int32_t j = 0; j < o->N; j++)
                if (chg[j] == kind) emit(o, node, j, kind << 8, 0u, 0u, now);
        free(chg);
    }
    free(snap);
    /* FailureDetector.garbage_collect (108-119) */
    int32_t *res = xcalloc(b->ndead + 1, sizeof(int32_t));
    int32_t nres = 0;
    for (int32_t q = 0; q < b->ndead; q++) {
        int32_t j = b->dead_order[q];
        if (now >= b->tod[j] + o->c.dead_grace_us) res[nres++] = j;
    }
    int32_t q9 = -1;
    for (int32_t r = 0; r < nres; r++) {
        int32_t j = res[r];
        dead_pop(b, j);
        if (!b->w[j].has) { q9 = j; break; }                          /* KeyError (118), Q9 */
        b->w[j].has = 0; b->w[j].has_last = 0; b->w[j].sum = 0.0; b->w[j].idx = 0; b->w[j].filled = 0;
    }
    if (q9 < 0)
        for (int32_t r = 0; r < nres; r++) remove_node(o, b, res[r]); /* 619-620 */
    free(res);
    return q9;
}

/* ------------------------------------------------ threaded phases (checker speed) */
/* A worker's view of the handle: the rows, configuration and sizes are shared (each thread touches its own
 * rows only), the scratch (digests, deltas, schedules, temporaries) and the statistics are its own. */
static void shadow_init(orc *sh, const orc *o) {
    *sh = *o;
    memset(&sh->st, 0, sizeof sh->st);
    sh->ev_on = 0; sh->ev = NULL; sh->ev_n = sh->ev_cap = 0;
    for (int d = 0; d < 2; d++) {
        sh->dg[d].has = xcalloc(o->N, 1);
        sh->dg[d].hb = xcalloc(o->N, sizeof(uint32_t));
        sh->dg[d].gc = xcalloc(o->N, sizeof(uint32_t));
        sh->dg[d].mv = xcalloc(o->N, sizeof(uint32_t));
        sh->dg[d].list = xcalloc(o->N, sizeof(int32_t));
        sh->sched[d] = xcalloc(o->N, 1);
        sh->dl[d].cap_nd = 64;
        sh->dl[d].nd = xcalloc(64, sizeof(ond));
        sh->dl[d].cap_kv = 256;
        sh->dl[d].kv = xcalloc(256, sizeof(okvu));
    }
    sh->tmp_stale = xcalloc(o->N, sizeof(int32_t));
    sh->tmp_from = xcalloc(o->N, sizeof(uint32_t));
    sh->tmp_keys = xcalloc(o->K, sizeof(int32_t));
}

static void shadow_fold(orc *o, orc *sh) {
    o->st.exchanges += sh->st.exchanges;
    o->st.node_deltas += sh->st.node_deltas;
    o->st.kvs_sent += sh->st.kvs_sent;
    o->st.delta_bytes += sh->st.delta_bytes;
    o->st.hb_reports += sh->st.hb_reports;
    o->st.truncated += sh->st.truncated;
    for (int d = 0; d < 2; d++) {
        free(sh->dg[d].has); free(sh->dg[d].hb); free(sh->dg[d].gc); free(sh->dg[d].mv); free(sh->dg[d].list);
        free(sh->sched[d]); free(sh->dl[d].nd); free(sh->dl[d].kv);
    }
    free(sh->tmp_stale); free(sh->tmp_from); free(sh->tmp_keys);
}

typedef struct {
    orc sh;
    int kind; /* 0 phase, 1 round start, 2 liveness */
    const int32_t *a, *b;
    const uint8_t *up;
    int32_t lo, hi, *q9;
    int64_t now;
} mt_job;

static void *mt_run(void *arg) {
    mt_job *j = arg;
    for (int32_t i = j->lo; i < j->hi; i++) {
        if (j->kind == 0) orc_exchange(&j->sh, j->a[i], j->b[i], j->now);
        else if (j->up[i] && j->kind == 1) orc_begin_round(&j->sh, i, j->now);
        else if (j->up[i]) j->q9[i] = orc_liveness(&j->sh, i, j->now);
    }
    return NULL;
}

static void mt_split(orc *o, int kind, const int32_t *a, const int32_t *b, const uint8_t *up, int32_t n, int64_t now,
                     int32_t threads, int32_t *q9) {
    if (o->ev_on) { fprintf(stderr, "oracle: threaded operations need hook events off\n"); abort(); }
    if (threads < 1) threads = 1;
    if (threads > n) threads = n > 0 ? n : 1;
    mt_job *jobs = xcalloc((size_t)threads, sizeof(mt_job));
    pthread_t *th = xcalloc((size_t)threads, sizeof(pthread_t));
    for (int32_t t = 0; t < threads; t++) {
        mt_job *j = &jobs[t];
        shadow_init(&j->sh, o);
        j->kind = kind; j->a = a; j->b = b; j->up = up; j->q9 = q9; j->now = now;
        j->lo = (int32_t)((int64_t)n * t / threads);
        j->hi = (int32_t)((int64_t)n * (t + 1) / threads);
        if (t > 0 && pthread_create(&th[t], NULL, mt_run, j)) { fprintf(stderr, "oracle: pthread_create\n"); abort(); }
    }
    mt_run(&jobs[0]);
    for (int32_t t = 1; t < threads; t++) pthread_join(th[t], NULL);
    for (int32_t t = 0; t < threads; t++) shadow_fold(o, &jobs[t].sh);
    free(jobs); free(th);
}

void orc_run_phase_mt(orc *o, const int32_t *a, const int32_t *b, int32_t n, int64_t now, int32_t threads) {
    /* the threads share rows only if the phase's exchanges are disjoint (a conflict-free phase): a node in two
     * pairs would race, so such a phase runs sequentially, in list order */
    uint8_t *seen = (uint8_t *)calloc((size_t)o->N, 1);
    int disjoint = seen != NULL;
    for (int32_t i = 0; i < n && disjoint; i++) {
        if (a[i] < 0 || b[i] < 0 || a[i] >= o->N || b[i] >= o->N || a[i] == b[i] || seen[a[i]] || seen[b[i]]) {
            disjoint = 0;
            break;
        }
        seen[a[i]] = seen[b[i]] = 1;
    }
    free(seen);
    if (!disjoint) {
        for (int32_t i = 0; i < n; i++) orc_exchange(o, a[i], b[i], now);
        return;
    }
    for (int32_t i = 0; i < n; i++) {  /* rows are allocated here, once, before the threads share the table */
        row(o, a[i]);
        row(o, b[i]);
    }
    mt_split(o, 0, a, b, NULL, n, now, threads, NULL);
}

void orc_begin_round_mt(orc *o, const uint8_t *up, int64_t now, int32_t threads) {
    mt_split(o, 1, NULL, NULL, up, o->N, now, threads, NULL);
}

void orc_liveness_mt(orc *o, const uint8_t *up, int64_t now, int32_t threads, int32_t *q9) {
    for (int32_t i = 0; i < o->N; i++) q9[i] = -1;
    mt_split(o, 2, NULL, NULL, up, o->N, now, threads, q9);
}

/* ------------------------------------------------------------- readback */
int32_t orc_node_count(const orc *o, int32_t i) { return o->obs[i].alloc ? o->obs[i].cnt : 0; }

void orc_node_order(const orc *o, int32_t i, int32_t *out) {
    if (o->obs[i].alloc) memcpy(out, o->obs[i].order, sizeof(int32_t) * o->obs[i].cnt);
}

void orc_view(const orc *o, int32_t i, int32_t j, uint32_t out[3]) {
    if (!o->obs[i].alloc) { out[0] = out[1] = out[2] = 0; return; }
    const oview *v = &o->obs[i].v[j];
    out[0] = v->hb; out[1] = v->mv; out[2] = v->gc;
}

void orc_view_kvs(const orc *o, int32_t i, int32_t j, int32_t *present, uint32_t *version, int32_t *status,
                  uint32_t *value_id, int64_t *ts) {
    if (!o->obs[i].alloc) { memset(present, 0, sizeof(int32_t) * o->K); return; }
    const okv *kv = &o->obs[i].kv[(size_t)j * o->K];
    for (int32_t k = 0; k < o->K; k++) {
        present[k] = kv[k].present; version[k] = kv[k].version; status[k] = kv[k].status;
        value_id[k] = kv[k].value_id; ts[k] = kv[k].ts;
    }
}

int32_t orc_fd_window(const orc *o, int32_t i, int32_t j, int64_t *last, int32_t *len, double *sum) {
    if (!o->obs[i].alloc) return 0;
    const owin *w = &o->obs[i].w[j];
    if (!w->has) return 0;
    *last = w->has_last ? w->last : -1;
    *len = win_len(w, o->c.window);
    *sum = w->sum;
    return 1;
}

int32_t orc_fd_phi(const orc *o, int32_t i, int32_t j, int64_t now, double *phi) {
    if (!o->obs[i].alloc) return 0;
    return win_phi(o, &o->obs[i].w[j], now, phi);
}

int32_t orc_fd_live(const orc *o, int32_t i, int32_t j) { return o->obs[i].alloc ? o->obs[i].live[j] : 0; }

int64_t orc_fd_dead_since(const orc *o, int32_t i, int32_t j) {
    if (!o->obs[i].alloc) return -1;
    return o->obs[i].dead_pos[j] >= 0 ? o->obs[i].tod[j] : -1;
}

void orc_get_stats(const orc *o, orc_stats *out) { *out = o->st; }

void orc_export_row(const orc *o, int32_t i, int32_t *pos, uint32_t *hb, uint32_t *mv, uint32_t *gc,
                    uint32_t *kv_version, int32_t *kv_status, uint32_t *kv_value_id, int64_t *kv_ts,
                    int64_t *fd_last, int32_t *fd_len, double *fd_sum, int32_t *live, int64_t *tod) {
    const oobs *b = &o->obs[i];
    const int32_t N = o->N, K = o->K;
    for (int32_t j = 0; j < N; j++) {
        pos[j] = b->alloc ? b->pos[j] : -1;
        const oview *v = b->alloc ? &b->v[j] : NULL;
        hb[j] = v ? v->hb : 0; mv[j] = v ? v->mv : 0; gc[j] = v ? v->gc : 0;
        for (int32_t k = 0; k < K; k++) {
            const okv *e = b->alloc ? &b->kv[(size_t)j * K + k] : NULL;
            const int pr = e && e->present;
            kv_version[(size_t)j * K + k] = pr ? e->version : 0;
            kv_status[(size_t)j * K + k] = pr ? e->status : 0;
            kv_value_id[(size_t)j * K + k] = pr ? e->value_id : 0;
            kv_ts[(size_t)j * K + k] = pr ? e->ts : 0;
        }
        const owin *w = b->alloc ? &b->w[j] : NULL;
        fd_last[j] = (w && w->has && w->has_last) ? w->last : -1;
        fd_len[j] = (w && w->has) ? win_len(w, o->c.window) : 0;
        fd_sum[j] = (w && w->has) ? w->sum : 0.0;
        live[j] = b->alloc ? b->live[j] : 0;
        tod[j] = (b->alloc && b->dead_pos[j] >= 0) ? b->tod[j] : -1;
    }
}

/* --------------------------------------------------- state injection */
void orc_load_row(orc *o, int32_t obs, int32_t cnt, const int32_t *order,
                  const uint32_t *hb, const uint32_t *mv, const uint32_t *gc,
                  const uint8_t *held_w, int32_t hist_cap,
                  const uint32_t *hist_version, const uint32_t *hist_value_id,
                  const int32_t *hist_value_len, const uint8_t *hist_status,
                  const uint32_t *fd_last_tick, const uint32_t *fd_sum_tick, const uint32_t *fd_len,
                  const uint32_t *fd_state, int64_t tick_us) {
    oobs *b = row(o, obs);
    const int32_t N = o->N, K = o->K;
    for (int32_t j = 0; j < N; j++) { b->pos[j] = -1; b->dead_pos[j] = -1; b->live[j] = 0; }
    b->ndead = 0;
    for (int32_t q = 0; q < cnt; q++) {
        int32_t j = order[q];
        b->pos[j] = q;
        b->order[q] = j;
        b->v[j].hb = hb[j]; b->v[j].mv = mv[j]; b->v[j].gc = gc[j];
        okv *kv = kvp(o, b, j);
        for (int32_t k = 0; k < K; k++) {
            uint32_t w = held_w[(size_t)j * K + k];
            memset(&kv[k], 0, sizeof(okv));
            if (!w) continue;
            size_t h = ((size_t)j * hist_cap + w) * K + k;
            kv[k].present = 1;
            kv[k].version = hist_version[h];
            kv[k].value_id = hist_value_id[h];
            kv[k].value_len = hist_value_len[h];
            kv[k].status = hist_status[h];
        }
        owin *win = &b->w[j];
        win->has = fd_last_tick[j] != 0xFFFFFFFFu;
        win->has_last = win->has;
        win->last = (int64_t)fd_last_tick[j] * tick_us;
        win->sum = (double)fd_sum_tick[j] * ((double)tick_us / 1e6);
        win->idx = win->has ? (int32_t)fd_len[j] : 0;
        win->filled = 0;
        uint32_t s = fd_state[j];
        if (s == 1) b->live[j] = 1;
        else if (s >= 2) {
            b->dead_pos[j] = b->ndead;
            b->dead_order[b->ndead++] = j;
            b->tod[j] = (int64_t)(s - 2) * tick_us;
        }
    }
    b->cnt = cnt;
}

void orc_set_row_ts(orc *o, int32_t obs, const uint32_t *ts_tick, int64_t tick_us) {
    oobs *b = row(o, obs);
    const int32_t N = o->N, K = o->K;
    for (int32_t j = 0; j < N; j++) {
        if (b->pos[j] < 0) continue;
        okv *kv = kvp(o, b, j);
        for (int32_t k = 0; k < K; k++) {
            const uint32_t t = ts_tick[(size_t)j * K + k];
            if (kv[k].present && kv[k].status != 0 && t != 0xFFFFFFFFu) kv[k].ts = (int64_t)t * tick_us;
        }
    }
}

/* The interval rings of a row loaded by orc_load_row (sampled ring rows of the device): ring_tick[N][W]
 * (ticks), cnt[N] = intervals appended since the last reset, kept below 2W (the device's encoding: the
 * next slot is cnt mod W, and the ring is full once cnt >= W).  BoundedArrayStats (failure_detector.py:
 * 131-162): _values, _index, _filled; _sum was set by orc_load_row. */
void orc_set_row_ring(orc *o, int32_t obs, const uint16_t *ring_tick, const uint32_t *cnt, int64_t tick_us) {
    oobs *b = row(o, obs);
    const int32_t N = o->N, W = o->c.window;
    for (int32_t j = 0; j < N; j++) {
        owin *w = &b->w[j];
        if (b->pos[j] < 0 || !w->has) continue;
        if (w->cap_alloc < W) {
            w->vals = realloc(w->vals, sizeof(double) * (size_t)W);
            if (!w->vals) abort();
            w->cap_alloc = W;
        }
        for (int32_t k = 0; k < W; k++) w->vals[k] = (double)((int64_t)ring_tick[(size_t)j * W + k] * tick_us) / 1e6;
        const uint32_t c = cnt[j];
        w->filled = c >= (uint32_t)W;
        w->idx = (int32_t)(c % (uint32_t)W);
    }
}

/* ------------------------------------------- method-level hooks (KAT ports) */
void orc_kat_set_view(orc *o, int32_t obs, int32_t owner, uint32_t hb, uint32_t mv, uint32_t gc) {
    oobs *b = row(o, obs);
    insert_node(o, b, owner);
    b->v[owner].hb = hb; b->v[owner].mv = mv; b->v[owner].gc = gc;
}

void orc_kat_set_kv(orc *o, int32_t obs, int32_t owner, int32_t key, uint32_t value_id, int32_t value_len,
                    uint32_t version, int32_t status, int64_t ts) {
    oobs *b = row(o, obs);
    insert_node(o, b, owner);
    okv *e = &kvp(o, b, owner)[key];
    e->present = 1; e->value_id = value_id; e->value_len = value_len; e->version = version;
    e->status = (uint8_t)status; e->ts = ts;
}

int32_t orc_kat_apply_heartbeat(orc *o, int32_t obs, int32_t owner, uint32_t h) {
    oobs *b = row(o, obs);
    insert_node(o, b, owner);
    oview *v = &b->v[owner];
    if (v->hb == 0) { v->hb = h; return 0; }
    if (h > v->hb) { v->hb = h; return 1; }
    return 0;
}

void orc_kat_apply_nodedelta(orc *o, int32_t obs, int32_t owner, uint32_t from, uint32_t gc, uint32_t mv,
                             int32_t nkv, const int32_t *keys, const uint32_t *vids, const int32_t *vlens,
                             const uint32_t *versions, const int32_t *statuses, int64_t now) {
    odelta dl;
    memset(&dl, 0, sizeof dl);
    ond nd = {owner, from, gc, mv, 0, nkv};
    okvu *kv = xcalloc(nkv ? nkv : 1, sizeof(okvu));
    for (int32_t x = 0; x < nkv; x++) {
        kv[x].key = keys[x]; kv[x].value_id = vids[x]; kv[x].value_len = vlens[x];
        kv[x].version = versions[x]; kv[x].status = statuses[x];
    }
    dl.nd = &nd; dl.nnd = 1; dl.kv = kv; dl.nkv = nkv;
    apply_delta(o, obs, &dl, now);
    free(kv);
}

void orc_kat_gc(orc *o, int32_t obs, int32_t owner, int64_t grace_us, int64_t now) {
    int64_t saved = o->c.tombstone_grace_us;
    o->c.tombstone_grace_us = grace_us;
    gc_view(o, row(o, obs), owner, now);
    o->c.tombstone_grace_us = saved;
}

int32_t orc_kat_compute_delta(orc *o, int32_t sender, int32_t n_digest, const int32_t *dg_node,
                              const uint32_t *dg_gc, const uint32_t *dg_mv, int32_t mtu,
                              int32_t *nd_node, uint32_t *nd_from, int32_t *nd_nkv, uint32_t *kv_versions,
                              int32_t max_out) {
    odigest *d = &o->dg[0];
    memset(d->has, 0, o->N);
    d->n = 0;
    for (int32_t q = 0; q < n_digest; q++) {
        int32_t j = dg_node[q];
        d->has[j] = 1; d->gc[j] = dg_gc[q]; d->mv[j] = dg_mv[q]; d->hb[j] = 0;
        d->list[d->n++] = j;
    }
    memset(o->sched[1], 0, o->N);
    int32_t saved = o->c.mtu;
    o->c.mtu = mtu;
    compute_delta(o, sender, d, o->sched[1], &o->dl[0]);
    o->c.mtu = saved;
    const odelta *dl = &o->dl[0];
    int32_t nk = 0;
    for (int32_t q = 0; q < dl->nnd && q < max_out; q++) {
        nd_node[q] = dl->nd[q].node; nd_from[q] = dl->nd[q].from; nd_nkv[q] = dl->nd[q].nkv;
        for (int32_t x = 0; x < dl->nd[q].nkv && nk < max_out; x++) kv_versions[nk++] = dl->kv[dl->nd[q].kv0 + x].version;
    }
    return dl->nnd;
}

void orc_kat_fd_report(orc *o, int32_t obs, int32_t target, int64_t now) { fd_report(o, row(o, obs), target, now); }

void orc_kat_fd_update(orc *o, int32_t obs, int32_t target, int64_t now) { fd_update(o, row(o, obs), target, now); }

void orc_kat_fd_reset(orc *o, int32_t obs, int32_t target) {
    owin *w = &row(o, obs)->w[target];
    w->sum = 0.0; w->idx = 0; w->filled = 0;
}

int32_t orc_kat_fd_gc(orc *o, int32_t obs, int64_t now, int32_t *out) {
    oobs *b = row(o, obs);
    int32_t nres = 0;
    for (int32_t q = 0; q < b->ndead; q++) {
        int32_t j = b->dead_order[q];
        if (now >= b->tod[j] + o->c.dead_grace_us) out[nres++] = j;
    }
    for (int32_t r = 0; r < nres; r++) {
        int32_t j = out[r];
        dead_pop(b, j);
        if (!b->w[j].has) return -1 - r;                              /* KeyError (Q9) */
        b->w[j].has = 0; b->w[j].has_last = 0; b->w[j].sum = 0.0; b->w[j].idx = 0; b->w[j].filled = 0;
    }
    return nres;
}

int32_t orc_kat_fd_scheduled(orc *o, int32_t obs, int64_t now, int32_t *out) {
    oobs *b = row(o, obs);
    fd_scheduled(o, b, now, o->sched[0]);
    int32_t n = 0;
    for (int32_t q = 0; q < b->ndead; q++)
        if (o->sched[0][b->dead_order[q]]) out[n++] = b->dead_order[q];
    return n;
}

void orc_kat_win_append(orc *o, int32_t obs, int32_t target, double x) {
    owin *w = &row(o, obs)->w[target];
    w->has = 1;
    win_append(w, o->c.window, x);
}
double orc_kat_win_sum(orc *o, int32_t obs, int32_t target) { return row(o, obs)->w[target].sum; }
int32_t orc_kat_win_len(orc *o, int32_t obs, int32_t target) { return win_len(&row(o, obs)->w[target], o->c.window); }
int32_t orc_kat_win_filled(orc *o, int32_t obs, int32_t target) { return row(o, obs)->w[target].filled; }

/* ------------------------------------------------------------- snapshots */
void orc_snapshot_row(orc *o, int32_t obs) {
    oobs *b = row(o, obs);
    const int32_t N = o->N;
    if (!b->snap) {
        b->snap = xcalloc(1, sizeof(oobs));
        oobs *c = b->snap;
        c->order = xcalloc(N, sizeof(int32_t)); c->pos = xcalloc(N, sizeof(int32_t));
        c->v = xcalloc(N, sizeof(oview)); c->kv = xcalloc((size_t)N * o->K, sizeof(okv));
        c->w = xcalloc(N, sizeof(owin)); c->live = xcalloc(N, 1);
        c->dead_order = xcalloc(N, sizeof(int32_t)); c->tod = xcalloc(N, sizeof(int64_t));
        c->dead_pos = xcalloc(N, sizeof(int32_t));
    }
    oobs *c = b->snap;
    c->cnt = b->cnt; c->ndead = b->ndead;
    memcpy(c->order, b->order, sizeof(int32_t) * N); memcpy(c->pos, b->pos, sizeof(int32_t) * N);
    memcpy(c->v, b->v, sizeof(oview) * N); memcpy(c->kv, b->kv, sizeof(okv) * (size_t)N * o->K);
    memcpy(c->w, b->w, sizeof(owin) * N); memcpy(c->live, b->live, N);
    memcpy(c->dead_order, b->dead_order, sizeof(int32_t) * N); memcpy(c->tod, b->tod, sizeof(int64_t) * N);
    memcpy(c->dead_pos, b->dead_pos, sizeof(int32_t) * N);
    /* ring storage is not copied: snapshots are taken of rows whose windows hold no ring yet */
    for (int32_t j = 0; j < N; j++) { c->w[j].vals = NULL; c->w[j].cap_alloc = 0; }
}

void orc_restore_row(orc *o, int32_t obs) {
    oobs *b = row(o, obs);
    oobs *c = b->snap;
    if (!c) return;
    const int32_t N = o->N;
    for (int32_t j = 0; j < N; j++) free(b->w[j].vals);
    b->cnt = c->cnt; b->ndead = c->ndead;
    memcpy(b->order, c->order, sizeof(int32_t) * N); memcpy(b->pos, c->pos, sizeof(int32_t) * N);
    memcpy(b->v, c->v, sizeof(oview) * N); memcpy(b->kv, c->kv, sizeof(okv) * (size_t)N * o->K);
    memcpy(b->w, c->w, sizeof(owin) * N); memcpy(b->live, c->live, N);
    memcpy(b->dead_order, c->dead_order, sizeof(int32_t) * N); memcpy(b->tod, c->tod, sizeof(int64_t) * N);
    memcpy(b->dead_pos, c->dead_pos, sizeof(int32_t) * N);
}
