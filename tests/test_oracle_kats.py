"""The reference's own unit tests, replayed against the C oracle (CPU).

Each test restates one test of /root/reference/tests with the same inputs and
assertions, driven through the oracle's method-level hooks:

* tests/test_state.py:19-223      (apply_delta, apply_heartbeat, GC, staleness, MTU trim)
* tests/test_node_state.py:15-61  (set / delete / TTL transitions)
* tests/test_failure_detector.py:24-177 (BoundedArrayStats, SamplingWindow, FailureDetector)

``_prepart_node`` (test_state.py:139-153) is dead code in the library (never
called) and is not restated.
"""

import ctypes as C
from random import Random

import pytest
from oracle import _Cfg, lib, us

from aiocluster_amd import pbsize

SET, DELETED, DAT = 0, 1, 2
H = 3600.0


class Kat:
    """A small oracle instance; node 0 observes, nodes 1.. are owners."""

    def __init__(self, n=4, k=4, mtu=65507, window=1000, max_interval=10.0, prior=5.0, dead_grace=24 * H,
                 nid_size=20, key_lens=None):
        self.L = lib()
        cfg = _Cfg(n, k, mtu, us(7200), 8.0, window, us(max_interval), us(prior), us(dead_grace))
        ns = (C.c_int32 * n)(*[nid_size] * n)
        kl = (C.c_int32 * k)(*(key_lens or [2] * k))
        self.h = self.L.orc_create(C.byref(cfg), ns, kl)
        self.values = {"": 0}

    def __del__(self):
        self.L.orc_destroy(self.h)

    def vid(self, v):
        return self.values.setdefault(v, len(self.values))

    def set_kv(self, obs, owner, key, value, version, status=SET, ts_s=0.0):
        self.L.orc_kat_set_kv(self.h, obs, owner, key, self.vid(value), len(value), version, status, us(ts_s))

    def kv(self, obs, owner, key):
        K = 4
        pres, ver, st = (C.c_int32 * K)(), (C.c_uint32 * K)(), (C.c_int32 * K)()
        vid, ts = (C.c_uint32 * K)(), (C.c_int64 * K)()
        self.L.orc_view_kvs(self.h, obs, owner, pres, ver, st, vid, ts)
        if not pres[key]:
            return None
        inv = {v: s for s, v in self.values.items()}
        return inv[vid[key]], ver[key], st[key]

    def get(self, obs, owner, key):  # NodeState.get: None for deleted statuses (state.py:115-119)
        v = self.kv(obs, owner, key)
        return None if v is None or v[2] != SET else v

    def view(self, obs, owner):
        out = (C.c_uint32 * 3)()
        self.L.orc_view(self.h, obs, owner, out)
        return tuple(out)

    def apply(self, obs, owner, frm, gc, kvs, mv, now_s=0.0):
        n = len(kvs)
        keys = (C.c_int32 * max(n, 1))(*[k for k, _, _, _ in kvs])
        vids = (C.c_uint32 * max(n, 1))(*[self.vid(v) for _, v, _, _ in kvs])
        vls = (C.c_int32 * max(n, 1))(*[len(v) for _, v, _, _ in kvs])
        vers = (C.c_uint32 * max(n, 1))(*[ver for _, _, ver, _ in kvs])
        sts = (C.c_int32 * max(n, 1))(*[st for _, _, _, st in kvs])
        self.L.orc_kat_apply_nodedelta(self.h, obs, owner, frm, gc, mv, n, keys, vids, vls, vers, sts, us(now_s))


# ---------------------------------------------------------------- tests/test_state.py
def test_apply_delta_creates_node():  # test_state.py:19-47
    k = Kat()
    assert k.view(0, 1) == (0, 0, 0)
    k.apply(0, 1, 0, 0, [(0, "v1", 1, SET)], 1)
    assert k.get(0, 1, 0)[0] == "v1"


def test_apply_delta_respects_per_key_versions():  # test_state.py:50-76
    k = Kat()
    k.set_kv(0, 1, 0, "old", 10)  # set_with_version("a", "old", 10)
    k.set_kv(0, 1, 1, "old", 1)  # set_with_version("b", "old", 1)
    k.L.orc_kat_set_view(k.h, 0, 1, 0, 10, 0)  # set_versioned raised max_version to 10
    k.apply(0, 1, 1, 0, [(1, "new", 11, SET)], 11)
    assert k.get(0, 1, 1) == ("new", 11, SET)


def test_apply_heartbeat():  # test_state.py:84-91
    k = Kat()
    assert k.L.orc_kat_apply_heartbeat(k.h, 0, 1, 5) == 0 and k.view(0, 1)[0] == 5
    assert k.L.orc_kat_apply_heartbeat(k.h, 0, 1, 3) == 0 and k.view(0, 1)[0] == 5
    assert k.L.orc_kat_apply_heartbeat(k.h, 0, 1, 6) == 1 and k.view(0, 1)[0] == 6


def test_apply_delta_skips_old_or_gc_versions():  # test_state.py:94-108
    k = Kat()
    k.L.orc_kat_set_view(k.h, 0, 1, 0, 2, 2)
    k.apply(0, 1, 0, 0, [(0, "v1", 1, SET), (1, "v2", 2, DAT), (2, "v3", 3, SET)], 3)
    assert k.get(0, 1, 0) is None
    assert k.get(0, 1, 1) is None
    assert k.get(0, 1, 2) is not None


def test_gc_marked_for_deletion_updates_last_gc_version():  # test_state.py:111-136
    k = Kat()
    now = 10.0
    k.L.orc_kat_set_view(k.h, 0, 1, 0, 0, 1)
    k.set_kv(0, 1, 0, "v1", 2, SET, now - 5)  # keep
    k.set_kv(0, 1, 1, "v2", 5, DELETED, now - 20)  # delete
    k.set_kv(0, 1, 2, "v3", 3, DAT, now - 2)  # wait
    k.L.orc_kat_gc(k.h, 0, 1, us(10), us(now))
    assert k.kv(0, 1, 1) is None
    assert k.kv(0, 1, 0) is not None
    assert k.kv(0, 1, 2) is not None
    assert k.view(0, 1)[2] == 5


def _delta(k, sender, digest, mtu, max_out=64):
    n = len(digest)
    dn = (C.c_int32 * max(n, 1))(*[x[0] for x in digest])
    dg = (C.c_uint32 * max(n, 1))(*[x[1] for x in digest])
    dm = (C.c_uint32 * max(n, 1))(*[x[2] for x in digest])
    nd_node, nd_from = (C.c_int32 * max_out)(), (C.c_uint32 * max_out)()
    nd_nkv, kv_ver = (C.c_int32 * max_out)(), (C.c_uint32 * max_out)()
    cnt = k.L.orc_kat_compute_delta(k.h, sender, n, dn, dg, dm, mtu, nd_node, nd_from, nd_nkv, kv_ver, max_out)
    return [(nd_node[i], nd_from[i], nd_nkv[i]) for i in range(cnt)], list(kv_ver[: sum(nd_nkv[:cnt])])


def test_staleness_score_decides_staleness():  # test_state.py:156-169 (as used at state.py:364)
    k = Kat()
    k.set_kv(0, 1, 0, "v1", 1)
    k.set_kv(0, 1, 1, "v2", 2)
    k.L.orc_kat_set_view(k.h, 0, 1, 0, 2, 0)
    assert _delta(k, 0, [(1, 0, 2)], 65507)[0] == []  # staleness_score(floor=2) is None
    nds, vers = _delta(k, 0, [], 65507)  # floor 0: unknown, 2 stale kvs
    assert nds == [(1, 0, 2)] and vers == [1, 2]


def test_compute_partial_delta_respecting_mtu_trims():  # test_state.py:172-223
    nid = pbsize.nodeid_size("node", 0, "localhost", 7001, None)
    k = Kat(nid_size=nid)
    k.set_kv(0, 1, 0, "v1", 1)
    k.set_kv(0, 1, 1, "v2", 2)
    k.L.orc_kat_set_view(k.h, 0, 1, 0, 2, 1)
    kv1 = pbsize.kv_size("k1", "v1", 1, 0)
    kv2 = pbsize.kv_size("k2", "v2", 2, 0)
    size1 = pbsize.delta_size([pbsize.nodedelta_size(nid, 0, 1, [kv1], 2)])
    size2 = pbsize.delta_size([pbsize.nodedelta_size(nid, 0, 1, [kv1, kv2], 2)])
    assert size2 > size1
    nds, vers = _delta(k, 0, [], size1 + 1)
    assert len(nds) == 1 and nds[0][2] == 1 and vers == [1]


# ---------------------------------------------------------------- tests/test_node_state.py
def _owner(k):
    k.L.orc_kat_set_view(k.h, 1, 1, 0, 1, 1)  # NodeState(node_id, 0, {}, 1, 1)


def test_node_set_delete():  # test_node_state.py:24-29
    k = Kat()
    _owner(k)
    k.L.orc_write(k.h, 1, 0, 0, k.vid("val_b"), 5, 0)
    k.L.orc_write(k.h, 1, 0, 1, 0, 0, 0)
    assert k.get(1, 1, 0) is None


def test_node_set_delete_after_ttl_set():  # test_node_state.py:32-40
    k = Kat()
    _owner(k)
    k.L.orc_write(k.h, 1, 0, 0, k.vid("val_b"), 5, 0)
    k.L.orc_write(k.h, 1, 0, 3, 0, 0, 0)
    k.L.orc_write(k.h, 1, 0, 0, k.vid("val_b2"), 6, 0)
    v = k.kv(1, 1, 0)
    assert v is not None and v[2] == SET and v[0] == "val_b2"


def test_node_set_with_ttl():  # test_node_state.py:43-48
    k = Kat()
    _owner(k)
    k.L.orc_write(k.h, 1, 0, 2, k.vid("val_b"), 5, 0)
    v = k.kv(1, 1, 0)
    assert v is not None and v[2] == DAT and v[0] == "val_b"


# ---------------------------------------------------------------- tests/test_failure_detector.py
def test_bounded_array():  # test_failure_detector.py:24-46
    from collections import deque

    cap = 5
    k = Kat(window=cap)
    L, h = k.L, k.h
    expected = deque(maxlen=cap)
    for i in range(1, cap):
        assert L.orc_kat_win_len(h, 0, 1) < cap and not L.orc_kat_win_filled(h, 0, 1)
        L.orc_kat_win_append(h, 0, 1, i * 0.1)
        expected.append(i * 0.1)
        assert L.orc_kat_win_len(h, 0, 1) == i
        assert L.orc_kat_win_sum(h, 0, 1) == sum(expected)
    assert not L.orc_kat_win_filled(h, 0, 1)
    for i in range(cap):
        L.orc_kat_win_append(h, 0, 1, i * 0.1)
        expected.append(i * 0.1)
        assert L.orc_kat_win_filled(h, 0, 1)
        assert L.orc_kat_win_len(h, 0, 1) == cap == len(expected)
        assert L.orc_kat_win_sum(h, 0, 1) == sum(expected)


def _phi(k, obs, tgt, t_s):
    p = C.c_double()
    return p.value if k.L.orc_fd_phi(k.h, obs, tgt, us(t_s), C.byref(p)) else None


def test_sampling_window():  # test_failure_detector.py:49-80
    k = Kat(window=10, max_interval=5.0, prior=2.0)
    rep = lambda t: k.L.orc_kat_fd_report(k.h, 0, 1, us(t))  # noqa: E731
    now = 1000.0
    rep(now)
    t1 = now + 3
    rep(t1)
    mean = (3.0 + 2.0 * 5.0) / (1.0 + 5.0)
    assert _phi(k, 0, 1, t1) == pytest.approx(0.0)
    t2 = t1 + 1
    assert _phi(k, 0, 1, t2) == pytest.approx(1.0 / mean)
    t3 = t2 + 5
    rep(t3)
    t4 = t3 + 2
    assert _phi(k, 0, 1, t4) == pytest.approx(2.0 / mean)
    t5 = t4 + 100
    k.L.orc_kat_fd_reset(k.h, 0, 1)
    rep(t5)
    assert _phi(k, 0, 1, now) is None
    t6 = t5 + 2
    rep(t6)
    t7 = t6 + 4
    new_mean = (2.0 + 2.0 * 5.0) / (1.0 + 5.0)
    assert _phi(k, 0, 1, t7) == pytest.approx(4.0 / new_mean)


def test_single_heartbeat_is_dead():  # test_failure_detector.py:83-92
    k = Kat()
    k.L.orc_kat_fd_report(k.h, 0, 1, us(100.0))
    k.L.orc_kat_fd_update(k.h, 0, 1, us(100.0))
    assert k.L.orc_fd_dead_since(k.h, 0, 1) >= 0 and not k.L.orc_fd_live(k.h, 0, 1)


def test_failure_detector():  # test_failure_detector.py:95-130
    rng = Random(1234)
    k = Kat(n=4)
    nodes = [1, 2, 3]
    t = 1_000_000.0
    for _ in range(100):
        node = rng.choice(nodes)
        t += 1
        k.L.orc_kat_fd_report(k.h, 0, node, us(t))
    for node in nodes:
        k.L.orc_kat_fd_update(k.h, 0, node, us(t))
    assert sum(k.L.orc_fd_live(k.h, 0, j) for j in nodes) == 3
    assert sum(k.L.orc_fd_dead_since(k.h, 0, j) >= 0 for j in nodes) == 0
    t += 50
    for node in nodes:
        k.L.orc_kat_fd_update(k.h, 0, node, us(t))
    assert sum(k.L.orc_fd_live(k.h, 0, j) for j in nodes) == 0
    assert sum(k.L.orc_fd_dead_since(k.h, 0, j) >= 0 for j in nodes) == 3
    out = (C.c_int32 * 8)()
    assert k.L.orc_kat_fd_gc(k.h, 0, us(t), out) == 0
    t += 25 * 3600
    assert k.L.orc_kat_fd_gc(k.h, 0, us(t), out) == 3
    assert sum(k.L.orc_fd_dead_since(k.h, 0, j) >= 0 for j in nodes) == 0
    assert sum(k.L.orc_fd_live(k.h, 0, j) for j in nodes) == 0


def test_bounded_array_stats_rollover_and_clear():  # test_failure_detector.py:133-144
    k = Kat(window=2)
    for x in (1.0, 2.0, 3.0):
        k.L.orc_kat_win_append(k.h, 0, 1, x)
    assert k.L.orc_kat_win_len(k.h, 0, 1) == 2 and k.L.orc_kat_win_sum(k.h, 0, 1) == 5.0
    k.L.orc_kat_fd_reset(k.h, 0, 1)
    assert k.L.orc_kat_win_len(k.h, 0, 1) == 0 and k.L.orc_kat_win_sum(k.h, 0, 1) == 0.0


def test_sampling_window_respects_max_interval():  # test_failure_detector.py:147-161
    k = Kat(window=2, max_interval=1.0, prior=1.0)
    t0 = 5000.0
    k.L.orc_kat_fd_report(k.h, 0, 1, us(t0))
    k.L.orc_kat_fd_report(k.h, 0, 1, us(t0 + 2))
    assert _phi(k, 0, 1, t0 + 2) is None
    k.L.orc_kat_fd_report(k.h, 0, 1, us(t0 + 2.5))
    assert _phi(k, 0, 1, t0 + 3) is not None


def test_failure_detector_garbage_collect_and_scheduled_nodes():  # test_failure_detector.py:164-177
    k = Kat(dead_grace=10.0)
    now = 7000.0
    k.L.orc_kat_fd_report(k.h, 0, 1, us(now))
    k.L.orc_kat_fd_update(k.h, 0, 1, us(now))
    out = (C.c_int32 * 8)()
    n = k.L.orc_kat_fd_scheduled(k.h, 0, us(now + 5), out)
    assert 1 in list(out[:n])
    assert k.L.orc_kat_fd_gc(k.h, 0, us(now + 11), out) == 1 and out[0] == 1
