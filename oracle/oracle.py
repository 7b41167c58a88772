"""ctypes wrapper of the C oracle (``oracle/gossip_oracle.c``).

TEST INFRASTRUCTURE: the checker for the HIP path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg import it.

``OracleSim`` implements the scenario backend protocol of
``aiocluster_amd.scenario.replay`` and dumps the same canonical state as
``oracle/refharness.py`` so the two compare byte for byte.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libgossip_oracle.so")
TICK_US = 15_625


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "gossip_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


class _Cfg(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int32),
        ("n_keys", C.c_int32),
        ("mtu", C.c_int32),
        ("tombstone_grace_us", C.c_int64),
        ("phi_threshold", C.c_double),
        ("window", C.c_int32),
        ("max_interval_us", C.c_int64),
        ("initial_interval_us", C.c_int64),
        ("dead_grace_us", C.c_int64),
    ]


class _Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in
                ("exchanges", "node_deltas", "kvs_sent", "delta_bytes", "hb_reports", "truncated")]


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        L = C.CDLL(build())
        P = C.c_void_p
        i32, i64, u32 = C.c_int32, C.c_int64, C.c_uint32
        pi32, pu32, pi64, pdbl = C.POINTER(i32), C.POINTER(u32), C.POINTER(i64), C.POINTER(C.c_double)
        sig = {
            "orc_create": (P, [C.POINTER(_Cfg), pi32, pi32]),
            "orc_destroy": (None, [P]),
            "orc_boot": (None, [P, i32]),
            "orc_init_warm": (None, [P]),
            "orc_write": (None, [P, i32, i32, i32, u32, i32, i64]),
            "orc_begin_round": (None, [P, i32, i64]),
            "orc_exchange": (None, [P, i32, i32, i64]),
            "orc_liveness": (i32, [P, i32, i64]),
            "orc_run_phase_mt": (None, [P, P, P, i32, i64, i32]),
            "orc_begin_round_mt": (None, [P, P, i64, i32]),
            "orc_liveness_mt": (None, [P, P, i64, i32, P]),
            "orc_node_count": (i32, [P, i32]),
            "orc_node_order": (None, [P, i32, pi32]),
            "orc_view": (None, [P, i32, i32, pu32]),
            "orc_view_kvs": (None, [P, i32, i32, pi32, pu32, pi32, pu32, pi64]),
            "orc_fd_window": (i32, [P, i32, i32, pi64, pi32, pdbl]),
            "orc_fd_phi": (i32, [P, i32, i32, i64, pdbl]),
            "orc_fd_live": (i32, [P, i32, i32]),
            "orc_fd_dead_since": (i64, [P, i32, i32]),
            "orc_get_stats": (None, [P, C.POINTER(_Stats)]),
            "orc_enable_events": (None, [P, i32]),
            "orc_drain_events": (i32, [P, P, i32]),
            "orc_export_row": (None, [P, i32] + [P] * 13),
            "orc_load_row": (None, [P, i32, i32, P, P, P, P, P, i32, P, P, P, P, P, P, P, P, i64]),
            "orc_set_row_ts": (None, [P, i32, P, i64]),
            "orc_set_row_ring": (None, [P, i32, P, P, i64]),
            "orc_snapshot_row": (None, [P, i32]),
            "orc_restore_row": (None, [P, i32]),
            "orc_kat_set_view": (None, [P, i32, i32, u32, u32, u32]),
            "orc_kat_set_kv": (None, [P, i32, i32, i32, u32, i32, u32, i32, i64]),
            "orc_kat_apply_heartbeat": (i32, [P, i32, i32, u32]),
            "orc_kat_apply_nodedelta": (None, [P, i32, i32, u32, u32, u32, i32, P, P, P, P, P, i64]),
            "orc_kat_gc": (None, [P, i32, i32, i64, i64]),
            "orc_kat_compute_delta": (i32, [P, i32, i32, P, P, P, i32, P, P, P, P, i32]),
            "orc_kat_fd_report": (None, [P, i32, i32, i64]),
            "orc_kat_fd_update": (None, [P, i32, i32, i64]),
            "orc_kat_fd_gc": (i32, [P, i32, i64, P]),
            "orc_kat_fd_scheduled": (i32, [P, i32, i64, P]),
            "orc_kat_fd_reset": (None, [P, i32, i32]),
            "orc_kat_win_append": (None, [P, i32, i32, C.c_double]),
            "orc_kat_win_sum": (C.c_double, [P, i32, i32]),
            "orc_kat_win_len": (i32, [P, i32, i32]),
            "orc_kat_win_filled": (i32, [P, i32, i32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def us(seconds: float) -> int:
    """``timedelta(seconds=...)`` in whole microseconds (round-half-even, as datetime does)."""
    from datetime import timedelta

    return timedelta(seconds=seconds) // timedelta(microseconds=1)


class OracleSim:
    """The C oracle as a scenario backend (``aiocluster_amd.scenario.replay``)."""

    def __init__(self, node_ids, keys, cfg: dict, init: str, initial_values, nid_sizes=None, threads: int = 1):
        """``threads`` > 1: phases, round starts and liveness sweeps split their rows over that many host
        threads (orc_*_mt: the sequential result, checker speed for the long whole-array tests; no hook
        events)."""
        from aiocluster_amd.pbsize import nodeid_size

        self.L = lib()
        self.n = len(node_ids)
        self.keys = list(keys)
        self.k = len(keys)
        self.cfg = cfg
        c = _Cfg(
            self.n, self.k, int(cfg["mtu"]), us(cfg["tombstone_grace_s"]), float(cfg["phi_threshold"]),
            int(cfg["window"]), us(cfg["max_interval_s"]), us(cfg["initial_interval_s"]), us(cfg["dead_grace_s"]),
        )
        if nid_sizes is None:
            nid_sizes = [nodeid_size(n.name, n.generation_id, n.gossip_advertise_addr[0],
                                     n.gossip_advertise_addr[1], n.tls_name) for n in node_ids]
        ns = (C.c_int32 * self.n)(*nid_sizes)
        kl = (C.c_int32 * self.k)(*[len(k.encode()) for k in keys])
        self.h = self.L.orc_create(C.byref(c), ns, kl)
        self.values = [""]
        self.value_ids = {"": 0}
        self.last_tick = 0
        self.q9_events = []
        self.threads = int(threads)
        self.events_on = False
        for j in range(self.n):
            self.L.orc_boot(self.h, j)
        if initial_values:
            for j in range(self.n):
                for k, v in initial_values.get(j, []):
                    self.write(0, j, k, 0, v)
        if init == "warm":
            self.L.orc_init_warm(self.h)

    def close(self):
        if self.h:
            self.L.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def intern(self, value: str) -> int:
        vid = self.value_ids.get(value)
        if vid is None:
            vid = len(self.values)
            self.values.append(value)
            self.value_ids[value] = vid
        return vid

    # -------------------------------------------------------- backend protocol
    def write(self, t: int, j: int, k: int, op: int, value: str):
        self.L.orc_write(self.h, j, k, op, self.intern(value), len(value.encode()), t * TICK_US)

    def _mt(self) -> bool:
        return self.threads > 1 and not self.events_on

    def begin_round(self, t: int, up):
        if self._mt():
            u = np.ascontiguousarray(np.asarray(up, dtype=np.uint8))
            self.L.orc_begin_round_mt(self.h, u.ctypes.data_as(C.c_void_p), t * TICK_US, self.threads)
            return
        for o in range(self.n):
            if up[o]:
                self.L.orc_begin_round(self.h, o, t * TICK_US)

    def run_phase(self, t: int, pairs):
        if self._mt():
            p = np.ascontiguousarray(np.asarray(list(pairs), dtype=np.int32).reshape(-1, 2).T)
            self.L.orc_run_phase_mt(self.h, p[0].ctypes.data_as(C.c_void_p), p[1].ctypes.data_as(C.c_void_p),
                                    p.shape[1], t * TICK_US, self.threads)
            return
        for a, b in pairs:
            self.L.orc_exchange(self.h, int(a), int(b), t * TICK_US)

    def exchange(self, a: int, b: int, t: int):
        self.L.orc_exchange(self.h, int(a), int(b), t * TICK_US)

    def liveness(self, t: int, up, r: int = -1):
        self.last_tick = t
        if self._mt():
            u = np.ascontiguousarray(np.asarray(up, dtype=np.uint8))
            q9 = np.empty(self.n, np.int32)
            self.L.orc_liveness_mt(self.h, u.ctypes.data_as(C.c_void_p), t * TICK_US, self.threads,
                                   q9.ctypes.data_as(C.c_void_p))
            for o in np.flatnonzero(q9 >= 0):
                self.q9_events.append([r, int(o), int(q9[o])])
            return
        for o in range(self.n):
            if up[o]:
                q = self.L.orc_liveness(self.h, o, t * TICK_US)
                if q >= 0:
                    self.q9_events.append([r, o, q])

    def enable_events(self):
        self.events_on = True
        self.L.orc_enable_events(self.h, 1)

    def drain_events(self) -> np.ndarray:
        """Events since the last drain in the device's format (times in ticks), in the reference's order
        (the oracle runs the reference's calls one at a time; join / leave in node order, see
        gossip_oracle.c orc_liveness)."""
        buf = np.zeros((1 << 22, 6), dtype=np.int64)
        n = self.L.orc_drain_events(self.h, buf.ctypes.data_as(C.c_void_p), buf.shape[0])
        assert n <= buf.shape[0]
        ev = buf[:n].copy()
        ev[:, 5] //= TICK_US
        return ev.astype(np.uint32)

    def stats(self) -> dict:
        s = _Stats()
        self.L.orc_get_stats(self.h, C.byref(s))
        return {n: getattr(s, n) for n, _ in _Stats._fields_}

    # ------------------------------------------------------------------ dump
    def order(self, o: int) -> list[int]:
        cnt = self.L.orc_node_count(self.h, o)
        buf = (C.c_int32 * max(cnt, 1))()
        self.L.orc_node_order(self.h, o, buf)
        return list(buf[:cnt])

    def view(self, o: int, j: int) -> tuple[int, int, int]:
        out = (C.c_uint32 * 3)()
        self.L.orc_view(self.h, o, j, out)
        return out[0], out[1], out[2]

    def view_kvs(self, o: int, j: int) -> list:
        K = self.k
        pres, ver, st = (C.c_int32 * K)(), (C.c_uint32 * K)(), (C.c_int32 * K)()
        vid, ts = (C.c_uint32 * K)(), (C.c_int64 * K)()
        self.L.orc_view_kvs(self.h, o, j, pres, ver, st, vid, ts)
        out = []
        for k in range(K):
            if pres[k]:
                out.append([self.keys[k], self.values[vid[k]], ver[k], st[k],
                            None if st[k] == 0 else ts[k] // TICK_US])
        out.sort()
        return out

    def observer_state(self, o: int) -> dict:
        now = self.last_tick * TICK_US
        nodes = []
        for j in self.order(o):
            hb, mv, gc = self.view(o, j)
            nodes.append([j, hb, mv, gc, self.view_kvs(o, j)])
        live, dead, wins = [], [], []
        last, ln, sm, phi = C.c_int64(), C.c_int32(), C.c_double(), C.c_double()
        for j in range(self.n):
            if self.L.orc_fd_live(self.h, o, j):
                live.append(j)
            tod = self.L.orc_fd_dead_since(self.h, o, j)
            if tod >= 0:
                dead.append([j, tod // TICK_US])
            if self.L.orc_fd_window(self.h, o, j, C.byref(last), C.byref(ln), C.byref(sm)):
                has = self.L.orc_fd_phi(self.h, o, j, now, C.byref(phi))
                wins.append([j, None if last.value < 0 else last.value // TICK_US, ln.value, sm.value,
                             phi.value if has else None])
        return {"nodes": nodes, "live": live, "dead": dead, "windows": wins}

    def state(self) -> list[dict]:
        return [self.observer_state(o) for o in range(self.n)]

    _EXPORT = (("pos", np.int32, 0), ("hb", np.uint32, 0), ("mv", np.uint32, 0), ("gc", np.uint32, 0),
               ("kv_version", np.uint32, 1), ("kv_status", np.int32, 1), ("kv_value_id", np.uint32, 1),
               ("kv_ts", np.int64, 1), ("fd_last", np.int64, 0), ("fd_len", np.int32, 0), ("fd_sum", np.float64, 0),
               ("live", np.int32, 0), ("tod", np.int64, 0))

    def export(self) -> dict:
        return self.export_rows(range(self.n))

    def export_rows(self, rows) -> dict:
        """Numpy arrays of the observer rows ``rows`` (see ``orc_export_row``), written in place; times in ticks."""
        rows = list(rows)
        R, N, K = len(rows), self.n, self.k
        a = {name: np.empty((R, N, K) if kv else (R, N), dt) for name, dt, kv in self._EXPORT}
        stride = {name: a[name].strides[0] for name, _, _ in self._EXPORT}
        base = {name: a[name].ctypes.data for name, _, _ in self._EXPORT}
        names = [name for name, _, _ in self._EXPORT]
        for i, o in enumerate(rows):
            self.L.orc_export_row(self.h, o, *[C.c_void_p(base[nm] + i * stride[nm]) for nm in names])
        for n in ("kv_ts", "fd_last", "tod"):
            x = a[n]
            np.floor_divide(x, TICK_US, out=x, where=x >= 0)
        return a

    def export_row(self, o: int) -> dict:
        """Numpy view of observer ``o`` (see ``orc_export_row``); times in ticks."""
        return {k: v[0] for k, v in self.export_rows([o]).items()}
