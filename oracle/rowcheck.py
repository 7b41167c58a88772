"""The C oracle on observer rows copied out of a device state -- full-size parity checks.

TEST INFRASTRUCTURE: the checker for the HIP path.  Only ``tests/`` and ``bench.py``'s
``cpu_baseline`` leg use it.

At 65,536 nodes the oracle cannot replay a whole run (N^2 views), but the
exchanges of one conflict-free phase touch only their own two rows.  ``RowOracle`` copies the
rows of sampled exchanges from a ``GossipSim`` (after ``gs_begin_round``), runs the same
exchanges and the liveness sweep of those rows in the oracle, and exports them in the
device's ``export()`` format, so ``tests/helpers.compare_exports`` checks the device rows the
same phase produced bit for bit: decoded heartbeats, max versions, last_gc versions, held keys
(versions, statuses, values, tombstone receive ticks), failure-detector windows, live/dead.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

import oracle as orc_mod

TICK_US = orc_mod.TICK_US

EXPORT_FIELDS = ("pos", "hb", "mv", "gc", "kv_version", "kv_status", "kv_value_id", "kv_ts", "fd_last", "fd_len",
                 "fd_sum", "live", "tod")


def compare_exports(got: dict, want: dict):
    """First mismatching (field, observer, index) between two ``export()`` dicts, or None."""
    for key in EXPORT_FIELDS:
        a, b = np.asarray(got[key]), np.asarray(want[key])
        if a.shape != b.shape:
            return f"{key}: shape {a.shape} != {b.shape}"
        if key == "kv_ts":
            mask = np.asarray(want["kv_status"]) != 0
            a, b = np.where(mask, a, 0), np.where(mask, b, 0)
        ne = np.argwhere(a != b)
        if len(ne):
            idx = tuple(int(x) for x in ne[0])
            return f"{key}{list(idx)}: got {a[idx]!r} want {b[idx]!r} ({len(ne)} mismatches)"
    return None


class RowOracle:
    """One oracle handle holding copies of selected observer rows of a ``GossipSim`` (one slice)."""

    def __init__(self, sim, cfg: dict):
        from aiocluster_amd.pbsize import nodeid_size

        self.sim = sim
        self.L = orc_mod.lib()
        n, K = sim.n, sim.k
        if sim.shards > 1:
            raise ValueError("RowOracle needs the whole matrix (one slice)")
        ids = sim.node_ids
        self._ns = (C.c_int32 * n)(*[nodeid_size(x.name, x.generation_id, x.gossip_advertise_addr[0],
                                                  x.gossip_advertise_addr[1], x.tls_name) for x in ids])
        self._kl = (C.c_int32 * K)(*[len(k.encode()) for k in sim.keys])
        self._cfg = orc_mod._Cfg(n, K, int(cfg["mtu"]), orc_mod.us(cfg["tombstone_grace_s"]),
                                 float(cfg["phi_threshold"]), int(cfg["window"]), orc_mod.us(cfg["max_interval_s"]),
                                 orc_mod.us(cfg["initial_interval_s"]), orc_mod.us(cfg["dead_grace_s"]))
        self.handles = []
        self.rows: list[int] = []

    def new_handle(self):
        h = self.L.orc_create(C.byref(self._cfg), self._ns, self._kl)
        self.handles.append(h)
        return h

    def close(self):
        for h in self.handles:
            self.L.orc_destroy(h)
        self.handles = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, rows, handles=None, owner=None):
        """Copy observer rows ``rows`` of the device's current state into every handle in ``handles``
        (default: one new handle), or, with ``owner`` (one handle per row), each row into its own
        handle only.  Returns the handles."""
        sim = self.sim
        rows = [int(o) for o in rows]
        handles = handles or [self.new_handle()]
        g = sim._host(rows)
        n, K, Cc = sim.n, sim.k, sim.hist_cap
        hist_ver = np.ascontiguousarray(g["HIST_VER"])
        hist_vid = np.ascontiguousarray(g["HIST_VID"])
        meta = g["HIST_META"]
        hist_vlen = np.ascontiguousarray((meta >> 18).astype(np.int32))
        hist_st = np.ascontiguousarray(((meta >> 16) & 3).astype(np.uint8))
        P = C.c_void_p
        for i, o in enumerate(rows):
            if sim.canonical:
                order = np.arange(n, dtype=np.int32)
            else:
                order = np.ascontiguousarray(g["ORD"][i, : g["ROW"][i, 0]].view(np.int32))

            def c(x, dt=np.uint32):
                return np.ascontiguousarray(np.asarray(x)[:n].astype(dt))

            hb, mv, gc = c(g["HB"][i]), c(g["MV"][i]), c(g["GC"][i])
            fl, fs, fc, st = c(g["FD_LAST"][i]), c(g["FD_SUM"][i]), c(g["FD_CNT"][i]), c(g["FD_STATE"][i])
            held = np.ascontiguousarray(g["HELD"][i, :n, :K])
            ts = np.ascontiguousarray(g["TS"][i, :n, :K]) if "TS" in g else None
            for h in (handles if owner is None else [owner[i]]):
                self.L.orc_load_row(h, o, len(order), order.ctypes.data_as(P), hb.ctypes.data_as(P),
                                    mv.ctypes.data_as(P), gc.ctypes.data_as(P), held.ctypes.data_as(P), Cc,
                                    hist_ver.ctypes.data_as(P), hist_vid.ctypes.data_as(P),
                                    hist_vlen.ctypes.data_as(P), hist_st.ctypes.data_as(P), fl.ctypes.data_as(P),
                                    fs.ctypes.data_as(P), fc.ctypes.data_as(P), st.ctypes.data_as(P), TICK_US)
                if ts is not None:
                    self.L.orc_set_row_ts(h, o, ts.ctypes.data_as(P), TICK_US)
        self.rows = rows
        return handles

    def exchange(self, h, a: int, b: int, tick: int):
        self.L.orc_exchange(h, int(a), int(b), tick * TICK_US)

    def liveness(self, h, o: int, tick: int) -> int:
        return self.L.orc_liveness(h, int(o), tick * TICK_US)

    def export_rows(self, h, rows) -> dict:
        """Rows ``rows`` of handle ``h`` in the device ``export()`` format (times in ticks)."""
        N, K = self.sim.n, self.sim.k
        out = {k: [] for k in EXPORT_FIELDS}
        for o in rows:
            a = {
                "pos": np.empty(N, np.int32), "hb": np.empty(N, np.uint32), "mv": np.empty(N, np.uint32),
                "gc": np.empty(N, np.uint32), "kv_version": np.empty((N, K), np.uint32),
                "kv_status": np.empty((N, K), np.int32), "kv_value_id": np.empty((N, K), np.uint32),
                "kv_ts": np.empty((N, K), np.int64), "fd_last": np.empty(N, np.int64),
                "fd_len": np.empty(N, np.int32), "fd_sum": np.empty(N, np.float64), "live": np.empty(N, np.int32),
                "tod": np.empty(N, np.int64),
            }
            order = list(out)
            self.L.orc_export_row(h, int(o), *[a[k].ctypes.data_as(C.c_void_p) for k in order])
            for k in ("kv_ts", "fd_last", "tod"):
                m = a[k] >= 0
                a[k][m] //= TICK_US
            for k in out:
                out[k].append(a[k])
        return {k: np.stack(v) for k, v in out.items()}

    def stats(self, h) -> dict:
        s = orc_mod._Stats()
        self.L.orc_get_stats(h, C.byref(s))
        return {n: getattr(s, n) for n, _ in orc_mod._Stats._fields_}


def check_phase_rows(sim, cfg: dict, rd: dict, sample: int = 64, phase: int = 0):
    """Full-size parity on a sample: ``sim`` has just run ``gs_begin_round`` of round ``rd``
    (``aiocluster_amd.driver.begin``).  Copies the rows of the first ``sample`` exchanges of phase
    ``phase`` into the oracle, runs that whole phase on the device and closes the round there
    (``gs_liveness`` one tick later), runs the same ``sample`` exchanges and the liveness sweep of
    their rows in the oracle, and returns ``(diff, info)``: the first mismatching (field, row, column)
    between the device rows and the oracle rows (None = bit-identical) and counts of what the
    sampled exchanges did."""
    from aiocluster_amd import driver

    a_all, b_all, n, t = rd["phases"][phase]
    a = a_all[:sample].cpu().numpy().tolist()
    b = b_all[:sample].cpu().numpy().tolist()
    rows = a + b
    assert len(set(rows)) == len(rows), "a phase's exchanges are disjoint"
    ro = RowOracle(sim, cfg)
    (h,) = ro.load(rows)
    driver.run_phases([sim], rd, phases=[rd["phases"][phase]])
    t_live = t + 1
    driver.end([sim], rd, tick=t_live)
    for x, y in zip(a, b):
        ro.exchange(h, x, y, t)
    for o in rows:
        if rd["up_host"][o]:
            ro.liveness(h, o, t_live)
    want = ro.export_rows(h, rows)
    got = sim.export_rows(rows)
    diff = compare_exports(got, want)
    info = {**ro.stats(h), "rows": len(rows)}
    ro.close()
    return diff, info
