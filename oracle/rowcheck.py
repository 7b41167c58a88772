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
    """One oracle handle holding copies of selected observer rows of a ``GossipSim``.

    An owner-column slice (``sim.shards > 1``, canonical) is checked on its own columns: the oracle holds
    the whole cluster's rows, with the slice's columns copied from the device and every other column
    *inert* -- known (canonical), heartbeat 0, max_version 0, no keys, no window, on every loaded row --
    so no exchange between two loaded rows merges, reports or sends anything for it.  That is exact for
    the slice's columns whenever the MTU cannot bind (config 4's contract: a slice's packing does not
    depend on the others); ``export_rows`` returns the slice's columns only."""

    def __init__(self, sim, cfg: dict):
        from aiocluster_amd.pbsize import nodeid_size

        self.sim = sim
        self.L = orc_mod.lib()
        n, K = sim.n, sim.k
        if sim.shards > 1 and not sim.canonical:
            raise ValueError("RowOracle on a slice needs the canonical layout")
        self.lo, self.nc = sim.col_lo, sim.ncol
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

    def load(self, rows, handles=None, owner=None, g=None):
        """Copy observer rows ``rows`` of the device's current state into every handle in ``handles``
        (default: one new handle), or, with ``owner`` (one handle per row), each row into its own
        handle only.  ``g``: host copies of those rows already taken (``join_host_rows``).  Returns the
        handles."""
        sim = self.sim
        rows = [int(o) for o in rows]
        handles = handles or [self.new_handle()]
        g = sim._host(rows) if g is None else g
        n, K = sim.n, sim.k
        lo, nc = self.lo, self.nc

        def full(x, fill=0):
            """owner-indexed array of the slice -> the whole cluster's (inert owners: ``fill``)"""
            x = np.asarray(x)
            if nc == n:
                return np.ascontiguousarray(x[:n])
            out = np.full((n,) + x.shape[1:], fill, dtype=x.dtype)
            out[lo:lo + nc] = x[:nc]
            return out

        Cc = g["HIST_VER"].shape[1]  # hist_cap, or fewer entries (host_rows trims what no loaded row holds)
        hist_ver = full(g["HIST_VER"])
        hist_vid = full(g["HIST_VID"])
        meta = full(g["HIST_META"])
        hist_vlen = np.ascontiguousarray((meta >> 18).astype(np.int32))
        hist_st = np.ascontiguousarray(((meta >> 16) & 3).astype(np.uint8))
        P = C.c_void_p
        for i, o in enumerate(rows):
            if sim.canonical:
                order = np.arange(n, dtype=np.int32)
            else:
                order = np.ascontiguousarray(g["ORD"][i, : g["ROW"][i, 0]].view(np.int32))

            def c(x, dt=np.uint32, fill=0):
                return full(np.asarray(x)[:nc].astype(dt), fill)

            hb, mv, gc = c(g["HB"][i]), c(g["MV"][i]), c(g["GC"][i])
            fl = c(g["FD_LAST"][i], fill=0xFFFFFFFF)
            fs, fc, st = c(g["FD_SUM"][i]), c(g["FD_CNT"][i]), c(g["FD_STATE"][i])
            held = full(g["HELD"][i, :nc, :K])
            ts = full(g["TS"][i, :nc, :K], 0xFFFFFFFF) if "TS" in g else None
            ring = self._ring(o)
            for h in (handles if owner is None else [owner[i]]):
                self.L.orc_load_row(h, o, len(order), order.ctypes.data_as(P), hb.ctypes.data_as(P),
                                    mv.ctypes.data_as(P), gc.ctypes.data_as(P), held.ctypes.data_as(P), Cc,
                                    hist_ver.ctypes.data_as(P), hist_vid.ctypes.data_as(P),
                                    hist_vlen.ctypes.data_as(P), hist_st.ctypes.data_as(P), fl.ctypes.data_as(P),
                                    fs.ctypes.data_as(P), fc.ctypes.data_as(P), st.ctypes.data_as(P), TICK_US)
                if ts is not None:
                    self.L.orc_set_row_ts(h, o, ts.ctypes.data_as(P), TICK_US)
                if ring is not None:  # the row's interval rings: exact eviction from here on
                    self.L.orc_set_row_ring(h, o, ring.ctypes.data_as(P), fc.ctypes.data_as(P), TICK_US)
        self.rows = rows
        return handles

    def _ring(self, o: int):
        """Observer row o's interval rings as u16 [N][W] ticks (whole-cluster owner indexing), if it has any:
        every row with GS_FD_RING, the sampled rows with gs_config.ring_rows; else None."""
        sim = self.sim
        from aiocluster_amd._lib import GS_FD_RING

        if sim.flags & GS_FD_RING:
            slot = o
        elif o in getattr(sim, "ring_rows", []):
            slot = sim.ring_rows.index(o)
        else:
            return None
        W = int(sim.cfg["window"])
        t = sim.regions["RING"].view(sim.torch.int16).view(-1, sim.np_, W)[slot, : self.nc]
        r = t.cpu().numpy().view(np.uint16)
        n = sim.n
        if self.nc == n:
            return np.ascontiguousarray(r)
        out = np.zeros((n, W), np.uint16)
        out[self.lo:self.lo + self.nc] = r
        return out

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
                out[k].append(a[k][self.lo:self.lo + self.nc])  # a slice: its own columns
        return {k: np.stack(v) for k, v in out.items()}

    def stats(self, h) -> dict:
        s = orc_mod._Stats()
        self.L.orc_get_stats(h, C.byref(s))
        return {n: getattr(s, n) for n, _ in orc_mod._Stats._fields_}


def check_round_rows(sim, cfg: dict, rd: dict, sample: int = 32, seed: int = 0, group=None, only_rows=None):
    """Full-size parity over EVERY phase of round ``rd`` (``sim`` has just run its ``gs_begin_round``).

    Phase p: ``sample`` exchanges drawn at random from the phase; their rows are copied into a fresh
    oracle handle after the device has applied the round's pending reports so far (``gs_flush_reports``:
    the windows then hold phases 0..p-1), the whole phase runs on the device and the sample in the oracle,
    the device applies the new reports, and the rows must be bit-identical (every field; membership only
    changes at liveness).  The last phase is closed by the liveness sweep on both sides instead.  Rows of
    later phases have been merged by several phases of this round.  ``only_rows``: sample only exchanges
    with an endpoint in this set and compare only those rows (e.g. the sampled ring rows: the partner's
    row is loaded to run the exchange, its windows are not compared).  Returns ``(diff, info)``."""
    from aiocluster_amd import driver

    rng = np.random.default_rng(seed)
    sims = group.slices if group is not None else [sim]
    phases = [p for p in rd["phases"] if p[2]]
    info = {"phases": len(phases), "rows": 0, "node_deltas": 0, "hb_reports": 0, "truncated": 0}
    keep = None if only_rows is None else set(int(x) for x in only_rows)
    for i, (a_all, b_all, n, t) in enumerate(phases):
        last = i == len(phases) - 1
        an, bn = a_all.cpu().numpy(), b_all.cpu().numpy()
        pool = np.arange(n) if keep is None else np.flatnonzero(
            np.isin(an, list(keep)) | np.isin(bn, list(keep)))
        pick = np.sort(rng.choice(pool, size=min(sample, len(pool)), replace=False))
        a = an[pick].tolist()
        b = bn[pick].tolist()
        rows = a + b
        cmp_rows = rows if keep is None else [o for o in rows if o in keep]
        for s_ in sims:
            s_.flush_reports(t - 1)
        ro = RowOracle(sim, cfg)
        (h,) = ro.load(rows) if rows else (ro.new_handle(),)
        driver.run_phases(sims, rd, phases=[(a_all, b_all, n, t)], group=group)
        if last:
            driver.end(sims, rd, tick=t + 1)
        else:
            for s_ in sims:
                s_.flush_reports(t)
        for x, y in zip(a, b):
            ro.exchange(h, x, y, t)
        if last:
            for o in rows:
                if rd["up_host"][o]:
                    ro.liveness(h, o, t + 1)
        # a phase with no sampled exchange on ``only_rows`` (a small third matching) still runs on the device
        diff = compare_exports(sim.export_rows(cmp_rows), ro.export_rows(h, cmp_rows)) if cmp_rows else None
        st = ro.stats(h)
        ro.close()
        info["rows"] += len(cmp_rows)
        for k in ("node_deltas", "hb_reports", "truncated"):
            info[k] += st[k]
        if diff is not None:
            return f"phase {i} (tick {t}): {diff}", info
    return None, info


def check_phase_rows(sim, cfg: dict, rd: dict, sample: int = 64, phase: int = 0, group=None):
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
    sims = group.slices if group is not None else [sim]
    driver.run_phases(sims, rd, phases=[rd["phases"][phase]], group=group)
    t_live = t + 1
    driver.end(sims, rd, tick=t_live)
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


# -- the whole cluster's rows from owner-column slices (multi-GPU bench parity: VERDICT r5 item 5)


class ClusterView:
    """The attributes ``RowOracle`` reads of a ``GossipSim``, for the WHOLE cluster of a sliced run: rows loaded
    from host copies joined over every slice (``join_host_rows``), so the oracle holds complete rows and the
    check is exact whatever the MTU does (no inert columns)."""

    def __init__(self, sim, hist_cap: int):
        self.n, self.k, self.hist_cap = sim.n, sim.k, hist_cap
        self.canonical, self.shards, self.col_lo, self.ncol = True, 1, 0, sim.n
        self.node_ids, self.keys = sim.node_ids, sim.keys
        self.flags, self.ring_rows = 0, []


def host_rows(sim, g: dict, cmax: int | None = None) -> dict:
    """Host copies ``g`` (``sim._host(rows)``) of observer rows of one slice, cut to the slice's own columns
    (``[:, :ncol]``), with the owner tables (HIST_*) cut to their first ``cmax`` write ordinals (default: all)."""
    nc = sim.ncol
    out = {"col_lo": sim.col_lo, "ncol": nc}
    for k, v in g.items():
        if k == "rows" or k in ("ROW", "ORD"):
            out[k] = v
        elif k.startswith("HIST_"):
            out[k] = np.ascontiguousarray(v[:, :cmax]) if cmax is not None else v
        else:
            out[k] = np.ascontiguousarray(v[:, :nc])
    return out


def join_host_rows(parts: list[dict]) -> dict:
    """``host_rows`` of every slice, in slice order, joined along the owner axis into whole-cluster rows."""
    parts = sorted(parts, key=lambda p: p["col_lo"])
    lo = 0
    for p in parts:
        if p["col_lo"] != lo:
            raise ValueError(f"slices do not tile the owner columns: {p['col_lo']} != {lo}")
        lo += p["ncol"]
    g = {"rows": parts[0]["rows"], "ROW": parts[0]["ROW"]}
    for k in parts[0]:
        if k in ("rows", "ROW", "ORD", "col_lo", "ncol"):
            continue
        g[k] = np.concatenate([p[k] for p in parts], axis=0 if k.startswith("HIST_") else 1)
    return g


def check_sliced_phase_rows(group, cfg: dict, rd: dict, sample: int = 16, phase: int = 0, comm=None):
    """Full-size parity of a SLICED cluster (one slice per rank, or G slices in this process): ``group`` (a
    ``ShardGroup``) has just run ``gs_begin_round`` of round ``rd``.  The rows of the first ``sample`` exchanges
    of phase ``phase`` are copied out of every slice and joined on rank 0 into whole-cluster rows (all owner
    columns: the MTU walk across slices is checked too, unlike the inert-column ``RowOracle`` of one slice); the
    whole phase then runs on the devices through the group's own sliced driver (count, gather, pack, chain steps)
    and the round is closed by the liveness sweep; rank 0 runs the sampled exchanges and the liveness of their
    rows in the oracle and compares every slice's columns of the device rows with the oracle's.

    ``comm``: object collectives ``gather(list) -> list | None`` (every slice's objects on rank 0) and
    ``allmax(int) -> int``; default: the slices of this process only.  Returns, on rank 0, a list with one dict
    per slice ({"slice", "cols": [lo, hi), "rows", "diff", "exact"}) and an info dict; ``(None, None)``
    elsewhere."""
    from aiocluster_amd import driver

    sims = group.slices
    gather = comm.gather if comm is not None else (lambda xs: xs)
    allmax = comm.allmax if comm is not None else (lambda x: x)
    a_all, b_all, n, t = rd["phases"][phase]
    a = a_all[:sample].cpu().numpy().tolist()
    b = b_all[:sample].cpu().numpy().tolist()
    rows = a + b
    assert len(set(rows)) == len(rows), "a phase's exchanges are disjoint"
    gs = [s_._host(rows) for s_ in sims]
    # the oracle's owner tables need the write ordinals the loaded rows hold (not hist_cap of them)
    cmax = allmax(max(int(g_["HELD"][:, : s_.ncol].max()) for s_, g_ in zip(sims, gs))) + 1
    before = gather([host_rows(s_, g_, cmax) for s_, g_ in zip(sims, gs)])
    del gs
    driver.run_phases(sims, rd, phases=[rd["phases"][phase]], group=group)
    driver.end(sims, rd, tick=t + 1)
    after = gather([(s_.col_lo, s_.ncol, s_.export_rows(rows)) for s_ in sims])
    if before is None:
        return None, None
    g = join_host_rows(before)
    view = ClusterView(sims[0], cmax)
    ro = RowOracle(view, cfg)
    (h,) = ro.load(rows, g=g)
    for x, y in zip(a, b):
        ro.exchange(h, x, y, t)
    for o in rows:
        if rd["up_host"][o]:
            ro.liveness(h, o, t + 1)
    want = ro.export_rows(h, rows)
    st = ro.stats(h)
    ro.close()
    res = []
    for i, (lo, nc, got) in enumerate(sorted(after, key=lambda x: x[0])):
        w = {k: v[:, lo:lo + nc] for k, v in want.items()}
        diff = compare_exports(got, w)
        res.append({"slice": i, "cols": [int(lo), int(lo + nc)], "rows": len(rows), "diff": diff,
                    "exact": diff is None})
    info = {"exchanges": len(a), "rows": len(rows), "tick": int(t), "hist_entries": int(cmax),
            **{k: int(st[k]) for k in ("node_deltas", "hb_reports", "truncated")}}
    return res, info
