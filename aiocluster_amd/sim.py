"""Host side of the MI355X batched gossip backend.

``GossipSim`` holds a whole simulated aiocluster cluster in HBM and drives the
hand-written gfx950 kernels of ``csrc/gossip_sim.hip`` through the C ABI of
``include/gossip_sim.h``.  PyTorch is used only to allocate the device regions
and to provide the HIP stream.  There is no CPU fallback: without the HIP
library (or without a GPU) construction raises.

The public methods mirror the reference call sites the backend replaces
(``aiocluster/server.py`` and ``aiocluster/state.py``):

==============================  ==========================================================
``GossipSim``                   reference
==============================  ==========================================================
``set/delete/set_with_ttl/      ``Cluster.set/...`` -> ``NodeState.set/...``
delete_after_ttl``              (server.py:193-215, state.py:137-180)
``begin_round``                 ``_gossip_multiple``: inc_heartbeat + gc_marked_for_deletion
                                (server.py:471-474)
``run_phase``                   ``_gossip`` / ``_handle_message`` for a set of disjoint pairs
                                (server.py:327-376, 523-568)
``update_node_liveness``        ``_update_node_liveness`` (server.py:606-620)
``node_state``, ``snapshot``,   ``ClusterState.node_state``, ``Cluster.snapshot``,
``live_nodes``, ``dead_nodes``, ``FailureDetector.live_nodes/dead_nodes/phi``
``phi``
==============================  ==========================================================
"""

from __future__ import annotations

import ctypes as C
import math
from datetime import timedelta

import numpy as np

from . import _lib
from ._lib import (GS_CANONICAL, GS_FD_RING, GS_HB8, GS_MV8, GS_NO_HELD, GS_NONE, GS_SLICED, GS_TOMBSTONES, REGION,
                   TICK_US, GsError)
from .entities import ClusterSnapshot, NodeId, NodeState, VersionedValue, VersionStatusEnum
from .pbsize import nodeid_size

OPS = {"set": 0, "delete": 1, "set_with_ttl": 2, "delete_after_ttl": 3}


def _us(seconds: float) -> int:
    return timedelta(seconds=seconds) // timedelta(microseconds=1)


def _ticks(seconds: float, what: str) -> int:
    us = _us(seconds)
    if us % TICK_US:
        raise ValueError(f"{what}={seconds}s is not a whole number of 1/64 s ticks")
    return us // TICK_US


def sched_delay_ticks(dead_grace_s: float) -> int:
    """Smallest tick count d with d*TICK_US >= dead_grace/2.0 as timedelta rounds it (half to even)."""
    g = _us(dead_grace_s)
    half = g // 2
    if (g & 1) and (half & 1):
        half += 1
    return -(-half // TICK_US)


FD_WIN, FD_OLD, FD_OLD_AGE = 4, 8, 1 << 15


def unpack_fd(st8, last16, sc, tick: int, sum_bits: int):
    """Host restatement of the device's fd_get (gossip_sim.hip): see GossipSim.unpack_fd."""
    st8 = np.asarray(st8).view(np.uint8).astype(np.uint32)
    l16 = np.asarray(last16).view(np.uint16).astype(np.int64)
    sc = np.asarray(sc).view(np.uint32)
    t = np.int64(tick)
    last = np.where(st8 & FD_OLD, t - FD_OLD_AGE, t - ((t - l16) & 0xFFFF)) & 0xFFFFFFFF
    last = np.where(st8 & FD_WIN, last, GS_NONE).astype(np.uint32)
    return last, sc & np.uint32((1 << sum_bits) - 1), sc >> np.uint32(sum_bits)


def fd_state_word(st8: np.ndarray, tod: np.ndarray) -> np.ndarray:
    """GS_R_FD_STATE (u8: 0 unknown, 1 live, 2 dead) + GS_R_FD_TOD (time of death) as one u32 per pair:
    0 unknown, 1 live, tick of death + 2 for a dead pair (the readback format of export / snapshot)."""
    st8 = np.asarray(st8).view(np.uint8) & np.uint8(3)
    tod = np.asarray(tod).view(np.uint32)
    return np.where(st8 == 2, tod + np.uint32(2), st8.astype(np.uint32)).astype(np.uint32)


def order_events(ev: np.ndarray, n: int, phases: dict, wmap: list) -> np.ndarray:
    """Permutation putting device event records (uint32 [m, 8], gs_set_events) in the reference's order:
    by tick; owner writes by call order (``wmap``: record seq -> call index); in a phase (``phases``:
    tick -> (initiators, responders)) by exchange index, the initiator's apply (SynAck delta,
    server.py:351-353) before the responder's (Ack delta, 372-376), then the NodeDelta order (seq = the
    sender's dict position, state.py:346-413), then kv version; join / leave by observer, joins first,
    then node (the reference iterates sets there, server.py:611-614)."""
    m = len(ev)
    t = ev[:, 5].astype(np.int64)
    kind = (ev[:, 2] >> 8).astype(np.int64)
    seq = ev[:, 6].astype(np.int64)
    obs = ev[:, 0].astype(np.int64)
    k1, k2, k3, k4 = (np.zeros(m, np.int64) for _ in range(4))
    lv = kind != 0
    k1[lv], k2[lv], k3[lv] = obs[lv], kind[lv], ev[lv, 1]
    kc = ~lv
    wm = np.asarray(wmap, dtype=np.int64)
    for tick in np.unique(t[kc]).tolist():
        sel = kc & (t == tick)
        ph = phases.get(tick)
        if ph is None:  # owner writes (a seq the map does not cover: after every mapped write, in seq order)
            sq = seq[sel]
            k1[sel] = np.where(sq < len(wm), wm[np.minimum(sq, len(wm) - 1)], len(wm) + sq) if len(wm) else sq
            continue
        a, b = (np.asarray(x, dtype=np.int64) for x in ph)
        ex = np.full(n, -1, np.int64)
        side = np.zeros(n, np.int64)
        ex[a] = np.arange(len(a))
        ex[b] = np.arange(len(b))
        side[b] = 1
        k1[sel], k2[sel], k3[sel], k4[sel] = ex[obs[sel]], side[obs[sel]], seq[sel], ev[sel, 4]
    return np.lexsort((k4, k3, k2, k1, t))


def make_config(n: int, k: int, cfg: dict, flags: int, hist_cap: int, shards: int = 1,
                shard: int = 0, ring_rows: int = 0) -> _lib.GsConfig:
    c = _lib.GsConfig()
    c.n_shards = shards
    c.shard = shard
    c.ring_rows = ring_rows
    c.n_nodes = n
    c.n_keys = k
    c.hist_cap = hist_cap
    c.mtu = int(cfg["mtu"])
    c.flags = flags
    c.window = int(cfg["window"])
    c.max_interval_ticks = _ticks(cfg["max_interval_s"], "max_interval")
    c.tombstone_grace_ticks = _ticks(cfg["tombstone_grace_s"], "marked_for_deletion_grace_period")
    c.dead_grace_ticks = _ticks(cfg["dead_grace_s"], "dead_node_grace_period")
    c.sched_delay_ticks = sched_delay_ticks(cfg["dead_grace_s"])
    c.phi_threshold = float(cfg["phi_threshold"])
    # SamplingWindow: _prev_weight * _prev_mean (failure_detector.py:22-23, 51)
    c.prior_weighted = 5.0 * timedelta(seconds=cfg["initial_interval_s"]).total_seconds()
    return c


def split_owner_batches(ops: list[tuple]) -> list[list[tuple]]:
    """Split owner writes ``(tick, owner, ...)`` into device batches of distinct owners.

    ``k_owner_writes`` runs one thread per write, so two writes of one owner must
    not share a batch; the i-th write of an owner goes to batch i, which keeps
    every owner's writes in call order (what NodeState.set/... sequences need).
    """
    batches: list[list[tuple]] = []
    seen: dict[int, int] = {}
    for op in ops:
        j = op[1]
        b = seen.get(j, 0)
        seen[j] = b + 1
        while len(batches) <= b:
            batches.append([])
        batches[b].append(op)
    return batches


class GossipSim:
    """A simulated cluster of ``len(node_ids)`` aiocluster nodes resident on one MI355X.

    With ``shards > 1`` this object holds one owner-column slice of the cluster (every
    observer row, columns ``[col_lo, col_lo + ncol)``); the slices of a cluster are
    driven together by ``aiocluster_amd.shard.ShardGroup``.
    """

    def __init__(self, node_ids: list[NodeId], keys: list[str], cfg: dict, init: str = "cold",
                 initial_values: dict[int, list[tuple[int, str]]] | None = None, *, device: str = "cuda:0",
                 tombstones: bool = True, fd_ring: bool | None = None, hist_cap: int = 64,
                 nid_sizes: list[int] | None = None, initial_ops: list[np.ndarray] | None = None,
                 canonical: bool | None = None, shards: int = 1, shard: int = 0, held: bool = True,
                 ring_rows=None, hb8: bool = False, mv8: bool = False, sliced: bool = False, esc_cols: int | None = None):
        import torch

        if not torch.cuda.is_available():
            raise GsError("GossipSim needs a ROCm GPU (no CPU fallback)")
        self.torch = torch
        self.L = _lib.load()
        self.device = torch.device(device)
        self.n = n = len(node_ids) if node_ids is not None else len(nid_sizes)
        self.node_ids = node_ids
        self.keys = list(keys)
        self.k = k = len(keys)
        self.cfg = dict(cfg)
        self.shards, self.shard = shards, shard
        self.col_lo, self.ncol = _lib.slice_columns(n, shards, shard)
        self.np_ = (self.ncol + 63) // 64 * 64
        self.kp = (k + 3) // 4 * 4
        self.hist_cap = hist_cap
        self.init = init
        flags = 0
        if canonical is None:
            canonical = init == "warm"
        if canonical and init != "warm":
            raise GsError("the canonical layout needs a warm start")
        if canonical:
            flags |= GS_CANONICAL
        if tombstones:
            flags |= GS_TOMBSTONES
        if not held:  # version-only: every view must stay a prefix S_j(max_version) (GS_NO_HELD)
            if tombstones:
                raise GsError("held=False (GS_NO_HELD) needs tombstones=False")
            flags |= GS_NO_HELD
        # 8-bit heartbeat views (GS_HB8: canonical record phases, K <= 16; exact while every view lags its owner
        # by < 2^8, swept every <= 64 round starts + phases, err_hb_lag at 128)
        self.hb8 = bool(hb8)
        if hb8:
            flags |= GS_HB8
        # 8-bit max_version views (GS_MV8, with GS_HB8 and no tombstones; exact while every view lags its owner
        # by < 2^7 versions, swept every <= 64 owner-write calls, err_hb_lag at 64)
        self.mv8 = bool(mv8)
        if mv8:
            flags |= GS_MV8
        # GS_SLICED: the sliced phase path (count, gather, pack) even with one slice -- the multi-GPU code on
        # one GPU (a world-1 RCCL communicator or process group); phases then go through ShardGroup
        self.sliced = shards > 1 or bool(sliced)
        if sliced:
            flags |= GS_SLICED
        W = int(cfg["window"])
        # sampled rings: these observer rows keep interval rings (exact eviction), the others compact windows
        self.ring_rows = sorted(set(int(x) for x in ring_rows)) if ring_rows else []
        if fd_ring is None:
            fd_ring = not self.ring_rows and n * ((n + 63) // 64 * 64) * W * 2 <= (1 << 30)  # whole-cluster rule
        if fd_ring:
            flags |= GS_FD_RING
        self.flags = flags
        self.canonical = bool(flags & GS_CANONICAL)
        c = make_config(n, k, cfg, flags, hist_cap, shards, shard, len(self.ring_rows))
        # escape slots for owner columns whose 8-bit views fall >= 2^7 behind (GS_MV8): 256 by default
        c.esc_cols = (256 if esc_cols is None else int(esc_cols)) if mv8 else 0
        self.c_esc_cols = c.esc_cols
        h = C.c_void_p()
        rc = self.L.gs_create(C.byref(c), C.byref(h))
        if rc:
            raise GsError(f"gs_create failed ({_lib.ERRORS.get(rc, rc)}): invalid config {cfg}")
        self.h = h
        self.regions = {}
        try:
            for name, idx in REGION.items():
                nb = C.c_uint64()
                self._chk(self.L.gs_region_bytes(h, idx, C.byref(nb)), "gs_region_bytes")
                if nb.value:
                    t = torch.empty(int(nb.value), dtype=torch.uint8, device=self.device)
                    self.regions[name] = t
                    self._chk(self.L.gs_bind(h, idx, C.c_void_p(t.data_ptr())), "gs_bind")
            self.stream = torch.cuda.current_stream(self.device)
            self._chk(self.L.gs_set_stream(h, C.c_void_p(self.stream.cuda_stream)), "gs_set_stream")
            if nid_sizes is None:
                nid_sizes = [nodeid_size(x.name, x.generation_id, x.gossip_advertise_addr[0],
                                         x.gossip_advertise_addr[1], x.tls_name) for x in node_ids]
            ns = np.asarray(nid_sizes, dtype=np.uint16)
            kl = np.asarray([len(s.encode()) for s in self.keys], dtype=np.uint8)
            self._chk(self.L.gs_boot(h, ns.ctypes.data_as(C.c_void_p), kl.ctypes.data_as(C.c_void_p)), "gs_boot")
            if self.ring_rows:
                rr = np.asarray(self.ring_rows, dtype=np.uint32)
                self._chk(self.L.gs_set_ring_rows(h, rr.ctypes.data_as(C.c_void_p), len(rr)), "gs_set_ring_rows")
        except Exception:
            self.close()
            raise
        self.values = [""]
        self.value_ids = {"": 0}
        self._pending: list[tuple] = []
        self._ev = self._ev_count = None  # hook events off (enable_events)
        self._ev_phases: dict = {}
        self._ev_wmap: list[int] = []
        self._ev_writes = 0
        self.last_tick = 0
        self.q9_events: list = []
        if initial_values:
            for j in range(n):
                for kk, v in initial_values.get(j, []):
                    self.write(0, j, kk, 0, v)
            self._flush()
        for batch in initial_ops or []:  # pre-interned boot writes (owner, key, op, value_id, value_len)
            self.owner_writes(batch, 0)
        if init == "warm":
            self._chk(self.L.gs_warm(h), "gs_warm")

    # ------------------------------------------------------------------ plumbing
    def _chk(self, rc: int, what: str):
        if rc:
            msg = self.L.gs_last_error(self.h).decode() if getattr(self, "h", None) else ""
            raise GsError(f"{what}: {_lib.ERRORS.get(rc, rc)} {msg}")

    def close(self):
        h = getattr(self, "h", None)
        if h:
            self.L.gs_destroy(h)
            self.h = None
        self.regions = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def region(self, name: str, dtype, shape):
        return self.regions[name].view(dtype).view(*shape)

    def intern(self, value: str) -> int:
        vid = self.value_ids.get(value)
        if vid is None:
            vid = len(self.values)
            self.values.append(value)
            self.value_ids[value] = vid
        return vid

    def _dev(self, arr: np.ndarray, dtype):
        return self.torch.from_numpy(np.ascontiguousarray(arr)).to(self.device, non_blocking=False).view(dtype)

    # --------------------------------------------------------------- owner writes
    def write(self, t: int, j: int, k: int, op: int, value: str):
        if op in (1, 2, 3) and not self.flags & GS_TOMBSTONES:
            raise GsError("deletes / TTL writes need tombstones=True (GS_TOMBSTONES)")
        # interned at call time, so ids follow the caller's write order (as the oracle's do)
        self._pending.append((t, j, k, op, self.intern(value), len(value.encode()), self._ev_writes))
        self._ev_writes += 1

    def set(self, t: int, owner: int, key: str, value: str):
        self.write(t, owner, self.keys.index(key), 0, value)

    def delete(self, t: int, owner: int, key: str):
        self.write(t, owner, self.keys.index(key), 1, "")

    def set_with_ttl(self, t: int, owner: int, key: str, value: str):
        self.write(t, owner, self.keys.index(key), 2, value)

    def delete_after_ttl(self, t: int, owner: int, key: str):
        self.write(t, owner, self.keys.index(key), 3, "")

    def _flush(self):
        if not self._pending:
            return
        batches = split_owner_batches(self._pending)
        self._pending = []
        for batch in batches:
            ticks = {x[0] for x in batch}
            for tick in sorted(ticks):
                rows = [[j, k, op, vid, vl] for t, j, k, op, vid, vl, _ in batch if t == tick]
                self.owner_writes(np.asarray(rows, dtype=np.uint32), tick,
                                  order=[w for t, *_, w in batch if t == tick])

    def owner_writes(self, ops: np.ndarray, tick: int, order: list[int] | None = None):
        """Device batch of owner writes; ``ops`` is uint32 [m, 5] (owner, key, op, value_id, value_len).
        ``order``: each op's index among the caller's writes (hook-event order); default: after every
        write so far, in row order."""
        if len(ops) == 0:
            return
        ops = np.ascontiguousarray(ops, dtype=np.uint32)
        if len(np.unique(ops[:, 0])) != len(ops):
            raise GsError("owner_writes: owners must be distinct within one batch")
        d = self._dev(ops.view(np.int32), self.torch.int32)
        self._chk(self.L.gs_owner_writes(self.h, C.c_void_p(d.data_ptr()), len(ops), tick), "gs_owner_writes")
        if self._ev is not None:  # gs_set_events: op i of this call has seq = ops issued before + i
            if order is None:
                order = list(range(self._ev_writes, self._ev_writes + len(ops)))
                self._ev_writes += len(ops)
            self._ev_wmap += list(order)

    # --------------------------------------------------------------- round driver
    def begin_round(self, t: int, up):
        self._flush()
        u = up if hasattr(up, "data_ptr") else self._dev(np.asarray(up, dtype=np.uint8), self.torch.uint8)
        self._chk(self.L.gs_begin_round(self.h, C.c_void_p(u.data_ptr()), t), "gs_begin_round")

    def run_phase(self, t: int, pairs):
        self._flush()
        if len(pairs) == 0:
            return
        arr = np.asarray(pairs, dtype=np.int32).reshape(-1, 2)
        self.run_phase_arrays(t, arr[:, 0], arr[:, 1])

    def _pairs_dev(self, initiators, responders):
        ini = initiators if hasattr(initiators, "data_ptr") else self._dev(np.asarray(initiators, np.int32),
                                                                           self.torch.int32)
        res = responders if hasattr(responders, "data_ptr") else self._dev(np.asarray(responders, np.int32),
                                                                           self.torch.int32)
        return ini, res

    def run_phase_arrays(self, t: int, initiators, responders):
        if self.sliced:
            raise GsError("a column slice runs phases through ShardGroup (gs_phase_count / gs_phase_pack)")
        ini, res = self._pairs_dev(initiators, responders)
        n = int(ini.numel())
        if n == 0:
            return
        if self._ev is not None:
            self._ev_phases[t] = (ini.cpu().numpy().astype(np.int64), res.cpu().numpy().astype(np.int64))
        self._chk(self.L.gs_run_phase(self.h, C.c_void_p(ini.data_ptr()), C.c_void_p(res.data_ptr()), n, t),
                  "gs_run_phase")

    # ------------------------------------------------------- sliced phases (shards > 1)
    def phase_count(self, t: int, ini, res, out=None):
        """gs_phase_count: pass 1 on this slice; returns the device u64 slice totals [n, 2] (as int64)."""
        n = int(ini.numel())
        if out is None:
            out = self.torch.empty((n, 2), dtype=self.torch.int64, device=self.device)
        self._chk(self.L.gs_phase_count(self.h, C.c_void_p(ini.data_ptr()), C.c_void_p(res.data_ptr()), n, t,
                                        C.c_void_p(out.data_ptr())), "gs_phase_count")
        return out

    def phase_pack(self, t: int, ini, res, step: int, tot_all, chain_all, chain):
        """gs_phase_pack step ``step``; ``tot_all``/``chain_all`` are the gathered [G, n, 2] tensors."""
        n = int(ini.numel())
        ca = C.c_void_p(chain_all.data_ptr()) if chain_all is not None else None
        self._chk(self.L.gs_phase_pack(self.h, C.c_void_p(ini.data_ptr()), C.c_void_p(res.data_ptr()), n, t, step,
                                       C.c_void_p(tot_all.data_ptr()), ca, C.c_void_p(chain.data_ptr())),
                  "gs_phase_pack")
        return chain

    @property
    def has_records(self) -> bool:
        """Candidate records are allocated (canonical layout): the compacted chain is available."""
        return "CAND" in self.regions

    def phase_overflow(self, tot_all, chain, list_buf, chainc, read: bool = True):
        """gs_phase_overflow: the overflowing slots into list_buf, this slice's states into chainc; with
        ``read`` (blocking) returns their number."""
        n = int(chain.shape[0])
        cnt = C.c_uint32()
        self._chk(self.L.gs_phase_overflow(self.h, n, C.c_void_p(tot_all.data_ptr()), C.c_void_p(chain.data_ptr()),
                                           C.c_void_p(list_buf.data_ptr()), C.c_void_p(chainc.data_ptr()),
                                           C.byref(cnt) if read else None), "gs_phase_overflow")
        return int(cnt.value) if read else None

    def phase_chain(self, t: int, ini, res, step: int, list_buf, count: int, chain_all, chain, chainc, tot_all):
        """gs_phase_chain step ``step`` over the ``count`` listed slots (chain_all = gathered [G, count + 1],
        entry count = that slice's pending slots; tot_all = the phase's gathered slice totals)."""
        n = int(ini.numel())
        self._chk(self.L.gs_phase_chain(self.h, C.c_void_p(ini.data_ptr()), C.c_void_p(res.data_ptr()), n, t, step,
                                        C.c_void_p(list_buf.data_ptr()), count, C.c_void_p(chain_all.data_ptr()),
                                        C.c_void_p(chain.data_ptr()), C.c_void_p(chainc.data_ptr()),
                                        C.c_void_p(tot_all.data_ptr())),
                  "gs_phase_chain")

    def phase_pending(self, n: int, list_buf, count: int, chain_all) -> tuple[int, int]:
        """gs_phase_pending: (the listed slots still pending over all slices -- -1 when the device count exceeds
        GS_CHAIN_CAP --, the count) after a chain step; ``count`` = GS_CHAIN_DEVICE reads it from ``list_buf``."""
        pend, cnt = C.c_uint64(), C.c_uint32()
        ca = chain_all if chain_all.device == self.device else chain_all.to(self.device)
        self._chk(self.L.gs_phase_pending(self.h, n, C.c_void_p(list_buf.data_ptr()), count, C.c_void_p(ca.data_ptr()),
                                          C.byref(pend), C.byref(cnt)), "gs_phase_pending")
        p = int(pend.value)
        return (-1 if p == (1 << 64) - 1 else p), int(cnt.value)

    def flush_reports(self, t: int):
        """gs_flush_reports: apply the open round's pending heartbeat reports to the windows now (a
        mid-round readback of GS_R_FD); the next phase must come after ``t``."""
        self._chk(self.L.gs_flush_reports(self.h, t), "gs_flush_reports")

    def update_node_liveness(self, t: int, up):
        self._flush()
        u = up if hasattr(up, "data_ptr") else self._dev(np.asarray(up, dtype=np.uint8), self.torch.uint8)
        self._chk(self.L.gs_liveness(self.h, C.c_void_p(u.data_ptr()), t), "gs_liveness")
        self.last_tick = t

    def liveness(self, t: int, up, r: int = -1):
        self.update_node_liveness(t, up)

    # --------------------------------------------------------------- counters
    def counters(self) -> dict:
        c = _lib.GsCounters()
        self._chk(self.L.gs_read_counters(self.h, C.byref(c)), "gs_read_counters")
        return {n: int(getattr(c, n)) for n in _lib.COUNTER_FIELDS}

    def reset_counters(self):
        self._chk(self.L.gs_reset_counters(self.h), "gs_reset_counters")

    def set_timing(self, on: bool = True):
        """gs_set_timing: HIP events around every pass-1 / packing / liveness launch (measurement)."""
        self._chk(self.L.gs_set_timing(self.h, 1 if on else 0), "gs_set_timing")

    def kernel_times(self) -> dict:
        """gs_kernel_times (blocking): {kind: (ms summed, launches)} since the previous call."""
        kt = _lib.GsKtimes()
        self._chk(self.L.gs_kernel_times(self.h, C.byref(kt)), "gs_kernel_times")
        return {k: (kt.ms[i], int(kt.launches[i])) for i, k in enumerate(_lib.KT_KINDS)}

    def check(self, accept_saturated: bool = False) -> dict:
        """Raise if any device-side check failed; return the counters.  With sampled rings (``ring_rows``) a
        compact row's window that would need an eviction is counted in fd_saturated: the ring rows stay exact,
        the compact rows do not (BoundedArrayStats, failure_detector.py:131-162), so that raises too unless the
        caller accepts the sampled-ring contract (``accept_saturated``)."""
        c = self.counters()
        errs = {k: v for k, v in c.items() if k.startswith("err_") and v}
        if c["fd_saturated"] and not accept_saturated:
            errs["fd_saturated"] = c["fd_saturated"]
        if errs.get("err_fd_gc"):
            raise GsError(f"FailureDetector.garbage_collect is due in a canonical (warm, index-order) state; "
                          f"removing nodes needs the general layout (init='cold' or canonical=False): {errs}")
        if errs:
            raise GsError(f"device checks failed: {errs}")
        return c

    def sync(self):
        self._chk(self.L.gs_sync(self.h), "gs_sync")

    def check_heartbeat_lag(self):
        """gs_check_heartbeat_lag: count views lagging their owner by >= 2^15 heartbeats in err_hb_lag
        (gs_begin_round also runs it every 2^14 round starts + phases)."""
        self._chk(self.L.gs_check_heartbeat_lag(self.h), "gs_check_heartbeat_lag")

    # --------------------------------------------------------------- hook events
    def enable_events(self, capacity: int = 1 << 20):
        """gs_set_events: record on_key_change / on_node_join / on_node_leave (see drain_events)."""
        torch = self.torch
        self._ev = torch.empty((capacity, 8), dtype=torch.int32, device=self.device)
        self._ev_phases = {}  # phase tick -> (initiators, responders): the exchange order of that phase
        self._ev_wmap = []    # owner-write seq -> index among the caller's writes since enable_events
        # writes queued before this call (not yet flushed) are the first ones of the new numbering
        self._pending = [(*w[:-1], i) for i, w in enumerate(self._pending)]
        self._ev_writes = len(self._pending)
        self._ev_count = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._chk(self.L.gs_set_events(self.h, C.c_void_p(self._ev.data_ptr()), capacity,
                                       C.c_void_p(self._ev_count.data_ptr())), "gs_set_events")

    def disable_events(self):
        self._chk(self.L.gs_set_events(self.h, None, 0, None), "gs_set_events")
        self._ev = self._ev_count = None

    def drain_events(self) -> np.ndarray:
        """The events since the last drain, uint32 [n, 6] = observer, owner (node index), key | kind << 8,
        old version (0 = none), new version, tick; in the reference's order (gossip_sim.h, gs_set_events):
        by tick; owner writes in call order; within a phase by exchange (its index in the phase), the
        initiator's apply before the responder's, the NodeDelta order (sender's dict position), kv version;
        liveness by observer, joins before leaves, then node.  Raises if the buffer overflowed."""
        self.sync()
        n = int(self._ev_count.item())
        if n > self._ev.shape[0]:
            # reset first, so the next drain starts clean (the caller can resize with enable_events)
            self._ev_count.zero_()
            self.sync()
            raise GsError(f"event buffer overflow: {n} events, capacity {self._ev.shape[0]} "
                          f"(the records of this drain are lost; enable_events with a larger capacity)")
        ev = self._ev[:n].cpu().numpy().view(np.uint32)
        self._ev_count.zero_()
        out = ev[order_events(ev, self.n, self._ev_phases, self._ev_wmap), :6]
        self._ev_phases.clear()
        return out


    def fd_census(self, up) -> dict:
        """gs_fd_census: live / dead sets of every up observer against the up mask (config 5's
        false-positive rate = up_dead / up_pairs)."""
        u = up if hasattr(up, "data_ptr") else self._dev(np.asarray(up, dtype=np.uint8), self.torch.uint8)
        c = _lib.GsCensus()
        self._chk(self.L.gs_fd_census(self.h, C.c_void_p(u.data_ptr()), C.byref(c)), "gs_fd_census")
        return {n: int(getattr(c, n)) for n in _lib.CENSUS_FIELDS}

    def materialize_held(self, row_lo: int = 0, row_hi: int | None = None):
        """Write out GS_R_HELD for the prefix views of rows [row_lo, row_hi) (readback only)."""
        hi = self.n if row_hi is None else row_hi
        self._chk(self.L.gs_materialize_held(self.h, row_lo, hi), "gs_materialize_held")

    def horizon(self, rounds: int | None = None) -> dict:
        """Headroom to the two bounds of the exact compact layout: the most intervals any
        sampling window holds since its last reset (compact windows: err_fd_overflow at W; the ring
        evicts exactly), and the most writes of any (owner, key) of this slice (err_hist_full at
        hist_cap - 1).  With ``rounds`` (rounds run so far) each bound is also projected linearly: the rounds
        left until the fastest-growing window / (owner, key) reaches it at the rate seen so far."""
        torch = self.torch
        sb = _lib.fd_sum_bits(int(self.cfg["window"]))
        fd = self.region("FD", torch.int32, (self.n, self.np_))
        mx = 0
        for r0 in range(0, self.n, 8192):
            blk = fd[r0:r0 + 8192, : self.ncol]
            mx = max(mx, int(((blk >> sb) & ((1 << (32 - sb)) - 1)).max().item()))
        lw = self.region("LAST_W", torch.uint8, (self.ncol, self.kp))[:, : self.k]
        mw = int(lw.max().item())
        c = self.counters()
        out = {"max_window_count": mx, "window": int(self.cfg["window"]),
               "fd_ring": "all rows" if self.flags & GS_FD_RING else f"{len(self.ring_rows)} sampled rows",
               "max_writes_per_owner_key": mw, "hist_cap_writes": self.hist_cap - 1,
               "fd_saturated": c["fd_saturated"], "err_fd_overflow": c["err_fd_overflow"],
               "err_hist_full": c["err_hist_full"], "err_hb_lag": c["err_hb_lag"]}
        if rounds:
            W = int(self.cfg["window"])
            out["rounds_run"] = int(rounds)
            # compact windows: appends since the last reset grow by at most one per report; ring windows evict
            out["projected_rounds_to_window"] = (None if self.flags & GS_FD_RING else
                                                 int((W - mx) * rounds / max(mx, 1)))
            out["projected_rounds_to_hist_cap"] = int((self.hist_cap - 1 - mw) * rounds / max(mw, 1))
        return out

    def inexact_views(self) -> int:
        """Views with holes (GS_MV_INEXACT set): those whose HELD row the exchange kernel keeps."""
        if self.mv8:
            mv = self.region("MV", self.torch.uint8, (self.n, self.np_))[:, : self.ncol]
            return int((mv >= 128).sum().item())
        mv = self.region("MV", self.torch.int16, (self.n, self.np_))[:, : self.ncol]
        return int((mv < 0).sum().item())

    def mv_words(self, rows=None):
        """Device int32 [rows, NP] max_version words (version | GS_MV_INEXACT) of observer rows ``rows`` (a
        slice or index tensor; default all): GS_R_MV as stored (u16), or decoded from GS_MV8's bytes (version
        mod 2^7 | inexact << 7) against the owners' own max_versions (GS_R_SELF_MV)."""
        torch = self.torch
        sel = slice(None) if rows is None else rows
        if not self.mv8:
            return self.region("MV", torch.int16, (self.n, self.np_))[sel].to(torch.int32) & 0xFFFF
        s = self.region("MV", torch.uint8, (self.n, self.np_))[sel].to(torch.int32)
        M = self.region("SELF_MV", torch.int32, (self.np_,))
        return (M - ((M - (s & 0x7F)) & 0x7F)) | ((s & 0x80) << 8)

    def hb_region(self):
        """GS_R_HB as a device tensor [N, NP]: int16 views (mod 2^16), or uint8 with GS_HB8 (mod 2^8)."""
        return self.region("HB", self.torch.uint8 if self.hb8 else self.torch.int16, (self.n, self.np_))

    def decode_heartbeats(self, hb: np.ndarray, rows=None) -> np.ndarray:
        """NodeState.heartbeat of host rows of GS_R_HB (u16, or u8 with GS_HB8; shape [rows, NP] or [NP]):
        the stored value is the heartbeat mod 2^16 (2^8), decoded against the owner's own heartbeat R
        (GS_R_SELF_HB).  ``rows``: the observer rows of ``hb`` (default: all rows, or the single row of a 1-D
        ``hb``); escaped owner columns (gs_config.esc_cols) are read from their 16-bit slots (GS_R_ESC16)."""
        R = self.region("SELF_HB", self.torch.int32, (self.np_,)).cpu().numpy().view(np.uint32)
        if self.hb8:
            s = np.asarray(hb).view(np.uint8).astype(np.uint32)
            out = (R - ((R - s) & np.uint32(0xFF))).astype(np.uint32)
        else:
            s = np.asarray(hb).view(np.uint16).astype(np.uint32)
            out = (R - ((R - s) & np.uint32(0xFFFF))).astype(np.uint32)
        if "ESC_SLOT" in self.regions:
            torch = self.torch
            slot = self.region("ESC_SLOT", torch.int32, (self.np_,)).cpu().numpy().view(np.uint32)
            cols = np.nonzero(slot != GS_NONE)[0]
            if len(cols):
                # only the requested rows' escaped slots cross to the host (ESC16 is N x esc_cols x 2 B)
                ec = int(self.c_esc_cols)
                esc = self.region("ESC16", torch.int16, (self.n, ec))
                if rows is not None or out.ndim == 1:
                    o = np.arange(self.n) if rows is None else np.asarray(rows, dtype=np.int64).reshape(-1)
                    esc = esc.index_select(0, torch.as_tensor(o, device=self.device))
                sl = torch.as_tensor(slot[cols].astype(np.int64), device=self.device)
                e = esc.index_select(1, sl).cpu().numpy().view(np.uint16).astype(np.uint32)  # [rows, escaped cols]
                v = (R[cols] - ((R[cols] - e) & np.uint32(0xFFFF))).astype(np.uint32)
                if out.ndim == 1:
                    out[cols] = v[0]
                else:
                    out[:, cols] = v
        return out

    def max_versions(self):
        """Device int32 [N, NP] NodeState.max_version of every view (GS_R_MV words: version | GS_MV_INEXACT)."""
        return self.mv_words() & 0x7FFF

    # --------------------------------------------------------------- readback
    def _host(self, rows=None):
        """Host copies of the state; ``rows`` = observer rows to read (default: all of them)."""
        n, NP, KP, K, Cc = self.n, self.np_, self.kp, self.k, self.hist_cap
        torch = self.torch
        if rows is None:
            self.materialize_held()
            sel = slice(None)
        else:
            rows = np.asarray(rows, dtype=np.int64)
            for o in rows.tolist():
                self.materialize_held(o, o + 1)
            sel = torch.as_tensor(rows, device=self.device)
        self.sync()

        def rd(name, dt, shape):
            t = self.region(name, dt, shape)
            return (t if rows is None else t.index_select(0, sel)).cpu().numpy()

        g = {"rows": np.arange(n) if rows is None else rows}
        g["HB"] = self.decode_heartbeats(rd("HB", torch.uint8 if self.hb8 else torch.int16, (n, NP)),
                                         None if rows is None else rows)
        for name in ("GC", "POS"):
            if name in self.regions:
                g[name] = rd(name, torch.int32, (n, NP)).view(np.uint32)
        st8 = rd("FD_STATE", torch.uint8, (n, NP))
        g["FD_STATE"] = fd_state_word(st8, rd("FD_TOD", torch.int32, (n, NP)))
        mv = (self.mv_words(None if rows is None else sel).cpu().numpy().astype(np.uint32))
        g["MV_INEXACT"] = (mv >> np.uint32(15)).astype(np.uint8)  # prefix-view flag (GS_MV_INEXACT)
        g["MV"] = mv & np.uint32(0x7FFF)
        nr = g["MV"].shape[0]
        if "GC" not in g:  # no tombstone GC: last_gc_version is 0 everywhere
            g["GC"] = np.zeros((nr, NP), dtype=np.uint32)
        g["FD_LAST"], g["FD_SUM"], g["FD_CNT"] = self.unpack_fd(st8, rd("FD_LAST", torch.int16, (n, NP)),
                                                                rd("FD", torch.int32, (n, NP)), self.latest_tick())
        nc = self.ncol
        hist = self.region("HIST", torch.int64, (nc, Cc, K)).cpu().numpy().view(np.uint64)
        g["HIST_VER"] = (hist & 0xFFFFFFFF).astype(np.uint32)
        if "HELD" in self.regions:
            g["HELD"] = rd("HELD", torch.uint8, (n, NP, KP))
        else:  # GS_NO_HELD: every view is S_j(max_version); count each key's writes <= max_version
            last_w = self.region("LAST_W", torch.uint8, (nc, KP)).cpu().numpy()[:, :K].astype(np.int64)
            M = g["MV"][:, :nc].astype(np.int64)
            held = np.zeros((nr, NP, KP), dtype=np.uint8)
            for w in range(1, Cc):
                ok = (w <= last_w) & (g["HIST_VER"][:, w, :] > 0)  # [nc, K]
                held[:, :nc, :K] += (ok[None, :, :] & (g["HIST_VER"][None, :, w, :] <= M[:, :, None])).astype(np.uint8)
            g["HELD"] = held
        g["HIST_META"] = (hist >> 32).astype(np.uint32)
        g["HIST_VID"] = self.region("HIST_VID", torch.int32, (nc, Cc, K)).cpu().numpy().view(np.uint32)
        g["ROW"] = rd("ROW", torch.int32, (n, 4)).view(np.uint32)
        if "TS" in self.regions:
            g["TS"] = rd("TS", torch.int32, (n, NP, KP)).view(np.uint32)
        if "ORD" in self.regions:
            g["ORD"] = rd("ORD", torch.int32, (n, NP)).view(np.uint32)
        return g

    def export(self, g=None) -> dict:
        """All observers as numpy arrays in the oracle's ``export_row`` format (times in ticks).

        A column slice exports its own owner columns (``ShardGroup.export`` joins them)."""
        g = self._host() if g is None else g
        n, K = self.ncol, self.k
        nr = g["MV"].shape[0]
        held = g["HELD"][:, :n, :K].astype(np.int64)
        jj = np.arange(n)[None, :, None]
        kk = np.arange(K)[None, None, :]
        ver = g["HIST_VER"][jj, held, kk]
        meta = g["HIST_META"][jj, held, kk]
        vid = g["HIST_VID"][jj, held, kk]
        present = held > 0
        out = {
            "hb": g["HB"][:, :n], "mv": g["MV"][:, :n], "gc": g["GC"][:, :n],
            "kv_version": np.where(present, ver, 0).astype(np.uint32),
            "kv_status": np.where(present, (meta >> 16) & 3, 0).astype(np.int32),
            "kv_value_id": np.where(present, vid, 0).astype(np.uint32),
        }
        if self.canonical:
            out["pos"] = np.broadcast_to(np.arange(self.col_lo, self.col_lo + n, dtype=np.int32), (nr, n)).copy()
        else:
            pos = g["POS"][:, :n].view(np.int32)
            out["pos"] = np.where(pos == -1, -1, pos).astype(np.int32)
        ts = g["TS"][:, :n, :K].astype(np.int64) if "TS" in g else np.zeros((nr, n, K), np.int64)
        out["kv_ts"] = np.where(out["kv_status"] != 0, ts, 0)
        last = g["FD_LAST"][:, :n]
        out["fd_last"] = np.where(last == GS_NONE, -1, last.astype(np.int64))
        cnt = g["FD_CNT"][:, :n].astype(np.int32)
        W = int(self.cfg["window"])
        # ring windows count appends up to 2W (len = min(cnt, W)); a compact window never holds more than W
        out["fd_len"] = np.where(last == GS_NONE, 0, np.minimum(cnt, W))
        out["fd_sum"] = np.where(last == GS_NONE, 0.0, g["FD_SUM"][:, :n] / 64.0)
        st = g["FD_STATE"][:, :n]
        out["live"] = (st == 1).astype(np.int32)
        out["tod"] = np.where(st >= 2, st.astype(np.int64) - 2, -1)
        return out

    def export_rows(self, rows) -> dict:
        """``export()`` of the observer rows ``rows`` only (full-size parity checks: a few rows of a
        65,536-node matrix)."""
        return self.export(self._host(rows))

    def latest_tick(self) -> int:
        """gs_latest_tick: the latest tick any operation on the handle used (decodes GS_R_FD_LAST)."""
        t = C.c_uint32()
        self._chk(self.L.gs_latest_tick(self.h, C.byref(t)), "gs_latest_tick")
        return int(t.value)

    def unpack_fd(self, st8: np.ndarray, last16: np.ndarray, sc: np.ndarray, tick: int):
        """Windows (GS_R_FD_STATE bits, GS_R_FD_LAST, GS_R_FD) as (last tick or GS_NONE, sum in ticks,
        appended count); 16-bit ticks decoded against ``tick`` (at or after every report recorded), a
        window marked old (>= 2^15 ticks) as tick - 2^15, as the device does (fd_get)."""
        return unpack_fd(st8, last16, sc, tick, _lib.fd_sum_bits(int(self.cfg["window"])))

    def read_rows(self, region: str, row_lo: int, row_hi: int) -> bytes:
        """gs_read_rows: the bytes of observer rows [row_lo, row_hi) of ``region`` (blocking copy-out)."""
        n = C.c_uint64()
        t = self.regions.get(region)
        rb = t.numel() * t.element_size() // self.n if t is not None else 0
        buf = (C.c_uint8 * max(1, rb * (row_hi - row_lo)))()
        self._chk(self.L.gs_read_rows(self.h, REGION[region], row_lo, row_hi, buf, len(buf), C.byref(n)),
                  "gs_read_rows")
        return bytes(buf)[: n.value]

    def phi_row(self, observer: int, tick: int | None = None) -> np.ndarray:
        """Device-computed phi (binary64) of every target of ``observer``; NaN = None."""
        t = self.last_tick if tick is None else tick
        out = self.torch.empty(self.ncol, dtype=self.torch.float64, device=self.device)
        self._chk(self.L.gs_phi_row(self.h, observer, t, C.c_void_p(out.data_ptr())), "gs_phi_row")
        return out.cpu().numpy()

    def _whole(self):
        if self.shards > 1:
            raise GsError("per-observer views need the whole matrix (shards == 1); use export() on a slice")

    def _order(self, g, o: int) -> list[int]:
        if self.canonical:
            return list(range(self.n))
        return [int(x) for x in g["ORD"][o, : g["ROW"][o, 0]]]

    def _kvs(self, g, o: int, j: int) -> list:
        out = []
        for k in range(self.k):
            w = int(g["HELD"][o, j, k])
            if not w:
                continue
            ver = int(g["HIST_VER"][j, w, k])
            meta = int(g["HIST_META"][j, w, k])
            st = (meta >> 16) & 3
            ts = int(g["TS"][o, j, k]) if (st and "TS" in g) else None
            out.append([self.keys[k], self.values[int(g["HIST_VID"][j, w, k])], ver, st, ts])
        out.sort()
        return out

    def _window_len(self, cnt: int) -> int:
        return min(cnt, int(self.cfg["window"]))

    def observer_state(self, o: int, g=None) -> dict:
        """Canonical dump, identical in format to ``oracle/refharness.py`` (golden fixtures)."""
        self._whole()
        g = self._host() if g is None else g
        nodes = []
        for j in self._order(g, o):
            nodes.append([j, int(g["HB"][o, j]), int(g["MV"][o, j]), int(g["GC"][o, j]), self._kvs(g, o, j)])
        st = g["FD_STATE"][o, : self.n]
        live = [int(j) for j in np.flatnonzero(st == 1)]
        dead = [[int(j), int(st[j]) - 2] for j in np.flatnonzero(st >= 2)]
        phis = self.phi_row(o)
        wins = []
        for j in np.flatnonzero(g["FD_LAST"][o, : self.n] != GS_NONE):
            j = int(j)
            phi = float(phis[j])
            wins.append([j, int(g["FD_LAST"][o, j]), self._window_len(int(g["FD_CNT"][o, j])),
                         int(g["FD_SUM"][o, j]) / 64.0, None if math.isnan(phi) else phi])
        return {"nodes": nodes, "live": live, "dead": dead, "windows": wins}

    def state(self) -> list[dict]:
        g = self._host()
        return [self.observer_state(o, g) for o in range(self.n)]

    # --------------------------------------------------------------- reference-shaped views
    def node_state(self, observer: int, owner: int) -> NodeState | None:
        """``ClusterState.node_state`` of ``observer`` for ``owner`` (state.py:295-296).  Reads only
        that view (a few bytes of the observer's row) and the owner's history rows."""
        self._whole()
        torch, n, K, KP, Cc = self.torch, self.n, self.k, self.kp, self.hist_cap
        o, j = int(observer), int(owner)
        if not self.canonical:
            pos = int(self.region("POS", torch.int32, (n, self.np_))[o, j].item())
            if pos == -1:
                return None
        self.materialize_held(o, o + 1)
        self.sync()
        hb = int(self.decode_heartbeats(self.hb_region()[o].cpu().numpy(), [o])[j])
        mv = int(self.mv_words(slice(o, o + 1))[0, j].item()) & 0x7FFF
        gc = int(self.region("GC", torch.int32, (n, self.np_))[o, j].item()) & 0xFFFFFFFF \
            if "GC" in self.regions else 0
        hist = self.region("HIST", torch.int64, (n, Cc, K))[j].cpu().numpy().view(np.uint64)
        hvid = self.region("HIST_VID", torch.int32, (n, Cc, K))[j].cpu().numpy().view(np.uint32)
        if "HELD" in self.regions:
            held = self.region("HELD", torch.uint8, (n, self.np_, KP))[o, j, :K].cpu().numpy()
        else:  # GS_NO_HELD: the view is S_j(max_version): each key's latest write <= mv
            ver = (hist & np.uint64(0xFFFFFFFF)).astype(np.int64)
            last_w = self.region("LAST_W", torch.uint8, (n, KP))[j, :K].cpu().numpy().astype(np.int64)
            w = np.arange(Cc)[:, None]
            held = (((w >= 1) & (w <= last_w[None, :]) & (ver > 0) & (ver <= mv)).sum(0)).astype(np.uint8)
        ts = self.region("TS", torch.int32, (n, self.np_, KP))[o, j, :K].cpu().numpy().view(np.uint32) \
            if "TS" in self.regions else None
        kvs = {}
        for k in range(K):
            w = int(held[k])
            if not w:
                continue
            e = int(hist[w, k])
            st = VersionStatusEnum((e >> 48) & 3)
            kvs[self.keys[k]] = VersionedValue(self.values[int(hvid[w, k])], e & 0xFFFFFFFF, st,
                                               int(ts[k]) if (st and ts is not None) else None)
        return NodeState(self.node_ids[j], hb, kvs, mv, gc)

    def snapshot(self, observer: int, cluster_id: str = "default") -> ClusterSnapshot:
        """``Cluster.snapshot`` of node ``observer`` (server.py:168-175), read from its rows only: its
        dict in insertion order, each NodeState with its key-values, the failure detector's live and
        dead nodes (live in target order; dead in time-of-death order, as the reference's dict)."""
        self._whole()
        torch, n, K, KP, Cc = self.torch, self.n, self.k, self.kp, self.hist_cap
        o = int(observer)
        self.materialize_held(o, o + 1)
        self.sync()

        def row(name, dt=torch.int32):
            return self.region(name, dt, (n, self.np_))[o, :n].cpu().numpy()

        hb = self.decode_heartbeats(self.hb_region()[o].cpu().numpy(), [o])[:n]
        mv = self.mv_words(slice(o, o + 1))[0, :n].cpu().numpy().astype(np.uint32) & np.uint32(0x7FFF)
        gc = row("GC").view(np.uint32) if "GC" in self.regions else np.zeros(n, np.uint32)
        st = fd_state_word(row("FD_STATE", torch.uint8), row("FD_TOD"))
        hist = self.region("HIST", torch.int64, (n, Cc, K)).cpu().numpy().view(np.uint64)
        if "HELD" in self.regions:
            held = self.region("HELD", torch.uint8, (n, self.np_, KP))[o, :n, :K].cpu().numpy()
        else:  # GS_NO_HELD: every view is S_j(max_version): count each key's writes <= the row's mv
            ver = (hist & np.uint64(0xFFFFFFFF)).astype(np.int64)  # [n, C, K]
            last_w = self.region("LAST_W", torch.uint8, (n, KP))[:, :K].cpu().numpy().astype(np.int64)
            held = np.zeros((n, K), dtype=np.uint8)
            for w in range(1, Cc):
                ok = (w <= last_w) & (ver[:, w, :] > 0) & (ver[:, w, :] <= mv.astype(np.int64)[:, None])
                held += ok.astype(np.uint8)
        ts = self.region("TS", torch.int32, (n, self.np_, KP))[o, :n, :K].cpu().numpy().view(np.uint32) \
            if "TS" in self.regions else None
        hvid = self.region("HIST_VID", torch.int32, (n, Cc, K)).cpu().numpy().view(np.uint32)
        if self.canonical:
            order = range(n)
        else:
            cnt = int(self.region("ROW", torch.int32, (n, 4))[o, 0].item())
            order = [int(x) for x in self.region("ORD", torch.int32, (n, self.np_))[o, :cnt].cpu().numpy()]
        states = {}
        for j in order:
            kvs = {}
            for k in range(K):
                w = int(held[j, k])
                if not w:
                    continue
                e = int(hist[j, w, k])
                status = VersionStatusEnum((e >> 48) & 3)
                kvs[self.keys[k]] = VersionedValue(self.values[int(hvid[j, w, k])], e & 0xFFFFFFFF, status,
                                                   int(ts[j, k]) if (status and ts is not None) else None)
            states[self.node_ids[j]] = NodeState(self.node_ids[j], int(hb[j]), kvs, int(mv[j]), int(gc[j]))
        live = [self.node_ids[j] for j in np.flatnonzero(st == 1)]
        dead_j = np.flatnonzero(st >= 2)
        if self.canonical:
            dead_j = sorted(dead_j.tolist(), key=lambda j: (int(st[j]), j))
        else:
            pos = row("POS").view(np.uint32)
            dead_j = sorted(dead_j.tolist(), key=lambda j: (int(st[j]), int(pos[j])))
        return ClusterSnapshot(cluster_id, self.node_ids[o], states, live, [self.node_ids[j] for j in dead_j])

    def live_nodes(self, observer: int) -> list[NodeId]:
        self._whole()
        st = self.region("FD_STATE", self.torch.uint8, (self.n, self.np_))[observer, : self.n].cpu().numpy()
        return [self.node_ids[j] for j in np.flatnonzero((st & 3) == 1)]

    def dead_nodes(self, observer: int) -> list[NodeId]:
        self._whole()
        st = self.region("FD_STATE", self.torch.uint8, (self.n, self.np_))[observer, : self.n].cpu().numpy()
        return [self.node_ids[j] for j in np.flatnonzero((st & 3) == 2)]

    def phi(self, observer: int, target: int, tick: int | None = None) -> float | None:
        v = float(self.phi_row(observer, tick)[target])
        return None if math.isnan(v) else v
