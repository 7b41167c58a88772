"""In-process driver of the REAL reference (``/root/reference``) -- fixture generation only.

TEST INFRASTRUCTURE.  This module runs only in the build container, where the
reference checkout exists; nothing on the GPU box or in the product path
imports it.  It produces the golden fixtures under ``tests/golden/`` that pin
the C oracle (``oracle/gossip_oracle.c``), which in turn is the checker for
the HIP path.

The reference targets Python >= 3.13 (``pyproject.toml:6``); this image has
3.10, so three compatibility patches are applied in-process before import
(SURVEY §8(c)): ``typing.Self``, ``datetime.UTC`` and ``LoggerAdapter``'s
``merge_extra`` keyword.  Nothing in the reference is modified.

Driving (SURVEY §8(c) harness contract), never starting sockets or tickers:

* boot: ``Cluster(config, initial_key_values)`` (``server.py:75-122``);
* round start, per up node: ``self_node_state().inc_heartbeat()`` and
  ``_cluster_state.gc_marked_for_deletion`` (``server.py:471-474``);
* exchange (a, b): ``a._make_syn_msg`` -> ``b.inc_heartbeat`` (``server.py:524``)
  -> ``b._handle_syn_msg`` -> ``a._handle_synac_msg`` -> ``b._handle_ack``
  (``server.py:327-376``), every packet round-tripped through its wire bytes;
* round end, per up node: ``_update_node_liveness`` (``server.py:606-620``).

The clock is virtual: ``aiocluster.state.utc_now`` and
``aiocluster.failure_detector.utc_now`` are replaced by the harness clock.
"""

from __future__ import annotations

import datetime as _dt
import logging
import os
import sys
import typing
from datetime import timedelta

REF_PATH = "/root/reference"
_REF = None


def import_reference():
    """Import the reference package with the 3.10 compatibility patches (cached)."""
    global _REF
    if _REF is not None:
        return _REF
    if not os.path.isdir(REF_PATH):
        raise RuntimeError("reference checkout not present (fixture generation runs in the build container only)")
    import typing_extensions

    if not hasattr(typing, "Self"):
        typing.Self = typing_extensions.Self
    if not hasattr(_dt, "UTC"):
        _dt.UTC = _dt.timezone.utc
    orig = logging.LoggerAdapter.__init__
    if "merge_extra" not in orig.__code__.co_varnames:

        def _init(self, logger, extra=None, merge_extra=False):  # noqa: ARG001
            orig(self, logger, extra)

        logging.LoggerAdapter.__init__ = _init
    sys.dont_write_bytecode = True
    if REF_PATH not in sys.path:
        sys.path.insert(0, REF_PATH)
    import aiocluster  # noqa: F401
    import aiocluster.entities as ent
    import aiocluster.failure_detector as fdm
    import aiocluster.server as srv
    import aiocluster.state as st
    from aiocluster.protos import messages_pb2 as pb

    class R:
        pass

    R.ent, R.fd, R.srv, R.state, R.pb = ent, fdm, srv, st, pb
    _REF = R
    return R


_EPOCH = _dt.datetime(2024, 1, 1, tzinfo=_dt.timezone.utc)
_TICK_US = 15_625


def tick_dt(t: int) -> _dt.datetime:
    return _EPOCH + timedelta(microseconds=t * _TICK_US)


def dt_tick(d: _dt.datetime) -> int:
    us = (d - _EPOCH) // timedelta(microseconds=1)
    assert us % _TICK_US == 0, d
    return us // _TICK_US


class RefSim:
    """N reference ``Cluster`` objects driven by an explicit schedule."""

    def __init__(self, node_ids, keys, cfg: dict, init: str, initial_values: dict[int, list[tuple[int, str]]]):
        R = import_reference()
        self.R = R
        self.now = tick_dt(0)
        R.state.utc_now = lambda: self.now
        R.fd.utc_now = lambda: self.now
        self.keys = keys
        self.ids = [
            R.ent.NodeId(n.name, n.generation_id, tuple(n.gossip_advertise_addr), n.tls_name) for n in node_ids
        ]
        self.idx = {nid: i for i, nid in enumerate(self.ids)}
        fdc = R.ent.FailureDetectorConfig(
            phi_threshhold=cfg["phi_threshold"],
            sampling_window_size=cfg["window"],
            max_interval=timedelta(seconds=cfg["max_interval_s"]),
            initial_interval=timedelta(seconds=cfg["initial_interval_s"]),
            dead_node_grace_period=timedelta(seconds=cfg["dead_grace_s"]),
        )
        self.grace = timedelta(seconds=cfg["tombstone_grace_s"])
        self.clusters = []
        for i, nid in enumerate(self.ids):
            conf = R.ent.Config(
                node_id=nid,
                marked_for_deletion_grace_period=cfg["tombstone_grace_s"],
                failure_detector=fdc,
                max_payload_size=cfg["mtu"],
            )
            kv = {keys[k]: v for k, v in initial_values.get(i, [])}
            self.clusters.append(R.srv.Cluster(conf, initial_key_values=kv))
        if init == "warm":
            self._warm()
        self.q9_events = []

    def _warm(self):
        """Every observer knows every owner, in index order, at the owner's boot state."""
        R = self.R
        own = [c.self_node_state() for c in self.clusters]
        for o, c in enumerate(self.clusters):
            states = {}
            for j, ns in enumerate(own):
                if j == o:
                    states[self.ids[j]] = ns
                else:
                    kvs = {
                        k: R.ent.VersionedValue(v.value, v.version, v.status, v.status_change_ts)
                        for k, v in ns.key_values.items()
                    }
                    states[self.ids[j]] = R.state.NodeState(
                        self.ids[j], ns.heartbeat, kvs, ns.max_version, ns.last_gc_version
                    )
            c._cluster_state._node_states = states

    def set_time(self, t: int):
        self.now = tick_dt(t)

    def write(self, t: int, j: int, k: int, op: int, value: str):
        self.set_time(t)
        c = self.clusters[j]
        key = self.keys[k]
        if op == 0:
            c.set(key, value)
        elif op == 1:
            c.delete(key)
        elif op == 2:
            c.set_with_ttl(key, value)
        elif op == 3:
            c.delete_after_ttl(key)
        else:
            raise ValueError(op)

    def begin_round(self, t: int, up):
        self.set_time(t)
        for o, c in enumerate(self.clusters):
            if up[o]:
                c.self_node_state().inc_heartbeat()
                c._cluster_state.gc_marked_for_deletion(self.grace)

    def run_phase(self, t: int, pairs):
        self.set_time(t)
        for a, b in pairs:
            self.exchange(a, b)

    def exchange(self, a: int, b: int):
        PacketPb = self.R.pb.PacketPb
        A, B = self.clusters[a], self.clusters[b]
        syn = PacketPb.FromString(A._make_syn_msg().SerializeToString())
        B.self_node_state().inc_heartbeat()
        synack = PacketPb.FromString(B._handle_syn_msg(syn).SerializeToString())
        ack = PacketPb.FromString(A._handle_synac_msg(synack).SerializeToString())
        B._handle_ack(ack)

    def liveness(self, t: int, up, r: int):
        self.set_time(t)
        for o, c in enumerate(self.clusters):
            if up[o]:
                try:
                    c._update_node_liveness()
                except KeyError as e:  # SURVEY Q9 (failure_detector.py:118)
                    self.q9_events.append([r, o, self.idx[e.args[0]]])

    # ------------------------------------------------------------------ dump
    def observer_state(self, o: int) -> dict:
        c = self.clusters[o]
        SET = self.R.ent.VersionStatusEnum.SET
        nodes = []
        for nid, ns in c._cluster_state._node_states.items():
            kvs = sorted(
                [key, vv.value, vv.version, int(vv.status), None if vv.status == SET else dt_tick(vv.status_change_ts)]
                for key, vv in ns.key_values.items()
            )
            nodes.append([self.idx[nid], ns.heartbeat, ns.max_version, ns.last_gc_version, kvs])
        fd = c._failure_detector
        live = sorted(self.idx[n] for n in fd._live_nodes)
        dead = sorted([self.idx[n], dt_tick(t)] for n, t in fd._dead_nodes.items())
        wins = []
        for n, sw in fd._node_samples.items():
            last = None if sw._last_heartbeat is None else dt_tick(sw._last_heartbeat)
            phi = fd.phi(n, ts=self.now)
            wins.append([self.idx[n], last, len(sw._intervals), sw._intervals.sum(), phi])
        wins.sort()
        return {"nodes": nodes, "live": live, "dead": dead, "windows": wins}

    def state(self) -> list[dict]:
        return [self.observer_state(o) for o in range(len(self.clusters))]

    def export(self) -> dict:
        """Every observer as numpy arrays in the ``GossipSim.export`` / ``OracleSim.export`` format
        (times in ticks; kv_value_id is left out: an owner's version identifies its write, hence the
        value).  Used for the compact per-round digests of large fixtures
        (``aiocluster_amd.scenario.export_digest``)."""
        import numpy as np

        n, K = len(self.clusters), len(self.keys)
        kidx = {k: i for i, k in enumerate(self.keys)}
        SET = self.R.ent.VersionStatusEnum.SET
        out = {
            "pos": np.full((n, n), -1, np.int32), "hb": np.zeros((n, n), np.uint32),
            "mv": np.zeros((n, n), np.uint32), "gc": np.zeros((n, n), np.uint32),
            "kv_version": np.zeros((n, n, K), np.uint32), "kv_status": np.zeros((n, n, K), np.int32),
            "kv_ts": np.zeros((n, n, K), np.int64), "fd_last": np.full((n, n), -1, np.int64),
            "fd_len": np.zeros((n, n), np.int32), "fd_sum": np.zeros((n, n), np.float64),
            "live": np.zeros((n, n), np.int32), "tod": np.full((n, n), -1, np.int64),
        }
        for o, c in enumerate(self.clusters):
            for p, (nid, ns) in enumerate(c._cluster_state._node_states.items()):
                j = self.idx[nid]
                out["pos"][o, j] = p
                out["hb"][o, j], out["mv"][o, j], out["gc"][o, j] = ns.heartbeat, ns.max_version, ns.last_gc_version
                for key, vv in ns.key_values.items():
                    k = kidx[key]
                    out["kv_version"][o, j, k] = vv.version
                    out["kv_status"][o, j, k] = int(vv.status)
                    if vv.status != SET:
                        out["kv_ts"][o, j, k] = dt_tick(vv.status_change_ts)
            fd = c._failure_detector
            for nid in fd._live_nodes:
                out["live"][o, self.idx[nid]] = 1
            for nid, t in fd._dead_nodes.items():
                out["tod"][o, self.idx[nid]] = dt_tick(t)
            for nid, sw in fd._node_samples.items():
                j = self.idx[nid]
                if sw._last_heartbeat is not None:
                    out["fd_last"][o, j] = dt_tick(sw._last_heartbeat)
                out["fd_len"][o, j] = len(sw._intervals)
                out["fd_sum"][o, j] = sw._intervals.sum()
        return out
