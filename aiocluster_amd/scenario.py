"""Backend-neutral scenario format and replay loop.

A *scenario* is plain JSON-able data: node identities, key names, hot-path
configuration, boot writes and, per round, the owner writes, the up-mask and
the explicit phase schedule.  The same scenario is replayed by

* the reference harness (``oracle/refharness.py``, container only) to make
  golden fixtures,
* the C oracle (``oracle/oracle.py``), and
* the HIP simulator (``aiocluster_amd.sim.GossipSim``),

and their canonical states are compared.  The round/tick model is documented
in ``aiocluster_amd/workload.py``.
"""

from __future__ import annotations

import hashlib
import json

from .entities import NodeId
from .workload import Workload, WorkloadSpec, liveness_tick, phase_tick, round_tick

DEFAULT_CFG = {
    "mtu": 65_507,  # Config.max_payload_size (entities.py:105)
    "tombstone_grace_s": 7200,  # Config.marked_for_deletion_grace_period (entities.py:101)
    "phi_threshold": 8.0,  # FailureDetectorConfig (entities.py:87-91)
    "window": 1000,
    "max_interval_s": 10.0,
    "initial_interval_s": 5.0,
    "dead_grace_s": 86400.0,
}


def make_scenario(name: str, spec: WorkloadSpec, rounds: int, cfg: dict | None = None) -> dict:
    wl = Workload(spec)
    c = dict(DEFAULT_CFG)
    c.update(cfg or {})
    iw, ivals = wl.initial_writes()
    scen = {
        "name": name,
        "n": spec.n,
        "k": spec.k,
        "nodes": [[n.name, n.generation_id, n.gossip_advertise_addr[0], n.gossip_advertise_addr[1], n.tls_name]
                  for n in wl.node_ids],
        "keys": wl.keys,
        "init": spec.init,
        "config": c,
        "initial": [[int(j), int(k), v] for (j, k, _), v in zip(iw.tolist(), ivals)],
        "rounds": [],
    }
    for _ in range(rounds):
        plan = wl.next_round()
        scen["rounds"].append(
            {
                "writes": [[int(j), int(k), int(o), v] for (j, k, o), v in zip(plan.writes.tolist(), plan.values)],
                "up": [int(x) for x in plan.up],
                "phases": [[[int(x), int(y)] for x, y in zip(a.tolist(), b.tolist())] for a, b in plan.phases],
            }
        )
    return scen


def scenario_node_ids(scen: dict) -> list[NodeId]:
    return [NodeId(n[0], n[1], (n[2], n[3]), n[4]) for n in scen["nodes"]]


def initial_by_owner(scen: dict) -> dict[int, list[tuple[int, str]]]:
    out: dict[int, list[tuple[int, str]]] = {}
    for j, k, v in scen["initial"]:
        out.setdefault(j, []).append((k, v))
    return out


def state_hash(state) -> str:
    return hashlib.sha256(json.dumps(state, separators=(",", ":")).encode()).hexdigest()


# fields of an ``export()`` dict that the compact digest covers, with their canonical dtypes
DIGEST_FIELDS = {
    "pos": "<i4", "hb": "<u4", "mv": "<u4", "gc": "<u4", "kv_version": "<u4", "kv_status": "<i4",
    "kv_ts": "<i8", "fd_last": "<i8", "fd_len": "<i4", "fd_sum": "<f8", "live": "<i4", "tod": "<i8",
}


def export_digest(ex: dict, fields=None) -> dict[str, str]:
    """SHA-256 per field of an ``export()`` dict (every observer row, every owner column), for
    fixtures too large to store as canonical JSON states (config 2: 1,024 x 1,024 views x 64 keys).
    Every backend's export has the same layout: ``pos`` = dict position or -1, times in ticks,
    ``kv_ts`` only where the status is not SET, ``fd_last`` -1 without a window; values are left
    out (an owner's version identifies its write, so the versions pin the values)."""
    import numpy as np

    out = {}
    for name, dt in (fields or DIGEST_FIELDS).items():
        a = np.asarray(ex[name])
        if name == "kv_ts":
            a = np.where(np.asarray(ex["kv_status"]) != 0, a, 0)
        out[name] = hashlib.sha256(np.ascontiguousarray(a.astype(dt)).tobytes()).hexdigest()
    return out


def replay(backend, scen: dict, on_round=None, rounds: int | None = None):
    """Drive ``backend`` through ``scen``'s rounds (backend already booted at tick 0).

    Backend protocol: ``write(t, j, k, op, value)``, ``begin_round(t, up)``,
    ``run_phase(t, pairs)``, ``liveness(t, up, r)``.
    """
    rs = scen["rounds"] if rounds is None else scen["rounds"][:rounds]
    for r in range(len(rs)):
        replay_round(backend, scen, r)
        if on_round is not None:
            on_round(r)


def replay_round(backend, scen: dict, r: int):
    """Round ``r`` of ``scen`` on ``backend`` (writes, round start, phases, liveness)."""
    rd = scen["rounds"][r]
    t = round_tick(r)
    up = rd["up"]
    for j, k, op, v in rd["writes"]:
        backend.write(t, j, k, op, v)
    backend.begin_round(t, up)
    for p, ph in enumerate(rd["phases"]):
        backend.run_phase(phase_tick(r, p), ph)
    backend.liveness(liveness_tick(r, len(rd["phases"])), up, r)
