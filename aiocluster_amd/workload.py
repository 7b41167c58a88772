"""Deterministic synthetic gossip workloads (node ids, owner writes, churn, schedules).

The reference picks peers with ``random.Random`` over Python ``set`` iteration
order (``aiocluster/server.py:441-469,685-717``), which is not reproducible
across processes.  The batched backend is therefore driven by an
explicit, seeded schedule that every backend replays identically: the device
simulator, the C oracle and the reference harness used to make golden fixtures.

Round model (one *step* of the bench), mirroring ``Cluster._gossip_multiple``
(``server.py:441-495``) for every node that is up:

* tick ``t_r = 64 * (r + 1)``: owner writes, then ``inc_heartbeat`` +
  ``gc_marked_for_deletion`` on every up node (``server.py:471-474``);
* phase ``p`` at tick ``t_r + 1 + p``: a conflict-free set of exchanges
  (each node in at most one), each a full Syn/SynAck/Ack
  (``server.py:327-376,523-568``);
* tick ``t_r + 1 + P``: ``_update_node_liveness`` on every up node
  (``server.py:606-620``).

Fanout: for each of ``F`` slots a random permutation ``sigma`` gives every
node exactly one initiation ``i -> sigma(i)``; the permutation's cycles are
edge-coloured into <= 3 matchings, so a round has ``3F`` phases.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .entities import NodeId

TICKS_PER_ROUND = 64
MAX_PHASES_PER_ROUND = TICKS_PER_ROUND - 2

OP_SET = 0
OP_DELETE = 1
OP_SET_WITH_TTL = 2
OP_DELETE_AFTER_TTL = 3


def round_tick(r: int) -> int:
    return TICKS_PER_ROUND * (r + 1)


def phase_tick(r: int, p: int) -> int:
    """Tick of phase p of round r.  Phases past the tick budget (a schedule by the reference's own selection, whose
    hubs need more phases than a round has ticks) are sub-phases at the budget's last tick: the reference runs
    every selected exchange (server.py:476-493), concurrently, so several at one time."""
    return round_tick(r) + 1 + min(p, MAX_PHASES_PER_ROUND - 1)


def liveness_tick(r: int, n_phases: int) -> int:
    return round_tick(r) + 1 + min(n_phases, MAX_PHASES_PER_ROUND)


def synthetic_node_ids(n: int) -> list[NodeId]:
    """``node-{i}``, host ``10.{i>>16}.{(i>>8)&255}.{i&255}``, port 7000, gen i+1."""
    return [
        NodeId(f"node-{i}", i + 1, (f"10.{i >> 16}.{(i >> 8) & 255}.{i & 255}", 7000), None)
        for i in range(n)
    ]


def simple_node_ids(n: int = 3) -> list[NodeId]:
    """``examples/simple.py:14-16``: simple1..3 on 127.0.0.1:7000-7002 (generation ids fixed)."""
    return [NodeId(f"simple{i + 1}", i + 1, ("127.0.0.1", 7000 + i), None) for i in range(n)]


def key_names(k: int) -> list[str]:
    return [f"key_{i:02d}" for i in range(k)]


def initial_value(j: int, k: int) -> str:
    return f"v{j}.{k}.i"


def write_value(j: int, k: int, r: int, op: int) -> str:
    if op == OP_DELETE or op == OP_DELETE_AFTER_TTL:
        return ""
    return f"{'t' if op == OP_SET_WITH_TTL else 'v'}{j}.{k}.{r}"


def permutation_phases(perm: np.ndarray) -> list[tuple[np.ndarray, np.ndarray]]:
    """Edge-colour the functional graph ``i -> perm[i]`` into <= 3 matchings.

    Along each cycle the edges alternate colours 0/1; an odd cycle's closing
    edge takes colour 2.  Fixed points (self loops) are dropped.
    """
    n = perm.shape[0]
    color = np.full(n, -1, dtype=np.int8)
    seen = np.zeros(n, dtype=bool)
    perm_l = perm.tolist()
    for s in range(n):
        if seen[s]:
            continue
        cyc = []
        i = s
        while not seen[i]:
            seen[i] = True
            cyc.append(i)
            i = perm_l[i]
        L = len(cyc)
        if L == 1:
            continue
        for m, node in enumerate(cyc):
            color[node] = m & 1
        if L & 1:
            color[cyc[-1]] = 2
    out = []
    idx = np.arange(n, dtype=np.int32)
    for c in range(3):
        sel = color == c
        out.append((idx[sel], perm[sel].astype(np.int32)))
    return out


@dataclass
class RoundPlan:
    r: int
    writes: np.ndarray  # int64 [m, 3]: owner, key, op
    values: list[str]   # value string per write ("" for deletes)
    up: np.ndarray      # bool [n]
    phases: list[tuple[np.ndarray, np.ndarray]]  # (initiators, responders) int32

    @property
    def n_exchanges(self) -> int:
        return int(sum(len(a) for a, _ in self.phases))


@dataclass
class WorkloadSpec:
    n: int
    k: int
    fanout: int = 3
    seed: int = 0
    init: str = "warm"  # "warm": every node knows every node in index order; "cold": self only
    write_frac: float = 0.05
    delete_frac: float = 0.0  # fraction of writes that are deletes
    ttl_frac: float = 0.0  # fraction of writes that are set_with_ttl / delete_after_ttl
    down_frac: float = 0.0  # steady-state fraction of nodes down
    down_rounds: int = 3  # a node that goes down stays down this many rounds
    partition: tuple[int, int] | None = None  # rounds [start, end) with the cluster split in halves
    node_style: str = "synthetic"
    initial_keys: int | None = None  # keys written at boot (default: all k)
    quiet_from: int | None = None  # rounds >= this: no writes, every node up (convergence checks)
    extra: dict = field(default_factory=dict)


class Workload:
    """Round-by-round plan generator; round ``r`` depends only on (seed, r) and the churn history."""

    def __init__(self, spec: WorkloadSpec):
        self.spec = spec
        n = spec.n
        self.node_ids = simple_node_ids(n) if spec.node_style == "simple" else synthetic_node_ids(n)
        self.keys = key_names(spec.k)
        self._down_until = np.zeros(n, dtype=np.int64)
        self._next_round = 0

    def initial_writes(self) -> tuple[np.ndarray, list[str]]:
        nk = self.spec.k if self.spec.initial_keys is None else self.spec.initial_keys
        n = self.spec.n
        owners = np.repeat(np.arange(n, dtype=np.int64), nk)
        keys = np.tile(np.arange(nk, dtype=np.int64), n)
        ops = np.zeros_like(owners)
        vals = [initial_value(int(j), int(k)) for j, k in zip(owners, keys)] if n * nk <= 1 << 20 else None
        return np.stack([owners, keys, ops], axis=1), vals

    def next_round(self, materialize_values: bool = True) -> RoundPlan:
        r = self._next_round
        self._next_round += 1
        s = self.spec
        n = s.n
        rng = np.random.default_rng([s.seed, r])
        # -- churn: nodes going down for `down_rounds` rounds
        up = self._down_until <= r
        if s.down_frac > 0:
            goes_down = up & (rng.random(n) < s.down_frac / max(1, s.down_rounds))
            self._down_until[goes_down] = r + s.down_rounds
            up = self._down_until <= r
        quiet = s.quiet_from is not None and r >= s.quiet_from
        if quiet:
            up = np.ones(n, dtype=bool)
        # -- owner writes (only up nodes write)
        m_w = 0 if quiet else int(round(s.write_frac * n))
        if m_w > 0:
            owners = rng.choice(n, size=m_w, replace=False).astype(np.int64)
            keys = rng.integers(0, s.k, size=m_w).astype(np.int64)
            u = rng.random(m_w)
            ops = np.full(m_w, OP_SET, dtype=np.int64)
            ops[u < s.delete_frac + s.ttl_frac] = OP_SET_WITH_TTL
            ops[u < s.delete_frac + s.ttl_frac / 2] = OP_DELETE_AFTER_TTL
            ops[u < s.delete_frac] = OP_DELETE
            keep = up[owners]
            owners, keys, ops = owners[keep], keys[keep], ops[keep]
            order = np.argsort(owners, kind="stable")
            owners, keys, ops = owners[order], keys[order], ops[order]
        else:
            owners = keys = ops = np.zeros(0, dtype=np.int64)
        writes = np.stack([owners, keys, ops], axis=1)
        values = (
            [write_value(int(j), int(k), r, int(o)) for j, k, o in writes] if materialize_values else []
        )
        # -- schedule
        phases = []
        part = s.partition is not None and s.partition[0] <= r < s.partition[1]
        for _ in range(s.fanout):
            perm = rng.permutation(n).astype(np.int32)
            for a, b in permutation_phases(perm):
                keep = up[a] & up[b]
                if part:
                    keep &= (a < n // 2) == (b < n // 2)
                phases.append((a[keep], b[keep]))
        assert len(phases) <= MAX_PHASES_PER_ROUND
        return RoundPlan(r, writes, values, up, phases)
