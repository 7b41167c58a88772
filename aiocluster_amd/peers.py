"""Peer selection on the device: ``select_nodes_for_gossip`` (``aiocluster/server.py:656-717``) for
every node of a simulated cluster, and the round's exchanges split into conflict-free phases.

``Cluster._gossip_multiple`` (``server.py:441-495``) picks its peers from the failure detector's
live / dead sets and its known peers at round start, before ``inc_heartbeat`` and the exchanges.
``run_selected_round`` drives one such round on a ``GossipSim``: owner writes, ``gs_begin_round``,
``gs_select_peers`` (from the previous round's liveness), ``gs_schedule_phases``, the phases, the
liveness sweep.  Everything stays on the device except the 17 phase offsets.

The reference draws from ``random.Random`` over Python ``set`` iteration order; here
the draws are Philox4x32-10 keyed by the run seed with counter (round, node, slot), so a schedule is
reproducible and its CPU restatement (``oracle/peer_select.py``) matches it exactly.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import MAX_SCHED_PHASES, GsError, sched_scratch_bytes


class PeerSelector:
    """Device buffers for one cluster's per-round peer selection and phase schedule."""

    def __init__(self, sim, fanout: int = 3, seeds=(), seed: int = 0, iters: int = 4,
                 max_phases: int = MAX_SCHED_PHASES):
        if sim.shards > 1:
            raise GsError("peer selection needs the whole matrix (one slice)")
        if not 1 <= fanout <= 8:
            raise GsError("fanout must be in 1..8")
        torch = sim.torch
        # the workload's tick model: phase p at round tick + 1 + min(p, MAX_PHASES_PER_ROUND - 1) -- the phases past
        # the tick budget are sub-phases at its last tick (workload.phase_tick), so every selected exchange runs
        # (server.py:476-493) -- and liveness after them, before the next round's tick
        if not 1 <= max_phases <= MAX_SCHED_PHASES:
            raise GsError(f"max_phases must be in 1..{MAX_SCHED_PHASES}")
        self.sim, self.fanout, self.seed, self.iters = sim, int(fanout), int(seed), int(iters)
        self.max_phases = int(max_phases)
        n, F = sim.n, self.fanout
        dev = sim.device
        self.seeds = torch.tensor(sorted(set(int(x) for x in seeds)) or [0], dtype=torch.int32, device=dev)
        self.n_seeds = len(set(seeds))
        self.targets = torch.empty((n, F + 2), dtype=torch.int32, device=dev)
        self.sel_scratch = torch.empty(4 * n * (F + 6), dtype=torch.uint8, device=dev)
        self.sched_scratch = torch.empty(sched_scratch_bytes(n, F, self.max_phases), dtype=torch.uint8, device=dev)
        self.ini = torch.empty(n * (F + 2), dtype=torch.int32, device=dev)
        self.res = torch.empty(n * (F + 2), dtype=torch.int32, device=dev)

    def select(self, up_dev, r: int):
        """gs_select_peers: targets[N][F+2] = F peers, the dead pick, the seed pick (-1 = none)."""
        s = self.sim
        s._chk(s.L.gs_select_peers(s.h, C.c_void_p(up_dev.data_ptr()), self.fanout,
                                   C.c_void_p(self.seeds.data_ptr()), self.n_seeds, self.seed, r,
                                   C.c_void_p(self.targets.data_ptr()), C.c_void_p(self.sel_scratch.data_ptr())),
               "gs_select_peers")
        return self.targets

    def schedule(self, up_dev, r: int):
        """gs_schedule_phases: ``(phases, offsets, unscheduled)`` -- [(initiators, responders, n)] per
        non-empty phase (device views), the phase offsets (``offsets[-1]`` = exchanges scheduled) and the
        number of selected exchanges with an up responder that did not fit in ``max_phases`` phases
        (``_gossip_multiple`` contacts every selected peer, server.py:476-493: callers assert 0)."""
        s = self.sim
        P = self.max_phases
        off = (C.c_uint32 * (P + 1))()
        left = C.c_uint32()
        s._chk(s.L.gs_schedule_phases(s.h, C.c_void_p(up_dev.data_ptr()), self.fanout,
                                      C.c_void_p(self.targets.data_ptr()), self.seed, r, self.iters, P,
                                      C.c_void_p(self.sched_scratch.data_ptr()), C.c_void_p(self.ini.data_ptr()),
                                      C.c_void_p(self.res.data_ptr()), off, C.byref(left)), "gs_schedule_phases")
        offs = np.frombuffer(off, dtype=np.uint32).astype(np.int64)
        nz = np.flatnonzero(offs[1:] > offs[:-1]).tolist()
        phases = [(self.ini[offs[p]:offs[p + 1]], self.res[offs[p]:offs[p + 1]], int(offs[p + 1] - offs[p]))
                  for p in nz]
        offs = offs.tolist()
        return phases, offs, int(left.value)

    def scheduled_pairs(self, phases) -> list[set]:
        """Host copy of a schedule: one set of (initiator, responder) per phase."""
        return [set(zip(a.cpu().numpy().tolist(), b.cpu().numpy().tolist())) for a, b, _ in phases]


def run_selected_round(sim, sel: PeerSelector, r: int, up, writes=None, tick0: int | None = None) -> dict:
    """One round with device peer selection (workload tick model: round tick 64 (r + 1))."""
    from .workload import liveness_tick, phase_tick, round_tick

    t = round_tick(r) if tick0 is None else tick0
    up_dev = up if hasattr(up, "data_ptr") else sim._dev(np.asarray(up, dtype=np.uint8), sim.torch.uint8)
    if writes is not None:
        for j, k, op, v in writes:
            sim.write(t, j, k, op, v)
    sim.begin_round(t, up_dev)
    sel.select(up_dev, r)  # live / dead sets of the previous round's liveness (server.py:448-469)
    phases, offs, left = sel.schedule(up_dev, r)
    if left:
        raise GsError(f"round {r}: {left} selected exchanges did not fit in {sel.max_phases} phases")
    # phases past the tick budget share its last tick (sub-phases: workload.phase_tick)
    for p, (a, b, n) in enumerate(phases):
        sim.run_phase_arrays(phase_tick(r, p), a, b)
    sim.update_node_liveness(liveness_tick(r, len(phases)), up_dev)
    return {"phases": len(phases), "exchanges": offs[-1]}
