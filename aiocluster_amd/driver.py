"""Round driver shared by the bench, the full-size parity tests and the config-5 tool.

``prepare`` turns a seeded ``Workload`` (``workload.py``) into per-round device inputs (write
batches, up masks, phase arrays) uploaded before any timing; ``run_round`` drives one round
on the slices a process holds, in the order ``Cluster._gossip_multiple`` runs it
(``aiocluster/server.py:441-495``): owner writes, ``inc_heartbeat`` + tombstone GC
(``gs_begin_round``), the conflict-free phases (``gs_run_phase``, or the sliced
count/gather/pack of ``shard.py``), then ``_update_node_liveness`` (``gs_liveness``).
"""

from __future__ import annotations

import ctypes as C

import numpy as np


def digits(x: np.ndarray) -> np.ndarray:
    return np.floor(np.log10(np.maximum(x, 1))).astype(np.int64) + 1


def boot_ops(n: int, k: int) -> list[np.ndarray]:
    """``Cluster(initial_key_values)``: key k of owner j = "v{j}.{k}.i", as K batches of distinct owners
    (owner, key, op, value_id, value_len); value ids 1 + k * n + j."""
    out = []
    for kk in range(k):
        ops = np.zeros((n, 5), dtype=np.uint32)
        ops[:, 0] = np.arange(n)
        ops[:, 1] = kk
        ops[:, 3] = 1 + kk * n + np.arange(n)
        ops[:, 4] = 3 + digits(np.arange(n)) + digits(np.full(n, kk)) + 1
        out.append(ops)
    return out


def prepare(spec, rounds: int, torch, dev) -> list[dict]:
    """Every round's device inputs (host schedule generation is not timed).  Write values are
    interned as ids 2^24 + i with the byte length of ``workload.write_value``."""
    from .workload import OP_DELETE, OP_DELETE_AFTER_TTL, Workload, liveness_tick, phase_tick, round_tick

    wl = Workload(spec)
    out = []
    vid = 1 << 24
    for _ in range(rounds):
        p = wl.next_round(materialize_values=False)
        w = p.writes
        ops = np.zeros((len(w), 5), dtype=np.int64)
        if len(w):
            # value "v{j}.{k}.{r}" / "t{j}.{k}.{r}" (deletes: ""): byte length without materialising strings
            ops[:, 0], ops[:, 1], ops[:, 2] = w[:, 0], w[:, 1], w[:, 2]
            ops[:, 3] = vid + np.arange(len(w))
            vid += len(w)
            ops[:, 4] = 3 + digits(w[:, 0]) + digits(w[:, 1]) + digits(np.full(len(w), p.r))
            dele = (w[:, 2] == OP_DELETE) | (w[:, 2] == OP_DELETE_AFTER_TTL)
            ops[dele, 3] = 0
            ops[dele, 4] = 0
        r = p.r
        out.append({
            "r": r,
            "t": round_tick(r),
            "ops": torch.from_numpy(ops.astype(np.int32)).to(dev),
            "nops": len(w),
            "up": torch.from_numpy(p.up.astype(np.uint8)).to(dev),
            "up_host": p.up.astype(np.uint8),
            "phases": [(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), len(a), phase_tick(r, i))
                       for i, (a, b) in enumerate(p.phases)],
            "t_live": liveness_tick(r, len(p.phases)),
            "exchanges": p.n_exchanges,
        })
    return out


def begin(sims, rd):
    """Owner writes + gs_begin_round of round ``rd`` on every slice."""
    for sim in sims:
        if rd["nops"]:
            sim._chk(sim.L.gs_owner_writes(sim.h, C.c_void_p(rd["ops"].data_ptr()), rd["nops"], rd["t"]),
                     "gs_owner_writes")
        sim._chk(sim.L.gs_begin_round(sim.h, C.c_void_p(rd["up"].data_ptr()), rd["t"]), "gs_begin_round")


def run_phases(sims, rd, events=None, group=None, phases=None):
    """The round's phases (``phases`` overrides the plan's: (a, b, n, tick) tuples)."""
    s0 = sims[0]
    for a, b, n, t in (rd["phases"] if phases is None else phases):
        if not n:
            continue
        for s_ in sims:
            if s_._ev is not None:  # hook events: order_events needs each phase's exchange order
                if group is not None:
                    raise ValueError("hook events on a sliced cluster are not supported (drain per slice)")
                s_._ev_phases[t] = (a.cpu().numpy().astype(np.int64), b.cpu().numpy().astype(np.int64))
        if events is not None:
            e0 = s0.torch.cuda.Event(enable_timing=True)
            e1 = s0.torch.cuda.Event(enable_timing=True)
            e0.record(s0.stream)
        if group is None:
            s0._chk(s0.L.gs_run_phase(s0.h, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), n, t),
                    "gs_run_phase")
        else:  # the group's own driver: shard.py's (its scratch kept across phases), or the library's (native)
            group.run_phase_arrays(t, a, b)
        if events is not None:
            e1.record(s0.stream)
            events.append((e0, e1))


def end(sims, rd, tick=None):
    """gs_liveness closing the round."""
    for sim in sims:
        sim._chk(sim.L.gs_liveness(sim.h, C.c_void_p(rd["up"].data_ptr()), rd["t_live"] if tick is None else tick),
                 "gs_liveness")


def run_round(sims, rd, events=None, group=None, sel=None):
    """One gossip round on the slices this process drives (one GossipSim when unsliced).  With ``sel``
    (a PeerSelector) the round's exchanges come from the device's select_nodes_for_gossip + phase
    schedule instead of the workload's explicit schedule (``rd`` gains "exchanges", "unscheduled")."""
    from .workload import TICKS_PER_ROUND, liveness_tick, phase_tick

    begin(sims, rd)
    phases = None
    if sel is not None:
        sel.select(rd["up"], rd["r"])
        ph, offs, left = sel.schedule(rd["up"], rd["r"])
        phases = [(a, b, n, phase_tick(rd["r"], p)) for p, (a, b, n) in enumerate(ph)]
        rd["exchanges"] = offs[-1]
        rd["unscheduled"] = left
        rd["t_live"] = liveness_tick(rd["r"], len(phases))  # sub-phases share the budget's last tick
        rd["phases_run"] = len(phases)
    if rd["t_live"] >= rd["t"] + TICKS_PER_ROUND:
        raise ValueError(f"round {rd['r']}: liveness tick {rd['t_live']} reaches the next round's tick")
    run_phases(sims, rd, events, group, phases)
    end(sims, rd)
