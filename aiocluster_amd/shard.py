"""Owner-column sharding of one simulated cluster (DESIGN.md "multi-GPU").

Every slice holds all N observer rows and a contiguous block of owner columns
(``gs_config.n_shards``/``shard``).  Heartbeat merges, failure-detector reports,
digests and stale-owner tests are per column, so they run on each slice with no
communication.  The only coupling is the MTU budget of each delta:
``compute_partial_delta_respecting_mtu`` (state.py:340-415) walks the sender's
stale owners in dict order — index order in the canonical layout, i.e. slice
order — and stops adding once the DeltaPb is full.  Per phase:

1. ``gs_phase_count`` on every slice: pass 1, plus the DeltaPb bytes of all the
   slice's stale owners per (exchange, direction) — ``u64 [n][2]``;
2. all-gather of those totals (16 B per exchange per slice; RCCL over xGMI);
3. ``gs_phase_pack(step 0)``: each slice packs and applies its owners starting
   at the byte count its predecessors reach when they all fit whole;
4. only for the (exchange, direction) slots whose totals sum past the MTU: chain
   steps, each an all-gather of those slots' chain states (8 bytes per
   overflowing slot and slice, plus each slice's pending count) and a
   ``gs_phase_chain`` that lets a pending slice continue where its nearest
   finished predecessor stopped, skipping slices that cannot add a NodeDelta
   (their smallest one exceeds the budget left: each total carries it); the
   steps stop once no slot is pending (usually after one).  ``gs_phase_overflow``
   lists the slots on the device -- the same list on every slice -- and returns
   their number: one host read per phase, and one per step.

The result equals ``gs_run_phase`` on a single handle bit for bit (tested on one
GPU with G in-process slices).  ``comm`` abstracts the gather: ``LocalComm``
(every slice in this process) or ``DistComm`` (one slice per rank,
``torch.distributed``: RCCL on GPUs, gloo in the CPU tests).
"""

from __future__ import annotations

import numpy as np

from ._lib import COUNTER_FIELDS, GS_CHAIN_CAP, GS_CHAIN_DEVICE, GsError, overflow_list_len

MAX_FIELDS = ("pack_groups_max", "pack_steps_max")  # counters that are maxima, not sums

CHAIN_PENDING = -1  # u64 ~0 viewed as int64 (gossip_sim.hip CHAIN_PENDING)
TOT_BYTES_MASK = (1 << 40) - 1  # a slice total's DeltaPb bytes (GS_TOT_BYTES); the smallest NodeDelta above


class LocalComm:
    """All G slices live in this process (tests; one GPU)."""

    def __init__(self, world: int):
        self.world = world
        self.rank = 0

    def gather(self, parts):
        import torch

        return torch.stack(parts)

    def sum_counters(self, per_slice: list[dict]) -> dict:
        return {k: (max if k in MAX_FIELDS else sum)(c[k] for c in per_slice) for k in COUNTER_FIELDS}

    def any(self, flag: bool) -> bool:
        return flag


class SoloComm:
    """Slice ``rank`` of a ``world``-slice cluster held alone (one GPU's share of a multi-GPU run): the
    other slices' gathered totals are zeros.  Exact for this slice's columns whenever the MTU cannot bind
    (config 4's contract: mtu above every delta), since a slice's packing then does not depend on the
    others; otherwise a timing rehearsal only."""

    def __init__(self, world: int, rank: int = 0):
        self.world = world
        self.rank = rank

    def gather(self, parts):
        import torch

        (x,) = parts
        out = torch.zeros((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        out[self.rank] = x
        return out

    def sum_counters(self, per_slice: list[dict]) -> dict:
        return per_slice[0]

    def any(self, flag: bool) -> bool:
        return flag


class DistComm:
    """One slice per rank of a ``torch.distributed`` process group."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

    def gather(self, parts):
        import torch

        (x,) = parts
        if self.dist.get_backend(self.group) == "gloo":  # CPU tests / rehearsals: gather through host memory
            xc = x.detach().to("cpu").contiguous()
            out = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype)
            self.dist.all_gather(list(out.unbind(0)), xc, group=self.group)
            return out.to(x.device)
        out = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        self.dist.all_gather_into_tensor(out, x.contiguous(), group=self.group)
        return out

    def sum_counters(self, per_slice: list[dict]) -> dict:
        import torch

        (c,) = per_slice
        dev = "cpu" if self.dist.get_backend(self.group) == "gloo" else "cuda"
        sums = [k for k in COUNTER_FIELDS if k not in MAX_FIELDS]
        v = torch.tensor([c[k] for k in sums], dtype=torch.int64, device=dev)
        m = torch.tensor([c[k] for k in MAX_FIELDS], dtype=torch.int64, device=dev)
        self.dist.all_reduce(v, group=self.group)
        self.dist.all_reduce(m, op=self.dist.ReduceOp.MAX, group=self.group)
        out = dict(zip(sums, (int(x) for x in v.tolist())))
        out.update(zip(MAX_FIELDS, (int(x) for x in m.tolist())))
        return {k: out[k] for k in COUNTER_FIELDS}

    def any(self, flag: bool) -> bool:
        return flag  # decided from gathered data, identical on every rank


def run_sliced_phase(slices, comm, mtu: int, t: int, ini, res, cache: dict | None = None) -> int:
    """One phase on the slices this process drives; returns the pack steps taken (1 = no chain).

    ``slices`` expose ``phase_count``, ``phase_pack``, ``phase_overflow``, ``phase_chain`` and ``phase_pending``
    (``GossipSim`` does).  ``cache``: the phase's scratch tensors kept across phases (per exchange count).
    """
    import torch

    n = int(ini.numel())
    if n == 0:
        return 0
    tots = [s.phase_count(t, ini, res) for s in slices]
    tot_all = comm.gather(tots)
    dev = tots[0].device
    # scratch sized for the largest phase seen on this device and slice count (peer-selected schedules change the
    # exchange count nearly every phase: views of one allocation, not a reallocation per phase)
    key = (str(dev), len(slices))
    buf = None if cache is None else cache.get(key)
    if buf is None or buf["n"] < n:
        buf = {
            "n": n,
            "chains": [torch.empty((n, 2), dtype=torch.int64, device=dev) for _ in slices],
            "lists": [torch.empty(overflow_list_len(n), dtype=torch.int32, device=dev) for _ in slices],
            # [2n + 1] (the listed slots' states, then the pending entry), at least GS_CHAIN_CAP + 1
            "chaincs": [torch.empty(max(2 * n, GS_CHAIN_CAP) + 1, dtype=torch.int64, device=dev) for _ in slices],
        }
        if cache is not None:
            cache[key] = buf
    buf = {"chains": [x[:n] for x in buf["chains"]], "lists": [x[: overflow_list_len(n)] for x in buf["lists"]],
           "chaincs": [x[: max(2 * n, GS_CHAIN_CAP) + 1] for x in buf["chaincs"]]}
    chains = buf["chains"]
    for s, ch in zip(slices, chains):
        s.phase_pack(t, ini, res, 0, tot_all, None, ch)
    if not all(s.has_records for s in slices):
        # fused count pass (GS_FUSED=1): every slot's chain state travels; one host read decides
        if not bool(((tot_all & TOT_BYTES_MASK).sum(0) > mtu).any()):
            return 1
        for step in range(1, comm.world):
            chain_all = comm.gather(chains)
            for s, ch in zip(slices, chains):
                s.phase_pack(t, ini, res, step, tot_all, chain_all, ch)
        return comm.world
    lists, chaincs = buf["lists"], buf["chaincs"]
    # the overflowing slots, listed on the device (the same list on every slice); no count read
    for i in range(len(slices) - 1, -1, -1):
        slices[i].phase_overflow(tot_all, chains[i], lists[i], chaincs[i], read=False)
    if comm.world < 2:
        return 1
    # step 1 on the device count (GS_CHAIN_DEVICE): a chain usually resolves in it, so one read -- the gathered
    # pending entries -- ends the phase; more slots than GS_CHAIN_CAP, or a chain still pending, go on from the host
    cap = GS_CHAIN_CAP
    chain_all = comm.gather([cc[: cap + 1] for cc in chaincs])
    for s, ch, lb, cc in zip(slices, chains, lists, chaincs):
        s.phase_chain(t, ini, res, 1, lb, GS_CHAIN_DEVICE, chain_all, ch, cc, tot_all)
    chain_all = comm.gather([cc[: cap + 1] for cc in chaincs])
    # the phase's one host read: the pending slots summed over the slices and the device count (gs_phase_pending:
    # one kernel writing a pinned host pair; -1 = more slots than the device step takes)
    p_, count = slices[0].phase_pending(n, lists[0], GS_CHAIN_DEVICE, chain_all)
    if p_ == 0:
        return 2 if count else 1
    steps = 1 if count > cap else 2
    for step in range(steps, comm.world):
        # every slice's chain states + pending count (entry count): the same on every rank, so all stop
        # together once no slot is pending
        chain_all = comm.gather([cc[: count + 1] for cc in chaincs])
        if int(chain_all[:, count].sum().item()) == 0:
            break
        for s, ch, lb, cc in zip(slices, chains, lists, chaincs):
            s.phase_chain(t, ini, res, step, lb, count, chain_all, ch, cc, tot_all)
        steps += 1
    return steps


class ShardGroup:
    """The owner-column slices of one simulated cluster, driven like one ``GossipSim``."""

    def __init__(self, slices, comm, mtu: int, native: bool = False):
        """``native``: the library drives each phase (gs_run_phase_group for the slices of this process,
        or gs_run_phase over the RCCL communicator of gs_comm_init, one slice per rank); otherwise this
        module does (run_sliced_phase, gathers through ``comm``)."""
        if not slices:
            raise GsError("ShardGroup needs at least one slice")
        self.slices = list(slices)
        self.comm = comm
        self.mtu = int(mtu)
        self.n = self.slices[0].n
        self.chain_phases = 0
        self.phase_steps: list[int] = []  # pack steps each phase of this driver took (1 = no chain)
        self._scratch: dict = {}  # run_sliced_phase's tensors, kept across phases
        self.native = native
        if native and len(self.slices) == 1 and isinstance(comm, DistComm):
            self._comm_init()

    def _comm_init(self):
        """gs_comm_id on rank 0, broadcast over the process group, gs_comm_init on every rank."""
        import ctypes as C

        s = self.slices[0]
        uid = (C.c_uint8 * 128)()
        if self.comm.rank == 0:
            s._chk(s.L.gs_comm_id(uid), "gs_comm_id")
        box = [bytes(uid)]
        self.comm.dist.broadcast_object_list(box, src=0, group=self.comm.group)
        uid = (C.c_uint8 * 128).from_buffer_copy(box[0])
        s._chk(s.L.gs_comm_init(s.h, uid, self.comm.world, self.comm.rank), "gs_comm_init")

    @classmethod
    def in_process(cls, node_ids, keys, cfg, shards: int, native: bool = False, **kw):
        from .sim import GossipSim

        sl = [GossipSim(node_ids, keys, cfg, shards=shards, shard=g, **kw) for g in range(shards)]
        return cls(sl, LocalComm(shards), cfg["mtu"], native=native)

    @classmethod
    def distributed(cls, node_ids, keys, cfg, group=None, native: bool = False, **kw):
        from .sim import GossipSim

        comm = DistComm(group)
        s = GossipSim(node_ids, keys, cfg, shards=comm.world, shard=comm.rank, **kw)
        return cls([s], comm, cfg["mtu"], native=native)

    # -- owner writes / round driver: every slice sees every call (each keeps its own columns)
    def write(self, t, j, k, op, value):
        for s in self.slices:
            s.write(t, j, k, op, value)

    def owner_writes(self, ops: np.ndarray, tick: int):
        for s in self.slices:
            s.owner_writes(ops, tick)

    def begin_round(self, t: int, up):
        for s in self.slices:
            s.begin_round(t, up)

    def run_phase(self, t: int, pairs):
        if len(pairs) == 0:
            return
        arr = np.asarray(pairs, dtype=np.int32).reshape(-1, 2)
        self.run_phase_arrays(t, arr[:, 0], arr[:, 1])

    def run_phase_arrays(self, t: int, initiators, responders):
        s0 = self.slices[0]
        for s in self.slices:
            s._flush()
            if s._ev is not None:
                raise GsError("hook events on a sliced cluster are not supported (order_events needs one handle)")
        ini, res = s0._pairs_dev(initiators, responders)
        if self.native:
            import ctypes as C

            n = int(ini.numel())
            if len(self.slices) == 1 and not isinstance(self.comm, SoloComm):
                s0._chk(s0.L.gs_run_phase(s0.h, C.c_void_p(ini.data_ptr()), C.c_void_p(res.data_ptr()), n, t),
                        "gs_run_phase")
            else:
                hs = (C.c_void_p * len(self.slices))(*[s.h for s in self.slices])
                s0._chk(s0.L.gs_run_phase_group(hs, len(self.slices), C.c_void_p(ini.data_ptr()),
                                                C.c_void_p(res.data_ptr()), n, t), "gs_run_phase_group")
            return
        steps = run_sliced_phase(self.slices, self.comm, self.mtu, t, ini, res, self._scratch)
        self.phase_steps.append(steps)
        if steps > 1:
            self.chain_phases += 1

    def flush_reports(self, t: int):
        for s in self.slices:
            s.flush_reports(t)

    def update_node_liveness(self, t: int, up):
        for s in self.slices:
            s.update_node_liveness(t, up)

    def liveness(self, t: int, up, r: int = -1):
        self.update_node_liveness(t, up)

    def sync(self):
        for s in self.slices:
            s.sync()

    # -- counters / readback
    def counters(self) -> dict:
        return self.comm.sum_counters([s.counters() for s in self.slices])

    def reset_counters(self):
        for s in self.slices:
            s.reset_counters()

    def check(self, accept_saturated: bool = False) -> dict:
        c = self.counters()
        errs = {k: v for k, v in c.items() if k.startswith("err_") and v}
        if c["fd_saturated"] and not accept_saturated:  # GossipSim.check: compact rows past W are inexact
            errs["fd_saturated"] = c["fd_saturated"]
        if errs:
            raise GsError(f"device checks failed: {errs}")
        return c

    def fd_census(self, up) -> dict:
        parts = [s.fd_census(up) for s in self.slices]
        local = {k: sum(p[k] for p in parts) for k in parts[0]}
        if isinstance(self.comm, DistComm):
            import torch

            from ._lib import CENSUS_FIELDS

            dev = "cpu" if self.comm.dist.get_backend(self.comm.group) == "gloo" else "cuda"
            v = torch.tensor([local[k] for k in CENSUS_FIELDS], dtype=torch.int64, device=dev)
            self.comm.dist.all_reduce(v, group=self.comm.group)
            local = dict(zip(CENSUS_FIELDS, (int(x) for x in v.tolist())))
        return local

    def export(self) -> dict:
        """The slices this process holds, joined along the owner axis (all of them in-process)."""
        parts = [s.export() for s in self.slices]
        return {k: np.concatenate([p[k] for p in parts], axis=1) for k in parts[0]}

    def phi_row(self, observer: int, tick: int | None = None) -> np.ndarray:
        return np.concatenate([s.phi_row(observer, tick) for s in self.slices])
