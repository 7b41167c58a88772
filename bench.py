"""Headline benchmark: simulated gossip exchanges/s at 65,536 nodes (BASELINE.json configs[2]).

Workload (synthetic, seeded; see aiocluster_amd/workload.py): 65,536 nodes x 16 keys,
fanout 3, warm start (every node knows every node, index order), every round 5% of
the nodes write one key and 5% churn up/down (down nodes neither initiate nor
answer), phi window 1000, mtu 65,507.  One step = one gossip round: owner writes,
heartbeat + tombstone GC, 9 conflict-free exchange phases, liveness sweep.  All
inputs (schedules, write batches, up masks) are uploaded to HBM before timing.

Multi-GPU: ``--gpus N`` under torch.distributed splits ONE 65,536-node cluster into N
owner-column slices, one per GPU (aiocluster_amd/shard.py; strong scaling): every rank
runs every exchange on its columns, and the ranks exchange only 16 bytes per exchange
(an RCCL all-gather of per-slice DeltaPb totals, plus chain states when a delta
overflows the MTU).  ``value`` is the cluster's exchanges / the slowest rank's time.
``--slices G`` rehearses the same sliced path with G slices in one process on one GPU.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (k_exchange,
HIP-event timed on the library's stream) and the CPU baseline (the C oracle on one
host core, timed on a bounded sample of exchanges whose rows are copied from the
device state).
"""

from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def digits(x: np.ndarray) -> np.ndarray:
    return np.floor(np.log10(np.maximum(x, 1))).astype(np.int64) + 1


def prepare(sim, spec, rounds, torch, dev):
    """Precompute every round's device inputs (host schedule generation is not timed)."""
    from aiocluster_amd.workload import Workload, liveness_tick, phase_tick, round_tick

    wl = Workload(spec)
    out = []
    vid = 1 << 24
    for _ in range(rounds):
        p = wl.next_round(materialize_values=False)
        w = p.writes
        ops = np.zeros((len(w), 5), dtype=np.int64)
        if len(w):
            # value "v{j}.{k}.{r}" (workload.write_value): byte length without materialising strings
            ops[:, 0], ops[:, 1], ops[:, 2] = w[:, 0], w[:, 1], w[:, 2]
            ops[:, 3] = vid + np.arange(len(w))
            vid += len(w)
            ops[:, 4] = 3 + digits(w[:, 0]) + digits(w[:, 1]) + digits(np.full(len(w), p.r))
        r = p.r
        out.append({
            "r": r,
            "t": round_tick(r),
            "ops": torch.from_numpy(ops.astype(np.int32)).to(dev),
            "nops": len(w),
            "up": torch.from_numpy(p.up.astype(np.uint8)).to(dev),
            "phases": [(torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), len(a), phase_tick(r, i))
                       for i, (a, b) in enumerate(p.phases)],
            "t_live": liveness_tick(r, len(p.phases)),
            "exchanges": p.n_exchanges,
        })
    return out


def run_round(sims, rd, events=None, group=None, sel=None):
    """One gossip round on the slices this process drives (one GossipSim when unsliced).  With ``sel``
    (a PeerSelector) the round's exchanges come from the device's select_nodes_for_gossip + phase
    schedule instead of the workload's explicit schedule."""
    from aiocluster_amd.shard import run_sliced_phase
    from aiocluster_amd.workload import phase_tick

    s0 = sims[0]
    for sim in sims:
        if rd["nops"]:
            sim._chk(sim.L.gs_owner_writes(sim.h, C.c_void_p(rd["ops"].data_ptr()), rd["nops"], rd["t"]),
                     "gs_owner_writes")
        sim._chk(sim.L.gs_begin_round(sim.h, C.c_void_p(rd["up"].data_ptr()), rd["t"]), "gs_begin_round")
    phases = rd["phases"]
    if sel is not None:
        sel.select(rd["up"], rd["r"])
        ph, offs = sel.schedule(rd["up"], rd["r"])
        phases = [(a, b, n, phase_tick(rd["r"], p)) for p, (a, b, n) in enumerate(ph)]
        rd["exchanges"] = offs[16]
        rd["t_live"] = rd["t"] + 1 + len(phases)
    for a, b, n, t in phases:
        if not n:
            continue
        if events is not None:
            e0 = s0.torch.cuda.Event(enable_timing=True)
            e1 = s0.torch.cuda.Event(enable_timing=True)
            e0.record(s0.stream)
        if group is None:
            s0._chk(s0.L.gs_run_phase(s0.h, C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), n, t),
                    "gs_run_phase")
        else:
            run_sliced_phase(sims, group.comm, group.mtu, t, a, b)
        if events is not None:
            e1.record(s0.stream)
            events.append((e0, e1))
    for sim in sims:
        sim._chk(sim.L.gs_liveness(sim.h, C.c_void_p(rd["up"].data_ptr()), rd["t_live"]), "gs_liveness")


def cpu_baseline(sim, spec, cfg, next_plan, sample: int, min_seconds: float = 10.0, threads: int = 1):
    """The C oracle (`threads` host cores) on `sample` exchanges whose two rows are copied from the device."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc_mod  # test infrastructure: the checker, timed here as the CPU baseline

    torch = sim.torch
    n, K, NP, KP, Cc = sim.n, sim.k, sim.np_, sim.kp, sim.hist_cap
    L = orc_mod.lib()
    from aiocluster_amd.workload import synthetic_node_ids
    from aiocluster_amd.pbsize import nodeid_size

    ids = synthetic_node_ids(n)
    ns = (C.c_int32 * n)(*[nodeid_size(x.name, x.generation_id, x.gossip_advertise_addr[0],
                                       x.gossip_advertise_addr[1], x.tls_name) for x in ids])
    kl = (C.c_int32 * K)(*[6] * K)
    oc = orc_mod._Cfg(n, K, int(cfg["mtu"]), orc_mod.us(cfg["tombstone_grace_s"]), float(cfg["phi_threshold"]),
                      int(cfg["window"]), orc_mod.us(cfg["max_interval_s"]), orc_mod.us(cfg["initial_interval_s"]),
                      orc_mod.us(cfg["dead_grace_s"]))
    # disjoint pairs from the first phase of the next round; `threads` host cores, one oracle handle
    # each (the oracle keeps per-handle scratch), pairs dealt round-robin (one
    # thread and threads over a phase, core count stated)
    a_all, b_all, _, t = next_plan["phases"][0]
    a_all, b_all = a_all.cpu().numpy(), b_all.cpu().numpy()
    pairs = list(zip(a_all[:sample].tolist(), b_all[:sample].tolist()))
    T = max(1, min(threads, len(pairs)))
    hs = [L.orc_create(C.byref(oc), ns, kl) for _ in range(T)]
    mine = [pairs[i::T] for i in range(T)]
    hist = sim.region("HIST", torch.int64, (n, Cc, K)).cpu().numpy().view(np.uint64)
    hist_ver = np.ascontiguousarray((hist & 0xFFFFFFFF).astype(np.uint32))
    hist_vid = sim.region("HIST_VID", torch.int32, (n, Cc, K)).cpu().numpy().view(np.uint32).copy()
    meta = (hist >> 32).astype(np.uint32)
    hist_vlen = (meta >> 18).astype(np.int32)
    hist_st = ((meta >> 16) & 3).astype(np.uint8)
    order = np.arange(n, dtype=np.int32)

    def rows(name, dt, shape):
        return sim.region(name, dt, shape)

    for a, b in pairs:  # prefix views keep no HELD row on the device: write them out for these rows
        sim.materialize_held(a, a + 1)
        sim.materialize_held(b, b + 1)
    hb16 = rows("HB", torch.int16, (n, NP))  # heartbeat mod 2^16 (decoded per row below)
    fst = rows("FD_STATE", torch.int32, (n, NP))
    mv16 = rows("MV", torch.int16, (n, NP))  # u16 max_version | GS_MV_INEXACT
    gc = rows("GC", torch.int32, (n, NP)) if "GC" in sim.regions else torch.zeros((n, NP), dtype=torch.int32)
    fdw = rows("FD", torch.int64, (n, NP))
    held = rows("HELD", torch.uint8, (n, NP, KP))
    P = C.c_void_p
    for h, prs in zip(hs, mine):
        for a, b in prs:
            for o in (a, b):
                def g(x):
                    return np.ascontiguousarray(x[o, :n].cpu().numpy().view(np.uint32))
                hb = np.ascontiguousarray(sim.decode_heartbeats(hb16[o].cpu().numpy())[:n])
                mv = np.ascontiguousarray((mv16[o, :n].cpu().numpy().view(np.uint16) & 0x7FFF).astype(np.uint32))
                fl, fs, fc = (np.ascontiguousarray(x) for x in sim.unpack_fd(fdw[o, :n].cpu().numpy()))
                hw = np.ascontiguousarray(held[o, :n, :K].cpu().numpy())
                L.orc_load_row(h, o, n, order.ctypes.data_as(P), hb.ctypes.data_as(P), mv.ctypes.data_as(P),
                               g(gc).ctypes.data_as(P), hw.ctypes.data_as(P), Cc, hist_ver.ctypes.data_as(P),
                               hist_vid.ctypes.data_as(P), hist_vlen.ctypes.data_as(P), hist_st.ctypes.data_as(P),
                               fl.ctypes.data_as(P), fs.ctypes.data_as(P), fc.ctypes.data_as(P),
                               g(fst).ctypes.data_as(P), 15625)
        for a, b in prs:
            L.orc_snapshot_row(h, a)
            L.orc_snapshot_row(h, b)

    def restore(i):
        for a, b in mine[i]:
            L.orc_restore_row(hs[i], a)
            L.orc_restore_row(hs[i], b)

    def run(i):
        for a, b in mine[i]:
            L.orc_exchange(hs[i], a, b, t * 15625)

    # one thread: every handle's pairs in turn, on restored rows, until ~min_seconds/3 are timed
    dt1, reps1 = 0.0, 0
    while dt1 < min_seconds / 3 or reps1 == 0:
        if reps1:
            for i in range(T):
                restore(i)
        t0 = time.perf_counter()
        for i in range(T):
            run(i)
        dt1 += time.perf_counter() - t0
        reps1 += 1
    # T threads (ctypes drops the GIL during each oracle call), a barrier around every timed pass
    import threading
    bar = threading.Barrier(T + 1)
    stop = [False]

    def worker(i):
        while True:
            bar.wait()  # restore
            if stop[0]:
                return
            restore(i)
            bar.wait()  # go
            run(i)
            bar.wait()  # done

    ths = [threading.Thread(target=worker, args=(i,), daemon=True) for i in range(T)]
    for th in ths:
        th.start()
    dtT, repsT = 0.0, 0
    while dtT < min_seconds or repsT == 0:
        bar.wait()
        bar.wait()
        t0 = time.perf_counter()
        bar.wait()
        dtT += time.perf_counter() - t0
        repsT += 1
    stop[0] = True
    bar.wait()
    for th in ths:
        th.join()
    nd = 0
    for h in hs:
        st = orc_mod._Stats()
        L.orc_get_stats(h, C.byref(st))
        nd += st.node_deltas
        L.orc_destroy(h)
    return {
        "value": len(pairs) * repsT / dtT,
        "unit": "exchanges/s",
        "cores": T,
        "kind": "port",
        "single_core_value": len(pairs) * reps1 / dt1,
        "sample": f"{len(pairs)} exchanges (disjoint pairs of the next round's first phase) at N={n}, K={K} on "
                  f"oracle rows copied from the device state after the timed rounds, dealt to {T} host threads "
                  f"(one oracle handle each) and run {repsT}x on restored rows ({dtT:.1f} s wall); one thread: "
                  f"{reps1}x ({dt1:.1f} s); {nd // (reps1 + repsT)} NodeDeltas per pass",
    }


class RehearsalComm:
    """One slice of a G-slice cluster on this GPU (``--rehearse-slices G``): the other slices' gathered
    totals are zeros, so the packing is NOT the cluster's -- a timing rehearsal of one GPU's share of a
    G-GPU run (memory footprint, kernel times), never a result."""

    def __init__(self, world: int):
        self.world = world
        self.rank = 0

    def gather(self, parts):
        import torch

        (x,) = parts
        return torch.cat([x[None], torch.zeros((self.world - 1,) + tuple(x.shape), dtype=x.dtype, device=x.device)])

    def sum_counters(self, per_slice):
        return per_slice[0]

    def any(self, flag):
        return flag


def aggregate(exchanges: float, elapsed: float, dist=None, dev=None) -> tuple[float, float]:
    """Whole-job totals: exchanges summed over ranks, time = the slowest rank's."""
    if dist is None:
        return float(exchanges), float(elapsed)
    import torch

    ex = torch.tensor([float(exchanges)], dtype=torch.float64, device=dev)
    tm = torch.tensor([float(elapsed)], dtype=torch.float64, device=dev)
    dist.all_reduce(ex, op=dist.ReduceOp.SUM)
    dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    return float(ex.item()), float(tm.item())


def copy_ceiling(torch, dev, nbytes: int = 1 << 30, reps: int = 20) -> float:
    """Measured streaming-copy ceiling: read + write bytes of a 1 GiB
    device-to-device copy over its HIP-event time, in GB/s."""
    src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev).fill_(1)
    dst = torch.empty_like(src)
    dst.copy_(src)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize(dev)
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del src, dst
    return gbs


def load_traffic(workload: str, exchanges_per_launch: float):
    """HBM bytes per k_exchange launch from the committed rocprofv3 PMC summary of this workload
    (tools/profile.sh + tools/pmc_summary.py): measured bytes per exchange x this run's exchanges per launch."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    try:
        e = json.load(open(path)).get(workload)
        if e is None or e.get("k_exchange_bytes_per_exchange") is None:
            return None
        return e["k_exchange_bytes_per_exchange"] * exchanges_per_launch
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=65536)
    ap.add_argument("--keys", type=int, default=16)
    ap.add_argument("--fanout", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--settle", type=int, default=20,
                    help="untimed rounds run as part of setup, before the warmup: the warm start has every view "
                         "equal to its owner, and the heartbeat / version lags reach their steady-state spread "
                         "only after ~15 rounds (SURVEY 8(d): time 20+ rounds after warm-up)")
    ap.add_argument("--cpu-sample", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=min(16, len(os.sched_getaffinity(0))),
                    help="host threads for the CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--slices", type=int, default=1, help="owner-column slices in this process (1-GPU rehearsal)")
    ap.add_argument("--mtu", type=int, default=65507)
    ap.add_argument("--peer-select", action="store_true",
                    help="schedule each round with the device's select_nodes_for_gossip (gs_select_peers) and "
                         "Luby phases (gs_schedule_phases) instead of the workload's permutation schedule")
    ap.add_argument("--rehearse-slices", type=int, default=0,
                    help="hold only slice 0 of G owner-column slices (one GPU's share of a G-GPU run; timing only)")
    ap.add_argument("--no-held", action="store_true",
                    help="version-only layout (GS_NO_HELD, config 4): needs an mtu no delta reaches")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.shard import DistComm, LocalComm, ShardGroup
    from aiocluster_amd.sim import GossipSim
    from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

    n, K = args.nodes, args.keys
    cfg = dict(DEFAULT_CFG)  # mtu 65507, window 1000, phi 8, max_interval 10 s, prior 5 s
    cfg["mtu"] = args.mtu
    spec = WorkloadSpec(n=n, k=K, fanout=args.fanout, seed=args.seed, init="warm", write_frac=0.05,
                        down_frac=0.05, down_rounds=3)
    workload = (f"N={n} K={K} F={args.fanout} warm, 5% writes + 5% down churn/round, window 1000, mtu {args.mtu}"
                + (", version-only views (GS_NO_HELD)" if args.no_held else "")
                + (", device peer selection (select_nodes_for_gossip, 8 seeds) + Luby phases" if args.peer_select
                   else ""))
    t_setup = time.perf_counter()
    ids = synthetic_node_ids(n)
    boot = []  # Cluster(initial_key_values): key k of owner j = "v{j}.{k}.i", as K batches of distinct owners
    for k in range(K):
        ops = np.zeros((n, 5), dtype=np.uint32)
        ops[:, 0] = np.arange(n)
        ops[:, 1] = k
        ops[:, 3] = 1 + k * n + np.arange(n)
        ops[:, 4] = 3 + digits(np.arange(n)) + digits(np.full(n, k)) + 1
        boot.append(ops)
    kw = dict(init="warm", device=str(dev), tombstones=False, fd_ring=False, hist_cap=16, initial_ops=boot,
              held=not args.no_held)
    if world > 1 and args.slices > 1:
        raise SystemExit("--slices is a one-process rehearsal; with --gpus N each rank holds one slice")
    group = None
    if world > 1:
        sims = [GossipSim(ids, key_names(K), cfg, shards=world, shard=rank, **kw)]
        group = ShardGroup(sims, DistComm(), cfg["mtu"])
    elif args.rehearse_slices > 1:
        sims = [GossipSim(ids, key_names(K), cfg, shards=args.rehearse_slices, shard=0, **kw)]
        group = ShardGroup(sims, RehearsalComm(args.rehearse_slices), cfg["mtu"])
    elif args.slices > 1:
        sims = [GossipSim(ids, key_names(K), cfg, shards=args.slices, shard=g, **kw) for g in range(args.slices)]
        group = ShardGroup(sims, LocalComm(args.slices), cfg["mtu"])
    else:
        sims = [GossipSim(ids, key_names(K), cfg, **kw)]
    sim = sims[0]
    R0 = args.settle + args.warmup  # first timed round
    plans = prepare(sim, spec, R0 + args.steps + 1, torch, dev)
    sel = None
    if args.peer_select:
        from aiocluster_amd.peers import PeerSelector

        if group is not None:
            raise SystemExit("--peer-select needs the whole matrix on one GPU")
        sel = PeerSelector(sim, fanout=args.fanout, seeds=list(range(0, n, max(1, n // 8))), seed=args.seed)
    torch.cuda.synchronize(dev)
    log(f"setup {time.perf_counter() - t_setup:.1f}s")

    for r in range(args.settle):
        ts = time.perf_counter()
        run_round(sims, plans[r], group=group, sel=sel)
        torch.cuda.synchronize(dev)
        log(f"settle round {r}: {(time.perf_counter() - ts) * 1e3:.1f} ms, {plans[r]['exchanges']} exchanges")
    for r in range(args.settle, R0):
        run_round(sims, plans[r], group=group, sel=sel)
    torch.cuda.synchronize(dev)
    for s_ in sims:
        s_.check()
        s_.reset_counters()
    events = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for r in range(R0, R0 + args.steps):
        run_round(sims, plans[r], events, group, sel)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    local = [s_.check() for s_ in sims]
    inexact = sum(s_.inexact_views() for s_ in sims)  # views with holes (HELD kept), GS_MV_INEXACT
    c = group.comm.sum_counters(local) if group is not None else local[0]
    exch = sum(plans[r]["exchanges"] for r in range(R0, R0 + args.steps))
    assert c["exchanges"] == exch, (c["exchanges"], exch)
    kern_ms = sum(e0.elapsed_time(e1) for e0, e1 in events)
    launches = len(events)
    # a sliced cluster: every rank runs the same exchanges on its columns -> count them once
    exch_total, elapsed_max = aggregate(exch if (group is None or rank == 0) else 0, elapsed, dist, dev)
    # this process's algorithmic bytes (all its slices) over its phase time
    alg_local = sum(x["alg_bytes"] for x in local)
    # algorithmic bytes per exchange, SURVEY.md §8(d): N(24 + 8) (read M, G, H of both rows, write both
    # H rows) + D (delta packing + apply bytes, counted in-kernel); the 32r failure-detector bytes are
    # priced into k_liveness, where this design performs the window updates
    ncols = sum(s_.ncol for s_ in sims)
    alg_survey = exch * 32 * ncols + sum(x["pack_bytes"] for x in local)
    achieved = alg_survey / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    achieved_in_kernel = alg_local / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    traffic = load_traffic(workload, exch / max(1, len(events))) if group is None else None
    copy_gbs = copy_ceiling(torch, dev) if rank == 0 else None
    cpu = None
    if rank == 0 and group is None and not args.no_cpu_baseline:
        cpu = cpu_baseline(sim, spec, cfg, plans[R0 + args.steps], args.cpu_sample, args.cpu_seconds,
                           args.cpu_threads)
    if rank == 0:
        line = {
            "metric": ("REHEARSAL (one GPU's slice of a %d-GPU run, packing not the cluster's): exchanges/s"
                       % args.rehearse_slices if args.rehearse_slices > 1 else
                       "simulated gossip exchanges/sec at 65,536 nodes, 1-8 GPUs; % HBM peak"),
            "value": exch_total / elapsed_max,
            "unit": "exchanges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if group is not None else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded workload generator; no dataset)",
            "config": {
                "workload": workload,
                "nodes": n,
                "keys": K,
                "fanout": args.fanout,
                "exchanges_per_step": exch / args.steps,
                "parallelism": (f"owner-column slices x{world} (RCCL all-gather of slice totals)" if world > 1
                                else f"slice 0 of {args.rehearse_slices} (rehearsal)" if args.rehearse_slices > 1
                                else f"owner-column slices x{args.slices} in one process" if group is not None
                                else "1 GPU"),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_exchange" if group is None else "sliced phase (count + gather + pack), per rank",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "measured_copy_ceiling": copy_gbs,
                # the PMC-measured HBM bytes of one launch over its HIP-event time, against the copy
                # ceiling ("achieved" prices the SURVEY formula's u32 rows; this layout moves fewer bytes)
                "traffic_gbs": traffic / (kern_ms / max(1, launches) / 1e3) / 1e9 if traffic and kern_ms else None,
                "traffic_frac_of_copy_ceiling": (traffic / (kern_ms / max(1, launches) / 1e3) / 1e9 / copy_gbs
                                                 if traffic and kern_ms and copy_gbs else None),
                "alg_bytes_per_launch": alg_survey / max(1, launches),
                "alg_bytes_formula": "exchanges x 32 x N + pack_bytes (SURVEY 8(d) minus the FD term, see DESIGN.md)",
                "in_kernel_bytes_per_launch": alg_local / max(1, launches),
                "achieved_in_kernel": achieved_in_kernel,
                "avg_launch_ms": kern_ms / max(1, launches),
                "launches": launches,
                "kernel_share_of_step": kern_ms / 1e3 / elapsed,
            },
            "cpu_baseline": cpu,
            **({"ABLATION_RESULTS_INVALID": os.environ["GS_ABLATE"]} if os.environ.get("GS_ABLATE") else {}),
            "counters": {**{k: v for k, v in c.items() if not k.startswith("err_")}, "inexact_views": inexact},
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
