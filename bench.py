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

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel (k_pass1; each phase is k_pass1,
then k_lite -- whole deltas sized from the owners' version logs and applied -- then the exact packer for
the rest; every kernel HIP-event timed on the library's stream, gs_kernel_times), the CPU baseline (the C oracle on 16 host threads and on one, timed
on a bounded sample of exchanges whose rows are copied from the device state after the timed rounds,
checked bit-exact against the device first) and 3 rounds scheduled by the device's own peer selection.
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


from aiocluster_amd.driver import digits, prepare, run_round  # noqa: E402,F401  (tools/ import them from here)


def cpu_baseline(sim, cfg, rd, sample: int, min_seconds: float = 10.0, threads: int = 1):
    """The C oracle (``threads`` host cores) on ``sample`` exchanges of the first phase of round ``rd``,
    on rows copied from the device after that round's ``gs_begin_round`` -- the same workload at full N.

    Before timing, the copied rows double as a full-size parity check (oracle/rowcheck.py): the device
    runs that phase (all of it) and closes the round, the oracle runs the sampled exchanges and the
    liveness sweep of their rows, and the rows must be bit-identical (raises otherwise).  Then the
    oracle's exchanges are timed alone, repeated on restored rows."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import rowcheck  # test infrastructure: the checker, timed here as the CPU baseline

    from aiocluster_amd import driver

    a_all, b_all, _, t = rd["phases"][0]
    pairs = list(zip(a_all[:sample].cpu().numpy().tolist(), b_all[:sample].cpu().numpy().tolist()))
    T = max(1, min(threads, len(pairs)))
    ro = rowcheck.RowOracle(sim, cfg)
    hs = [ro.new_handle() for _ in range(T)]
    mine = [pairs[i::T] for i in range(T)]
    rows, owner = [], []
    for i, prs in enumerate(mine):
        for a, b in prs:
            rows += [a, b]
            owner += [hs[i], hs[i]]
    ro.load(rows, hs, owner=owner)
    L = ro.L
    for h, prs in zip(hs, mine):
        for a, b in prs:
            L.orc_snapshot_row(h, a)
            L.orc_snapshot_row(h, b)
    # -- full-size parity on the sample (untimed)
    driver.run_phases([sim], rd, phases=[rd["phases"][0]])
    driver.end([sim], rd, tick=t + 1)
    for h, prs in zip(hs, mine):
        for a, b in prs:
            ro.exchange(h, a, b, t)
        for a, b in prs:
            ro.liveness(h, a, t + 1)
            ro.liveness(h, b, t + 1)
    got = sim.export_rows(rows)
    parts = [ro.export_rows(h, [x for a, b in prs for x in (a, b)]) for h, prs in zip(hs, mine)]
    want = {k: np.concatenate([p_[k] for p_ in parts]) for k in parts[0]}
    diff = rowcheck.compare_exports(got, want)
    if diff is not None:
        raise SystemExit(f"full-size parity FAILED on the CPU-baseline sample: device vs oracle: {diff}")
    nd_check = sum(ro.stats(h)["node_deltas"] for h in hs)

    def restore(i):
        for a, b in mine[i]:
            L.orc_restore_row(hs[i], a)
            L.orc_restore_row(hs[i], b)

    def run(i):
        for a, b in mine[i]:
            L.orc_exchange(hs[i], a, b, t * rowcheck.TICK_US)

    # host cores: thread i pinned to the i-th CPU this process may use (the main thread to the next one)
    cpus = sorted(os.sched_getaffinity(0))
    pin = cpus[: T + 1] if len(cpus) > T else None

    def pin_to(k):
        if pin is not None:
            os.sched_setaffinity(0, {pin[k]})  # Linux: pid 0 = the calling thread

    load0 = os.getloadavg()[0]
    # one thread: every handle's pairs in turn, each timed right after its own rows are restored -- as each of
    # the T threads below restores its handle just before its timed pass (like for like: cache-warm rows in
    # both legs; VERDICT r4: restoring all handles first left the single thread's rows cold)
    dt1, reps1, rate1 = 0.0, 0, []
    pin_to(0)  # the threaded leg's first core (a different core made the two legs incomparable)
    while dt1 < min_seconds / 3 or reps1 < 3:
        dt = 0.0
        for i in range(T):
            restore(i)
            t0 = time.perf_counter()
            run(i)
            dt += time.perf_counter() - t0
        dt1 += dt
        reps1 += 1
        rate1.append(len(pairs) / dt)
    pin_to(T)  # the main thread (it only waits at the barriers) off the workers' cores
    # T threads (ctypes drops the GIL during each oracle call), a barrier around every timed pass
    import threading
    bar = threading.Barrier(T + 1)
    stop = [False]

    def worker(i):
        pin_to(i)
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
    dtT, repsT, rateT = 0.0, 0, []
    while dtT < min_seconds or repsT < 3:
        bar.wait()
        bar.wait()
        t0 = time.perf_counter()
        bar.wait()
        dt = time.perf_counter() - t0
        dtT += dt
        repsT += 1
        rateT.append(len(pairs) / dt)
    stop[0] = True
    bar.wait()
    for th in ths:
        th.join()
    if pin is not None:
        os.sched_setaffinity(0, set(cpus))
    ro.close()
    n, K = sim.n, sim.k
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), model)
    except OSError:
        pass
    q = lambda xs, f: float(np.percentile(np.asarray(xs), f))  # noqa: E731
    return {
        "value": q(rateT, 50),
        "unit": "exchanges/s",
        "cores": T,
        "kind": "port",
        "statistic": f"median of {repsT} timed passes (p10 {q(rateT, 10):.0f}, p90 {q(rateT, 90):.0f}; mean "
                     f"{len(pairs) * repsT / dtT:.0f})",
        "single_core_value": q(rate1, 50),
        "threaded_per_core_value": q(rateT, 50) / T,
        "single_core_statistic": f"median of {reps1} passes (p10 {q(rate1, 10):.0f}, p90 {q(rate1, 90):.0f}); each "
                                 f"handle timed right after its own rows are restored, as in the threaded leg",
        "host": {"cpu_model": model, "cpus_allowed": len(cpus),
                 "pinning": (f"thread i on CPU {pin[0]}+i, the single-thread leg on CPU {pin[0]} (thread 0's)"
                             if pin is not None
                             else "unpinned (fewer allowed CPUs than threads)"),
                 "loadavg_1min_before": load0},
        "sample": f"{len(pairs)} exchanges (disjoint pairs of the first phase of the round after the timed ones) "
                  f"at N={n}, K={K}, on oracle rows copied from the device state after that round's "
                  f"gs_begin_round, dealt to {T} host threads (one oracle handle each) and run {repsT}x on "
                  f"restored rows ({dtT:.1f} s wall); one thread: {reps1}x ({dt1:.1f} s); {nd_check} NodeDeltas "
                  f"per pass",
        "parity_check": f"{len(rows)} device rows after that phase + liveness == oracle rows (bit-exact)",
    }


class ObjComm:
    """Object collectives for the sliced parity check over a gloo group of the bench's ranks (host pickles, so
    the same code runs beside an RCCL group): ``gather`` collects every rank's list on rank 0, ``allmax``."""

    def __init__(self, dist):
        self.dist = dist
        self.group = dist.new_group(backend="gloo")
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def gather(self, xs: list):
        out = [None] * self.world if self.rank == 0 else None
        self.dist.gather_object(xs, out, dst=0, group=self.group)
        return [x for part in out for x in part] if self.rank == 0 else None

    def allmax(self, x: int) -> int:
        import torch

        t = torch.tensor([int(x)], dtype=torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def bcast(self, obj):
        box = [obj]
        self.dist.broadcast_object_list(box, src=0, group=self.group)
        return box[0]


def sliced_parity(group, cfg, rd, sample: int, dist) -> dict | None:
    """Bit-exact check of a sliced run (every rank calls it; rank 0 returns the result): oracle/rowcheck's
    ``check_sliced_phase_rows`` -- the rows of ``sample`` exchanges of ``rd``'s first phase, copied out of every
    slice and joined into whole-cluster rows, vs the same exchanges + liveness in the C oracle.  Raises on a
    mismatch, on every rank, like the single-GPU CPU-baseline check."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import rowcheck  # test infrastructure: the checker

    comm = ObjComm(dist) if dist is not None else None
    t0 = time.perf_counter()
    res, info = rowcheck.check_sliced_phase_rows(group, cfg, rd, sample=sample, comm=comm)
    ok = all(r["exact"] for r in res) if res is not None else None
    if comm is not None:
        ok = comm.bcast(ok)
    if not ok:
        raise SystemExit(f"sliced full-size parity FAILED: {res}")
    if res is None:
        return None
    return {"exact": True, "per_slice": res, **info, "seconds": time.perf_counter() - t0,
            "what": "rows of the sampled exchanges of the first phase of the round after the timed ones, copied "
                    "from every slice after gs_begin_round and joined into whole-cluster rows (every owner column, "
                    "so the MTU walk across slices is covered); the phase ran on the devices through the sliced "
                    "driver, then the liveness sweep; each slice's columns == the C oracle's (bit-exact)"}


def aggregate(exchanges: float, elapsed: float, dist=None, dev=None) -> tuple[float, float]:
    """Whole-job totals: exchanges summed over ranks, time = the slowest rank's."""
    if dist is None:
        return float(exchanges), float(elapsed)
    import torch

    dev = dev if dist.get_backend() == "nccl" else "cpu"  # (gloo rehearsals: host tensors)
    ex = torch.tensor([float(exchanges)], dtype=torch.float64, device=dev)
    tm = torch.tensor([float(elapsed)], dtype=torch.float64, device=dev)
    dist.all_reduce(ex, op=dist.ReduceOp.SUM)
    dist.all_reduce(tm, op=dist.ReduceOp.MAX)
    return float(ex.item()), float(tm.item())


def copy_ceiling(torch, dev, stream, nbytes: int = 2 << 30, reps: int = 10) -> float:
    """Measured streaming-copy ceiling: read + write bytes of a 2 GiB copy by the
    library's hand-written 16-B-per-lane kernel (gs_stream_copy) over its HIP-event time, in GB/s."""
    from aiocluster_amd import _lib

    L = _lib.load()
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty_like(src)
    P = C.c_void_p

    def go():
        rc = L.gs_stream_copy(P(dst.data_ptr()), P(src.data_ptr()), nbytes, P(stream.cuda_stream))
        assert rc == 0, rc

    go()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        go()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del src, dst
    return gbs


def kernel_source_hash() -> str:
    """SHA-256 (16 hex) of the HIP source + header: ties a committed PMC summary to the kernels it measured."""
    import hashlib

    h = hashlib.sha256()
    for f in (os.path.join(REPO, "aiocluster_amd", "csrc", "gossip_sim.hip"), os.path.join(REPO, "include",
                                                                                          "gossip_sim.h")):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load_traffic(workload: str, kernel: str, units_per_launch: float):
    """HBM bytes per launch of ``kernel`` from the rocprofv3 PMC summary (tools/profile.sh +
    tools/pmc_summary.py), only if it measured THESE kernels (same source hash): measured bytes per unit
    (exchange for the phase kernels, launch for k_liveness) x this run's units per launch.
    Returns (bytes or None, provenance note)."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None, "no PMC summary"
    try:
        e = json.load(open(path)).get(workload)
    except Exception as x:  # noqa: BLE001
        return None, f"unreadable PMC summary: {x}"
    if e is None or kernel not in e.get("kernels", {}):
        return None, f"no PMC summary of {kernel} for this workload"
    src = kernel_source_hash()
    if e.get("source_hash") != src:
        return None, f"PMC summary is stale (kernels {e.get('source_hash')} != {src})"
    k = e["kernels"][kernel]
    return k["hbm_bytes_per_unit"] * units_per_launch, (
        f"rocprofv3 PMC run {e.get('tag')} of these kernels ({src}): (FETCH_SIZE x {k.get('fetch_factor')} + "
        f"WRITE_SIZE x {k.get('write_factor')}) per {k.get('unit')}, factors calibrated on known-byte streams "
        f"({e.get('calibration')}), x this run's units per launch")


KERNEL_OF = {"pass1": "k_pass1", "pack": "k_pack_slice", "liveness": "k_liveness", "count": "k_settle", "lite": "k_lite"}


def pass1_kernel(wide_views: bool) -> str:
    """The pass-1 kernel the library launches (gs_create: GS_MV8 record phases run k_pass1v unless env GS_P1=old or
    GS_PACK asks for another packing mode)."""
    if wide_views or os.environ.get("GS_P1") == "old" or os.environ.get("GS_PACK", "split") != "split":
        return "k_pass1"
    return "k_pass1v"


def roofline(sims, local_c, exch, kt, elapsed, torch, dev, rank, group, workload, p1name="k_pass1",
             steps: int = 1) -> dict:
    """Roofline of the dominant kernel (by summed time; HBM-bound integer/byte work, no MFMA) plus the
    same figures for the other kernels of the round.

    Times: the library's HIP events around every launch of each kind, on the stream the kernels run on
    (gs_set_timing / gs_kernel_times).  Bytes (``achieved``): the layout's algorithmic HBM bytes per
    launch, counted in-kernel (C_ALG: element bytes of HBM-resident regions the kernel must load and
    store; pass-3 part C_PACKB), DESIGN.md §4/§7.  The SURVEY §8(d) formula (u32 M/G/H rows) is kept as
    a secondary figure: this layout stores heartbeats and max versions as u16 and has no last_gc
    region without tombstones, so that formula overstates the bytes."""
    alg = sum(x["alg_bytes"] for x in local_c)
    packb = sum(x["pack_bytes"] for x in local_c)
    liteb = sum(x["lite_bytes"] for x in local_c)  # k_lite's part of pack_bytes
    liveb = sum(x["live_bytes"] for x in local_c)  # k_liveness's element bytes
    ncols = sum(s_.ncol for s_ in sims)
    fused = kt["pack"][1] == 0
    # k_pass1v with k_lite's slot work in its epilogue (round 5; no k_lite launches): its bytes are pass 1's too
    # (one slice only: a sliced count pass runs the slot work in k_settle<1, LITE> by default, GS_P1LITE < 2)
    lite_in_p1 = group is None and kt.get("lite", (0.0, 0))[1] == 0 and liteb > 0 and not fused
    per = {}
    for kind, (ms, launches) in kt.items():
        if not launches:
            continue
        avg_s = ms / launches / 1e3
        b = None
        if kind == "pass1":
            b = (alg if fused else alg - packb + (liteb if lite_in_p1 else 0)) / launches
        elif kind == "pack":
            b = (packb - liteb) / launches
        elif kind == "lite":
            b = liteb / launches
        elif kind == "liveness":
            b = liveb / launches
        kname = p1name if kind == "pass1" else KERNEL_OF[kind]
        shown = kname + (" (+ k_lite slot work in its epilogue)" if kind == "pass1" and lite_in_p1 else "")
        ent = {"kernel": ("k_pass1<fused>: pass 1, then packing + apply_delta in the same workgroup"
                          if (fused and kind == "pass1") else shown),
               "avg_launch_ms": avg_s * 1e3, "launches": launches, "share_of_step": ms / 1e3 / elapsed}
        if b is not None:
            ent.update(alg_bytes_per_launch=b, achieved=b / avg_s / 1e9, frac=b / avg_s / 1e9 / HBM_PEAK_GBPS)
        units = exch / launches if kind != "liveness" else 1.0
        if group is None:
            tr, note = load_traffic(workload, kname, units)
            ent.update(traffic=tr, traffic_source=note, traffic_gbs=tr / avg_s / 1e9 if tr else None)
        per[kind] = ent
    dom = max(per, key=lambda k: kt[k][0])
    d = per[dom]
    copy_gbs = copy_ceiling(torch, dev, sims[0].stream) if rank == 0 else None
    launches = kt["pass1"][1] or 1
    survey = (exch * 32 * ncols + packb) / launches
    # the whole step: every phase kernel's and k_liveness' in-kernel algorithmic bytes of the timed rounds over
    # the step's wall time (kernels not counted -- lag sweeps, round starts, owner writes -- add time, not bytes)
    step_bytes = (alg + liveb) / max(steps, 1)
    step_s = elapsed / max(steps, 1)
    return {
        "bound": "hbm",
        "kernel": d["kernel"] if group is None else d["kernel"] + " (one owner-column slice, per rank)",
        "achieved": d.get("achieved"),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": d.get("frac"),
        "traffic": d.get("traffic"),
        "traffic_source": d.get("traffic_source", "sliced run: not profiled"),
        "alg_bytes_per_launch": d.get("alg_bytes_per_launch"),
        "alg_bytes_basis": "in-kernel element bytes of HBM-resident regions: pass 1 (C_ALG - C_PACKB): both rows' "
                           "heartbeat + max_version views read (1 B each with GS_HB8 + GS_MV8), changed 16-column "
                           "heartbeat groups written, report bit planes, candidate records and overflow bitmap words "
                           "written; k_lite / packer (C_LITEB / C_PACKB - C_LITEB): records, version-log entries, "
                           "NodeId sizes, history rows, max_version stores; k_liveness (C_LIVEB): windows, state bytes, "
                           "times of death read and written, report planes replayed",
        "avg_launch_ms": d["avg_launch_ms"],
        "launches": d["launches"],
        "kernel_share_of_step": d["share_of_step"],
        "measured_copy_ceiling": copy_gbs,
        "achieved_frac_of_copy_ceiling": d["achieved"] / copy_gbs if copy_gbs and d.get("achieved") else None,
        "traffic_gbs": d.get("traffic_gbs"),
        "kernels": per,
        "note": ("k_pass1v streams 8-bit heartbeat + max_version views (GS_HB8 + GS_MV8), 16 columns per lane, and "
                 "runs pass 1's per-column rules on 4 views per 32-bit word (DESIGN.md §4)") if d["kernel"].startswith("k_pass1v")
                else None,
        "step_alg_bytes": step_bytes,
        "step_achieved": step_bytes / step_s / 1e9,
        "step_frac": step_bytes / step_s / 1e9 / HBM_PEAK_GBPS,
        "step_basis": "(C_ALG + C_LIVEB) per timed round / ms_per_step: pass 1, k_lite, the exact packer and "
                      "k_liveness in-kernel bytes over the whole round's wall time (launch gaps and kernels without a byte count "
                      "kernels included)",
        # the SURVEY §8(d) formula prices u32 heartbeat / max_version / last_gc rows (32 B per column per exchange);
        # this layout streams 1-byte views, so this is what the u32 layout would have to move at this pass-1 time,
        # an equivalent rate, NOT an achieved one (it exceeds the HBM peak)
        "u32_layout_equiv_bytes_per_phase": survey,
        "u32_layout_equiv_gbs_not_achieved": survey / (kt["pass1"][0] / launches / 1e3) / 1e9 if kt["pass1"][0] else None,
    }


C4_NODES, C4_GPUS = 262144, 8


def config4_leg(args, world: int, rank: int, dist, dev) -> dict:
    """BASELINE config 4: 262,144 nodes over 8 GPUs, one owner-column slice of 32,768 columns per rank
    (all 262,144 observer rows: ~170 GB of HBM per GPU), config 4's contract: warm start, no
    deletes, version-only views (GS_NO_HELD), mtu 2^30 above every delta (no truncation).  Same workload
    shape as the headline (K = 16, F = 3, 5 % writes + 5 % up/down churn per round, window 1000).  With 8
    ranks the slices gather their DeltaPb totals per phase over RCCL (torch.distributed "nccl");
    ``world == 1`` holds slice 0 of 8 alone (``SoloComm``: exact for its columns under this contract,
    tests/test_gpu_config4.py) and reports one GPU's share.  Weak in the sense of fixed work per GPU:
    every rank runs every exchange on its own columns."""
    import torch

    from aiocluster_amd import driver
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.shard import DistComm, ShardGroup, SoloComm
    from aiocluster_amd.sim import GossipSim
    from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

    n, K = C4_NODES, args.keys
    cfg = dict(DEFAULT_CFG)
    cfg["mtu"] = 1 << 30
    spec = WorkloadSpec(n=n, k=K, fanout=args.fanout, seed=args.seed, init="warm", write_frac=0.05,
                        down_frac=0.05, down_rounds=3)
    t0 = time.perf_counter()
    shard = rank if world == C4_GPUS else 0
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", device=str(dev), tombstones=False,
                    fd_ring=False, hist_cap=16, initial_ops=driver.boot_ops(n, K), held=False, shards=C4_GPUS,
                    shard=shard, hb8=not args.wide_views, mv8=not args.wide_views)
    comm = DistComm() if world == C4_GPUS else SoloComm(C4_GPUS, 0)
    grp = ShardGroup([sim], comm, cfg["mtu"])
    S, W, T = args.config4_settle, 1, args.config4_steps
    plans = driver.prepare(spec, S + W + T + 1, torch, dev)
    torch.cuda.synchronize(dev)
    setup = time.perf_counter() - t0
    for r in range(S + W):
        driver.run_round([sim], plans[r], group=grp)
    torch.cuda.synchronize(dev)
    sim.check()
    sim.reset_counters()
    sim.set_timing(True)
    sim.kernel_times()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for r in range(S + W, S + W + T):
        driver.run_round([sim], plans[r], group=grp)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t1
    kt = sim.kernel_times()
    sim.set_timing(False)
    c = grp.check()
    exch = sum(plans[r]["exchanges"] for r in range(S + W, S + W + T))
    assert c["exchanges"] == exch, (c["exchanges"], exch)
    _, el_max = aggregate(0.0, el, dist, dev)
    # parity of this leg: the next round's first phase, sampled rows vs the C oracle
    par = None
    if args.parity_sample:
        rd = plans[S + W + T]
        driver.begin([sim], rd)
        if world == C4_GPUS:  # whole-cluster rows joined from the 8 slices
            par = sliced_parity(grp, cfg, rd, min(args.parity_sample, 8), dist)
        else:  # slice 0 alone: the other columns inert in the oracle, exact under config 4's mtu (no truncation)
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import rowcheck

            diff, info = rowcheck.check_phase_rows(sim, cfg, rd, sample=min(args.parity_sample, 8), group=grp)
            if diff is not None:
                raise SystemExit(f"config-4 slice parity FAILED: {diff}")
            par = {"exact": True, "scope": "slice 0's columns (the others inert; exact: mtu 2^30)",
                   **{k: int(info[k]) for k in ("rows", "node_deltas", "hb_reports")}}
    hz = sim.horizon(rounds=S + W + T + (1 if par is not None else 0))
    sim.close()
    del sim, grp
    torch.cuda.empty_cache()
    return {
        "metric": "simulated gossip exchanges/sec at 262,144 nodes (BASELINE config 4)",
        "value": exch / el_max if world == C4_GPUS else None,
        "one_gpu_share_exchanges_per_s": exch / el if world != C4_GPUS else None,
        "unit": "exchanges/s",
        "n_gpus": world if world == C4_GPUS else 1,
        "slices": C4_GPUS,
        "scope": ("the whole 262,144-node cluster, one slice per GPU" if world == C4_GPUS else
                  "slice 0 of 8 held alone on one GPU: every exchange of the cluster on 32,768 owner columns "
                  "(one GPU's share of the 8-GPU run; exact for those columns under config 4's contract)"),
        "steps": T, "warmup": W, "settle": S,
        "ms_per_step": el_max / T * 1e3,
        "exchanges_per_step": exch / T,
        "setup_s": setup,
        "config": {"workload": f"N={n} K={K} F={args.fanout} warm, 5% writes + 5% down churn/round, window 1000, "
                               f"mtu 2^30 (no truncation), version-only views (GS_NO_HELD)",
                   "parallelism": f"owner-column slices x{C4_GPUS}" + (" (RCCL all-gather of slice totals)"
                                                                       if world == C4_GPUS else ", slice 0 only")},
        "kernel_ms_per_step": {k: v[0] / T for k, v in kt.items() if v[1]},
        "counters": {k: v for k, v in c.items() if not k.startswith("err_")},
        "exactness": hz,
        "parity_check": par,
    }


def peer_select_rounds(sims, plans, r0: int, steps: int, args, n: int, dev) -> dict:
    """Rounds r0 .. r0 + steps (the first untimed) on the headline's state, each scheduled on the device:
    gs_select_peers (select_nodes_for_gossip for every up node from its failure detector's live / dead
    sets, server.py:441-495, 656-717; 8 seeds) and gs_schedule_phases (Luby matchings into conflict-free
    phases; the exchanges that do not fit in its phase budget are counted, not dropped silently)."""
    import torch

    from aiocluster_amd import driver
    from aiocluster_amd.peers import PeerSelector

    sel = PeerSelector(sims[0], fanout=args.fanout, seeds=list(range(0, n, max(1, n // 8))), seed=args.seed)
    driver.run_round(sims, plans[r0], sel=sel)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for r in range(r0 + 1, r0 + 1 + steps):
        driver.run_round(sims, plans[r], sel=sel)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    rds = [plans[r] for r in range(r0 + 1, r0 + 1 + steps)]
    exch = sum(rd["exchanges"] for rd in rds)
    return {
        "value": exch / dt,
        "unit": "exchanges/s",
        "steps": steps,
        "ms_per_step": dt / steps * 1e3,
        "exchanges_per_step": exch / steps,
        "phases_per_round": [rd["phases_run"] for rd in rds],
        "unscheduled_exchanges": sum(rd["unscheduled"] for rd in rds),
        "note": "same cluster state and workload as the headline; the schedule comes from the device's "
                "select_nodes_for_gossip + Luby phases instead of the workload generator's permutations "
                "(selection, scheduling and the phase-offset read back are inside the timed region); phases past the "
                "round's 62-tick budget run as sub-phases at its last tick, so every selected exchange runs",
    }


def mark(sim, which: int) -> None:
    """An empty marker dispatch (gs_mark: k_mark_begin / k_mark_end) on the library's stream: rocprofv3 traces then
    show exactly which dispatches the timed rounds made (tools/pmc_summary.py selects them by position)."""
    from aiocluster_amd import _lib

    rc = _lib.load().gs_mark(which, C.c_void_p(sim.stream.cuda_stream))
    assert rc == 0, rc


def launch_ranks(n: int) -> int:
    """``--gpus N`` without a torch.distributed launcher: start N ranks (one per GPU) with
    torch.distributed.run as a child process -- before this process touches the GPU -- and return its
    exit code."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


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
    ap.add_argument("--parity-sample", type=int, default=16,
                    help="sliced runs (--gpus N > 1, --slices G): after the timed rounds, check this many exchanges "
                         "of the next round's first phase against the C oracle on whole-cluster rows joined from "
                         "every slice (0 = skip)")
    ap.add_argument("--peer-select", action="store_true",
                    help="schedule each round with the device's select_nodes_for_gossip (gs_select_peers) and "
                         "Luby phases (gs_schedule_phases) instead of the workload's permutation schedule")
    ap.add_argument("--peer-select-steps", type=int, default=3,
                    help="after the headline: time this many more rounds scheduled by the device's "
                         "select_nodes_for_gossip (gs_select_peers) + Luby phases (gs_schedule_phases), reported "
                         "as the line's peer_select object (0 = skip)")
    ap.add_argument("--rehearse-slices", type=int, default=0,
                    help="hold only slice 0 of G owner-column slices (one GPU's share of a G-GPU run; timing only "
                         "unless the mtu cannot bind)")
    ap.add_argument("--config4-steps", type=int, default=3,
                    help="with --gpus 8: after the headline, time this many rounds of BASELINE config 4 (262,144 "
                         "nodes, one owner-column slice of 32,768 columns per GPU, version-only views, mtu 2^30), "
                         "reported as the line's config4 object (0 = skip)")
    ap.add_argument("--config4-settle", type=int, default=3, help="untimed config-4 rounds before its warmup")
    ap.add_argument("--config4", action="store_true",
                    help="on one GPU: also run the config-4 leg as slice 0 of 8 held alone (one GPU's share)")
    ap.add_argument("--native-comm", action="store_true",
                    help="--gpus N: the library drives each sliced phase over its own RCCL communicator "
                         "(gs_comm_init + gs_run_phase) instead of aiocluster_amd/shard.py over torch.distributed; "
                         "--slices G: gs_run_phase_group")
    ap.add_argument("--wide-views", action="store_true", default=bool(os.environ.get("GS_WIDE_VIEWS")),
                    help="16-bit heartbeat and max_version views (default: GS_HB8 + GS_MV8, 8-bit views decoded "
                         "against the owner's own values, exact while every view lags < 2^8 / 2^7; swept)")
    ap.add_argument("--hist-cap", type=int, default=64, help="writes kept per (owner, key) (gs_config.hist_cap)")
    ap.add_argument("--no-held", action="store_true",
                    help="version-only layout (GS_NO_HELD, config 4): needs an mtu no delta reaches")
    args = ap.parse_args()

    # --peer-select keeps the 8-bit views: the reference's selection routes the first rounds' seed picks to 8 hub
    # columns whose views fall up to ~280 heartbeats behind (r4b census, tools/hb_lag.py); the lag sweeps move
    # such columns to 16-bit escape slots (gs_config.esc_cols) and back, so the run stays exact
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0:
        if args.gpus > 1:  # plain `python bench.py --gpus N`: become the launcher of N ranks
            raise SystemExit(launch_ranks(args.gpus))
        world = 1
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch

    dist = None
    # GS_BENCH_BACKEND=gloo: a rehearsal of the multi-rank run on fewer GPUs than ranks (ranks share devices,
    # the gathers go through host memory) -- the bench's rank plumbing end to end, not a measurement
    backend = os.environ.get("GS_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from aiocluster_amd import driver
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.shard import DistComm, LocalComm, ShardGroup, SoloComm
    from aiocluster_amd.sim import GossipSim
    from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

    n, K = args.nodes, args.keys
    cfg = dict(DEFAULT_CFG)  # mtu 65507, window 1000, phi 8, max_interval 10 s, prior 5 s
    cfg["mtu"] = args.mtu
    spec = WorkloadSpec(n=n, k=K, fanout=args.fanout, seed=args.seed, init="warm", write_frac=0.05,
                        down_frac=0.05, down_rounds=3)
    workload = (f"N={n} K={K} F={args.fanout} warm, 5% writes + 5% down churn/round, window 1000, mtu {args.mtu}"
                + (", version-only views (GS_NO_HELD)" if args.no_held else "")
                + ("" if args.wide_views else ", 8-bit heartbeat + max_version views (GS_HB8 + GS_MV8)")
                + (", device peer selection (select_nodes_for_gossip, 8 seeds) + Luby phases" if args.peer_select
                   else ""))
    t_setup = time.perf_counter()
    ids = synthetic_node_ids(n)
    # hist_cap 64: HIST is 8 B x N x C x K (0.5 GB at 64); at 16 the writes per (owner, key) reached the cap's
    # projection in ~100 rounds, well before the window horizon
    kw = dict(init="warm", device=str(dev), tombstones=False, fd_ring=False, hist_cap=args.hist_cap,
              initial_ops=driver.boot_ops(n, K), held=not args.no_held, hb8=not args.wide_views,
              mv8=not args.wide_views)
    if world > 1 and args.slices > 1:
        raise SystemExit("--slices is a one-process rehearsal; with --gpus N each rank holds one slice")
    group = None
    if world > 1:
        sims = [GossipSim(ids, key_names(K), cfg, shards=world, shard=rank, **kw)]
        group = ShardGroup(sims, DistComm(), cfg["mtu"], native=args.native_comm)
    elif args.rehearse_slices > 1:
        sims = [GossipSim(ids, key_names(K), cfg, shards=args.rehearse_slices, shard=0, **kw)]
        group = ShardGroup(sims, SoloComm(args.rehearse_slices), cfg["mtu"], native=args.native_comm)
    elif args.slices > 1:
        sims = [GossipSim(ids, key_names(K), cfg, shards=args.slices, shard=g, **kw) for g in range(args.slices)]
        group = ShardGroup(sims, LocalComm(args.slices), cfg["mtu"], native=args.native_comm)
    else:
        sims = [GossipSim(ids, key_names(K), cfg, **kw)]
    sim = sims[0]
    R0 = args.settle + args.warmup  # first timed round
    ps_steps = args.peer_select_steps if (group is None and not args.peer_select) else 0
    plans = driver.prepare(spec, R0 + args.steps + 1 + (1 + ps_steps if ps_steps else 0), torch, dev)
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
        driver.run_round(sims, plans[r], group=group, sel=sel)
        torch.cuda.synchronize(dev)
        log(f"settle round {r}: {(time.perf_counter() - ts) * 1e3:.1f} ms, {plans[r]['exchanges']} exchanges"
            + (f", {plans[r]['phases_run']} phases" if sel is not None else ""))
    for r in range(args.settle, R0):
        driver.run_round(sims, plans[r], group=group, sel=sel)
    torch.cuda.synchronize(dev)
    for s_ in sims:
        s_.check()
        s_.reset_counters()
        s_.set_timing(True)
        s_.kernel_times()  # clear
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    mark(sims[0], 0)  # k_mark_begin / k_mark_end bracket the timed dispatches in a kernel trace (tools/pmc_summary.py)
    t0 = time.perf_counter()
    for r in range(R0, R0 + args.steps):
        driver.run_round(sims, plans[r], None, group, sel)
    mark(sims[0], 1)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    local_c = [s_.check() for s_ in sims]
    inexact = sum(s_.inexact_views() for s_ in sims)  # views with holes (HELD kept), GS_MV_INEXACT
    c = group.comm.sum_counters(local_c) if group is not None else local_c[0]
    exch = sum(plans[r]["exchanges"] for r in range(R0, R0 + args.steps))
    unscheduled = sum(plans[r].get("unscheduled", 0) for r in range(R0, R0 + args.steps))
    assert c["exchanges"] == exch, (c["exchanges"], exch)
    kt = sims[0].kernel_times()  # slice 0's kernels (each rank: its own slice)
    for s_ in sims:
        s_.set_timing(False)
    # a sliced cluster: every rank runs the same exchanges on its columns -> count them once
    exch_total, elapsed_max = aggregate(exch if (group is None or rank == 0) else 0, elapsed, dist, dev)
    roof = roofline(sims[:1], local_c[:1], exch, kt, elapsed, torch, dev, rank, group, workload,
                    pass1_kernel(args.wide_views), steps=args.steps)
    cpu = None
    if rank == 0 and group is None and not args.no_cpu_baseline:
        rd = plans[R0 + args.steps]
        driver.begin(sims, rd)
        cpu = cpu_baseline(sim, cfg, rd, args.cpu_sample, args.cpu_seconds, args.cpu_threads)
    par = None
    if group is not None and args.rehearse_slices <= 1 and args.parity_sample:
        # the sliced run's own parity evidence: the round after the timed ones, phase 0's
        # first exchanges, whole-cluster rows joined from every slice vs the C oracle
        rd = plans[R0 + args.steps]
        driver.begin(sims, rd)
        par = sliced_parity(group, cfg, rd, args.parity_sample, dist)
    ps = None
    if ps_steps:
        ps = peer_select_rounds(sims, plans, R0 + args.steps + 1, ps_steps, args, n, dev)
        # the state after the selected rounds: a lag sweep now, and every device check counter (8-bit views
        # are exact only while every lag stays below the sweep bound: reported, not assumed)
        sims[0].check_heartbeat_lag()
        errs = {k: v for k, v in sims[0].counters().items() if k.startswith("err_") and v}
        ps["device_errors"] = errs
        ps["exact"] = not errs
    rounds_run = (R0 + args.steps + (1 if (cpu is not None or par is not None) else 0)
                  + (ps_steps + 1 if ps is not None else 0))
    horizon = sims[0].horizon(rounds=rounds_run)
    sliced = group is not None  # (the config-4 leg below releases the headline's handles first)
    c4 = None
    if args.config4_steps and (world == C4_GPUS or args.config4):
        for s_ in sims:
            s_.close()
        del sims, sim, group
        torch.cuda.empty_cache()
        c4 = config4_leg(args, world, rank, dist, dev)
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
            "scaling": "strong" if sliced else "weak",
            "vs_baseline": None,
            # the state is integer: heartbeat and max_version views stored as u8 (GS_HB8 + GS_MV8; exact
            # decode against the owners' own values, guarded: DESIGN.md §3), computed in u32; phi in binary64
            "dtype": ("u16" if args.wide_views else "u8") + "/u32 int (phi f64)",
            "data": "synthetic (seeded workload generator; no dataset)",
            "config": {
                "workload": workload,
                "nodes": n,
                "keys": K,
                "fanout": args.fanout,
                "exchanges_per_step": exch / args.steps,
                "parallelism": (f"owner-column slices x{world} (RCCL all-gather of slice totals"
                                + (", library-driven: gs_comm_init)" if args.native_comm else ")") if world > 1
                                else f"slice 0 of {args.rehearse_slices} (rehearsal)" if args.rehearse_slices > 1
                                else f"owner-column slices x{args.slices} in one process" if sliced
                                else "1 GPU"),
                **({"unscheduled_exchanges": unscheduled,
                    # every round of the run, settle and warmup included (round 5 dropped the exchanges past 62
                    # phases in the settle rounds, where the seed hubs are busiest: VERDICT r5)
                    "unscheduled_exchanges_all_rounds": sum(plans[r].get("unscheduled", 0)
                                                            for r in range(R0 + args.steps)),
                    "max_phases_per_round": max(plans[r].get("phases_run", 0) for r in range(R0 + args.steps)),
                    "rounds_with_sub_phases": sum(plans[r].get("phases_run", 0) > 62 for r in range(R0 + args.steps))}
                   if sel is not None else {}),
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            **({"parity_check": par} if par is not None else {}),
            "peer_select": ps,
            **({"ABLATION_RESULTS_INVALID": os.environ["GS_ABLATE"]} if os.environ.get("GS_ABLATE") else {}),
            "counters": {**{k: v for k, v in c.items() if not k.startswith("err_")}, "inexact_views": inexact},
            # headroom to the exact layout's two bounds: err_fd_overflow at a window count of W (compact
            # windows), err_hist_full at hist_cap - 1 writes of one (owner, key); each projected in rounds at
            # the growth rate of this run; fd_saturated (sampled rings' inexact compact rows) raises in check()
            "exactness": horizon,
            "config4": c4,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
