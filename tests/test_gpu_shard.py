"""Owner-column sharding invariance on one GPU (SURVEY.md §8(c) "config 4 is checked for sharding
invariance"): G in-process slices driven through gs_phase_count / gs_phase_pack must end every
round in exactly the state of a single handle (and of the C oracle), including deltas that the MTU
cuts across slice boundaries (the chain steps).  GPU only.
"""

import numpy as np
import pytest
from helpers import compare_exports, make_backend
from oracle import OracleSim

from aiocluster_amd.scenario import initial_by_owner, make_scenario, replay_round, scenario_node_ids
from aiocluster_amd.shard import ShardGroup
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec

pytestmark = pytest.mark.gpu


def sharded(scen, G, **kw):
    return ShardGroup.in_process(scenario_node_ids(scen), scen["keys"], scen["config"], G, init=scen["init"],
                                 initial_values=initial_by_owner(scen), **kw)


@pytest.mark.parametrize("n,G,mtu,tomb", [(256, 2, 1800, True), (384, 3, 3000, False), (512, 4, 1200, True),
                                          (200, 2, 65507, True)])
def test_slices_match_single_handle(n, G, mtu, tomb):
    spec = WorkloadSpec(n=n, k=8, fanout=3, seed=n + G, init="warm", write_frac=0.3,
                        delete_frac=0.1 if tomb else 0.0, ttl_frac=0.05 if tomb else 0.0,
                        down_frac=0.05, down_rounds=2)
    scen = make_scenario(f"shard{n}x{G}", spec, 8, {"mtu": mtu, "tombstone_grace_s": 2})
    kw = dict(tombstones=tomb, fd_ring=False)
    one = make_backend(GossipSim, scen, **kw)
    grp = sharded(scen, G, **kw)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round(grp, scen, r)
        diff = compare_exports(grp.export(), one.export())
        assert diff is None, f"round {r}: {diff}"
    c1, cg = one.check(), grp.check()
    for k in ("exchanges", "hb_reports", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "hb_writes",
              "live_pairs", "tomb_gc"):
        assert cg[k] == c1[k], (k, cg[k], c1[k])
    if mtu < 65507:
        assert c1["truncated"] > 0 and grp.chain_phases > 0  # deltas were cut, chains ran
    o = n // 3
    assert np.array_equal(grp.phi_row(o), one.phi_row(o), equal_nan=True)


@pytest.mark.parametrize("n,G,mtu", [(256, 2, 1800), (384, 3, 3000), (512, 4, 1200)])
def test_native_group_matches_single_handle(n, G, mtu):
    """The library-driven sliced phase (gs_run_phase_group: the driver gs_run_phase runs over RCCL after
    gs_comm_init, with device-copy gathers) vs one handle, MTU cuts across slices included."""
    spec = WorkloadSpec(n=n, k=8, fanout=3, seed=n * G, init="warm", write_frac=0.3, delete_frac=0.1,
                        ttl_frac=0.05, down_frac=0.05, down_rounds=2)
    scen = make_scenario(f"native{n}x{G}", spec, 8, {"mtu": mtu, "tombstone_grace_s": 2})
    kw = dict(tombstones=True, fd_ring=False)
    one = make_backend(GossipSim, scen, **kw)
    grp = sharded(scen, G, native=True, **kw)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round(grp, scen, r)
        diff = compare_exports(grp.export(), one.export())
        assert diff is None, f"round {r}: {diff}"
    c1, cg = one.check(), grp.check()
    for k in ("exchanges", "hb_reports", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "hb_writes"):
        assert cg[k] == c1[k], (k, cg[k], c1[k])
    assert c1["truncated"] > 0


@pytest.mark.parametrize("mv8", [False, True], ids=["hb16", "hb8mv8"])
def test_eight_slices_skip_chain_steps_and_match_single_handle(mv8):
    """G = 8 in-process slices (LocalComm) with a binding mtu: deltas cut across slice boundaries, and the
    skipping chain (a pending slice resumes from its nearest finished predecessor when the slices between
    cannot add a NodeDelta) must give exactly one handle's state, while some chained phase resolves in
    fewer than G pack steps."""
    n, G = 512, 8
    spec = WorkloadSpec(n=n, k=8, fanout=3, seed=88, init="warm", write_frac=0.3, down_frac=0.05, down_rounds=3)
    scen = make_scenario("skip512x8", spec, 10, {"mtu": 900})
    kw = dict(tombstones=False, fd_ring=False, hb8=mv8, mv8=mv8)
    one = make_backend(GossipSim, scen, **kw)
    grp = sharded(scen, G, **kw)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round(grp, scen, r)
        diff = compare_exports(grp.export(), one.export())
        assert diff is None, f"round {r}: {diff}"
    c1, cg = one.check(), grp.check()
    for k in ("exchanges", "hb_reports", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "hb_writes"):
        assert cg[k] == c1[k], (k, cg[k], c1[k])
    chained = [s for s in grp.phase_steps if s > 1]
    assert c1["truncated"] > 0 and chained, grp.phase_steps
    assert min(chained) < G, f"no chained phase skipped a step: {sorted(set(chained))}"


def test_read_rows_copies_out_regions():
    """gs_read_rows (blocking copy-out of observer rows) returns the bytes of the bound regions, and
    complete HELD rows for prefix views (materialized first)."""
    import torch

    from aiocluster_amd import _lib

    spec = WorkloadSpec(n=160, k=8, fanout=3, seed=3, init="warm", write_frac=0.3, down_frac=0.05, down_rounds=2)
    scen = make_scenario("rows160", spec, 6, {"mtu": 1500})
    sim = make_backend(GossipSim, scen, tombstones=False, fd_ring=False)
    for r in range(len(scen["rounds"])):
        replay_round(sim, scen, r)
    lo, hi = 17, 45
    for name, dt in (("HB", torch.int16), ("MV", torch.int16), ("FD", torch.int64), ("FD_STATE", torch.uint8),
                     ("FD_TOD", torch.int32), ("ROW", torch.int32)):
        got = sim.read_rows(name, lo, hi)
        t = sim.regions[name]
        rb = t.numel() * t.element_size() // sim.n
        want = t.view(torch.uint8).reshape(sim.n, rb)[lo:hi].cpu().numpy().tobytes()
        assert got == want, name
    held = np.frombuffer(sim.read_rows("HELD", lo, hi), np.uint8).reshape(hi - lo, sim.np_, sim.kp)
    g = sim._host(list(range(lo, hi)))
    assert np.array_equal(held, g["HELD"])
    assert held.any()
    with pytest.raises(_lib.GsError):
        sim.read_rows("HIST", 0, 1)  # indexed by owner, not observer row


def test_slices_match_oracle_with_ring():
    spec = WorkloadSpec(n=192, k=16, fanout=3, seed=5, init="warm", write_frac=0.2, delete_frac=0.1,
                        down_frac=0.1, down_rounds=3)
    scen = make_scenario("shard192", spec, 10, {"mtu": 2200, "window": 4, "tombstone_grace_s": 3,
                                                "initial_interval_s": 1.0, "phi_threshold": 3.0})
    grp = sharded(scen, 3, fd_ring=True)
    orc = make_backend(OracleSim, scen)
    for r in range(len(scen["rounds"])):
        replay_round(grp, scen, r)
        replay_round(orc, scen, r)
        diff = compare_exports(grp.export(), orc.export())
        assert diff is None, f"round {r}: {diff}"
    s, c = orc.stats(), grp.check()
    assert c["node_deltas"] == s["node_deltas"] and c["truncated"] == s["truncated"] > 0
    assert c["delta_bytes"] == s["delta_bytes"] and c["exchanges"] == s["exchanges"]


def _dist_worker(rank, world, port, scen, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        grp = ShardGroup.distributed(scenario_node_ids(scen), scen["keys"], scen["config"], init=scen["init"],
                                     initial_values=initial_by_owner(scen), fd_ring=False)
        for r in range(len(scen["rounds"])):
            replay_round(grp, scen, r)
        c = grp.check()
        q.put((rank, grp.export(), c, grp.chain_phases))
    finally:
        dist.destroy_process_group()


def test_distributed_slices_two_processes_match_single_handle():
    """DistComm end to end: two processes (gloo for the gather; both slices on cuda:0) vs one handle."""
    import socket

    import torch.multiprocessing as mp

    spec = WorkloadSpec(n=256, k=8, fanout=3, seed=9, init="warm", write_frac=0.3, delete_frac=0.1,
                        down_frac=0.05, down_rounds=2)
    scen = make_scenario("dist256", spec, 6, {"mtu": 1500, "tombstone_grace_s": 2})
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_worker, args=(r, 2, port, scen, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    one = make_backend(GossipSim, scen, fd_ring=False)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
    want = one.export()
    got = {k: np.concatenate([res[0][1][k], res[1][1][k]], axis=1) for k in want}
    assert compare_exports(got, want) is None
    c1 = one.check()
    for k in ("exchanges", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "hb_reports"):
        assert res[0][2][k] == c1[k], k  # counters summed over the ranks
    assert c1["truncated"] > 0 and res[0][3] > 0


def test_version_only_slices_match_single_handle():
    """Config 4's layout (GS_NO_HELD, owner-column slices, mtu above every delta) at a size one GPU holds."""
    spec = WorkloadSpec(n=512, k=16, fanout=3, seed=44, init="warm", write_frac=0.1, down_frac=0.05,
                        down_rounds=3)
    scen = make_scenario("vo512x4", spec, 8, {"mtu": 1 << 30})
    kw = dict(tombstones=False, fd_ring=False, held=False)
    one = make_backend(GossipSim, scen, **kw)
    grp = sharded(scen, 4, **kw)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round(grp, scen, r)
        diff = compare_exports(grp.export(), one.export())
        assert diff is None, f"round {r}: {diff}"
    c1, cg = one.check(), grp.check()
    assert c1["err_holes"] == cg["err_holes"] == 0
    for k in ("exchanges", "node_deltas", "kvs_sent", "delta_bytes", "hb_reports"):
        assert cg[k] == c1[k], k


def _native_group_run(n, G, mtu, seed):
    """(diff or None, one handle's counters, the group's) for G in-process slices in the headline's layout (8-bit
    views, prefix views, no tombstones: the batched group driver's case) through the library's group driver
    (native=True) vs one handle, every round."""
    spec = WorkloadSpec(n=n, k=8, fanout=3, seed=seed, init="warm", write_frac=0.3, down_frac=0.08, down_rounds=3)
    scen = make_scenario(f"grp{n}x{G}", spec, 8, {"mtu": mtu})
    kw = dict(tombstones=False, fd_ring=False, hb8=True, mv8=True)
    one = make_backend(GossipSim, scen, **kw)
    grp = sharded(scen, G, native=True, **kw)
    diff = None
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round(grp, scen, r)
        diff = compare_exports(grp.export(), one.export())
        if diff is not None:
            diff = f"round {r}: {diff}"
            break
    c1, cg = one.check(), grp.check()
    one.close()
    for s in grp.slices:
        s.close()
    return diff, c1, cg


GROUP_KEYS = ("exchanges", "hb_reports", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "hb_writes",
              "lite_slots")


@pytest.mark.parametrize("n,G,mtu", [(256, 2, 700), (512, 8, 900)])
def test_batched_group_driver_hb8mv8_matches_single_handle(n, G, mtu):
    """gs_run_phase_group's batched path (one launch per step for all slices: GroupArgs, the GRP
    instantiations of k_pass1v / k_settle / k_chain_step, k_ov_count / k_ov_write / k_pending) runs only for
    8-bit views without tombstones -- the headline's layout, which the tombstone case above never reaches.  With
    a binding mtu (chains across slices) it must give one handle's state every round."""
    diff, c1, cg = _native_group_run(n, G, mtu, seed=n + G)
    assert diff is None, diff
    for k in GROUP_KEYS:
        if k == "lite_slots":
            continue  # the sliced count pass sizes slots per slice
        assert cg[k] == c1[k], (k, cg[k], c1[k])
    assert c1["truncated"] > 0


def test_batched_group_driver_with_lite_in_pass1_matches_single_handle():
    """The same with env GS_GRP_P1LITE=1 (the lite slot work in k_pass1v's epilogue, the count launch only for the
    slots it leaves) -- read once per process, so a child process runs it."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    code = ("import sys; sys.path[:0] = [%r, %r, %r]\n"
            "from test_gpu_shard import _native_group_run\n"
            "d, c1, cg = _native_group_run(512, 8, 900, seed=77)\n"
            "assert d is None, d\n"
            "assert all(cg[k] == c1[k] for k in ('exchanges', 'node_deltas', 'kvs_sent', 'truncated', 'delta_bytes')), "
            "(c1, cg)\n"
            "assert c1['truncated'] > 0\n"
            "print('ok', c1['truncated'])\n") % (here, os.path.dirname(here), os.path.join(os.path.dirname(here),
                                                                                           "oracle"))
    env = dict(os.environ, GS_GRP_P1LITE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("ok")


def test_lone_slice_other_than_zero_is_refused_by_the_group_driver():
    """slice g > 0 held alone would pack from a zero predecessor total (silently wrong once the mtu
    binds): gs_run_phase_group refuses it; slice 0 alone is exact (its NodeDeltas start every delta)."""
    from aiocluster_amd._lib import GsError
    from aiocluster_amd.shard import SoloComm

    spec = WorkloadSpec(n=256, k=8, fanout=3, seed=3, init="warm", write_frac=0.3, down_frac=0.05, down_rounds=2)
    scen = make_scenario("lone256", spec, 3, {"mtu": 700})
    kw = dict(tombstones=False, fd_ring=False, hb8=True, mv8=True)
    one = make_backend(GossipSim, scen, **kw)
    ids, keys, cfg = scenario_node_ids(scen), scen["keys"], scen["config"]
    s0 = GossipSim(ids, keys, cfg, init=scen["init"], initial_values=initial_by_owner(scen), shards=4, shard=0, **kw)
    s2 = GossipSim(ids, keys, cfg, init=scen["init"], initial_values=initial_by_owner(scen), shards=4, shard=2, **kw)
    g0 = ShardGroup([s0], SoloComm(4, 0), cfg["mtu"], native=True)
    g2 = ShardGroup([s2], SoloComm(4, 2), cfg["mtu"], native=True)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round(g0, scen, r)
    want = one.export()
    got = g0.export()
    assert compare_exports(got, {k: v[:, : s0.ncol] for k, v in want.items()}) is None
    assert one.check()["truncated"] > 0
    with pytest.raises(GsError, match="held alone"):
        replay_round(g2, scen, 0)
    for x in (one, s0, s2):
        x.close()


def _bench_cluster(n, G, mtu, rounds, native=False):
    """The bench's layout (8-bit views, prefix views, no tombstones, warm, churn) as G in-process slices driven by
    the bench's round driver, and its plans (one more round than ``rounds``)."""
    import torch

    from aiocluster_amd import driver
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.workload import key_names, synthetic_node_ids

    K = 16
    cfg = dict(DEFAULT_CFG)
    cfg["mtu"] = mtu
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=11, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3)
    kw = dict(init="warm", device="cuda:0", tombstones=False, fd_ring=False, hist_cap=16,
              initial_ops=driver.boot_ops(n, K), hb8=True, mv8=True)
    ids = synthetic_node_ids(n)
    sims = [GossipSim(ids, key_names(K), cfg, shards=G, shard=g, **kw) for g in range(G)]
    from aiocluster_amd.shard import LocalComm

    grp = ShardGroup(sims, LocalComm(G), mtu, native=native)
    plans = driver.prepare(spec, rounds + 1, torch, sims[0].device)
    for r in range(rounds):
        driver.run_round(sims, plans[r], group=grp)
    grp.check()
    return grp, cfg, plans


@pytest.mark.parametrize("native", [False, True], ids=["shard_py", "library"])
def test_sliced_parity_check_on_whole_cluster_rows(native):
    """bench.py's multi-GPU parity evidence on one GPU: rowcheck.check_sliced_phase_rows joins
    the sampled rows of every slice into whole-cluster rows, runs the phase through the group's sliced driver and
    compares each slice's columns with the C oracle -- bit-exact, with deltas the mtu cuts across slices."""
    from rowcheck import check_sliced_phase_rows

    from aiocluster_amd import driver

    grp, cfg, plans = _bench_cluster(1024, 4, 500, 8, native=native)
    rd = plans[8]
    driver.begin(grp.slices, rd)
    res, info = check_sliced_phase_rows(grp, cfg, rd, sample=rd["phases"][0][2])
    assert [r["slice"] for r in res] == [0, 1, 2, 3]
    assert all(r["exact"] for r in res), res
    assert res[-1]["cols"][1] == 1024
    assert info["node_deltas"] > 0 and info["truncated"] > 0, info
    for s in grp.slices:
        s.close()


def test_sliced_parity_check_reports_a_corrupted_slice(monkeypatch):
    """The same check must name the slice whose columns differ: a view of slice 2 changed after the phase (before
    the rows are read back) is reported there, and only there."""
    import torch
    from rowcheck import check_sliced_phase_rows

    from aiocluster_amd import driver

    grp, cfg, plans = _bench_cluster(512, 4, 1500, 4)
    rd = plans[4]
    driver.begin(grp.slices, rd)
    a0 = int(rd["phases"][0][0][0].item())
    s2 = grp.slices[2]
    real_end = driver.end

    def end(sims, rd_, tick=None):
        real_end(sims, rd_, tick)
        mv = s2.region("MV", torch.uint8, (s2.n, s2.np_))
        mv[a0, 5] = mv[a0, 5] ^ 1  # the version's low bit of one view of slice 2 (column col_lo + 5)

    monkeypatch.setattr(driver, "end", end)
    res, _ = check_sliced_phase_rows(grp, cfg, rd, sample=8)
    assert [r["exact"] for r in res] == [True, True, False, True], res
    assert "mv" in res[2]["diff"]
    for s in grp.slices:
        s.close()


def test_bench_two_ranks_gloo_rehearsal_reports_parity_per_slice():
    """`GS_BENCH_BACKEND=gloo python bench.py --gpus 2` (both ranks on this GPU, gathers through host memory): the
    multi-rank bench's rank plumbing end to end, with its own parity evidence -- the line carries parity_check,
    bit-exact for each slice."""
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GS_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--nodes", "4096", "--steps", "2",
           "--warmup", "1", "--settle", "4", "--mtu", "3000", "--parity-sample", "32"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=repo)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(next(x for x in r.stdout.splitlines() if x.startswith("{")))
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    pc = line["parity_check"]
    assert pc["exact"] and [s["slice"] for s in pc["per_slice"]] == [0, 1], pc
    assert all(s["exact"] and s["diff"] is None for s in pc["per_slice"]), pc
    assert pc["per_slice"][1]["cols"][1] == 4096 and pc["node_deltas"] > 0, pc
