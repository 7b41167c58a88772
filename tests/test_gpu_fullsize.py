"""Full-size parity (GPU only): BASELINE configs 3 and 5 at their real sizes.

The oracle cannot replay a 65,536-node run (N^2 views), but one conflict-free phase touches only
its own rows: after ~20 settle rounds on the device, the rows of sampled exchanges of a phase are
copied into the C oracle (``oracle/rowcheck.py``), the whole phase runs on the device and in the
oracle (the sample), and the rows must be bit-identical: decoded heartbeats, max versions, last_gc
versions, held keys (version, status, value, tombstone tick), failure-detector windows (last report,
length, binary64 sum), live/dead.  ``check_round_rows`` does that for EVERY phase of a round (random
exchanges, the device's pending reports applied before each copy), so rows merged by several phases
of the round are compared too, closing with the liveness sweep; two rounds per config.  The owner
tables the row copies carry (HIST / LAST_W / HIST_VID) are first checked against the workload's write
stream restated on the host (``oracle/owner_tables.py``), so the oracle does not inherit them unchecked.
The reference semantics checked: ``aiocluster/state.py:190-233, 340-415``, ``server.py:327-376,
599-620``, ``failure_detector.py:12-128``.
"""

import numpy as np
import pytest
from owner_tables import check_owner_tables, plan_batches
from rowcheck import check_phase_rows, check_round_rows

from aiocluster_amd import driver
from aiocluster_amd.scenario import DEFAULT_CFG
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

pytestmark = pytest.mark.gpu


def _run(sim, plans, rounds):
    for r in range(rounds):
        driver.run_round([sim], plans[r])
    sim.check()


def _write_burst(sim, torch, tick, calls=70, per_call=2048, seed=7):
    """``calls`` owner-write batches at ``tick`` (distinct owners per batch, any key): more than the 64
    gs_owner_writes calls between GS_MV8 lag sweeps, so the sweep inside gs_owner_writes runs, while no
    owner writes often enough (a few versions each) for a view to reach the 2^6 sweep bound."""
    rng = np.random.default_rng(seed)
    vid = 1 << 25
    for _ in range(calls):
        ops = np.zeros((per_call, 5), dtype=np.int32)
        ops[:, 0] = rng.permutation(sim.n)[:per_call]
        ops[:, 1] = rng.integers(0, sim.k, per_call)
        ops[:, 3] = vid + np.arange(per_call)
        ops[:, 4] = 12
        vid += per_call
        sim.owner_writes(ops.view(np.uint32), tick)


@pytest.mark.parametrize("layout", ["hb16", "hb8", "hb8mv8"])
def test_config3_65536_every_phase_of_two_rounds_matches_oracle(layout):
    """BASELINE config 3 (the bench workload): 65,536 nodes x 16 keys, fanout 3, warm, 5 % writes + 5 %
    up/down churn, window 1000, mtu 65,507, prefix-view layout with HELD rows for views with holes, in
    three view widths: 16-bit heartbeat + max_version views, 8-bit heartbeats (GS_HB8), and the bench's
    own layout, 8-bit heartbeats + 8-bit max_versions (GS_HB8 + GS_MV8, ``bench.py`` default); 20 settle
    rounds, the owner tables vs the write stream, then every phase of rounds 20 and 21 on 16 random
    exchanges each.  In the bench's layout round 21 starts with a burst of 70 owner-write batches, so the
    max_version lag sweep of gs_owner_writes runs (every 64 calls) and the phases then spread the new
    versions, checked against the oracle; no view may reach the sweep bound (err_hb_lag = 0)."""
    import torch

    n, K = 65536, 16
    cfg = dict(DEFAULT_CFG)
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=0, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3)
    boot = driver.boot_ops(n, K)
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=False, fd_ring=False,
                    hist_cap=16, initial_ops=boot, hb8=layout != "hb16", mv8=layout == "hb8mv8")
    dev = sim.device
    plans = driver.prepare(spec, 22, torch, dev)
    _run(sim, plans, 20)
    assert check_owner_tables(sim, plan_batches(K, n, plans[:20], boot)) is None
    for r in (20, 21):
        rd = plans[r]
        if r == 21 and layout == "hb8mv8":
            sweeps = sim.check()["lag_sweeps"]
            _write_burst(sim, torch, rd["t"])
            c = sim.check()  # err_hb_lag = 0: the sweeps found every max_version lag < 2^6
            assert c["lag_sweeps"] > sweeps, (sweeps, c["lag_sweeps"])
        driver.begin([sim], rd)
        diff, info = check_round_rows(sim, cfg, rd, sample=16, seed=r)
        assert diff is None, f"round {r}: {diff}"
        # the sample did real work: deltas, heartbeat reports (the oracle's counts), every phase
        assert info["phases"] >= 8 and info["node_deltas"] > 0 and info["hb_reports"] > 0, info
    c = sim.check()
    assert c["exchanges"] > 0
    assert (c["lag_sweeps"] > 0) == (layout != "hb16")  # 8-bit views: swept every <= 64 round starts + phases
    sim.close()


def test_config5_16384_partition_heal_every_phase_matches_oracle():
    """BASELINE config 5: 16,384 nodes, K = 16, 5 % writes (1 % deletes), tombstone grace 10 rounds,
    mtu 65,507, partition into halves for rounds 10-29, heal from round 30.  Every phase of the last
    partitioned round (dead-marked peers: false positives) and of the first healed round (the heal burst:
    MTU-truncated NodeDeltas, tombstones collected) on 24 random exchanges each."""
    import torch

    n, K = 16384, 16
    cfg = dict(DEFAULT_CFG)
    cfg["tombstone_grace_s"] = 10
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=5, init="warm", write_frac=0.05, delete_frac=0.01,
                        partition=(10, 30))
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=True, fd_ring=False,
                    hist_cap=32, initial_ops=driver.boot_ops(n, K))
    plans = driver.prepare(spec, 31, torch, sim.device)
    _run(sim, plans, 29)
    assert check_owner_tables(sim, plan_batches(K, n, plans[:29], driver.boot_ops(n, K))) is None
    rd = plans[29]
    driver.begin([sim], rd)
    diff, info = check_round_rows(sim, cfg, rd, sample=24, seed=29)
    assert diff is None, f"partitioned round: {diff}"
    cen = sim.fd_census(rd["up"])
    assert cen["up_dead"] > 0  # the partition left peers dead-marked
    rd = plans[30]
    driver.begin([sim], rd)
    before = sim.check()
    diff, info = check_round_rows(sim, cfg, rd, sample=24, seed=30)
    assert diff is None, f"healed round: {diff}"
    c = sim.check()
    assert c["truncated"] - before["truncated"] > 0 and info["truncated"] > 0, (info, c["truncated"])
    assert c["tomb_gc"] > 0
    sim.close()


def test_fullsize_check_detects_a_corrupted_row():
    """The check is not vacuous: after a matching phase, one changed device value in a sampled row (a
    heartbeat, a live flag) is reported."""
    import torch

    import rowcheck

    n, K = 4096, 8
    cfg = dict(DEFAULT_CFG)
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=1, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3)
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=False, fd_ring=False,
                    hist_cap=16, initial_ops=driver.boot_ops(n, K))
    plans = driver.prepare(spec, 6, torch, sim.device)
    _run(sim, plans, 5)
    rd = plans[5]
    driver.begin([sim], rd)
    a, b, _, t = rd["phases"][0]
    rows = a[:8].cpu().numpy().tolist() + b[:8].cpu().numpy().tolist()
    ro = rowcheck.RowOracle(sim, cfg)
    (h,) = ro.load(rows)
    driver.run_phases([sim], rd, phases=[rd["phases"][0]])
    driver.end([sim], rd, tick=t + 1)
    for x, y in zip(rows[:8], rows[8:]):
        ro.exchange(h, x, y, t)
    for o in rows:
        ro.liveness(h, o, t + 1)
    want = ro.export_rows(h, rows)
    assert rowcheck.compare_exports(sim.export_rows(rows), want) is None
    hb = sim.region("HB", torch.int16, (n, sim.np_))
    o, j = rows[3], (rows[3] + 11) % n
    hb[o, j] -= 1
    d = rowcheck.compare_exports(sim.export_rows(rows), want)
    assert d is not None and d.startswith("hb[3, "), d
    hb[o, j] += 1
    st = sim.region("FD_STATE", torch.uint8, (n, sim.np_))
    tod = sim.region("FD_TOD", torch.int32, (n, sim.np_))
    o, j = rows[12], (rows[12] + 5) % n
    st[o, j] = (st[o, j] & 0xFC) | 2  # dead since t (membership bits only; the window bits stay)
    tod[o, j] = t
    d = rowcheck.compare_exports(sim.export_rows(rows), want)
    assert d is not None and d.startswith("live[12, "), d
    ro.close()
    sim.close()


def test_config3_65536_whole_array_converges_after_churn():
    """Whole-array properties at the headline size (the sampled-row checks above cover single exchanges): the
    bench's layout (GS_HB8 + GS_MV8, prefix views) through 10 rounds of writes + churn, then quiet rounds (no
    writes, every node up).  Anti-entropy (aiocluster/state.py:340-415, server.py:441-495) must then bring EVERY
    observer's view of EVERY owner to the owner's max_version, no view may ever be above it, and every up observer's
    failure detector must hold every other node live (failure_detector.py:89-106) -- checked on all 65,536 x 65,536
    pairs, with every device check counter 0."""
    import torch

    def versions():
        """(views above their owner's max_version, views below it, views with holes) over the whole matrix"""
        own = sim.region("SELF_MV", torch.int32, (sim.np_,))[:n]
        above = below = holes = 0
        for r0 in range(0, n, 8192):
            w = sim.mv_words(slice(r0, r0 + 8192))[:, :n]
            v = w & 0x7FFF
            above += int((v > own[None, :]).sum().item())
            below += int((v < own[None, :]).sum().item())
            holes += int((w >= 0x8000).sum().item())
        return above, below, holes

    n, K = 65536, 16
    cfg = dict(DEFAULT_CFG)
    settle, quiet = 10, 22
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=9, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3,
                        quiet_from=settle)
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=False, fd_ring=False,
                    hist_cap=16, initial_ops=driver.boot_ops(n, K), hb8=True, mv8=True)
    plans = driver.prepare(spec, settle + quiet, torch, sim.device)
    _run(sim, plans, settle)
    above, below, holes = versions()
    assert above == 0 and below > 0 and holes > 0, (above, below, holes)  # in flight: views behind, none ahead
    for r in range(settle, settle + quiet):
        driver.run_round([sim], plans[r])
    c = sim.check()  # every err_* = 0
    above, below, holes = versions()
    # converged (views with holes keep them: their max_version already equals the owner's, so no digest asks for
    # the missing keys -- SURVEY Q1, the reference's own behaviour)
    assert above == 0 and below == 0, (above, below, holes)
    census = sim.fd_census(plans[-1]["up_host"])
    assert census["up_pairs"] == n * (n - 1) and census["up_dead"] == 0, census
    assert census["up_live"] == census["up_pairs"], census
    assert c["truncated"] > 0 and c["exchanges"] > 0  # the mtu bound during the churn rounds
    sim.close()
