"""8-bit heartbeat and max_version views (GS_HB8, GS_MV8; GPU only).

GS_R_HB holds each view's heartbeat mod 2^8, decoded against the owner's own heartbeat (GS_R_SELF_HB):
exact while no view lags its owner by 2^8 or more.  gs_begin_round sweeps the lags at least every 64
round starts + phases and counts a lag >= 2^7 in err_hb_lag, so a run either decodes
exactly or is reported inexact.  GS_MV8 does the same for max_version views (version mod 2^7 | the
inexact flag, decoded against the owner's own max_version, GS_R_SELF_MV): a view only falls behind when its
owner writes, gs_owner_writes sweeps at least every 64 calls and counts a lag >= 2^6.  The headline and
config 4 run with both (bench.py; the heartbeat-lag census, tools/hb_lag.py, peaks at 49 there).
"""

import numpy as np
import pytest
from helpers import compare_exports, load_scenario, make_backend, replay_and_compare
from oracle import OracleSim

from aiocluster_amd.scenario import DEFAULT_CFG
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec, key_names, liveness_tick, phase_tick, round_tick, synthetic_node_ids

pytestmark = pytest.mark.gpu

SCHED = [[(0, 1), (2, 3), (4, 5), (6, 7)], [(1, 2), (3, 4), (5, 6), (7, 0)], [(0, 4), (1, 5), (2, 6), (3, 7)],
         [(5, 0), (6, 1), (7, 2), (4, 3)]]


@pytest.mark.parametrize("mv8", [False, True], ids=["hb8", "hb8mv8"])
@pytest.mark.parametrize("name", ["sched16", "warm128"])
def test_hb8_matches_reference_golden(name, mv8):
    """The warm golden scenarios (MTU truncation, holes, churn) in the 8-bit layouts: the reference's
    canonical state after every round."""
    scen = load_scenario(name)
    exp = scen["expect"]
    sim = make_backend(GossipSim, scen, tombstones=False, hb8=True, mv8=mv8)
    res = replay_and_compare(sim, scen, exp["states"], exp["hashes"])
    assert res is None, f"{name}: first mismatch at round {res[0]}: {res[1]}"
    assert sim.check()["err_hb_lag"] == 0


@pytest.mark.parametrize("mv8", [False, True], ids=["hb8", "hb8mv8"])
def test_hb8_heartbeats_past_2_8_with_a_long_absence_match_oracle(mv8):
    """Eight nodes, 400 rounds: every heartbeat wraps mod 2^8 several times, and node 7 is down for 25
    rounds (its views of the others fall ~75 behind, its windows go silent), then returns; the device
    matches the C oracle (unbounded heartbeats) array for array, and the automatic lag sweeps ran clean.
    With GS_MV8 pass 1 is k_pass1v: the lagging views make their row hot (per-column path) until a sweep
    finds them caught up."""
    import torch

    n, rounds, down0, down1 = 8, 400, 150, 175
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8, hb8=True,
                    mv8=mv8)
    orc = OracleSim(ids, keys, dict(DEFAULT_CFG), "warm", init)
    for r in range(rounds):
        up = np.ones(n, np.uint8)
        if down0 <= r < down1:
            up[7] = 0
        up_dev = torch.from_numpy(up).to(gpu.device)
        t = round_tick(r)
        gpu.begin_round(t, up_dev)
        orc.begin_round(t, up)
        for p in range(2):
            pairs = [(a, b) for a, b in SCHED[(r + p) % len(SCHED)] if up[a] and up[b]]
            gpu.run_phase(phase_tick(r, p), pairs)
            orc.run_phase(phase_tick(r, p), pairs)
        gpu.liveness(liveness_tick(r, 2), up_dev)
        orc.liveness(liveness_tick(r, 2), up)
        if r in (20, down1 - 1, down1 + 5, rounds - 1):
            want = orc.export()
            diff = compare_exports(gpu.export(), want)
            assert diff is None, f"round {r}: {diff}"
    assert np.asarray(want["hb"]).min() > 256, "every heartbeat must have wrapped mod 2^8"
    c = gpu.check()
    assert c["err_hb_lag"] == 0


def test_hb8_lag_sweep_flags_views_at_2_7():
    """A view lagging its owner by >= 2^7 heartbeats (injected) trips err_hb_lag; 2^7 - 1 does not."""
    import torch

    from aiocluster_amd._lib import GsError

    n = 8
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8, hb8=True)
    up_dev = torch.ones(n, dtype=torch.uint8, device=gpu.device)
    gpu.begin_round(round_tick(0), up_dev)
    gpu.liveness(liveness_tick(0, 0), up_dev)
    R = gpu.region("SELF_HB", torch.int32, (gpu.np_,))
    hb = gpu.hb_region()
    R[3] = 1000
    for o in range(n):
        hb[o, 3] = (1000 - 10) & 0xFF
    hb[3, 3] = 1000 & 0xFF
    hb[5, 3] = (1000 - 127) & 0xFF  # lag 2^7 - 1: exact, not flagged
    gpu.check_heartbeat_lag()
    assert gpu.check()["err_hb_lag"] == 0
    assert gpu.node_state(5, 3).heartbeat == 1000 - 127
    hb[6, 3] = (1000 - 128) & 0xFF  # lag 2^7
    gpu.check_heartbeat_lag()
    with pytest.raises(GsError, match="err_hb_lag"):
        gpu.check()


def test_hb8_refused_outside_the_record_phases():
    """GS_HB8 needs the canonical layout and K <= 16 (the record phases' pass 1 reads it)."""
    from aiocluster_amd._lib import GsError

    ids = synthetic_node_ids(8)
    with pytest.raises(GsError):
        GossipSim(ids, key_names(2), dict(DEFAULT_CFG), "cold", None, tombstones=False, hb8=True)
    with pytest.raises(GsError):
        GossipSim(ids, key_names(20), dict(DEFAULT_CFG), "warm", None, tombstones=False, hb8=True)


def test_mv8_versions_past_2_7_with_an_absence_match_oracle():
    """Eight nodes each writing a key every round they are up, 170 rounds: every owner's max_version passes
    2^7 (views wrap mod 2^7), node 7 is down for 20 rounds (its views fall 20 versions behind), and MTU
    truncation leaves holes (the inexact flag in the byte); the device matches the C oracle array for array
    and the automatic sweeps ran clean."""
    import torch

    n, rounds, down0, down1 = 8, 170, 100, 120
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    cfg = dict(DEFAULT_CFG, mtu=300)
    gpu = GossipSim(ids, keys, cfg, "warm", init, tombstones=False, fd_ring=True, hist_cap=100, hb8=True, mv8=True)
    orc = OracleSim(ids, keys, cfg, "warm", init)
    for r in range(rounds):
        up = np.ones(n, np.uint8)
        if down0 <= r < down1:
            up[7] = 0
        up_dev = torch.from_numpy(up).to(gpu.device)
        t = round_tick(r)
        for j in range(n):
            if up[j]:
                gpu.write(t, j, r % 2, 0, f"v{j}.{r}")
                orc.write(t, j, r % 2, 0, f"v{j}.{r}")
        gpu.begin_round(t, up_dev)
        orc.begin_round(t, up)
        for p in range(2):
            pairs = [(a, b) for a, b in SCHED[(r + p) % len(SCHED)] if up[a] and up[b]]
            gpu.run_phase(phase_tick(r, p), pairs)
            orc.run_phase(phase_tick(r, p), pairs)
        gpu.liveness(liveness_tick(r, 2), up_dev)
        orc.liveness(liveness_tick(r, 2), up)
        if r in (30, down1 - 1, down1 + 3, rounds - 1):
            want = orc.export()
            diff = compare_exports(gpu.export(), want)
            assert diff is None, f"round {r}: {diff}"
    assert np.asarray(want["mv"]).max() > 128, "max_versions must pass 2^7"
    c = gpu.check()
    assert c["err_hb_lag"] == 0 and c["truncated"] > 0


def test_mv8_lag_sweep_flags_views_at_2_6():
    """A max_version view lagging its owner by >= 2^6 versions (injected) trips err_hb_lag; 2^6 - 1 does
    not, and decodes exactly (the inexact flag kept apart)."""
    import torch

    from aiocluster_amd._lib import GsError

    n = 8
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8,
                    hb8=True, mv8=True)
    up_dev = torch.ones(n, dtype=torch.uint8, device=gpu.device)
    gpu.begin_round(round_tick(0), up_dev)
    gpu.liveness(liveness_tick(0, 0), up_dev)
    M = gpu.region("SELF_MV", torch.int32, (gpu.np_,))
    PK = gpu.region("SELF_PK", torch.int32, (gpu.np_,))  # pass 1's and the sweep's packed copy
    R3 = int(gpu.region("SELF_HB", torch.int32, (gpu.np_,))[3].item())
    mv = gpu.region("MV", torch.uint8, (n, gpu.np_))
    M[3] = 1000
    PK[3] = (R3 & 0x7FFF) | (1000 << 16)
    for o in range(n):
        mv[o, 3] = (1000 - 5) & 0x7F
    mv[3, 3] = 1000 & 0x7F
    mv[5, 3] = ((1000 - 63) & 0x7F) | 0x80  # lag 2^6 - 1, with holes: exact, not flagged
    gpu.check_heartbeat_lag()
    assert gpu.check()["err_hb_lag"] == 0
    w = int(gpu.mv_words(slice(5, 6))[0, 3].item())
    assert w == (1000 - 63) | 0x8000
    mv[6, 3] = (1000 - 64) & 0x7F  # lag 2^6
    gpu.check_heartbeat_lag()
    with pytest.raises(GsError, match="err_hb_lag"):
        gpu.check()


def test_mv8_refused_without_hb8_or_with_tombstones():
    from aiocluster_amd._lib import GsError

    ids = synthetic_node_ids(8)
    with pytest.raises(GsError):
        GossipSim(ids, key_names(2), dict(DEFAULT_CFG), "warm", None, tombstones=False, mv8=True)
    with pytest.raises(GsError):
        GossipSim(ids, key_names(2), dict(DEFAULT_CFG), "warm", None, tombstones=True, hb8=True, mv8=True)


def _long_round(gpu, orc, phases, t0):
    """One round of ``phases`` phases at ticks t0 + 1 .. t0 + phases: node 1 answers in every phase (its
    own heartbeat rises by one per phase), nodes 6 and 7 are up but take part in none (their views of 1
    fall behind by one per phase)."""
    import torch

    n = gpu.n
    up = np.ones(n, np.uint8)
    up_dev = torch.from_numpy(up).to(gpu.device)
    gpu.begin_round(t0, up_dev)
    if orc is not None:
        orc.begin_round(t0, up)
    for p in range(phases):
        pairs = [(0, 1), (2, 3), (4, 5)] if p % 2 == 0 else [(2, 1), (4, 3), (0, 5)]
        gpu.run_phase(t0 + 1 + p, pairs)
        if orc is not None:
            orc.run_phase(t0 + 1 + p, pairs)
    gpu.liveness(t0 + 1 + phases, up_dev)
    if orc is not None:
        orc.liveness(t0 + 1 + phases, up)


def test_hb8_round_of_100_phases_matches_oracle():
    """A round may hold more phases than the 64 round starts + phases between lag sweeps: the
    phases sweep too, so the views of an idle node, lagging ~100 behind by the round's end, stay exact;
    the device matches the C oracle array for array and the mid-round sweeps ran clean."""
    n = 8
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8,
                    hb8=True, mv8=True)
    orc = OracleSim(ids, keys, dict(DEFAULT_CFG), "warm", init)
    _long_round(gpu, orc, 100, round_tick(0))
    want = orc.export()
    assert np.asarray(want["hb"])[1, 1] - np.asarray(want["hb"])[7, 1] >= 100  # the idle view's lag
    diff = compare_exports(gpu.export(), want)
    assert diff is None, diff
    c = gpu.check()
    assert c["err_hb_lag"] == 0 and c["lag_sweeps"] >= 1 and c["plane_flushes"] >= 1


def test_hb8_round_of_300_phases_is_reported_not_silently_wrong():
    """300 phases in one round: the idle nodes' views of node 1 would fall 2^8 behind and decode wrongly.
    A mid-round sweep counts them in err_hb_lag (at 2^7) before that happens, so the run raises."""
    from aiocluster_amd._lib import GsError

    n = 8
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8,
                    hb8=True)
    _long_round(gpu, None, 300, round_tick(0))
    with pytest.raises(GsError, match="err_hb_lag"):
        gpu.check()


def test_hb8mv8_round_of_300_phases_escapes_and_matches_oracle():
    """The same 300-phase round with GS_MV8 (k_pass1v and escape slots, gs_config.esc_cols): the lag sweep that
    finds the idle nodes' views of node 1 at >= 2^7 moves column 1 to 16-bit views, so the round stays exact;
    the device matches the C oracle array for array, and the column goes back to bytes once caught up."""
    import torch

    n = 8
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8,
                    hb8=True, mv8=True)
    orc = OracleSim(ids, keys, dict(DEFAULT_CFG), "warm", init)
    _long_round(gpu, orc, 300, round_tick(0))
    want = orc.export()
    assert np.asarray(want["hb"])[1, 1] - np.asarray(want["hb"])[7, 1] >= 256  # beyond what a byte holds
    diff = compare_exports(gpu.export(), want)
    assert diff is None, diff
    c = gpu.check()
    assert c["err_hb_lag"] == 0 and c["hb_escapes"] >= 1, c
    # a normal round lets the idle nodes catch up: the next sweeps move the column back
    up = np.ones(n, np.uint8)
    up_dev = torch.from_numpy(up).to(gpu.device)
    for r in range(6, 30):
        t = round_tick(r)
        gpu.begin_round(t, up_dev)
        orc.begin_round(t, up)
        for p in range(2):
            pairs = SCHED[(r + p) % len(SCHED)]
            gpu.run_phase(phase_tick(r, p), pairs)
            orc.run_phase(phase_tick(r, p), pairs)
        gpu.liveness(liveness_tick(r, 2), up_dev)
        orc.liveness(liveness_tick(r, 2), up)
    gpu.check_heartbeat_lag()
    diff = compare_exports(gpu.export(), orc.export())
    assert diff is None, diff
    c = gpu.check()
    assert c["hb_releases"] >= 1 and c["err_hb_lag"] == 0, c


def test_hb8mv8_100_selected_rounds_at_16384_match_oracle():
    """the reference's own peer selection (select_nodes_for_gossip, 8 seeds; the first rounds
    after a warm start route every node's seed pick to 8 hub columns, whose views then lag by up to ~280
    heartbeats) drives 101 rounds of a 16,384-node cluster in the 8-bit layout (GS_HB8 + GS_MV8 with escape
    slots).  Every phase of round 6 (hub columns escaped) and of round 100 is checked on sampled rows against
    the C oracle, and no device check fires."""
    import torch
    from rowcheck import check_round_rows

    from aiocluster_amd import driver
    from aiocluster_amd.peers import PeerSelector
    from aiocluster_amd.workload import TICKS_PER_ROUND, phase_tick as ptick

    n, K = 16384, 16
    cfg = dict(DEFAULT_CFG)
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=4, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3)
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=False, fd_ring=False,
                    hist_cap=16, initial_ops=driver.boot_ops(n, K), hb8=True, mv8=True)
    plans = driver.prepare(spec, 101, torch, sim.device)
    sel = PeerSelector(sim, fanout=3, seeds=list(range(0, n, n // 8)), seed=4)
    escaped_seen = 0
    for r in range(101):
        rd = plans[r]
        if r in (6, 100):
            driver.begin([sim], rd)
            sel.select(rd["up"], rd["r"])
            ph, offs, left = sel.schedule(rd["up"], rd["r"])
            assert left == 0
            rd["phases"] = [(a, b, m, ptick(rd["r"], p)) for p, (a, b, m) in enumerate(ph)]
            rd["t_live"] = liveness_tick(rd["r"], len(ph))
            assert rd["t_live"] < rd["t"] + TICKS_PER_ROUND
            if r == 6:
                slot = sim.region("ESC_SLOT", torch.int32, (sim.np_,))
                escaped_seen = int((slot != -1).sum().item())
            diff, info = check_round_rows(sim, cfg, rd, sample=16, seed=r)
            assert diff is None, f"round {r}: {diff}"
            assert info["phases"] >= 8 and info["hb_reports"] > 0, info
        else:
            driver.run_round([sim], rd, sel=sel)
    sim.check_heartbeat_lag()
    c = sim.check()
    assert escaped_seen > 0 and c["hb_escapes"] > 0, (escaped_seen, c["hb_escapes"])
    assert c["err_hb_lag"] == 0
    sim.close()
