"""Device peer selection (gs_select_peers, gs_schedule_phases) vs its CPU restatement
(oracle/peer_select.py), and rounds driven by it vs the C oracle.  GPU only.

select_nodes_for_gossip (aiocluster/server.py:656-717) draws from random.Random over set order
(SURVEY Q11): parity is exact against the restatement of the same Philox draws, distributional
against the reference's probabilities (dead probe p = dead / (live + 1), F distinct live peers).
"""

import numpy as np
import pytest
import peer_select
from helpers import compare_exports, make_backend
from oracle import OracleSim

from aiocluster_amd.peers import PeerSelector, run_selected_round
from aiocluster_amd.scenario import make_scenario, replay_round
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec, liveness_tick, phase_tick, round_tick

pytestmark = pytest.mark.gpu


def _state(orc):
    ex = orc.export()
    return ex["live"], ex["tod"], (ex["pos"] >= 0)


def _warm_cluster(n=160, rounds=8, seed=3, init="warm"):
    spec = WorkloadSpec(n=n, k=4, fanout=3, seed=seed, init=init, write_frac=0.1, down_frac=0.15, down_rounds=4)
    scen = make_scenario(f"sel{n}", spec, rounds + 1, {"initial_interval_s": 1.0, "phi_threshold": 3.0})
    gpu = make_backend(GossipSim, scen, fd_ring=False)
    orc = make_backend(OracleSim, scen)
    for r in range(rounds):
        replay_round(gpu, scen, r)
        replay_round(orc, scen, r)
    assert compare_exports(gpu.export(), orc.export()) is None
    return scen, gpu, orc


@pytest.mark.parametrize("init,iters,max_phases", [("warm", 4, 62), ("cold", 4, 62), ("warm", 1, 62),
                                                   ("warm", 3, 62), ("warm", 1, 8), ("cold", 2, 16)])
def test_selection_and_schedule_match_restatement(init, iters, max_phases):
    """Odd `iters` and phase caps included: the Luby minimum buffers alternate by the global iteration
    index, so every iteration starts from fresh minima as the restatement does."""
    scen, gpu, orc = _warm_cluster(init=init)
    up = np.asarray(scen["rounds"][-1]["up"], dtype=np.uint8)
    seeds = [0, 5, 77]
    sel = PeerSelector(gpu, fanout=3, seeds=seeds, seed=1234, iters=iters, max_phases=max_phases)
    up_dev = gpu._dev(up, gpu.torch.uint8)
    got = sel.select(up_dev, 9).cpu().numpy()
    live, tod, known = _state(orc)
    want = peer_select.select_peers(live, tod, known, up, 3, seeds, 1234, 9)
    assert np.array_equal(got, want)
    assert (got[:, 3] >= 0).any() and (got[:, 4] >= 0).any()  # dead probes and seed probes happened
    phases, offs, left = sel.schedule(up_dev, 9)
    eph = peer_select.schedule_phases(want, up, 1234, 9, iters, max_phases)
    W = want.shape[1]
    want_sets = [set() for _ in range(max_phases)]
    for e in np.flatnonzero(eph >= 0):
        want_sets[eph[e]].add((int(e // W), int(want.reshape(-1)[e])))
    got_sets = sel.scheduled_pairs(phases)
    assert got_sets == [x for x in want_sets if x]
    for ph in got_sets:  # conflict-free
        nodes = [x for pr in ph for x in pr]
        assert len(nodes) == len(set(nodes))
    flat = want.reshape(-1)
    valid = sum(1 for e in range(want.size) if flat[e] >= 0 and up[flat[e]])
    assert offs[-1] == int((eph >= 0).sum())
    assert left == valid - offs[-1]  # reported, never silently dropped
    if max_phases == 62:
        assert left == 0  # _gossip_multiple contacts every selected peer (server.py:476-493)
    else:
        assert max_phases > 8 or left > 0  # 8 phases cannot hold every node's exchanges


def test_rounds_with_device_peer_selection_match_oracle():
    """Whole rounds whose schedule comes from gs_select_peers / gs_schedule_phases: the oracle replays
    the same phases and must end every round in the same state."""
    scen, gpu, orc = _warm_cluster(n=128, rounds=3, seed=9)
    sel = PeerSelector(gpu, fanout=3, seeds=[1, 2], seed=77)
    rng = np.random.default_rng(5)
    for r in range(3, 12):
        up = (rng.random(128) > 0.1).astype(np.uint8)
        t = round_tick(r)
        up_dev = gpu._dev(up, gpu.torch.uint8)
        gpu.begin_round(t, up_dev)
        orc.begin_round(t, up)
        sel.select(up_dev, r)
        phases, _, left = sel.schedule(up_dev, r)
        assert left == 0
        sets = sel.scheduled_pairs(phases)
        for p, (a, b, n) in enumerate(phases):
            gpu.run_phase_arrays(phase_tick(r, p), a, b)
            orc.run_phase(phase_tick(r, p), sorted(sets[p]))
        gpu.update_node_liveness(liveness_tick(r, len(phases)), up_dev)
        orc.liveness(liveness_tick(r, len(phases)), up, r)
        diff = compare_exports(gpu.export(), orc.export())
        assert diff is None, f"round {r}: {diff}"
    assert gpu.check()["exchanges"] > 0


def test_dead_probe_and_sample_distribution():
    """Frequencies of the device draws against select_nodes_for_gossip's probabilities."""
    scen, gpu, orc = _warm_cluster(n=256, rounds=8, seed=4)
    up = np.asarray(scen["rounds"][-1]["up"], dtype=np.uint8)
    live, tod, known = _state(orc)
    sel = PeerSelector(gpu, fanout=3, seeds=[], seed=99)
    up_dev = gpu._dev(up, gpu.torch.uint8)
    hits, expect, picks = 0, 0.0, 0
    for r in range(40):
        tg = sel.select(up_dev, 100 + r).cpu().numpy()
        for o in np.flatnonzero(up):
            kn = known[o].copy()
            kn[o] = False
            L = int((kn & (live[o] == 1)).sum())
            D = int((kn & (tod[o] >= 0)).sum())
            expect += min(1.0, D / (L + 1))
            hits += tg[o, 3] >= 0
            row = tg[o, :3]
            assert len(set(row[row >= 0])) == (row >= 0).sum() == min(3, L if L else int(kn.sum()))
            assert all(live[o, x] == 1 for x in row[row >= 0]) if L else True
            picks += 1
    assert abs(hits - expect) < 4 * np.sqrt(expect) + 1, (hits, expect)
    assert expect > 20


def test_run_selected_round_helper():
    scen, gpu, orc = _warm_cluster(n=96, rounds=2, seed=12)
    sel = PeerSelector(gpu, fanout=2, seeds=[0], seed=5)
    for r in range(2, 6):
        info = run_selected_round(gpu, sel, r, np.ones(96, dtype=np.uint8))
        assert 1 <= info["phases"] <= 16 and info["exchanges"] > 0
    gpu.check()


@pytest.mark.parametrize("fanout,flushes", [(8, False), (11, True)])
def test_rounds_with_many_phases_match_oracle(fanout, flushes):
    """Fanout 8 = 24 phases per round fit the 32 report planes (no mid-round replay); fanout 11 = 33
    phases: phases more than 32 ticks after the round start replay the pending planes into the windows
    mid-round (plane_flushes, one per round); every round vs the oracle."""
    spec = WorkloadSpec(n=96, k=4, fanout=fanout, seed=31, init="warm", write_frac=0.1, down_frac=0.1,
                        down_rounds=3)
    scen = make_scenario(f"f{fanout}", spec, 6, {"initial_interval_s": 1.0, "phi_threshold": 3.0, "mtu": 800})
    assert max(len(rd["phases"]) for rd in scen["rounds"]) > (32 if flushes else 16)
    gpu = make_backend(GossipSim, scen, fd_ring=False)
    orc = make_backend(OracleSim, scen)
    for r in range(len(scen["rounds"])):
        replay_round(gpu, scen, r)
        replay_round(orc, scen, r)
        diff = compare_exports(gpu.export(), orc.export())
        assert diff is None, f"round {r}: {diff}"
    c = gpu.check()
    # a round replays its planes mid-round when it runs a phase more than 32 ticks after the round start
    late = sum(1 for rd in scen["rounds"] if any(len(ph) for ph in rd["phases"][32:]))
    assert c["plane_flushes"] == late and (late > 0) == flushes


@pytest.mark.parametrize("rounds", [0, 6])
def test_canonical_selection_past_one_scan_step_matches_restatement(rounds):
    """k_sel_row16 (the canonical layout's counts, ranks and resolve from one read of each row) ranks a row's
    columns in steps of 4,096: at 4,500 nodes a row spans two, the second partial, so the ranks carried from
    the first step into the second are checked.  Round 0 (no liveness yet: every observer draws from its
    known set) and after 6 rounds with down churn (live and dead sets, dead probes)."""
    n = 4500
    spec = WorkloadSpec(n=n, k=4, fanout=3, seed=5, init="warm", write_frac=0.05, down_frac=0.1, down_rounds=3)
    scen = make_scenario(f"selstep{n}", spec, rounds + 1, {"initial_interval_s": 1.0, "phi_threshold": 3.0})
    gpu = make_backend(GossipSim, scen, fd_ring=False)
    assert gpu.canonical
    for r in range(rounds):
        replay_round(gpu, scen, r)
    up = np.asarray(scen["rounds"][rounds]["up"], dtype=np.uint8)
    seeds = [0, 4099, 4321]
    sel = PeerSelector(gpu, fanout=3, seeds=seeds, seed=77)
    got = sel.select(gpu._dev(up, gpu.torch.uint8), rounds).cpu().numpy()
    st = gpu._host()["FD_STATE"][:, :n]  # the device's own live / dead sets (export()'s decoding)
    live = (st == 1).astype(np.int32)
    tod = np.where(st >= 2, st.astype(np.int64) - 2, -1)
    want = peer_select.select_peers(live, tod, np.ones((n, n), dtype=bool), up, 3, seeds, 77, rounds)
    assert np.array_equal(got, want)
    if rounds:
        assert (got[:, 3] >= 0).any()  # dead probes happened
    gpu.close()
