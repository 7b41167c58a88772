"""Heartbeats past 2^16 (GPU only).

GS_R_HB holds each view's heartbeat mod 2^16, decoded against the owner's own heartbeat
(GS_R_SELF_HB): exact while no view lags its owner by 2^16 or more.  Here
eight nodes gossip every round for ~34,000 rounds, so every heartbeat crosses 65,536 while
the views stay close behind; the device must match the C oracle (unbounded heartbeats)
array for array, heartbeats, failure-detector windows and live sets included.
"""

import numpy as np
import pytest
from helpers import compare_exports
from oracle import OracleSim

from aiocluster_amd.scenario import DEFAULT_CFG
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import key_names, liveness_tick, phase_tick, round_tick, synthetic_node_ids

pytestmark = pytest.mark.gpu

SCHED = [[(0, 1), (2, 3), (4, 5), (6, 7)], [(1, 2), (3, 4), (5, 6), (7, 0)], [(0, 4), (1, 5), (2, 6), (3, 7)],
         [(5, 0), (6, 1), (7, 2), (4, 3)]]


def test_heartbeats_past_2_16_match_oracle():
    import torch

    n, rounds = 8, 34000
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8)
    orc = OracleSim(ids, keys, dict(DEFAULT_CFG), "warm", init)
    up = np.ones(n, np.uint8)
    up_dev = torch.from_numpy(up).to(gpu.device)
    dev_sched = [(torch.tensor([a for a, _ in s], dtype=torch.int32, device=gpu.device),
                  torch.tensor([b for _, b in s], dtype=torch.int32, device=gpu.device)) for s in SCHED]
    for r in range(rounds):
        t = round_tick(r)
        gpu.begin_round(t, up_dev)
        orc.begin_round(t, up)
        for p in range(2):
            i = (r + p) % len(SCHED)
            gpu.run_phase_arrays(phase_tick(r, p), *dev_sched[i])
            orc.run_phase(phase_tick(r, p), SCHED[i])
        gpu.liveness(liveness_tick(r, 2), up_dev)
        orc.liveness(liveness_tick(r, 2), up)
        if r in (100, rounds // 2, rounds - 1):
            want = orc.export()
            diff = compare_exports(gpu.export(), want)
            assert diff is None, f"round {r}: {diff}"
    hb = np.asarray(want["hb"])
    assert hb.min() > 65536, "every heartbeat must have crossed 2^16"
    c = gpu.check()  # raises on err_hb_lag: the automatic sweeps (every 2^14 rounds + phases) ran clean
    assert c["exchanges"] == rounds * 8 and c["err_hb_lag"] == 0


def test_heartbeat_lag_sweep_flags_views_near_the_16_bit_bound():
    """A view that lags its owner by >= 2^15 heartbeats (injected into GS_R_HB; in a run: an observer
    cut off from an owner for ~2^15 of the owner's increments) trips err_hb_lag, so check() raises before
    a 16-bit decode can go wrong; a lag just below the bound does not."""
    import torch

    from aiocluster_amd._lib import GsError

    n = 8
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=True, hist_cap=8)
    up_dev = torch.ones(n, dtype=torch.uint8, device=gpu.device)
    gpu.begin_round(round_tick(0), up_dev)
    gpu.liveness(liveness_tick(0, 0), up_dev)
    R = gpu.region("SELF_HB", torch.int32, (gpu.np_,))
    hb = gpu.region("HB", torch.int16, (n, gpu.np_))
    def s16(v):  # a heartbeat as GS_R_HB stores it (mod 2^16), viewed as int16
        v &= 0xFFFF
        return v - 65536 if v >= 32768 else v

    R[3] = 50000
    hb[3, 3] = s16(50000)  # the owner's own view (diagonal)
    hb[5, 3] = s16(50000 - 32767)  # lag 2^15 - 1: exact, not flagged
    hb[6, 3] = s16(50000 - 32000)
    for o in (0, 1, 2, 4, 7):
        hb[o, 3] = s16(50000 - 10)
    gpu.check_heartbeat_lag()
    assert gpu.check()["err_hb_lag"] == 0
    hb[6, 3] = s16(50000 - 32768)  # lag 2^15
    gpu.check_heartbeat_lag()
    with pytest.raises(GsError, match="err_hb_lag"):
        gpu.check()


def test_windows_silent_past_2_15_ticks_decide_exactly():
    """16-bit last-report ticks (GS_R_FD_LAST): node 7 is down for 700 rounds (44,800 ticks > 2^15), so
    every window about it and every window of its own row goes unreported past the 2^15-tick bound and
    is marked old (k_fd_age); liveness decisions (dead while silent, a report after the silence appends
    no interval) stay exact, and once node 7 is back every window is fresh again: the export matches
    the C oracle array for array.  Windows are compared mid-silence too, with the old windows' report
    tick left out (it reads back only as "2^15 ticks or more ago")."""
    import torch

    n, down0, down1, rounds = 8, 10, 710, 740
    ids, keys = synthetic_node_ids(n), key_names(2)
    init = {j: [(0, f"v{j}")] for j in range(n)}
    gpu = GossipSim(ids, keys, dict(DEFAULT_CFG), "warm", init, tombstones=False, fd_ring=False, hist_cap=8)
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
        if r == down1 - 1:  # mid-silence: the old windows' tick is the only thing not kept
            got, want = gpu.export(), orc.export()
            old = (want["fd_last"] >= 0) & (liveness_tick(r, 2) - want["fd_last"] >= 1 << 15)
            assert old[:, 7].sum() == n - 1 and old[7].sum() == n - 1
            got["fd_last"] = np.where(old, want["fd_last"], got["fd_last"])
            diff = compare_exports(got, want)
            assert diff is None, f"round {r}: {diff}"
    diff = compare_exports(gpu.export(), orc.export())
    assert diff is None, f"after the silence: {diff}"
    assert gpu.check()["exchanges"] == orc.stats()["exchanges"]
