"""Sampled interval rings at full size (GPU only): SURVEY §7(b)'s fallback for windows past W intervals.

The compact window layout is exact only until a window holds W intervals since its last reset; at the
headline's ~1.8 reports per pair and round, W = 1000 lasts ~560 rounds.  With ``ring_rows`` a sample of
observer rows keeps every window's interval ring, so their ``BoundedArrayStats`` roll over exactly
(``aiocluster/failure_detector.py:131-162``: subtract the evicted interval, then add), forever; the other
rows' full windows are counted in ``fd_saturated`` (documented inexact, not an error).  Here W = 8 at
65,536 nodes, so every ring row's windows roll over within a few rounds, and every phase of a round on
exchanges touching a ring row must equal the C oracle (whose rings are loaded from the device's) on the
ring rows, including the liveness decisions that the rolled-over means drive."""

import numpy as np
import pytest
from rowcheck import check_round_rows

from aiocluster_amd import driver
from aiocluster_amd.scenario import DEFAULT_CFG
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

pytestmark = pytest.mark.gpu


def test_sampled_ring_rows_roll_over_exactly_at_65536():
    import torch

    n, K, W = 65536, 16, 8
    cfg = dict(DEFAULT_CFG, window=W)
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=7, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3)
    ring = sorted(np.random.default_rng(7).choice(n, size=64, replace=False).tolist())
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=False, fd_ring=False,
                    hist_cap=16, initial_ops=driver.boot_ops(n, K), ring_rows=ring)
    plans = driver.prepare(spec, 13, torch, sim.device)
    for r in range(12):
        driver.run_round([sim], plans[r], group=None)
    from aiocluster_amd._lib import GsError

    with pytest.raises(GsError, match="fd_saturated"):  # inexact compact rows are loud by default
        sim.check()
    c = sim.check(accept_saturated=True)  # the sampled-ring contract: counted, the ring rows exact
    assert c["err_fd_overflow"] == 0 and c["fd_saturated"] > 0, c
    # the ring rows' windows rolled over (appends since the last reset >= W, held below 2W)
    sb = 32 - 5  # W = 8: the count takes 5 bits
    fd = sim.region("FD", torch.int32, (n, sim.np_))[torch.as_tensor(ring, device=sim.device), :n]
    cnt = (fd >> sb) & 31
    assert int((cnt >= W).sum().item()) > 1000
    rd = plans[12]
    driver.begin([sim], rd)
    diff, info = check_round_rows(sim, cfg, rd, sample=16, seed=12, only_rows=ring)
    assert diff is None, diff
    assert info["rows"] >= 64 and info["hb_reports"] > 0, info
    sim.close()
