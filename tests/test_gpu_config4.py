"""BASELINE config 4 at its real size, on one GPU: 262,144 nodes, one owner-column slice of 8 (GPU only).

Config 4's contract: warm start, no deletes, version-only views
(GS_NO_HELD; 8-bit heartbeat and max_version views, GS_HB8 + GS_MV8, as bench.py runs it) and an mtu above every delta, so no
NodeDelta is ever truncated.  Then a slice's packing
does not depend on the other slices (every stale owner is sent whole), and slice 0 of 8 held alone
(``SoloComm``: the others' totals are zeros) is exact for its 32,768 owner columns over all 262,144
observer rows -- 152+ GB of the 288 GB HBM, the share one GPU of the 8-GPU run holds.  Checked:

* every device check counter is 0 (``err_holes`` included) and the exchange count is the plan's;
* the owner tables equal the host restatement of the write stream (``oracle/owner_tables.py``);
* every view's max_version is at most its owner's, and the version matrix converges once writes stop
  (every observer holds every owner's max_version: anti-entropy, ``aiocluster/state.py:340-415``);
* every phase of one round, on sampled exchanges, equals the C oracle on the slice's columns
  (``rowcheck.check_round_rows``; the other columns are loaded inert on both sides).

The round: ``aiocluster/server.py:441-495``.
"""

import numpy as np
import pytest
from owner_tables import check_owner_tables, plan_batches
from rowcheck import check_round_rows

from aiocluster_amd import driver
from aiocluster_amd.scenario import DEFAULT_CFG
from aiocluster_amd.shard import ShardGroup, SoloComm
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

pytestmark = pytest.mark.gpu


def _max_version_checks(sim, converged: bool) -> tuple[int, int]:
    """(views above their owner's max_version, views below it); row chunks keep the temporaries small.
    The owner's max_version is GS_R_SELF_MV (its own latest write).  With GS_MV8 a view decodes to at most
    that by construction, and the bound that keeps the decode exact (lag < 2^7) is the lag sweep's
    (err_hb_lag, checked by every grp.check()); "below" -- convergence -- is the real check there."""
    torch = sim.torch
    nc = sim.ncol
    own = sim.region("SELF_MV", torch.int32, (sim.np_,))[:nc]
    above = below = 0
    for r0 in range(0, sim.n, 16384):
        blk = sim.mv_words(slice(r0, r0 + 16384))[:, :nc]  # decoded words, the inexact bit included: never set here
        above += int((blk > own[None, :]).sum().item())
        if converged:
            below += int((blk < own[None, :]).sum().item())
    return above, below


def test_config4_262144_slice0_of_8():
    import torch

    n, K, G = 262144, 16, 8
    cfg = dict(DEFAULT_CFG)
    cfg["mtu"] = 1 << 30  # above every delta: no truncation (config 4's contract)
    settle, quiet = 6, 12
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=4, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3,
                        quiet_from=settle + 1)
    boot = driver.boot_ops(n, K)
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=False, fd_ring=False,
                    hist_cap=16, initial_ops=boot, held=False, shards=G, shard=0, hb8=True,
                    mv8=True)  # bench.py's layout
    assert (sim.col_lo, sim.ncol) == (0, 32768)
    grp = ShardGroup([sim], SoloComm(G), cfg["mtu"])
    plans = driver.prepare(spec, settle + 1 + quiet, torch, sim.device)
    for r in range(settle):
        driver.run_round([sim], plans[r], group=grp)
    c = grp.check()  # every err_* = 0, err_holes included
    assert c["exchanges"] == sum(plans[r]["exchanges"] for r in range(settle))
    assert c["node_deltas"] > 0 and c["truncated"] == 0
    assert check_owner_tables(sim, plan_batches(K, n, plans[:settle], boot)) is None
    above, _ = _max_version_checks(sim, converged=False)
    assert above == 0
    # every phase of the next round (the last one with writes) vs the oracle on the slice's columns
    rd = plans[settle]
    driver.begin([sim], rd)
    diff, info = check_round_rows(sim, cfg, rd, sample=12, seed=4, group=grp)
    assert diff is None, diff
    assert info["node_deltas"] > 0 and info["hb_reports"] > 0, info
    # writes and churn stop: the version matrix converges
    for r in range(settle + 1, settle + 1 + quiet):
        driver.run_round([sim], plans[r], group=grp)
    grp.check()
    above, below = _max_version_checks(sim, converged=True)
    assert above == 0 and below == 0, (above, below)
    sim.close()
