"""Distribution of the peer-selection restatement (the device's algorithm, oracle/peer_select.py)
against the REAL reference's select_nodes_for_gossip (aiocluster/server.py:656-717), whose
frequencies over 20,000 seeded draws per case are in tests/golden/peer_select_freq.json
(oracle/gen_peer_fixture.py).  CPU only.  The device kernels are pinned to the restatement
bit for bit by tests/test_gpu_peers.py.
"""

import json
import os

import numpy as np
import peer_select
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "peer_select_freq.json")
CASES = json.load(open(GOLDEN))
TRIALS = 6000


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"L{c['L']}D{c['D']}X{c['X']}S{c['S']}F{c['F']}")
def test_frequencies_match_reference(case):
    L, D, X, S, F = case["L"], case["D"], case["X"], case["S"], case["F"]
    n = 1 + L + D + X
    live = np.zeros((n, n), dtype=np.int64)
    tod = np.full((n, n), -1, dtype=np.int64)
    live[0, 1:1 + L] = 1
    tod[0, 1 + L:1 + L + D] = 7
    known = np.ones((n, n), dtype=bool)
    up = np.zeros(n, dtype=np.uint8)
    up[0] = 1
    pool = list(range(1, 1 + L)) if case["seeds_live"] else (list(range(1 + L, n)) or list(range(1, 1 + L)))
    seeds = pool[:S]
    dead_hits = seed_hits = total = 0
    inc = np.zeros(n)
    for r in range(TRIALS):
        t = peer_select.select_peers(live, tod, known, up, F, seeds, 2024, r)[0]
        picks = t[:F][t[:F] >= 0]
        total += len(picks)
        inc[picks] += 1
        dead_hits += t[F] >= 0
        seed_hits += t[F + 1] >= 0
    def close(p_got, p_ref):  # two binomial estimates (6,000 and 20,000 draws): 5 sigma
        sd = np.sqrt(max(p_ref * (1 - p_ref), 1e-4) * (1 / TRIALS + 1 / case["trials"]))
        return abs(p_got - p_ref) <= 5 * sd + 1e-9
    assert close(dead_hits / TRIALS, case["p_dead"]), (dead_hits / TRIALS, case["p_dead"])
    assert close(seed_hits / TRIALS, case["p_seed"]), (seed_hits / TRIALS, case["p_seed"])
    assert total / TRIALS == pytest.approx(case["mean_sampled"])
    chosen = inc[inc > 0] / TRIALS
    assert len(chosen) == case["distinct"]
    mean = case["mean_sampled"] / case["distinct"]
    assert np.all(np.abs(chosen - mean) <= 5 * np.sqrt(mean * (1 - mean) / TRIALS) + 1e-9)
