"""The C oracle against the REAL reference's golden fixtures (CPU).

Each fixture (tests/golden/scen_*.json.gz, made by oracle/gen_golden.py from the
reference's own Cluster handlers) holds a scenario and the reference's canonical
state after every round.  The oracle must reproduce every round byte for byte:
versions, key-values, tombstones, heartbeats, dict order, live/dead sets,
time of death, sampling windows (len, float sum) and phi.
"""

import pytest
from helpers import SCENARIOS, load_scenario, make_backend, replay_and_compare
from oracle import OracleSim


@pytest.mark.parametrize("name", SCENARIOS)
def test_oracle_matches_reference(name):
    scen = load_scenario(name)
    exp = scen["expect"]
    sim = make_backend(OracleSim, scen)
    res = replay_and_compare(sim, scen, exp["states"], exp["hashes"])
    assert res is None, f"{name}: first mismatch at round {res[0]}: {res[1]}"
    assert sim.q9_events == exp["q9"]


def test_fixtures_exercise_the_quirks():
    """The fixtures cover truncation, tombstone GC, scheduled-for-deletion and FD GC."""
    trunc = load_scenario("trunc8")
    sim = make_backend(OracleSim, trunc)
    from aiocluster_amd.scenario import replay

    replay(sim, trunc)
    assert sim.stats()["truncated"] > 0  # Q1: NodeDeltas cut by the MTU
    # tombstones were garbage collected somewhere (last_gc_version > 0)
    assert any(nd[3] > 0 for o in trunc["expect"]["final"] for nd in o["nodes"])
    # FD garbage collection removed nodes from some dict (fdgc12)
    fd = load_scenario("fdgc12")["expect"]["states"]
    assert min(sum(len(o["nodes"]) for o in st) for st in fd[5:]) < 144


def replay_digests(sim, scen):
    """Replay the rounds the config-2 fixture pins and compare the per-round export digests; returns the
    last export."""
    import numpy as np

    from aiocluster_amd.scenario import export_digest, replay_round

    exp = scen["expect"]
    ex = None
    for r in range(exp["rounds_done"]):
        replay_round(sim, scen, r)
        ex = sim.export()
        got = export_digest(ex)
        bad = [k for k, v in exp["digests"][r].items() if got[k] != v]
        assert not bad, f"round {r}: digest mismatch in {bad}"
    assert np.array_equal(ex["mv"], np.asarray(exp["final_mv"], dtype=ex["mv"].dtype))
    holes = int(((ex["kv_version"] == 0) & (ex["pos"] >= 0)[:, :, None]).sum())
    assert holes == exp["final_holes"]
    return ex


def test_oracle_matches_reference_config2_digests():
    """BASELINE config 2 (1,024 nodes x 64 keys, cold start): the reference's per-round SHA-256 of every
    export field (tests/golden/scen_config2.json.gz, the rounds it pins) and its final max_version
    matrix."""
    scen = load_scenario("config2")
    replay_digests(make_backend(OracleSim, scen), scen)
