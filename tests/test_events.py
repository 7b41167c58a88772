"""Hook events (on_key_change / on_node_join / on_node_leave) per round against the REAL reference's
(tests/golden/events_*.json.gz, oracle/gen_events_fixture.py): the C oracle on the CPU, the device
event stream (gs_set_events) on the GPU."""

import gzip
import json
import os

import numpy as np
import pytest
from helpers import load_scenario, make_backend
from oracle import OracleSim

from aiocluster_amd.scenario import replay_round

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["trunc8", "fdgc12", "simple3", "cold64"]


def golden_events(name):
    with gzip.open(os.path.join(GOLDEN, f"events_{name}.json.gz"), "rt") as f:
        return json.load(f)


def _check(backend, name):
    scen = load_scenario(name)
    want = golden_events(name)
    backend.enable_events()
    kinds = set()
    for r in range(len(scen["rounds"])):
        replay_round(backend, scen, r)
        got = backend.drain_events().astype(np.int64).tolist()
        assert got == want[r], f"{name} round {r}: {len(got)} events vs {len(want[r])}"
        kinds |= {e[2] >> 8 for e in got}
    return kinds


@pytest.mark.parametrize("name", NAMES)
def test_oracle_events_match_reference(name):
    scen = load_scenario(name)
    kinds = _check(make_backend(OracleSim, scen), name)
    assert 0 in kinds


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_device_events_match_reference(name):
    from aiocluster_amd.sim import GossipSim

    scen = load_scenario(name)
    kinds = _check(make_backend(GossipSim, scen), name)
    assert 0 in kinds
    if name == "fdgc12":
        assert {1, 2} <= kinds


@pytest.mark.gpu
def test_device_events_prefix_views():
    """Prefix views (no tombstones) take the per-key apply path while events are on."""
    from aiocluster_amd.sim import GossipSim

    scen = load_scenario("fdgc12")
    kinds = _check(make_backend(GossipSim, scen, tombstones=False), "fdgc12")
    assert {0, 1, 2} <= kinds
