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


class _SeqRecorder:
    """Proxies an OracleSim and turns its (reference-ordered) events into device-format records
    (gs_set_events: 8 words, seq as the device computes it) call by call."""

    def __init__(self, orc):
        self.orc, self.recs, self.phases, self.writes = orc, [], {}, 0

    def _take(self, seq_of):
        for e in self.orc.drain_events().astype(np.int64).tolist():
            self.recs.append(e + [seq_of(e), 0])

    def write(self, t, j, k, op, v):
        self.orc.write(t, j, k, op, v)

    def begin_round(self, t, up):
        w0 = self.writes

        def seq(e):  # the write's index among all writes (call order)
            nonlocal w0
            w0 += 1
            return w0 - 1

        self.orc.begin_round(t, up)  # flushes the writes
        self._take(seq)
        self.writes = w0

    def run_phase(self, t, pairs):
        self.orc.run_phase(t, pairs)
        peer = {}
        for a, b in pairs:
            peer[a], peer[b] = b, a
        self.phases[t] = ([a for a, _ in pairs], [b for _, b in pairs])
        order = {}

        def seq(e):  # the sender's dict position of the owner
            s = peer[e[0]]
            if s not in order:
                order[s] = {j: q for q, j in enumerate(self.orc.order(s))}
            return order[s][e[1]]

        self._take(seq)

    def liveness(self, t, up, r):
        self.orc.liveness(t, up, r)
        self._take(lambda e: 0)


@pytest.mark.parametrize("name", NAMES)
def test_order_events_restores_reference_order(name):
    """aiocluster_amd.sim.order_events (the device stream's host-side order) puts shuffled records,
    carrying the seq words the kernels write, back into the reference's hook order."""
    from aiocluster_amd.sim import order_events

    scen = load_scenario(name)
    rec = _SeqRecorder(make_backend(OracleSim, scen))
    rec.orc.enable_events()
    want = golden_events(name)
    rng = np.random.default_rng(7)
    for r in range(len(scen["rounds"])):
        rec.recs, rec.phases = [], {}
        replay_round(rec, scen, r)
        ev = np.asarray(rec.recs, dtype=np.int64).reshape(-1, 8)
        assert ev[:, :6].tolist() == want[r]
        shuf = ev[rng.permutation(len(ev))].astype(np.uint32)
        got = shuf[order_events(shuf, rec.orc.n, rec.phases, list(range(rec.writes)))]
        assert got[:, :6].astype(np.int64).tolist() == want[r], f"{name} round {r}"
