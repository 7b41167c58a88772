"""Wire-format emitter on the device vs the REAL reference's bytes (GPU only).

Each golden scenario is replayed on the device; after every captured round the emitter produces,
for the fixture's (s, r) pairs, ``_make_syn_msg().SerializeToString()`` of s (the DigestPb from
``gs_emit_digest`` in the host's PacketPb framing) and the DeltaPb of s's
``compute_partial_delta_respecting_mtu`` against r's digest (``gs_emit_delta``).  Both must equal
the reference's bytes (``oracle/gen_wire_fixture.py``) exactly -- including MTU-truncated NodeDeltas,
tombstones, scheduled-for-deletion targets and general-layout dict orders.  The emitter must not
change the state (the replay continues and is checked against the golden state hashes).
"""

import pytest
from helpers import load_scenario, make_backend
from test_wire_host import load_wire

from aiocluster_amd.scenario import replay_round, state_hash
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.wire import WireEmitter

pytestmark = pytest.mark.gpu

CASES = [("trunc8", True), ("sched16", True), ("fdgc12", True), ("simple3", True), ("cold64", True),
         ("sched16", False), ("fdgc12", False)]


@pytest.mark.parametrize("name,tomb", CASES)
def test_device_wire_bytes_match_reference(name, tomb):
    scen = load_scenario(name)
    w = load_wire(name)
    by_round = {}
    for r, s, q, syn, delta in w["cases"]:
        by_round.setdefault(r, []).append((s, q, syn, delta))
    sim = make_backend(GossipSim, scen, tombstones=tomb)
    em = WireEmitter(sim, cluster_id="default-cluster")
    checked = 0
    for r in range(len(scen["rounds"])):
        replay_round(sim, scen, r)
        for s, q, syn, delta in by_round.get(r, []):
            t = w["tick"][str(r)]
            got = em.syn(s, t)
            assert got.hex() == syn, f"round {r} syn of {s}: {got.hex()} != {syn}"
            got = em.delta(s, q, t)
            assert got.hex() == delta, f"round {r} delta {s}->{q}: {got.hex()} != {delta}"
            checked += 1
        assert state_hash(sim.state()) == scen["expect"]["hashes"][r], f"round {r}: emitter changed the state"
    assert checked == len(w["cases"])
