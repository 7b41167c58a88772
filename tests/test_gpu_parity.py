"""Parity of the HIP path (through the C ABI) with the reference and the C oracle.  GPU only.

* golden: the device reproduces the REAL reference's canonical state after every
  round of every golden fixture (byte-identical JSON, phi computed on the device);
* oracle: larger seeded scenarios (cold/general and warm/canonical layouts, MTU
  truncation, deletes + TTL + tombstone GC, churn, ring and compact windows) are
  compared array by array with the C oracle after every round.
Integer state must be bit-exact; phi is binary64 and is compared exactly too
(the north-star tolerance is 1e-9 relative; the tick model makes it exact).
"""

import numpy as np
import pytest
from helpers import SCENARIOS, compare_exports, load_scenario, make_backend, replay_and_compare
from oracle import OracleSim

from aiocluster_amd._lib import GsError
from aiocluster_amd.scenario import make_scenario, replay, replay_round
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec

pytestmark = pytest.mark.gpu

PHI_RTOL = 1e-9  # north_star tolerance for phi


@pytest.mark.parametrize("name", SCENARIOS)
def test_gpu_matches_reference_golden(name):
    scen = load_scenario(name)
    exp = scen["expect"]
    sim = make_backend(GossipSim, scen)
    res = replay_and_compare(sim, scen, exp["states"], exp["hashes"])
    assert res is None, f"{name}: first mismatch at round {res[0]}: {res[1]}"
    c = sim.check()
    assert c["q9"] == len(exp["q9"])  # garbage_collect KeyErrors


SET_ONLY = ["sched16", "fdgc12", "q9x10", "warm128"]  # golden scenarios without deletes / TTL writes


@pytest.mark.parametrize("name", SET_ONLY)
def test_prefix_views_match_reference_golden(name):
    """Without GS_TOMBSTONES views are tracked as prefixes of the owner's writes (GS_MV_INEXACT);
    the packer skips HELD for them.  Same golden states as the tombstone-tracking layout."""
    scen = load_scenario(name)
    exp = scen["expect"]
    sim = make_backend(GossipSim, scen, tombstones=False)
    res = replay_and_compare(sim, scen, exp["states"], exp["hashes"])
    assert res is None, f"{name}: first mismatch at round {res[0]}: {res[1]}"
    c = sim.check()
    assert c["q9"] == len(exp["q9"])
    if name == "sched16":
        assert c["truncated"] > 0 and sim.inexact_views() > 0  # holes: the HELD path ran


def test_fd_garbage_collection_in_canonical_layout_fails_loudly():
    """Removing nodes needs the general layout: a canonical (warm, index-order) state must refuse."""
    spec = WorkloadSpec(n=16, k=2, fanout=2, seed=3, init="warm", write_frac=0.1, down_frac=0.4, down_rounds=12)
    scen = make_scenario("gcwarm", spec, 30, {"dead_grace_s": 4.0, "phi_threshold": 2.0, "initial_interval_s": 1.0})
    sim = make_backend(GossipSim, scen)
    with pytest.raises(GsError, match="garbage_collect"):
        replay(sim, scen, on_round=lambda r: sim.check())


def test_warm_general_layout_with_fd_gc_vs_oracle():
    """A warm start run in the general layout so FD garbage collection can remove and re-add nodes."""
    spec = WorkloadSpec(n=48, k=4, fanout=2, seed=21, init="warm", write_frac=0.2, delete_frac=0.2,
                        down_frac=0.4, down_rounds=10)
    scen = make_scenario("gcwarm48", spec, 36, {"dead_grace_s": 5.0, "phi_threshold": 2.0,
                                                 "initial_interval_s": 1.0, "tombstone_grace_s": 3, "mtu": 1500})
    gpu, orc, c = lockstep_vs_oracle(scen, canonical=False)
    assert c["fd_gc"] > 0 and c["q9"] == len(orc.q9_events)


def lockstep_vs_oracle(scen, every=1, **kw):
    gpu = make_backend(GossipSim, scen, **kw)
    orc = make_backend(OracleSim, scen)
    for r in range(len(scen["rounds"])):
        replay_round(gpu, scen, r)
        replay_round(orc, scen, r)
        if r % every == 0 or r == len(scen["rounds"]) - 1:
            diff = compare_exports(gpu.export(), orc.export())
            assert diff is None, f"round {r}: {diff}"
            c = gpu.check()
    return gpu, orc, c


def test_cold_general_layout_vs_oracle():
    spec = WorkloadSpec(n=200, k=8, fanout=3, seed=11, init="cold", write_frac=0.2, delete_frac=0.15,
                        ttl_frac=0.1, down_frac=0.1, down_rounds=3)
    cfg = {"mtu": 700, "tombstone_grace_s": 2, "window": 6, "max_interval_s": 2.0, "initial_interval_s": 1.0,
           "phi_threshold": 3.0}
    scen = make_scenario("cold200", spec, 14, cfg)
    gpu, orc, c = lockstep_vs_oracle(scen)
    s = orc.stats()
    assert c["exchanges"] == s["exchanges"] and c["node_deltas"] == s["node_deltas"]
    assert c["kvs_sent"] == s["kvs_sent"] and c["truncated"] == s["truncated"] > 0
    assert c["delta_bytes"] == s["delta_bytes"] and c["hb_reports"] == s["hb_reports"]


def test_warm_canonical_compact_fd_vs_oracle():
    spec = WorkloadSpec(n=512, k=16, fanout=3, seed=12, init="warm", write_frac=0.05, down_frac=0.05,
                        down_rounds=3)
    scen = make_scenario("warm512", spec, 10, {"mtu": 2500})
    gpu, orc, c = lockstep_vs_oracle(scen, tombstones=False, fd_ring=False)
    s = orc.stats()
    assert c["node_deltas"] == s["node_deltas"] and c["truncated"] == s["truncated"]
    assert c["delta_bytes"] == s["delta_bytes"]


def test_phi_matches_oracle_within_tolerance():
    spec = WorkloadSpec(n=64, k=4, fanout=2, seed=13, init="warm", write_frac=0.1, down_frac=0.2, down_rounds=4)
    scen = make_scenario("phi64", spec, 12, {"initial_interval_s": 1.0, "phi_threshold": 3.0})
    gpu = make_backend(GossipSim, scen)
    orc = make_backend(OracleSim, scen)
    replay(gpu, scen)
    replay(orc, scen)
    t = gpu.last_tick
    import ctypes

    got = np.stack([gpu.phi_row(o, t) for o in range(64)])
    want = np.full((64, 64), np.nan)
    phi = ctypes.c_double()
    for o in range(64):
        for j in range(64):
            if orc.L.orc_fd_phi(orc.h, o, j, t * 15625, ctypes.byref(phi)):
                want[o, j] = phi.value
    assert np.array_equal(np.isnan(got), np.isnan(want))
    m = ~np.isnan(want)
    assert m.sum() > 0
    np.testing.assert_allclose(got[m], want[m], rtol=PHI_RTOL, atol=0)


def test_config2_cold_1024x64_converges_bit_exact():
    """BASELINE config 2: 1,024 nodes x 64 keys, fanout 3, cold start, run to version convergence."""
    spec = WorkloadSpec(n=1024, k=64, fanout=3, seed=2, init="cold", write_frac=0.0)
    scen = make_scenario("config2", spec, 24, {})
    gpu, orc, c = lockstep_vs_oracle(scen, every=6, tombstones=False, fd_ring=False)
    ex = gpu.export()
    owner_mv = np.diag(ex["mv"])
    assert np.all(ex["mv"] <= owner_mv[None, :])
    assert np.all(ex["mv"] == owner_mv[None, :]), "version matrix did not converge"


def test_config2_matches_reference_digests():
    """BASELINE config 2 (1,024 x 64, cold) against the REAL reference: per-round SHA-256 of every export
    field and the final max_version matrix (tests/golden/scen_config2.json.gz, the rounds it pins)."""
    from test_oracle_golden import replay_digests

    scen = load_scenario("config2")
    for tomb in (True, False):  # tombstone layout and prefix views
        replay_digests(make_backend(GossipSim, scen, tombstones=tomb, fd_ring=False), scen)


def test_config5_partition_heal_small_vs_oracle():
    """BASELINE config 5 in miniature: MTU-truncated deltas, deletes + tombstone GC, a partition into
    halves that heals; every round vs the oracle, and the device's failure-detector census (false-
    positive rate) vs the one counted from the oracle's live / dead sets."""
    spec = WorkloadSpec(n=256, k=8, fanout=3, seed=55, init="warm", write_frac=0.1, delete_frac=0.1,
                        partition=(6, 22))
    scen = make_scenario("c5_256", spec, 30, {"mtu": 1400, "tombstone_grace_s": 4, "initial_interval_s": 1.0,
                                               "phi_threshold": 3.0})
    gpu = make_backend(GossipSim, scen, fd_ring=False)
    orc = make_backend(OracleSim, scen)
    saw_fp = False
    for r in range(len(scen["rounds"])):
        replay_round(gpu, scen, r)
        replay_round(orc, scen, r)
        ex = orc.export()
        diff = compare_exports(gpu.export(), ex)
        assert diff is None, f"round {r}: {diff}"
        up = np.asarray(scen["rounds"][r]["up"], dtype=bool)
        off = ~np.eye(256, dtype=bool) & up[:, None]
        tu = up[None, :]
        want = {"up_pairs": int((off & tu).sum()), "up_dead": int((off & tu & (ex["tod"] >= 0)).sum()),
                "up_live": int((off & tu & (ex["live"] == 1)).sum()), "down_pairs": int((off & ~tu).sum()),
                "down_live": int((off & ~tu & (ex["live"] == 1)).sum())}
        got = gpu.fd_census(scen["rounds"][r]["up"])
        assert got == want, (r, got, want)
        saw_fp |= got["up_dead"] > 0
    c = gpu.check()
    assert saw_fp and c["truncated"] > 0 and c["tomb_gc"] > 0
    assert got["up_dead"] == 0  # healed: nobody is dead any more


@pytest.mark.parametrize("name", ["fdgc12", "q9x10"])
def test_version_only_layout_matches_reference_golden(name):
    """GS_NO_HELD (config 4's layout): no HELD region at all; exact while no NodeDelta is truncated."""
    scen = load_scenario(name)
    exp = scen["expect"]
    sim = make_backend(GossipSim, scen, tombstones=False, held=False)
    assert "HELD" not in sim.regions
    res = replay_and_compare(sim, scen, exp["states"], exp["hashes"])
    assert res is None, f"{name}: first mismatch at round {res[0]}: {res[1]}"
    c = sim.check()
    assert c["err_holes"] == 0 and c["truncated"] == 0
    last = exp["states"][-1]
    for o in range(scen["n"]):  # single-view reads and snapshots derive held keys from max_version
        for j, hb, mv, gc, kvs in last[o]["nodes"]:
            ns = sim.node_state(o, j)
            got = sorted([k, v.value, v.version, int(v.status), v.status_change_ts] for k, v in ns.key_values.items())
            assert [ns.heartbeat, ns.max_version, ns.last_gc_version, got] == [hb, mv, gc, kvs], (o, j)
        snap = sim.snapshot(o)
        assert len(snap.node_states) == len(last[o]["nodes"])


def test_version_only_layout_vs_oracle_and_refuses_holes():
    spec = WorkloadSpec(n=384, k=16, fanout=3, seed=17, init="warm", write_frac=0.2, down_frac=0.05,
                        down_rounds=3)
    scen = make_scenario("vo384", spec, 10, {"mtu": 1 << 30})
    gpu, orc, c = lockstep_vs_oracle(scen, tombstones=False, held=False, fd_ring=False)
    assert c["err_holes"] == 0 and c["node_deltas"] > 0
    # the same cluster with a small mtu truncates NodeDeltas: views get holes, which this layout refuses
    scen2 = make_scenario("vo384t", spec, 10, {"mtu": 1500})
    sim = make_backend(GossipSim, scen2, tombstones=False, held=False, fd_ring=False)
    with pytest.raises(GsError, match="err_holes"):
        replay(sim, scen2, on_round=lambda r: sim.check())


@pytest.mark.parametrize("name", ["trunc8", "fdgc12", "warm128"])
def test_snapshot_matches_reference_golden(name):
    """Cluster.snapshot (server.py:168-175) of every node, read from its device rows, against the
    reference's states after the last round."""
    scen = load_scenario(name)
    exp = scen["expect"]
    sim = make_backend(GossipSim, scen)
    replay(sim, scen)
    last = exp["states"][-1] if exp["states"] else exp["final"]
    idx = {nid: j for j, nid in enumerate(sim.node_ids)}
    for o in range(scen["n"]):
        snap = sim.snapshot(o)
        assert snap.self_node_id == sim.node_ids[o]
        nodes = []
        for nid, ns in snap.node_states.items():
            kvs = sorted([k, v.value, v.version, int(v.status), v.status_change_ts]
                         for k, v in ns.key_values.items())
            nodes.append([idx[nid], ns.heartbeat, ns.max_version, ns.last_gc_version, kvs])
        assert nodes == last[o]["nodes"], (o, nodes[:3], last[o]["nodes"][:3])
        # ClusterState.node_state (state.py:295-296) of single views, read without the whole matrix
        for j, hb, mv, gc, kvs in last[o]["nodes"][:4]:
            ns = sim.node_state(o, j)
            got = sorted([k, v.value, v.version, int(v.status), v.status_change_ts] for k, v in ns.key_values.items())
            assert [ns.heartbeat, ns.max_version, ns.last_gc_version, got] == [hb, mv, gc, kvs], (o, j)
        assert sorted(idx[x] for x in snap.live_nodes) == last[o]["live"]
        assert sorted(idx[x] for x in snap.dead_nodes) == [d[0] for d in last[o]["dead"]]
