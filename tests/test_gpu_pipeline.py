"""gs_run_phases_group (round 6): a round's sliced phases in one library call, pipelined -- phase p + 1's pass 1 is
queued behind a device gate before the host reads phase p's pending count, and runs again when a chain of phase p
outlived chain step 1 (``phase_reruns``).  Every round must end in one handle's state, bit for bit, with deltas the
mtu cuts across slices, for the batched in-process group and for slice 0 held alone.  GPU only."""

import numpy as np
import pytest
from helpers import compare_exports, make_backend

from aiocluster_amd.scenario import initial_by_owner, make_scenario, replay_round, scenario_node_ids
from aiocluster_amd.shard import ShardGroup, SoloComm
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec, liveness_tick, phase_tick, round_tick

pytestmark = pytest.mark.gpu

KW = dict(tombstones=False, fd_ring=False, hb8=True, mv8=True)  # the headline's layout: the pipelined path's case


def replay_round_batched(grp, scen, r):
    """replay_round with the round's phases in one gs_run_phases_group call (device arrays back to back)."""
    import torch

    rd = scen["rounds"][r]
    t = round_tick(r)
    up = rd["up"]
    for j, k, op, v in rd["writes"]:
        grp.write(t, j, k, op, v)
    grp.begin_round(t, up)
    phases = [np.asarray(ph, dtype=np.int32).reshape(-1, 2) for ph in rd["phases"]]
    offs = np.zeros(len(phases) + 1, dtype=np.uint32)
    offs[1:] = np.cumsum([len(p) for p in phases])
    allp = np.concatenate(phases) if phases else np.zeros((0, 2), np.int32)
    dev = grp.slices[0].device
    ini = torch.from_numpy(np.ascontiguousarray(allp[:, 0])).to(dev)
    res = torch.from_numpy(np.ascontiguousarray(allp[:, 1])).to(dev)
    ticks = np.array([phase_tick(r, p) for p in range(len(phases))], dtype=np.uint32)
    assert grp.run_phases(ini, res, offs, ticks)
    grp.liveness(liveness_tick(r, len(phases)), up, r)


def _scenario(n, mtu, seed, rounds=8):
    spec = WorkloadSpec(n=n, k=8, fanout=3, seed=seed, init="warm", write_frac=0.3, down_frac=0.08, down_rounds=3)
    return make_scenario(f"pipe{n}", spec, rounds, {"mtu": mtu})


@pytest.mark.parametrize("n,G,mtu", [(256, 2, 700), (512, 8, 900), (1024, 8, 400), (10240, 8, 250)])
def test_pipelined_group_matches_single_handle(n, G, mtu):
    """The remaining chain steps run on the device count after every phase; the gate fires only when a phase's
    overflow list is longer than GS_CHAIN_CAP (the host's steps) -- 10,240 nodes at mtu 250: most slots overflow."""
    scen = _scenario(n, mtu, seed=n * G + mtu, rounds=3 if n > 4096 else 8)
    one = make_backend(GossipSim, scen, **KW)
    grp = ShardGroup.in_process(scenario_node_ids(scen), scen["keys"], scen["config"], G, init=scen["init"],
                                initial_values=initial_by_owner(scen), native=True, **KW)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round_batched(grp, scen, r)
        diff = compare_exports(grp.export(), one.export())
        assert diff is None, f"round {r}: {diff}"
    c1, cg = one.check(), grp.check()
    for k in ("exchanges", "hb_reports", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "hb_writes"):
        assert cg[k] == c1[k], (k, cg[k], c1[k])
    assert c1["truncated"] > 0
    if n > 4096:  # more than GS_CHAIN_CAP overflowing slots in a phase: the gate fired and those phases ran again
        assert cg["phase_reruns"] > 0, cg["phase_reruns"]
    print(f"n={n} G={G} mtu={mtu}: truncated {c1['truncated']}, phase_reruns {cg['phase_reruns']}")
    one.close()
    for s in grp.slices:
        s.close()


def test_pipelined_lone_slice_zero_matches_single_handle_columns():
    """Slice 0 of 4 held alone (the rehearsal of one GPU's share, SoloComm): its columns equal one handle's."""
    scen = _scenario(512, 600, seed=5, rounds=5)
    one = make_backend(GossipSim, scen, **KW)
    ids, keys, cfg = scenario_node_ids(scen), scen["keys"], scen["config"]
    s0 = GossipSim(ids, keys, cfg, init=scen["init"], initial_values=initial_by_owner(scen), shards=4, shard=0, **KW)
    g0 = ShardGroup([s0], SoloComm(4, 0), cfg["mtu"], native=True)
    for r in range(len(scen["rounds"])):
        replay_round(one, scen, r)
        replay_round_batched(g0, scen, r)
    want = one.export()
    assert compare_exports(g0.export(), {k: v[:, : s0.ncol] for k, v in want.items()}) is None
    assert one.check()["truncated"] > 0
    for x in (one, s0):
        x.close()
