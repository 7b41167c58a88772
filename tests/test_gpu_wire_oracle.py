"""Wire emitter vs the C oracle at larger sizes (GPU only).

The golden fixtures pin the emitted bytes to the reference at up to 64 nodes
(``test_gpu_wire.py``).  Here seeded 1,024-node (warm, canonical layout) and 256-node (cold,
general layout) clusters run with a small MTU, so deltas are truncated; after several rounds
the device's DigestPb and DeltaPb bytes are parsed and compared with the oracle's state and
with the oracle's ``compute_partial_delta_respecting_mtu`` restatement (``orc_kat_compute_delta``,
pinned to the reference by ``tests/test_oracle_golden.py``): same NodeDeltas in the same order,
same from_version_excluded, same kv versions; and every DeltaPb fits the MTU.  No node goes
down, so nothing is scheduled for deletion (the oracle KAT takes an empty scheduled set).
"""

import ctypes as C
import random

import numpy as np
import pytest
from helpers import make_backend
from oracle import OracleSim
from pbread import fields

from aiocluster_amd.scenario import make_scenario, replay_round
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.wire import WireEmitter, node_id_pb
from aiocluster_amd.workload import WorkloadSpec, liveness_tick

pytestmark = pytest.mark.gpu


def parse_digest(b, nid_index):
    out = []
    for _, _, nd in fields(b):
        f = dict((x[0], x[2]) for x in fields(nd))
        out.append((nid_index[f[1]], f.get(2, 0), f.get(3, 0), f.get(4, 0)))
    return out


def parse_delta(b, nid_index):
    out = []
    for _, _, nd in fields(b):
        sub = fields(nd)
        f = dict((x[0], x[2]) for x in sub if x[0] != 4)
        vers = [dict((g[0], g[2]) for g in fields(x[2])).get(3, 0) for x in sub if x[0] == 4]
        out.append((nid_index[f[1]], f.get(2, 0), vers))
    return out


@pytest.mark.parametrize("n,k,init,mtu", [(1024, 16, "warm", 3000), (256, 8, "cold", 2000)])
def test_emitter_matches_oracle_delta_at_size(n, k, init, mtu):
    spec = WorkloadSpec(n=n, k=k, fanout=3, seed=11, init=init, write_frac=0.3, down_frac=0.0)
    scen = make_scenario(f"wire{n}", spec, 8, {"mtu": mtu})
    gpu = make_backend(GossipSim, scen)
    orc = make_backend(OracleSim, scen)
    em = WireEmitter(gpu)
    nid_index = {node_id_pb(x): i for i, x in enumerate(gpu.node_ids)}
    rng = random.Random(n)
    cap = 4 * n * k
    nd_node, nd_from = np.zeros(cap, np.int32), np.zeros(cap, np.uint32)
    nd_nkv, kv_ver = np.zeros(cap, np.int32), np.zeros(cap, np.uint32)
    P = C.c_void_p
    checked = 0
    for r in range(len(scen["rounds"])):
        replay_round(gpu, scen, r)
        replay_round(orc, scen, r)
        if r < 2:
            continue
        t = liveness_tick(r, len(scen["rounds"][r]["phases"]))
        for _ in range(24):
            s, q = rng.sample(range(n), 2)
            # digest of q (the receiver) from the device bytes vs the oracle's row in dict order
            dq = parse_digest(em.digest(q, t), nid_index)
            row = orc.export_row(q)
            order = np.argsort(np.where(row["pos"] >= 0, row["pos"], 1 << 30))[: int((row["pos"] >= 0).sum())]
            want = [(int(j), int(row["hb"][j]), int(row["gc"][j]), int(row["mv"][j])) for j in order]
            assert dq == want, f"round {r}: digest of {q}"
            # delta s -> q vs the oracle's compute_partial_delta_respecting_mtu for that digest
            raw = em.delta(s, q, t)
            assert len(raw) <= mtu
            got = parse_delta(raw, nid_index)
            dg = np.array([x[0] for x in dq], np.int32)
            dgc = np.array([x[2] for x in dq], np.uint32)
            dmv = np.array([x[3] for x in dq], np.uint32)
            nn = orc.L.orc_kat_compute_delta(orc.h, s, len(dg), dg.ctypes.data_as(P), dgc.ctypes.data_as(P),
                                             dmv.ctypes.data_as(P), mtu, nd_node.ctypes.data_as(P),
                                             nd_from.ctypes.data_as(P), nd_nkv.ctypes.data_as(P),
                                             kv_ver.ctypes.data_as(P), cap)
            want, x = [], 0
            for i in range(nn):
                c = int(nd_nkv[i])
                want.append((int(nd_node[i]), int(nd_from[i]), [int(v) for v in kv_ver[x:x + c]]))
                x += c
            assert got == want, f"round {r}: delta {s}->{q}"
            checked += 1
    assert checked == 24 * (len(scen["rounds"]) - 2)
    assert gpu.check()["truncated"] > 0  # the MTU bound was exercised by the exchanges themselves
