"""Generate golden fixtures from the REAL reference -- build container only.

TEST INFRASTRUCTURE (see ``oracle/refharness.py``).  Writes, under
``tests/golden/``:

* ``pbsize.json``   -- ``ByteSize()`` of random ``NodeIdPb`` / ``KeyValueUpdatePb``
  / ``NodeDeltaPb`` / ``DeltaPb`` built with the reference's generated classes
  (``aiocluster/protos/messages_pb2.py``), pinning ``aiocluster_amd/pbsize.py``
  and the device/oracle size formulas;
* ``scen_<name>.json.gz`` -- a scenario (input) plus the reference's state after
  every round (small N: full canonical state; larger N: SHA-256 per round and
  the full final state).

Run:  python oracle/gen_golden.py [names...]
"""

from __future__ import annotations

import gzip
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from aiocluster_amd.scenario import (  # noqa: E402
    export_digest,
    initial_by_owner,
    make_scenario,
    replay,
    scenario_node_ids,
    state_hash,
)
from aiocluster_amd.workload import WorkloadSpec  # noqa: E402
from refharness import RefSim, import_reference  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")

# name -> (spec, rounds, cfg overrides, full per-round states?)
SCENARIOS = {
    # config 1: examples/simple.py, 3 in-process nodes, 16 keys/node, 50 seeded rounds
    "simple3": (
        WorkloadSpec(n=3, k=16, fanout=2, seed=1, init="cold", write_frac=0.34, delete_frac=0.2, ttl_frac=0.2,
                     node_style="simple"),
        50,
        {"tombstone_grace_s": 4},
        True,
    ),
    # MTU truncation (Q1, Q4), deletes + short tombstone grace (Q2, Q3), FD ring eviction
    # (window 5), max_interval filter, up/down churn
    "trunc8": (
        WorkloadSpec(n=8, k=8, fanout=2, seed=2, init="cold", write_frac=0.5, delete_frac=0.25, ttl_frac=0.1,
                     down_frac=0.3, down_rounds=4),
        40,
        {"mtu": 300, "tombstone_grace_s": 3, "window": 5, "max_interval_s": 1.0, "initial_interval_s": 1.0,
         "phi_threshold": 3.0},
        True,
    ),
    # scheduled-for-deletion (dead >= grace/2 leaves digests and deltas), warm start
    "sched16": (
        WorkloadSpec(n=16, k=4, fanout=2, seed=3, init="warm", write_frac=0.25, down_frac=0.3, down_rounds=15),
        30,
        {"dead_grace_s": 30.0, "phi_threshold": 3.0, "initial_interval_s": 1.0, "mtu": 900},
        True,
    ),
    # FD garbage collection, remove_node and re-discovery (incl. Q9 KeyError)
    "fdgc12": (
        WorkloadSpec(n=12, k=4, fanout=2, seed=4, init="cold", write_frac=0.25, down_frac=0.3, down_rounds=12),
        45,
        {"dead_grace_s": 8.0, "phi_threshold": 2.0, "initial_interval_s": 1.0},
        True,
    ),
    # FD garbage collection that raises KeyError for windowless dead targets
    "q9x10": (
        WorkloadSpec(n=10, k=2, fanout=1, seed=4, init="cold", write_frac=0.2, down_frac=0.5, down_rounds=10),
        40,
        {"dead_grace_s": 4.0, "phi_threshold": 1.5, "initial_interval_s": 1.0},
        True,
    ),
    # cold start at moderate N with truncation and deletes (hashes per round)
    "cold64": (
        WorkloadSpec(n=64, k=16, fanout=3, seed=5, init="cold", write_frac=0.05, delete_frac=0.1, ttl_frac=0.05),
        24,
        {"mtu": 4000, "tombstone_grace_s": 6},
        False,
    ),
    # warm start, 5% writes + 5% down churn (the bench workload shape, small N)
    "warm128": (
        WorkloadSpec(n=128, k=16, fanout=3, seed=6, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3),
        16,
        {"mtu": 6000},
        False,
    ),
    # SURVEY 8(c) tier "N=64/256": cold start at 256 nodes with deletes, TTL writes, tombstone GC,
    # MTU truncation and churn (hashes per round, full final state)
    "cold256": (
        WorkloadSpec(n=256, k=8, fanout=3, seed=7, init="cold", write_frac=0.08, delete_frac=0.1, ttl_frac=0.05,
                     down_frac=0.05, down_rounds=3),
        18,
        {"mtu": 3000, "tombstone_grace_s": 5},
        False,
    ),
    # BASELINE config 2: 1,024 nodes x 64 keys, fanout 3, cold start to version convergence (the
    # workload of tests/test_gpu_parity.py::test_config2_cold_1024x64_converges_bit_exact): per-round
    # digests of the whole export (scenario.export_digest) and the final max_version matrix
    "config2": (
        WorkloadSpec(n=1024, k=64, fanout=3, seed=2, init="cold", write_frac=0.0),
        24,
        {},
        "digest",
    ),
}


def gen_pbsize(n_cases: int = 400) -> dict:
    R = import_reference()
    pb = R.pb
    rng = random.Random(1234)

    def rstr(maxlen):
        return "".join(rng.choice("abcdefghijklmnopqrstuvwxyz0123456789.-_é") for _ in range(rng.randint(0, maxlen)))

    def rint():
        return rng.choice([0, 1, 127, 128, 16383, 16384, rng.randint(0, 1 << 20), rng.randint(0, 1 << 40)])

    cases = []
    for _ in range(n_cases):
        nid = [rstr(20), rint(), rstr(16), rng.choice([0, 1, 7000, 65535]), rstr(6) or None]
        kvs = [[rstr(12) or "k", rstr(40), rint(), rng.choice([0, 1, 2])] for _ in range(rng.randint(0, 5))]
        frm, gc, mv = rint(), rint(), rint()
        nid_pb = pb.NodeIdPb(name=nid[0], generation_id=nid[1],
                             gossip_advertise_addr=pb.AddressPb(host=nid[2], port=nid[3]), tls_name=nid[4] or "")
        kv_pbs = [pb.KeyValueUpdatePb(key=k, value=v, version=ver, status=st) for k, v, ver, st in kvs]
        nd = pb.NodeDeltaPb(node_id=nid_pb, from_version_excluded=frm, last_gc_version=gc, key_values=kv_pbs,
                            max_version=mv)
        cases.append({
            "nid": nid, "kvs": kvs, "from": frm, "gc": gc, "mv": mv,
            "nid_size": nid_pb.ByteSize(), "kv_sizes": [k.ByteSize() for k in kv_pbs],
            "nd_size": nd.ByteSize(), "delta_size": pb.DeltaPb(node_deltas=[nd, nd]).ByteSize(),
        })
    return {"cases": cases}


def gen_scenario(name: str) -> dict:
    spec, rounds, cfg, full = SCENARIOS[name]
    scen = make_scenario(name, spec, rounds, cfg)
    sim = RefSim(scenario_node_ids(scen), scen["keys"], scen["config"], scen["init"], initial_by_owner(scen))
    states, hashes = [], []
    t0 = time.time()
    if full == "digest":
        # The reference's MTU packing re-serialises the growing delta per kv (state.py:395), so a
        # cold 1,024 x 64 round takes ~1.5 h here: the fixture is rewritten after every round and
        # pins the rounds completed so far ("rounds_done"), with the max_version matrix after the last.
        digests = []

        def on_digest(r):
            ex = sim.export()
            digests.append(export_digest(ex))
            scen["expect"] = {
                "digests": digests,
                "rounds_done": r + 1,
                "final_mv": ex["mv"].tolist(),
                "final_holes": int(((ex["kv_version"] == 0) & (ex["pos"] >= 0)[:, :, None]).sum()),
                "q9": sim.q9_events,
                "generator": "oracle/gen_golden.py via oracle/refharness.py (reference @ /root/reference)",
            }
            with gzip.open(os.path.join(GOLDEN, f"scen_{name}.json.gz"), "wt") as f:
                json.dump(scen, f, separators=(",", ":"))
            print(f"{name}: round {r} done, {time.time() - t0:.0f}s (fixture written)", flush=True)

        replay(sim, scen, on_round=on_digest)
        print(f"{name}: {rounds} rounds, {time.time() - t0:.1f}s")
        return scen

    def on_round(r):
        st = sim.state()
        hashes.append(state_hash(st))
        if full:
            states.append(st)

    replay(sim, scen, on_round=on_round)
    scen["expect"] = {
        "hashes": hashes,
        "states": states if full else None,
        "final": sim.state(),
        "q9": sim.q9_events,
        "generator": "oracle/gen_golden.py via oracle/refharness.py (reference @ /root/reference)",
    }
    print(f"{name}: {rounds} rounds, {sum(len(p) for rd in scen['rounds'] for p in rd['phases'])} exchanges, "
          f"q9={len(sim.q9_events)}, {time.time() - t0:.1f}s")
    return scen


def main(argv):
    os.makedirs(GOLDEN, exist_ok=True)
    names = argv or ["pbsize", *SCENARIOS]
    for name in names:
        if name == "pbsize":
            with open(os.path.join(GOLDEN, "pbsize.json"), "w") as f:
                json.dump(gen_pbsize(), f, separators=(",", ":"))
            print("pbsize: ok")
            continue
        scen = gen_scenario(name)
        with gzip.open(os.path.join(GOLDEN, f"scen_{name}.json.gz"), "wt") as f:
            json.dump(scen, f, separators=(",", ":"))


if __name__ == "__main__":
    main(sys.argv[1:])
