"""BASELINE config 5 on one MI355X: 16,384 nodes, MTU-truncated deltas, deletes + tombstone GC,
and a network partition into halves that heals, with the failure detector's false-positive rate.

Workload (aiocluster_amd/workload.py, seeded): warm start, K = 16 keys, fanout 3, every round 5 %
of the nodes write one key and 1 % of those writes are deletes; tombstone grace = 10 rounds
(Config.marked_for_deletion_grace_period = 10 s at one round per second); mtu 65,507; rounds
[warm, warm + partition) split the cluster into halves (no exchange crosses), then it heals.

Per round it reports the failure detector's census (gs_fd_census: false-positive rate = pairs whose
target is up but in the observer's dead set / pairs whose target is up, observer != target) and
the round's counters (NodeDeltas, truncated NodeDeltas, tombstones collected), and at the end
whether the version matrix converged (every view's max_version = the owner's).

Usage: python tools/config5.py [--nodes 16384] [--warm 10] [--partition 30] [--heal 30] [--out f.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=16384)
    ap.add_argument("--keys", type=int, default=16)
    ap.add_argument("--fanout", type=int, default=3)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--warm", type=int, default=10)
    ap.add_argument("--partition", type=int, default=30)
    ap.add_argument("--heal", type=int, default=30)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    from aiocluster_amd.driver import boot_ops, prepare, run_round
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.sim import GossipSim
    from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

    n, K = args.nodes, args.keys
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rounds = args.warm + args.partition + args.heal
    cfg = dict(DEFAULT_CFG)
    cfg["tombstone_grace_s"] = 10
    spec = WorkloadSpec(n=n, k=K, fanout=args.fanout, seed=args.seed, init="warm", write_frac=0.05,
                        delete_frac=0.01, partition=(args.warm, args.warm + args.partition))
    boot = boot_ops(n, K)
    t0 = time.perf_counter()
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", device=str(dev), tombstones=True,
                    fd_ring=False, hist_cap=32, initial_ops=boot)
    plans = prepare(spec, rounds, torch, dev)
    torch.cuda.synchronize(dev)
    print(f"setup {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    per_round = []
    prev = sim.check()
    busy = 0.0
    exch = 0
    for r in range(rounds):
        rd = plans[r]
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        run_round([sim], rd)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - a
        busy += dt
        exch += rd["exchanges"]
        cen = sim.fd_census(rd["up"])
        c = sim.check()
        d = {k: c[k] - prev[k] for k in ("exchanges", "node_deltas", "truncated", "tomb_gc", "delta_bytes",
                                          "hb_reports")}
        prev = c
        stage = "warm" if r < args.warm else "partition" if r < args.warm + args.partition else "heal"
        fp = cen["up_dead"] / max(1, cen["up_pairs"])
        per_round.append({"round": r, "stage": stage, "ms": dt * 1e3, "fp_rate": fp, **cen, **d})
        print(f"r{r:3d} {stage:9s} {dt * 1e3:7.1f} ms  fp {fp:.4f}  nd {d['node_deltas']}  trunc {d['truncated']}"
              f"  tombgc {d['tomb_gc']}", file=sys.stderr, flush=True)
    # version-matrix convergence: every observer's max_version of every owner = the owner's own
    mv = sim.max_versions()[:, :n]
    own = torch.diagonal(mv).clone()
    lag_views = int((mv != own[None, :]).sum().item())
    part = [x for x in per_round if x["stage"] == "partition"]
    heal = [x for x in per_round if x["stage"] == "heal"]
    out = {
        "config": "BASELINE config 5",
        "workload": f"N={n} K={K} F={args.fanout} warm, 5% writes (1% deletes), tombstone grace 10 rounds, "
                    f"mtu 65507, partition into halves for rounds [{args.warm}, {args.warm + args.partition}) "
                    f"then heal for {args.heal} rounds",
        "exchanges_per_s": exch / busy,
        "exchanges": exch,
        "fp_rate_max_partition": max(x["fp_rate"] for x in part) if part else None,
        "fp_rate_end_of_partition": part[-1]["fp_rate"] if part else None,
        "fp_rate_end": per_round[-1]["fp_rate"],
        "first_heal_round_fp_zero": next((x["round"] for x in heal if x["up_dead"] == 0), None),
        "truncated_total": sum(x["truncated"] for x in per_round),
        "tomb_gc_total": sum(x["tomb_gc"] for x in per_round),
        "views_lagging_at_end": lag_views,
        "rounds": per_round,
    }
    s = json.dumps(out, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s)
    print(json.dumps({k: v for k, v in out.items() if k != "rounds"}))


if __name__ == "__main__":
    main()
