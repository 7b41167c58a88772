"""Heartbeat-lag census of the headline workload (GPU): after each round, the largest lag R_j - hb[o][j]
of any view behind its owner's own heartbeat, the count of views at or above 64 / 128, and how they
concentrate: observer rows / owner columns holding any view at or above 64, and the up state of those rows.
Sizes the 8-bit heartbeat layout (GS_HB8) and its escape path.

    python tools/hb_lag.py [--nodes 65536] [--rounds 40] [--down-rounds 3] [--peer-select]
"""

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    from aiocluster_amd import driver
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.sim import GossipSim
    from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=40)
    ap.add_argument("--down-rounds", type=int, default=3)
    ap.add_argument("--partition", type=int, nargs=2, default=None, help="rounds [a, b) split into halves")
    ap.add_argument("--peer-select", action="store_true", help="rounds scheduled by the device's select_nodes_for_gossip")
    ap.add_argument("--every", type=int, default=1, help="census every this many rounds")
    a = ap.parse_args()
    n, K = a.nodes, 16
    cfg = dict(DEFAULT_CFG)
    kw = {}
    if a.partition:
        kw = dict(partition=tuple(a.partition))
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=0, init="warm", write_frac=0.05, down_frac=0.05,
                        down_rounds=a.down_rounds, **kw)
    sim = GossipSim(synthetic_node_ids(n), key_names(K), cfg, init="warm", tombstones=False, fd_ring=False,
                    hist_cap=16, initial_ops=driver.boot_ops(n, K))
    plans = driver.prepare(spec, a.rounds, torch, sim.device)
    sel = None
    if a.peer_select:
        from aiocluster_amd.peers import PeerSelector

        sel = PeerSelector(sim, fanout=3, seeds=list(range(0, n, max(1, n // 8))), seed=0)
    hb = sim.region("HB", torch.int16, (n, sim.np_))
    out = []
    for r in range(a.rounds):
        driver.run_round([sim], plans[r], group=None, sel=sel)
        if (r + 1) % a.every:
            continue
        R = sim.region("SELF_HB", torch.int32, (sim.np_,))[:n].to(torch.int64)
        mx, c64, c128 = 0, 0, 0
        rows64 = torch.zeros(n, dtype=torch.bool, device=sim.device)
        cols64 = torch.zeros(n, dtype=torch.bool, device=sim.device)
        for o0 in range(0, n, 4096):
            s = hb[o0:o0 + 4096, :n].to(torch.int64) & 0xFFFF
            lag = (R.unsqueeze(0) - s) & 0xFFFF
            mx = max(mx, int(lag.max().item()))
            big = lag >= 64
            c64 += int(big.sum().item())
            c128 += int((lag >= 128).sum().item())
            rows64[o0:o0 + 4096] = big.any(1)
            cols64 |= big.any(0)
        up = plans[r]["up"].to(torch.bool)
        rec = {"round": r, "max_lag": mx, "views_ge_64": c64, "views_ge_128": c128,
               "rows_with_ge_64": int(rows64.sum().item()), "of_them_down": int((rows64 & ~up).sum().item()),
               "cols_with_ge_64": int(cols64.sum().item()), "max_R": int(R.max().item()),
               "phases": len(plans[r]["phases"]) if sel is None else None}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    sim.check()
    sim.close()


if __name__ == "__main__":
    main()
