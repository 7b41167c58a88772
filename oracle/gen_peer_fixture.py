"""Frequencies of the REAL reference's select_nodes_for_gossip (aiocluster/server.py:656-717) over
many seeded draws, for the distributional test of the device peer selection
(tests/test_peer_select.py).  Build container only (imports /root/reference via refharness).

Output: tests/golden/peer_select_freq.json -- per case (live L, dead D, peers P, seeds S, whether
the seeds are live, fanout F): P(dead probe), P(seed probe), mean sampled count, and the per-peer
inclusion frequency spread (uniformity).
"""

from __future__ import annotations

import json
import os
import random

from refharness import import_reference

CASES = [
    # L, D, P(extra known but neither live nor dead), S, seeds_live, F
    (20, 5, 0, 2, True, 3),
    (20, 5, 0, 2, False, 3),
    (3, 10, 0, 1, False, 3),
    (0, 4, 6, 2, False, 3),
    (2, 0, 0, 3, True, 3),
    (50, 50, 0, 5, False, 2),
    (8, 1, 0, 1, True, 4),
]
TRIALS = 20000


def main():
    import_reference()
    from aiocluster.server import select_nodes_for_gossip

    out = []
    for L, D, X, S, seeds_live, F in CASES:
        live = {("10.0.0.1", 7000 + i) for i in range(L)}
        dead = {("10.0.1.1", 7000 + i) for i in range(D)}
        other = {("10.0.2.1", 7000 + i) for i in range(X)}
        peers = live | dead | other
        pool = sorted(live) if seeds_live else sorted(dead | other) or sorted(live)
        seeds = set(pool[:S])
        rng = random.Random(12345)
        dead_hits = seed_hits = total = 0
        inc = {}
        for _ in range(TRIALS):
            nodes, dn, sn = select_nodes_for_gossip(peers, live, dead, seeds, rng=rng, gossip_count=F)
            total += len(nodes)
            dead_hits += dn is not None
            seed_hits += sn is not None
            for x in nodes:
                inc[x] = inc.get(x, 0) + 1
        vals = list(inc.values())
        out.append({"L": L, "D": D, "X": X, "S": S, "seeds_live": seeds_live, "F": F, "trials": TRIALS,
                    "p_dead": dead_hits / TRIALS, "p_seed": seed_hits / TRIALS, "mean_sampled": total / TRIALS,
                    "incl_min": min(vals) / TRIALS, "incl_max": max(vals) / TRIALS, "distinct": len(vals)})
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                        "peer_select_freq.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
