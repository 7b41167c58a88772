"""Hook events of the REAL reference (Cluster._emit_key_change / _emit_node_join / _emit_node_leave,
aiocluster/server.py:217-257, 611-616) per round of golden scenarios, for the event-stream parity tests.
Build container only (imports /root/reference via refharness).

Output: tests/golden/events_<name>.json.gz = per round the list of
[observer, owner, key | kind << 8, old version (0 = None), new version, tick], kind 0/1/2 =
key change / node join / node leave, in the order the reference's hooks were called.  One
canonicalisation: _update_node_liveness emits its joins, then its leaves, by iterating Python sets
(server.py:611-614), whose order follows the hash-seeded NodeId hashes and so differs from run to
run; within each observer's join block and leave block the fixture orders by node index.
"""

from __future__ import annotations

import gzip
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from refharness import RefSim, dt_tick  # noqa: E402

from aiocluster_amd.scenario import initial_by_owner, replay_round, scenario_node_ids  # noqa: E402

NAMES = ["trunc8", "fdgc12", "simple3", "cold64"]


def canonical_liveness(events):
    """Each maximal run of join / leave events (one or more consecutive _update_node_liveness calls)
    ordered by (observer, kind, node); key-change events keep their positions."""
    out, run = [], []
    for e in events:
        if e[2] >> 8:
            run.append(e)
            continue
        out += sorted(run, key=lambda x: (x[0], x[2] >> 8, x[1]))
        run = []
        out.append(e)
    return out + sorted(run, key=lambda x: (x[0], x[2] >> 8, x[1]))


def capture(name):
    from helpers import load_scenario

    scen = load_scenario(name)
    ref = RefSim(scenario_node_ids(scen), scen["keys"], scen["config"], scen["init"], initial_by_owner(scen))
    events = []
    kidx = {k: i for i, k in enumerate(scen["keys"])}

    def hook(o):
        c = ref.clusters[o]

        def key_change(node_id, key, old_vv, new_vv):
            events.append([o, ref.idx[node_id], kidx[key], 0 if old_vv is None else old_vv.version, new_vv.version,
                           dt_tick(ref.now)])

        def join(node_id):
            events.append([o, ref.idx[node_id], 1 << 8, 0, 0, dt_tick(ref.now)])

        def leave(node_id):
            events.append([o, ref.idx[node_id], 2 << 8, 0, 0, dt_tick(ref.now)])

        c._emit_key_change = key_change
        c._emit_node_join = join
        c._emit_node_leave = leave

    for o in range(len(ref.clusters)):
        hook(o)
    per_round = []
    for r in range(len(scen["rounds"])):
        replay_round(ref, scen, r)
        per_round.append(canonical_liveness(events))
        events.clear()
    return per_round


def main():
    for name in NAMES:
        pr = capture(name)
        path = os.path.join(REPO, "tests", "golden", f"events_{name}.json.gz")
        with gzip.open(path, "wt") as f:
            json.dump(pr, f, separators=(",", ":"))
        print(name, sum(len(x) for x in pr), "events", os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
