"""Shared test helpers: load golden scenarios, replay a backend, diff canonical states."""

import gzip
import json
import os

from rowcheck import compare_exports  # noqa: F401  (re-exported for the tests)

from aiocluster_amd.scenario import initial_by_owner, replay, scenario_node_ids, state_hash

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCENARIOS = ["simple3", "trunc8", "sched16", "fdgc12", "q9x10", "cold64", "warm128", "cold256"]


def load_scenario(name):
    with gzip.open(os.path.join(GOLDEN, f"scen_{name}.json.gz"), "rt") as f:
        return json.load(f)


def first_diff(a, b, path="state"):
    """Human-readable location of the first difference between two canonical states."""
    if type(a) is not type(b):
        return f"{path}: {a!r} != {b!r}"
    if isinstance(a, dict):
        for k in a:
            if k not in b:
                return f"{path}.{k} missing"
            d = first_diff(a[k], b[k], f"{path}.{k}")
            if d:
                return d
        return None
    if isinstance(a, list):
        if len(a) != len(b):
            return f"{path}: len {len(a)} != {len(b)}: {a[:6]!r} vs {b[:6]!r}"
        for i, (x, y) in enumerate(zip(a, b)):
            d = first_diff(x, y, f"{path}[{i}]")
            if d:
                return d
        return None
    return None if a == b else f"{path}: {a!r} != {b!r}"


def replay_and_compare(backend, scen, expect_states=None, expect_hashes=None, rounds=None, state_fn=None):
    """Replay; return (round, diff) of the first mismatch against the expectations, or None."""
    state_fn = state_fn or backend.state
    bad = []

    def on_round(r):
        if bad:
            return
        st = state_fn()
        if expect_hashes is not None and state_hash(st) != expect_hashes[r]:
            diff = first_diff(st, expect_states[r]) if expect_states else "hash mismatch"
            bad.append((r, diff))
        elif expect_states is not None and expect_hashes is None and st != expect_states[r]:
            bad.append((r, first_diff(st, expect_states[r])))

    replay(backend, scen, on_round=on_round, rounds=rounds)
    return bad[0] if bad else None


def make_backend(cls, scen, **kw):
    return cls(scenario_node_ids(scen), scen["keys"], scen["config"], scen["init"], initial_by_owner(scen), **kw)
