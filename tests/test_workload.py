"""Deterministic workload/schedule generator (CPU)."""

import numpy as np

from aiocluster_amd.workload import Workload, WorkloadSpec, permutation_phases


def test_phases_are_matchings_and_cover_every_initiation():
    rng = np.random.default_rng(7)
    for n in (2, 3, 5, 64, 1000):
        perm = rng.permutation(n).astype(np.int32)
        phases = permutation_phases(perm)
        seen = []
        for a, b in phases:
            nodes = np.concatenate([a, b])
            assert len(np.unique(nodes)) == len(nodes)  # each node at most once per phase
            assert np.all(perm[a] == b)
            seen.extend(a.tolist())
        fixed = np.flatnonzero(perm == np.arange(n))
        assert sorted(seen + fixed.tolist()) == list(range(n))


def test_workload_is_deterministic():
    spec = WorkloadSpec(n=200, k=8, seed=3, down_frac=0.1, write_frac=0.1, delete_frac=0.2)
    a, b = Workload(spec), Workload(spec)
    for _ in range(5):
        ra, rb = a.next_round(), b.next_round()
        assert np.array_equal(ra.writes, rb.writes) and ra.values == rb.values
        assert np.array_equal(ra.up, rb.up)
        for (x1, y1), (x2, y2) in zip(ra.phases, rb.phases):
            assert np.array_equal(x1, x2) and np.array_equal(y1, y2)
        # down nodes neither initiate nor answer; writers are up and distinct
        for x, y in ra.phases:
            assert ra.up[x].all() and ra.up[y].all()
        assert len(np.unique(ra.writes[:, 0])) == len(ra.writes)
        assert ra.up[ra.writes[:, 0]].all()
