"""The C oracle keeps all of its state per handle, so bench.py's CPU baseline may run one
handle per host thread: two handles replayed concurrently on two threads end bit-identical
to a third replayed alone (CPU only; the oracle is test infrastructure, see oracle/oracle.py)."""

import threading

from helpers import compare_exports, make_backend
from oracle import OracleSim

from aiocluster_amd.scenario import make_scenario, replay
from aiocluster_amd.workload import WorkloadSpec


def test_oracle_handles_are_independent_across_threads():
    spec = WorkloadSpec(n=96, k=8, fanout=3, seed=13, init="warm", write_frac=0.2, delete_frac=0.1,
                        down_frac=0.1, down_rounds=3)
    scen = make_scenario("thr96", spec, 12, {"mtu": 700, "window": 4, "tombstone_grace_s": 3,
                                             "initial_interval_s": 1.0, "phi_threshold": 3.0})
    alone = make_backend(OracleSim, scen)
    replay(alone, scen)
    want = alone.export()
    pair = [make_backend(OracleSim, scen) for _ in range(2)]
    errs = []

    def run(b):
        try:
            replay(b, scen)
        except Exception as e:  # surfaced below
            errs.append(e)

    ths = [threading.Thread(target=run, args=(b,)) for b in pair]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errs, errs
    for b in pair:
        assert compare_exports(b.export(), want) is None
    st = alone.stats()
    assert st["exchanges"] > 1000 and st["truncated"] > 0, st
    for b in (alone, *pair):
        b.close()


def test_threaded_phases_equal_sequential():
    """orc_run_phase_mt / orc_begin_round_mt / orc_liveness_mt (rows split over host threads, each with
    scratch of its own: the long whole-array GPU tests' checker) end every round bit-identical to the
    sequential oracle, statistics and Q9 events included."""
    spec = WorkloadSpec(n=80, k=6, fanout=3, seed=21, init="cold", write_frac=0.2, delete_frac=0.1,
                        down_frac=0.15, down_rounds=3)
    scen = make_scenario("mt80", spec, 14, {"mtu": 600, "window": 5, "tombstone_grace_s": 2,
                                             "initial_interval_s": 1.0, "phi_threshold": 2.0, "dead_grace_s": 4})
    seq = make_backend(OracleSim, scen)
    par = make_backend(OracleSim, scen, threads=5)
    from aiocluster_amd.scenario import replay_round

    for r in range(len(scen["rounds"])):
        replay_round(seq, scen, r)
        replay_round(par, scen, r)
        assert compare_exports(par.export(), seq.export()) is None, r
    assert par.stats() == seq.stats()
    assert par.q9_events == seq.q9_events
    assert seq.stats()["truncated"] > 0
    for b in (seq, par):
        b.close()


def test_threaded_phase_with_overlapping_pairs_runs_sequentially():
    """orc_run_phase_mt on a pair list that is NOT conflict-free (node 3 in two pairs) must not race: it falls back
    to the sequential order, so the result equals orc_exchange pair by pair."""
    spec = WorkloadSpec(n=64, k=6, fanout=3, seed=5, init="warm", write_frac=0.3, down_frac=0.0, down_rounds=1)
    scen = make_scenario("ovl64", spec, 3, {"mtu": 900})
    seq = make_backend(OracleSim, scen)
    par = make_backend(OracleSim, scen, threads=4)
    from aiocluster_amd.scenario import replay_round

    for r in range(len(scen["rounds"])):
        replay_round(seq, scen, r)
        replay_round(par, scen, r)
    t = seq.last_tick + 1
    pairs = [(3, 10), (11, 12), (3, 20), (21, 22), (20, 30), (40, 41)]
    seq.begin_round(t, [1] * 64)
    par.begin_round(t, [1] * 64)
    for a, b in pairs:
        seq.exchange(a, b, t + 1)
    par.run_phase(t + 1, pairs)
    assert compare_exports(par.export(), seq.export()) is None
    for b in (seq, par):
        b.close()
