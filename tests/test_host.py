"""Host-side logic that needs no GPU (CPU): write batching, window packing, config, multi-rank aggregation."""

import os
import socket

import numpy as np
import pytest

from aiocluster_amd import _lib
from aiocluster_amd.scenario import DEFAULT_CFG
from aiocluster_amd.sim import make_config, split_owner_batches


def test_split_owner_batches_keeps_per_owner_order():
    ops = [(0, 1, "a"), (0, 2, "b"), (0, 1, "c"), (0, 1, "d"), (0, 3, "e"), (0, 2, "f")]
    batches = split_owner_batches(ops)
    for b in batches:
        owners = [op[1] for op in b]
        assert len(owners) == len(set(owners))
    flat = {}
    for b in batches:
        for op in b:
            flat.setdefault(op[1], []).append(op[2])
    assert flat == {1: ["a", "c", "d"], 2: ["b", "f"], 3: ["e"]}


def test_fd_window_decode():
    """GS_R_FD (sum | cnt << sum_bits) + GS_R_FD_LAST (tick mod 2^16) + GS_R_FD_STATE bits (window, old):
    the host decode restates the device's fd_get; exact while the last report is < 2^16 ticks old."""
    from aiocluster_amd.sim import FD_OLD, FD_OLD_AGE, FD_WIN, unpack_fd

    W = 1000
    sb = _lib.fd_sum_bits(W)
    assert sb == 21 and W * 640 < (1 << sb)
    rng = np.random.default_rng(0)
    t = 5_000_000
    last = t - rng.integers(0, 1 << 16, 100, dtype=np.int64)
    sm = rng.integers(0, 1 << sb, 100, dtype=np.uint64)
    cnt = rng.integers(0, 2 * W, 100, dtype=np.uint64)
    sc = (sm | (cnt << np.uint64(sb))).astype(np.uint32)
    st = np.full(100, FD_WIN | 1, np.uint8)
    st[:3] = 0  # no window
    st[3:6] |= FD_OLD
    l2, s2, c2 = unpack_fd(st, (last & 0xFFFF).astype(np.uint16), sc, t, sb)
    assert np.all(l2[:3] == _lib.GS_NONE)
    assert np.all(l2[3:6] == t - FD_OLD_AGE)
    assert np.array_equal(l2[6:], last[6:].astype(np.uint32))
    assert np.array_equal(s2, sm.astype(np.uint32)) and np.array_equal(c2, cnt.astype(np.uint32))


def test_make_config_ticks_and_rejects_fractional_ticks():
    c = make_config(100, 16, DEFAULT_CFG, 0, 32)
    assert c.max_interval_ticks == 640 and c.tombstone_grace_ticks == 7200 * 64
    assert c.dead_grace_ticks == 86400 * 64 and c.prior_weighted == 25.0
    bad = dict(DEFAULT_CFG, max_interval_s=0.01)
    with pytest.raises(ValueError):
        make_config(100, 16, bad, 0, 32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    ex, tm = bench.aggregate(1000 * (rank + 1), 2.0 + rank, dist, "cpu")
    q.put((rank, ex, tm))
    dist.destroy_process_group()


def test_multi_rank_aggregation_gloo():
    """bench.py's N>1 reduction (exchanges summed, time = max over ranks), world_size 2 on gloo."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
    assert [o[1:] for o in out] == [(3000.0, 3.0), (3000.0, 3.0)]
