"""Host side of the multi-GPU bench's parity evidence (bench.sliced_parity, oracle/rowcheck.check_sliced_phase_rows),
on CPU: the slices' row copies join into whole-cluster rows, and the object collectives work over gloo with two
ranks (the GPU part runs in tests/test_gpu_shard.py)."""

import os
import socket

import numpy as np
import torch.multiprocessing as mp
from rowcheck import host_rows, join_host_rows


class _Slice:
    def __init__(self, lo, nc):
        self.col_lo, self.ncol = lo, nc


def _whole(rows, n, C, K, seed=0):
    rng = np.random.default_rng(seed)
    NP = (n + 63) // 64 * 64
    g = {"rows": np.arange(rows), "ROW": rng.integers(0, 9, (rows, 4)).astype(np.uint32)}
    for k in ("HB", "MV", "GC", "FD_STATE", "FD_LAST", "FD_SUM", "FD_CNT"):
        g[k] = rng.integers(0, 1 << 20, (rows, NP)).astype(np.uint32)
    g["HELD"] = rng.integers(0, C, (rows, NP, 16)).astype(np.uint8)
    for k in ("HIST_VER", "HIST_META", "HIST_VID"):
        g[k] = rng.integers(0, 1 << 30, (n, C, K)).astype(np.uint32)
    return g


def test_slices_join_into_whole_cluster_rows():
    n, C, K, rows = 200, 6, 5, 3
    whole = _whole(rows, n, C, K)
    blk = 64
    parts = []
    for lo in range(0, n, blk):
        nc = min(blk, n - lo)
        s = _Slice(lo, nc)
        NPs = (nc + 63) // 64 * 64
        g = {"rows": whole["rows"], "ROW": whole["ROW"]}
        for k in ("HB", "MV", "GC", "FD_STATE", "FD_LAST", "FD_SUM", "FD_CNT"):
            x = np.zeros((rows, NPs), np.uint32)
            x[:, :nc] = whole[k][:, lo:lo + nc]
            g[k] = x
        h = np.zeros((rows, NPs, 16), np.uint8)
        h[:, :nc] = whole["HELD"][:, lo:lo + nc]
        g["HELD"] = h
        for k in ("HIST_VER", "HIST_META", "HIST_VID"):
            g[k] = whole[k][lo:lo + nc]
        parts.append(host_rows(s, g, cmax=4))
    joined = join_host_rows(parts[::-1])  # any order: joined by column
    for k in ("HB", "MV", "GC", "FD_STATE", "FD_LAST", "FD_SUM", "FD_CNT"):
        assert np.array_equal(joined[k], whole[k][:, :n]), k
    assert np.array_equal(joined["HELD"], whole["HELD"][:, :n])
    for k in ("HIST_VER", "HIST_META", "HIST_VID"):
        assert np.array_equal(joined[k], whole[k][:, :4]), k  # cut to the first cmax write ordinals
    assert np.array_equal(joined["ROW"], whole["ROW"])


def test_join_refuses_slices_that_do_not_tile():
    import pytest

    g = _whole(2, 128, 3, 2)
    a = host_rows(_Slice(0, 64), {k: (v[:64] if k.startswith("HIST_") else v) for k, v in g.items()})
    with pytest.raises(ValueError, match="tile"):
        join_host_rows([a, dict(a, col_lo=100)])


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bench import ObjComm

        c = ObjComm(dist)
        got = c.gather([("slice", rank, np.full(3, rank))])
        m = c.allmax(10 * rank + 3)
        ok = c.bcast(rank == 0 and got is not None and len(got) == world)
        q.put((rank, None if got is None else [(x[0], x[1], x[2].tolist()) for x in got], m, ok))
    finally:
        dist.destroy_process_group()


def test_object_collectives_over_gloo_two_ranks():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=120) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][1] == [("slice", 0, [0, 0, 0]), ("slice", 1, [1, 1, 1])]
    assert res[1][1] is None
    assert res[0][2] == res[1][2] == 13
    assert res[0][3] is True and res[1][3] is True
