"""Host protocol of owner-column sharding (aiocluster_amd/shard.py), on CPU.

The device kernels are replaced by a toy slice whose packing follows the same
rules as ``k_pack_slice`` (greedy whole-fit prefix, then first-fit) over a list
of candidate sizes per (exchange, direction); the protocol must make the
slices' union equal one sequential pass over all slices in order.  Runs both
in-process (LocalComm) and as two gloo ranks (DistComm).
"""

import os

import numpy as np
import pytest
import torch

from aiocluster_amd._lib import GS_CHAIN_CAP, GS_CHAIN_DEVICE
from aiocluster_amd.shard import CHAIN_PENDING, TOT_BYTES_MASK, LocalComm, run_sliced_phase

MTU = 100


def seq_pack(cands, S=0, tail=False, stop=False, mtu=MTU):
    """Sequential packing of (id, size) candidates; returns (sent ids, S, tail, stop)."""
    sent = []
    for cid, size in cands:
        if stop:
            break
        if not tail:
            if S + size <= mtu:
                S += size
                sent.append(cid)
            else:
                tail = True
        if tail and cid not in sent and size <= mtu - S:
            S += size
            sent.append(cid)
        if S >= mtu:
            stop = True
    return sent, S, tail, stop


def enc(S, tail, stop):
    return S | (int(tail) << 32) | (int(stop) << 33)


def dec(v):
    return v & 0xFFFFFFFF, bool((v >> 32) & 1), bool((v >> 33) & 1)


class ToySlice:
    """has_records = True: the compacted chain (gs_phase_overflow + gs_phase_chain); False: the fused
    protocol (every slot's chain state gathered per step)."""

    def __init__(self, g, cands, has_records=True):
        self.g = g
        self.cands = cands  # cands[e][dir] = [(id, size), ...] of this slice
        self.sent = {}
        self.has_records = has_records

    def phase_overflow(self, tot_all, chain, list_buf, chainc, read=True):
        tot = (tot_all & TOT_BYTES_MASK).sum(0).reshape(-1)
        idx = (tot > MTU).nonzero().flatten()
        list_buf[: len(idx)] = idx.to(list_buf.dtype)
        chainc[: len(idx)] = chain.reshape(-1)[idx]
        chainc[len(idx)] = int((chain.reshape(-1)[idx] == CHAIN_PENDING).sum())  # pending entry
        list_buf[-1] = len(idx)  # the count entry (GS_OVERFLOW_LIST_LEN's last word)
        return len(idx)

    def phase_chain(self, t, ini, res, step, list_buf, count, chain_all, chain, chainc, tot_all):
        """k_chain_step: resume from the nearest finished predecessor f, skipping the pending slices between
        that cannot add a candidate (delta complete, or their smallest candidate above the budget left)."""
        flat = chain.view(-1)
        if count == GS_CHAIN_DEVICE:  # the count from the list (gs_phase_overflow's entry); nothing above the cap
            count = int(list_buf[-1])
            if count > GS_CHAIN_CAP:
                return
        for i in range(count):
            slot = int(list_buf[i])
            e, d = slot // 2, slot % 2
            if self.g == 0 or int(flat[slot]) != CHAIN_PENDING:
                continue
            f = self.g - 1
            while f >= 0 and int(chain_all[f, i]) == CHAIN_PENDING:
                f -= 1
            if f < 0:
                continue
            S, tail, stop = dec(int(chain_all[f, i]))
            ok = all(stop or S >= MTU or (tail and ((int(tot_all[h, e, d]) & (1 << 64) - 1) >> 40) > MTU - S)
                     for h in range(f + 1, self.g))
            if not ok:
                continue
            sent, S, tail, stop = seq_pack(self.cands[e][d], S, tail, stop)
            self.sent[(e, d)] = sent
            flat[slot] = chainc[i] = enc(S, tail, stop)
        chainc[count] = sum(int(flat[int(list_buf[i])]) == CHAIN_PENDING for i in range(count))

    def phase_pending(self, n, list_buf, count, chain_all):
        """gs_phase_pending: (pending slots summed over the slices, or -1 above the device cap; the count)"""
        if count == GS_CHAIN_DEVICE:
            count = int(list_buf[-1])
            if count > GS_CHAIN_CAP:
                return -1, count
        return int(chain_all[:, count].sum()), count

    def phase_count(self, t, ini, res):
        """slice totals: bytes | the smallest candidate << 40 (0xFFFFFF: none), as gs_phase_count"""
        n = int(ini.numel())

        def word(c):  # u64 as the device writes it, viewed as int64
            w = sum(s for _, s in c) | (min((s for _, s in c), default=0xFFFFFF) << 40)
            return w - (1 << 64) if w >= 1 << 63 else w

        return torch.tensor([[word(self.cands[e][d]) for d in range(2)] for e in range(n)], dtype=torch.int64)

    def phase_pack(self, t, ini, res, step, tot_all, chain_all, chain):
        n = int(ini.numel())
        for e in range(n):
            for d in range(2):
                if step == 0:
                    P = int((tot_all[: self.g, e, d] & TOT_BYTES_MASK).sum()) if self.g else 0
                    if P > MTU:
                        chain[e, d] = CHAIN_PENDING
                        continue
                    st = (P, False, False)
                else:
                    if self.g == 0 or int(chain[e, d]) != CHAIN_PENDING:
                        continue
                    prev = int(chain_all[self.g - 1, e, d])
                    if prev == CHAIN_PENDING:
                        continue
                    st = dec(prev)
                sent, S, tail, stop = seq_pack(self.cands[e][d], *st)
                self.sent[(e, d)] = sent
                chain[e, d] = enc(S, tail, stop)
        return chain


def make_cands(rng, G, n, per=6):
    """cands[g][e][d]: candidate (id, size) lists; ids increase with slice (dict order)."""
    out = [[[[] for _ in range(2)] for _ in range(n)] for _ in range(G)]
    for e in range(n):
        for d in range(2):
            cid = 0
            for g in range(G):
                for _ in range(rng.integers(0, per)):
                    out[g][e][d].append((cid, int(rng.integers(5, 45))))
                    cid += 1
    return out


def check(slices, cands, G, n):
    for e in range(n):
        for d in range(2):
            allc = [c for g in range(G) for c in cands[g][e][d]]
            want = seq_pack(allc)[0]
            got = [c for s in slices for c in s.sent.get((e, d), [])]
            assert got == want, (e, d, got, want)


@pytest.mark.parametrize("G,records", [(2, True), (3, True), (5, True), (8, True), (3, False)])
def test_chain_protocol_in_process(G, records):
    rng = np.random.default_rng(G)
    n = 40
    cands = make_cands(rng, G, n)
    slices = [ToySlice(g, cands[g], records) for g in range(G)]
    ini = torch.zeros(n, dtype=torch.int32)
    steps = run_sliced_phase(slices, LocalComm(G), MTU, 0, ini, ini)
    # these inputs overflow the MTU somewhere; the compacted chain stops once nothing is pending
    assert (2 <= steps <= G) if records else steps == G
    check(slices, cands, G, n)


@pytest.mark.parametrize("big", [45, 80])
def test_chain_skips_slices_that_cannot_fit(big):
    """Eight slices whose owners are all larger than any budget left after the MTU is crossed (big = 80:
    every pending slice is skipped, one chain step), or a mix (big = 45 with small owners in some slices:
    those cannot be skipped and the chain takes more steps) -- either way the union equals one sequential
    pass."""
    G, n = 8, 12
    rng = np.random.default_rng(big)
    cands = [[[[] for _ in range(2)] for _ in range(n)] for _ in range(G)]
    for e in range(n):
        for d in range(2):
            cid = 0
            for g in range(G):
                for _ in range(3):
                    small = big == 45 and g % 3 == 2 and rng.random() < 0.5
                    cands[g][e][d].append((cid, int(rng.integers(2, 6)) if small else big))
                    cid += 1
    slices = [ToySlice(g, cands[g]) for g in range(G)]
    ini = torch.zeros(n, dtype=torch.int32)
    steps = run_sliced_phase(slices, LocalComm(G), MTU, 0, ini, ini)
    if big == 80:
        assert steps == 2, steps
    check(slices, cands, G, n)


def test_no_chain_when_everything_fits():
    G, n = 3, 10
    cands = [[[[(g, 5)], [(g, 6)]] for _ in range(n)] for g in range(G)]
    slices = [ToySlice(g, cands[g]) for g in range(G)]
    ini = torch.zeros(n, dtype=torch.int32)
    assert run_sliced_phase(slices, LocalComm(G), MTU, 0, ini, ini) == 1
    check(slices, cands, G, n)


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist

    from aiocluster_amd.shard import DistComm

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(7 + world)
        n = 30
        cands = make_cands(rng, world, n)
        s = ToySlice(rank, cands[rank])
        ini = torch.zeros(n, dtype=torch.int32)
        steps = run_sliced_phase([s], DistComm(), MTU, 0, ini, ini)
        counters = DistComm().sum_counters([{k: rank + 1 for k in __import__("aiocluster_amd._lib").
                                             _lib.COUNTER_FIELDS}])
        q.put((rank, steps, {k: v for k, v in s.sent.items()}, (counters["exchanges"], counters["pack_steps_max"])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_chain_protocol_gloo(world):
    """The compacted, skipping chain over torch.distributed (gloo): every rank reads the same gathered
    pending counts, so all stop at the same step, and the ranks' union equals one sequential pass."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    rng = np.random.default_rng(7 + world)
    n = 30
    cands = make_cands(rng, world, n)
    slices = [ToySlice(g, cands[g]) for g in range(world)]
    steps0 = res[0][1]
    for (rank, steps, sent, ex), s in zip(res, slices):
        assert steps == steps0 and 2 <= steps <= world  # the same stop on every rank
        assert ex[0] == world * (world + 1) // 2  # 1 + 2 + ... summed over the ranks
        assert ex[1] == world  # a maximum counter: the largest over the ranks, not the sum
        s.sent = sent
    check(slices, cands, world, n)
