"""CPU restatement of the device peer selection and phase schedule (gs_select_peers /
gs_schedule_phases in aiocluster_amd/csrc/gossip_sim.hip).

TEST INFRASTRUCTURE: the checker for the HIP path; only tests/ import it.

Selection follows select_nodes_for_gossip (aiocluster/server.py:656-717) as _gossip_multiple
(server.py:441-469) feeds it: peers = known nodes but self, live / dead = the failure detector's sets
(failure_detector.py:63-67).  ``rng.sample(live or peers, min(F, n))`` is Floyd's algorithm over
ranks in column order; ``select_dead_node_to_gossip_with`` (656-667) draws with probability
dead / (live + 1); ``select_seed_node_to_gossip_with`` (670-682) under the condition of 710-716.
The draws are Philox4x32-10 (key = run seed, counter = (round, node, slot)) instead of
random.Random: the reference's choice depends on set iteration order, so parity is
exact against this restatement of the same draws, and distributional against the reference.
"""

from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF
SEL_DEAD, SEL_SEED = 14, 15


def philox4x32(c, k0, k1):
    c = list(c)
    for _ in range(10):
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c[3] ^ k1) & M32, p0 & M32]
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c


def sel_rand(seed, r, node, slot):
    return philox4x32([r & M32, node, slot, 0], seed & M32, (seed >> 32) & M32)


def below(x, n):
    return (x * n) >> 32


def unit53(a, b):
    return float(((a << 21) ^ (b >> 11)) & ((1 << 53) - 1)) / 9007199254740992.0


def select_peers(live, tod, known, up, fanout, seeds, seed, r):
    """targets[N][F+2] (-1 = none) from per-observer arrays live[o][j] (0/1), tod[o][j] (>= 0 dead),
    known[o][j] (in the observer's dict)."""
    n = live.shape[0]
    F = fanout
    out = np.full((n, F + 2), -1, dtype=np.int64)
    for o in range(n):
        if not up[o]:
            continue
        kn = known[o].astype(bool).copy()
        kn[o] = False
        lv = kn & (live[o] == 1)
        dd = kn & (tod[o] >= 0)
        L, D, P = int(lv.sum()), int(dd.sum()), int(kn.sum())
        pool = np.flatnonzero(lv if L else kn)
        npool = L if L else P
        k = min(F, npool)
        ranks = []
        for i in range(k):
            t = npool - k + i
            c = sel_rand(seed, r, o, i)
            x = below(c[0], t + 1)
            if x in ranks:
                x = t
            ranks.append(x)
        for i, x in enumerate(ranks):
            out[o, i] = pool[x]
        if D:
            c = sel_rand(seed, r, o, SEL_DEAD)
            if D / (L + 1) > unit53(c[0], c[1]):
                out[o, F] = np.flatnonzero(dd)[below(c[2], D)]
        sl = [s for s in seeds if s != o]
        S = len(sl)
        has_seed = any(out[o, i] in sl for i in range(F) if out[o, i] >= 0)
        if S and (not has_seed or L < S):
            c = sel_rand(seed, r, o, SEL_SEED)
            ps = 1.0 if L + D == 0 else S / (L + D)
            if L == 0 or unit53(c[0], c[1]) <= ps:
                out[o, F + 1] = sl[below(c[2], S)]
    return out


def fmix32(h):
    h &= M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def luby_key(seed, r, e, p, it):
    inner = fmix32(((r * 0x9E3779B9) + (p * 0x632BE5AB) + it) & M32)
    h = fmix32(e ^ fmix32((seed & M32) ^ inner))
    return (h << 32) | e


def schedule_phases(targets, up, seed, r, iters, max_phases=16):
    """Phase of every exchange slot e = o * (F + 2) + s (-1 = not scheduled after max_phases)."""
    n, W = targets.shape
    E = n * W
    flat = targets.reshape(-1)
    eph = np.full(E, -1, dtype=np.int64)
    busy = np.zeros(n, dtype=np.int64)
    cand = [e for e in range(E) if flat[e] >= 0 and up[flat[e]]]
    for p in range(max_phases):
        for it in range(iters):
            best = {}
            act = []
            for e in cand:
                if eph[e] >= 0:
                    continue
                a, b = e // W, int(flat[e])
                if (busy[a] >> p) & 1 or (busy[b] >> p) & 1:
                    continue
                k = luby_key(seed, r, e, p, it)
                act.append((e, a, b, k))
                best[a] = min(best.get(a, 1 << 64), k)
                best[b] = min(best.get(b, 1 << 64), k)
            for e, a, b, k in act:
                if best[a] == k and best[b] == k:
                    eph[e] = p
                    busy[a] |= 1 << p
                    busy[b] |= 1 << p
    return eph
