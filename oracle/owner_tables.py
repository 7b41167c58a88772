"""Owner write tables restated on the host from the workload's write stream.

TEST INFRASTRUCTURE: the checker for the device's per-owner key logs (GS_R_LAST_W, GS_R_HIST,
GS_R_HIST_VID), which ``rowcheck.RowOracle`` copies into the oracle.  Checking them here against the
write stream the workload generated means a device error in the owner history cannot be inherited by the
full-size row checks unnoticed.

Semantics restated (``aiocluster/state.py:124-180``, ``NodeState.set / delete / set_with_ttl /
delete_after_ttl`` on the owner's own view; ``k_owner_writes`` in gossip_sim.hip follows the same rules):
every effective write gets version = the owner's max_version + 1; a set of the same value with the same
status is a no-op (140-141, 146-151); a delete of an absent key is a no-op (163-164, 175-176); a delete
clears the value (171) and marks the key DELETED; delete_after_ttl keeps the value and marks it
DELETE_AFTER_TTL, as set_with_ttl does.  Entry meta = KeyValueUpdatePb size | status << 16 | value bytes
<< 18 (include/gossip_sim.h, GS_R_HIST).
"""

from __future__ import annotations

import numpy as np

SET, DELETE, SET_WITH_TTL, DELETE_AFTER_TTL = 0, 1, 2, 3


def _vlen(x: int) -> int:
    n = 1
    while x >= 0x80:
        x >>= 7
        n += 1
    return n


def _sfield(n: int) -> int:
    return 0 if n == 0 else 1 + _vlen(n) + n


def _ufield(x: int) -> int:
    return 0 if x == 0 else 1 + _vlen(x)


def owner_tables(n_owners: int, key_len: list[int], hist_cap: int, batches, col_lo: int = 0, n_cols: int | None = None):
    """Replay ``batches`` -- an iterable of uint32/int arrays [m, 5] (owner, key, op, value_id, value_len), in
    call order, each with distinct owners -- and return (last_w [NC][K] u8, hist_ver [NC][C][K] u32,
    hist_meta [NC][C][K] u32, hist_vid [NC][C][K] u32) for owners [col_lo, col_lo + n_cols)."""
    K = len(key_len)
    nc = n_owners - col_lo if n_cols is None else n_cols
    last_w = np.zeros((nc, K), np.int64)
    ver = np.zeros((nc, hist_cap, K), np.uint32)
    meta = np.zeros((nc, hist_cap, K), np.uint32)
    vid = np.zeros((nc, hist_cap, K), np.uint32)
    mv = np.zeros(nc, np.int64)
    for ops in batches:
        ops = np.asarray(ops).astype(np.int64)
        if len(ops) == 0:
            continue
        sel = (ops[:, 0] >= col_lo) & (ops[:, 0] < col_lo + nc)
        for j_g, k, op, v_id, v_len in ops[sel].tolist():
            j = j_g - col_lo
            w = int(last_w[j, k])
            if op in (SET, SET_WITH_TTL):
                st = 0 if op == SET else 2
                if w and vid[j, w, k] == v_id and ((meta[j, w, k] >> 16) & 3) == st:
                    continue
                new_vid, new_vl = v_id, v_len
            else:
                if not w:
                    continue
                st = 1 if op == DELETE else 2
                new_vid = 0 if op == DELETE else int(vid[j, w, k])
                new_vl = 0 if op == DELETE else int(meta[j, w, k]) >> 18
            nw = w + 1
            if nw >= hist_cap:
                raise ValueError(f"owner {j_g} key {k}: more than hist_cap - 1 = {hist_cap - 1} writes")
            v = int(mv[j]) + 1
            mv[j] = v
            kvlen = _sfield(key_len[k]) + _sfield(new_vl) + _ufield(v) + _ufield(st)
            ver[j, nw, k] = v
            meta[j, nw, k] = kvlen | (st << 16) | (new_vl << 18)
            vid[j, nw, k] = new_vid
            last_w[j, k] = nw
    return last_w.astype(np.uint8), ver, meta, vid


def plan_batches(k: int, n: int, plans, boot=None):
    """The write batches of ``aiocluster_amd.driver.prepare`` plans (boot batches first), as host arrays."""
    out = list(boot or [])
    for rd in plans:
        if rd["nops"]:
            out.append(rd["ops"].cpu().numpy().view(np.uint32)[:, :5])
    return out


def check_owner_tables(sim, batches) -> str | None:
    """Compare the device's owner tables of ``sim`` (its owner columns) with the host restatement."""
    torch = sim.torch
    nc, K, KP, Cc = sim.ncol, sim.k, sim.kp, sim.hist_cap
    key_len = [len(x.encode()) for x in sim.keys]
    want = owner_tables(sim.n, key_len, Cc, batches, sim.col_lo, nc)
    lw = sim.region("LAST_W", torch.uint8, (nc, KP))[:, :K].cpu().numpy()
    hist = sim.region("HIST", torch.int64, (nc, Cc, K)).cpu().numpy().view(np.uint64)
    hvid = sim.region("HIST_VID", torch.int32, (nc, Cc, K)).cpu().numpy().view(np.uint32)
    got = (lw, (hist & np.uint64(0xFFFFFFFF)).astype(np.uint32), (hist >> np.uint64(32)).astype(np.uint32), hvid)
    valid = np.arange(Cc)[None, :, None] <= want[0].astype(np.int64)[:, None, :]  # entries 1..last_w are defined
    for name, g, w in zip(("LAST_W", "HIST version", "HIST meta", "HIST_VID"), got, want):
        if name != "LAST_W":
            g, w = np.where(valid, g, 0), np.where(valid, w, 0)
        ne = np.argwhere(g != w)
        if len(ne):
            idx = tuple(int(x) for x in ne[0])
            return f"{name}{list(idx)}: device {g[idx]} host {w[idx]} ({len(ne)} mismatches)"
    return None
