"""The word tricks of k_sel_row16 (aiocluster_amd/csrc/gossip_sim.hip), restated in numpy and checked
exhaustively against the per-column rules they replace (k_sel_resolve16's loop: live = membership 1,
dead = membership bit 1, a column counts only inside the row and off the observer's own column).

* bit 0 of each of a word's 4 bytes -> 4 adjacent bits: (x * 0x204081) >> 21 & 0xF for x whose set bits are
  a subset of 0x01010101 (bytes 0..3 land on bits 21..24 from the 2^21, 2^14, 2^7, 1 terms; no other term
  reaches bits 21..24 and no two terms share a bit, so nothing carries);
* the pool and dead counts scanned together as count_pool | count_dead << 16: each lane's counts are at most 16,
  so a 64-lane inclusive scan of the packed word stays below 2^16 in its low half (no carry into the high one).
"""

import numpy as np

FD_MEMB = 3


def memb_live4(w):
    m = w & 0x03030303
    return m & ~(m >> 1) & 0x01010101


def memb_dead4(w):
    return (w >> 1) & 0x01010101


def gather4(x):
    return ((x * 0x204081) >> 21) & 0xF


def keep_mask(jq, ncol, js):
    keep = 0x01010101
    if jq + 4 > ncol:
        keep = 0 if jq >= ncol else (keep >> (8 * (jq + 4 - ncol)))
    if 0 <= js < 4:
        keep &= ~(0x01 << (8 * js)) & 0xFFFFFFFF
    return keep


def test_byte_bit_gather_matches_the_per_column_rules():
    rng = np.random.default_rng(5)
    words = rng.integers(0, 2**32, size=4096, dtype=np.uint64).astype(np.int64)
    # every membership pattern of the 4 bytes too (2 bits each)
    pats = np.array([sum(((p >> (2 * b)) & 3) << (8 * b) for b in range(4)) for p in range(256)], dtype=np.int64)
    for w in np.concatenate([words, pats, pats | 0xFCFCFCFC]):
        w = int(w)
        for jq, ncol, js in [(0, 64, -1), (60, 63, -1), (60, 61, -1), (64, 64, -1), (8, 64, 2), (0, 4, 0), (4, 8, 3)]:
            keep = keep_mask(jq, ncol, js)
            a = gather4(memb_live4(w) & keep)
            b = gather4(memb_dead4(w) & keep)
            ea = eb = 0
            for k in range(4):
                st = (w >> (8 * k)) & FD_MEMB
                valid = jq + k < ncol and k != js
                ea |= int(valid and st == 1) << k
                eb |= int(valid and st >= 2) << k
            assert (a, b) == (ea, eb), (hex(w), jq, ncol, js)


def test_packed_pool_dead_scan_has_no_carry():
    rng = np.random.default_rng(6)
    for _ in range(200):
        cp = rng.integers(0, 17, size=64)
        cd = rng.integers(0, 17, size=64)
        packed = np.cumsum(cp | (cd << 16))
        assert np.array_equal(packed & 0xFFFF, np.cumsum(cp))
        assert np.array_equal(packed >> 16, np.cumsum(cd))
    full = np.cumsum(np.full(64, 16 | (16 << 16)))  # the extreme: every lane's 16 columns in both sets
    assert full[-1] & 0xFFFF == 1024 and full[-1] >> 16 == 1024
