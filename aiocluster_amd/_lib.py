"""ctypes binding of ``libgossip_sim.so`` (C ABI: ``include/gossip_sim.h``).

The shared library is built in-tree by ``__graft_entry__.build()`` (hipcc,
``--offload-arch=gfx950``).  There is no fallback: if the library is missing
or fails to load, every entry point of the package raises.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
LIB_DIR = os.path.join(PKG, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libgossip_sim.so")
SRC = os.path.join(PKG, "csrc", "gossip_sim.hip")
HEADER = os.path.join(REPO, "include", "gossip_sim.h")

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared"]

GS_CANONICAL = 1
GS_TOMBSTONES = 2
GS_FD_RING = 4
GS_NO_HELD = 8
GS_HB8 = 16  # 8-bit heartbeat views (include/gossip_sim.h)
GS_MV8 = 32  # 8-bit max_version views
GS_SLICED = 64  # the sliced phase path with one slice (a world-1 run of the multi-GPU code)
GS_NONE = 0xFFFFFFFF
GS_E_INVALID = -1
GS_MV_INEXACT = 0x8000
TICK_US = 15_625


def slice_columns(n: int, shards: int, shard: int) -> tuple[int, int]:
    """Owner columns ``(col_lo, n_cols)`` of slice ``shard`` of ``shards`` (gs_config.n_shards)."""
    if shards <= 1:
        return 0, n
    blk = (-(-n // shards) + 63) // 64 * 64
    if (shards - 1) * blk >= n:
        raise ValueError(f"{shards} slices of {blk} columns leave a slice of a {n}-node cluster empty")
    lo = shard * blk
    return lo, min(blk, n - lo)


GS_CHAIN_DEVICE = 0xFFFFFFFF  # gs_phase_chain: the count stays on the device
GS_CHAIN_CAP = 1024  # ... for at most this many overflowing slots


def overflow_list_len(n: int) -> int:
    """u32 words of gs_phase_overflow's list for a phase of ``n`` exchanges (GS_OVERFLOW_LIST_LEN)."""
    return 2 * n + (2 * n + 1023) // 1024 + 1


def fd_sum_bits(window: int) -> int:
    """Bits of the packed window's interval sum (include/gossip_sim.h, GS_R_FD)."""
    cnt_bits = 1
    while (1 << cnt_bits) <= 2 * window:
        cnt_bits += 1
    return 32 - cnt_bits

REGIONS = [
    "HB", "MV", "GC", "HELD", "FD", "FD_STATE", "TS", "RING", "POS", "ORD", "ROW",
    "LAST_W", "HIST", "HIST_VID", "NID_SIZE", "KEY_LEN", "STAMP", "COUNTERS", "SLICE_BITS", "PEND", "PEND_STAMP", "LATEST",
    "SELF_HB", "CAND", "CAND_N", "FD_TOD", "FD_LAST", "SLOT_STAT", "RING_SLOT", "SELF_MV", "SELF_PK", "VLOG",
    "P1FLAGS", "ESC16", "ESC_SLOT", "ESC_OWNER", "ESC_REQ",
]
REGION = {n: i for i, n in enumerate(REGIONS)}

ERRORS = {-1: "GS_E_INVALID", -2: "GS_E_UNBOUND", -3: "GS_E_HIP", -4: "GS_E_DEVICE", -5: "GS_E_UNSUPPORTED"}

COUNTER_FIELDS = [
    "exchanges", "hb_reports", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "alg_bytes", "hb_writes",
    "candidates", "live_pairs", "tomb_gc", "err_fd_overflow", "err_hist_full", "err_bad_index", "err_conflict",
    "err_fd_gc", "err_insert", "fd_gc", "q9", "pack_bytes", "err_holes", "err_hb_lag", "plane_flushes",
    "fd_saturated", "lite_slots", "lag_sweeps", "lite_bytes", "live_bytes", "hb_escapes", "hb_releases",
    "pack_groups_max", "pack_steps_max",  # maxima (gs_read_counters takes the largest; sum_counters too)
    "heavy_slots",
]

# Every symbol include/gossip_sim.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "gs_create", "gs_destroy", "gs_last_error", "gs_api_version", "gs_region_bytes", "gs_bind", "gs_set_stream",
    "gs_boot", "gs_warm", "gs_owner_writes", "gs_begin_round", "gs_run_phase", "gs_liveness", "gs_phi_row",
    "gs_read_counters", "gs_reset_counters", "gs_sync", "gs_shard_columns", "gs_phase_count", "gs_phase_pack", "gs_materialize_held", "gs_fd_census",
    "gs_select_peers", "gs_schedule_phases", "gs_set_events", "gs_emit_scratch_bytes", "gs_emit_digest", "gs_emit_delta",
    "gs_check_heartbeat_lag", "gs_stream_copy", "gs_stream_read", "gs_stream_write", "gs_set_timing", "gs_kernel_times",
    "gs_phase_overflow", "gs_phase_chain", "gs_phase_pending", "gs_comm_id", "gs_comm_init", "gs_run_phase_group", "gs_read_rows",
    "gs_latest_tick", "gs_flush_reports", "gs_set_ring_rows", "gs_mark",
]

API_VERSION = 20
MAX_PHASES = 64  # GS_MAX_PHASES
MAX_SCHED_PHASES = 65536  # GS_MAX_SCHED_PHASES


def sched_scratch_bytes(n: int, fanout: int, max_phases: int) -> int:
    """GS_SCHED_SCRATCH_BYTES: gs_schedule_phases' device scratch."""
    return 4 * n * (fanout + 2) + 12 * max_phases + 32 + 24 * n


class GsConfig(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32),
        ("n_keys", C.c_uint32),
        ("hist_cap", C.c_uint32),
        ("mtu", C.c_uint32),
        ("flags", C.c_uint32),
        ("window", C.c_uint32),
        ("max_interval_ticks", C.c_uint32),
        ("tombstone_grace_ticks", C.c_uint32),
        ("dead_grace_ticks", C.c_uint32),
        ("sched_delay_ticks", C.c_uint32),
        ("phi_threshold", C.c_double),
        ("prior_weighted", C.c_double),
        ("n_shards", C.c_uint32),
        ("shard", C.c_uint32),
        ("ring_rows", C.c_uint32),
        ("esc_cols", C.c_uint32),
    ]


class GsCounters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in COUNTER_FIELDS] + [("reserved", C.c_uint64 * (40 - len(COUNTER_FIELDS)))]


CENSUS_FIELDS = ["up_pairs", "up_dead", "up_live", "down_pairs", "down_live"]


KT_KINDS = ["pass1", "pack", "liveness", "count", "lite"]  # GS_KT_PASS1, GS_KT_PACK, GS_KT_LIVENESS, GS_KT_COUNT, GS_KT_LITE
KT_SLOTS = 8  # GS_KT_KINDS


class GsKtimes(C.Structure):
    _fields_ = [("ms", C.c_double * KT_SLOTS), ("launches", C.c_uint64 * KT_SLOTS)]


class GsCensus(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in CENSUS_FIELDS]


class GsWire(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("node_ids", "node_id_off", "keys", "key_off", "values", "value_off")]


class GsError(RuntimeError):
    pass


def source_hash() -> str:
    """SHA-256 of the HIP source, the header and the compile flags: what the built library is stamped with."""
    import hashlib

    h = hashlib.sha256(" ".join(HIPCC_FLAGS).encode())
    for f in (SRC, HEADER):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the HIP library for gfx950 in-tree (cross-compiles without a GPU).  Rebuilds whenever the
    sources' hash differs from the one stamped next to the library (LIB_PATH + ".srchash")."""
    os.makedirs(LIB_DIR, exist_ok=True)
    stamp = LIB_PATH + ".srchash"
    want = source_hash()
    have = open(stamp).read().strip() if os.path.exists(stamp) else None
    if force or not os.path.exists(LIB_PATH) or have != want:
        tmp = LIB_PATH + ".tmp"
        cmd = ["hipcc", *HIPCC_FLAGS, "-o", tmp, SRC, "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(tmp, LIB_PATH)
        with open(stamp, "w") as fh:
            fh.write(want + "\n")
    return LIB_PATH


_LIB = None


def load():
    """Load (never silently replace) the HIP library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # GS_LIB: an in-tree build variant (tuning sweeps); still the HIP library, never a fallback
    path = os.environ.get("GS_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise GsError(f"{path} missing: run __graft_entry__.build() (hipcc, gfx950)")
    L = C.CDLL(path)
    P, u32, i32, u64 = C.c_void_p, C.c_uint32, C.c_int32, C.c_uint64
    sig = {
        "gs_api_version": (C.c_int, []),
        "gs_create": (C.c_int, [C.POINTER(GsConfig), C.POINTER(P)]),
        "gs_destroy": (None, [P]),
        "gs_last_error": (C.c_char_p, [P]),
        "gs_region_bytes": (C.c_int, [P, C.c_int, C.POINTER(u64)]),
        "gs_bind": (C.c_int, [P, C.c_int, P]),
        "gs_set_stream": (C.c_int, [P, P]),
        "gs_boot": (C.c_int, [P, P, P]),
        "gs_warm": (C.c_int, [P]),
        "gs_owner_writes": (C.c_int, [P, P, u32, u32]),
        "gs_begin_round": (C.c_int, [P, P, u32]),
        "gs_run_phase": (C.c_int, [P, P, P, u32, u32]),
        "gs_liveness": (C.c_int, [P, P, u32]),
        "gs_phi_row": (C.c_int, [P, u32, u32, P]),
        "gs_read_counters": (C.c_int, [P, C.POINTER(GsCounters)]),
        "gs_reset_counters": (C.c_int, [P]),
        "gs_set_timing": (C.c_int, [P, C.c_int]),
        "gs_phase_overflow": (C.c_int, [P, u32, P, P, P, P, C.POINTER(u32)]),
        "gs_phase_chain": (C.c_int, [P, P, P, u32, u32, u32, P, u32, P, P, P, P]),
        "gs_phase_pending": (C.c_int, [P, u32, P, u32, P, C.POINTER(u64), C.POINTER(u32)]),
        "gs_comm_id": (C.c_int, [P]),
        "gs_comm_init": (C.c_int, [P, P, u32, u32]),
        "gs_run_phase_group": (C.c_int, [P, u32, P, P, u32, u32]),
        "gs_read_rows": (C.c_int, [P, C.c_int, u32, u32, P, u64, C.POINTER(u64)]),
        "gs_latest_tick": (C.c_int, [P, C.POINTER(u32)]),
        "gs_flush_reports": (C.c_int, [P, u32]),
        "gs_set_ring_rows": (C.c_int, [P, P, u32]),
        "gs_kernel_times": (C.c_int, [P, C.POINTER(GsKtimes)]),
        "gs_sync": (C.c_int, [P]),
        "gs_shard_columns": (C.c_int, [P, C.POINTER(u32), C.POINTER(u32)]),
        "gs_phase_count": (C.c_int, [P, P, P, u32, u32, P]),
        "gs_phase_pack": (C.c_int, [P, P, P, u32, u32, u32, P, P, P]),
        "gs_materialize_held": (C.c_int, [P, u32, u32]),
        "gs_fd_census": (C.c_int, [P, P, C.POINTER(GsCensus)]),
        "gs_set_events": (C.c_int, [P, P, u32, P]),
        "gs_select_peers": (C.c_int, [P, P, u32, P, u32, C.c_uint64, u32, P, P]),
        "gs_schedule_phases": (C.c_int, [P, P, u32, P, C.c_uint64, u32, u32, u32, P, P, P, C.POINTER(u32),
                                         C.POINTER(u32)]),
        "gs_check_heartbeat_lag": (C.c_int, [P]),
        "gs_stream_copy": (C.c_int, [P, P, u64, P]),
        "gs_stream_read": (C.c_int, [P, u64, u32, P, P]),
        "gs_stream_write": (C.c_int, [P, u64, u32, P]),
        "gs_mark": (C.c_int, [u32, P]),
        "gs_emit_scratch_bytes": (C.c_int, [P, C.POINTER(u64)]),
        "gs_emit_digest": (C.c_int, [P, C.POINTER(GsWire), u32, u32, P, u64, C.POINTER(u64), P]),
        "gs_emit_delta": (C.c_int, [P, C.POINTER(GsWire), u32, u32, u32, P, u64, C.POINTER(u64), P]),
    }
    missing = []
    for name, (res, args) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            if not os.environ.get("GS_LIB"):
                raise GsError(f"{path} lacks {name}: rebuild it (__graft_entry__.build())")
            missing.append(name)  # an older A/B build named by GS_LIB: that entry point is absent
            continue
        f.restype = res
        f.argtypes = args
    if missing:
        import sys

        print(f"[aiocluster_amd] GS_LIB={path} lacks {', '.join(missing)} (older A/B build): calls to them raise",
              file=sys.stderr, flush=True)
    L.gs_missing = frozenset(missing)
    del i32
    _LIB = L
    return L
