"""The C-ABI library builds for gfx950, loads, and exports every symbol the header declares (CPU).

No compute call is made here: the container has no GPU.
"""

import ctypes
import os
import re

import pytest

from aiocluster_amd import _lib


def header_functions():
    src = open(_lib.HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*(gs_\w+)\s*\(", src, re.M)))


def test_header_declares_what_the_binding_binds():
    assert header_functions() == sorted(_lib.EXPORTS)


def test_library_loads_and_exports_every_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    L = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(L, name), name
    lib = _lib.load()
    assert lib.gs_api_version() == _lib.API_VERSION


def test_create_validates_config_without_gpu():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.sim import make_config

    lib = _lib.load()
    h = ctypes.c_void_p()
    good = make_config(1000, 16, DEFAULT_CFG, 0, 32)
    assert lib.gs_create(ctypes.byref(good), ctypes.byref(h)) == 0
    nb = ctypes.c_uint64()
    assert lib.gs_region_bytes(h, _lib.REGION["HB"], ctypes.byref(nb)) == 0
    assert nb.value == 1000 * 1024 * 2
    assert lib.gs_region_bytes(h, _lib.REGION["POS"], ctypes.byref(nb)) == 0 and nb.value == 1000 * 1024 * 4
    # no tombstone GC: last_gc_version is 0 everywhere and not stored
    assert lib.gs_region_bytes(h, _lib.REGION["GC"], ctypes.byref(nb)) == 0 and nb.value == 0
    assert lib.gs_region_bytes(h, _lib.REGION["PEND"], ctypes.byref(nb)) == 0 and nb.value == 1000 * 1024 * 4  # 32 planes
    lib.gs_destroy(h)
    withgc = make_config(1000, 16, DEFAULT_CFG, _lib.GS_TOMBSTONES, 32)
    assert lib.gs_create(ctypes.byref(withgc), ctypes.byref(h)) == 0
    assert lib.gs_region_bytes(h, _lib.REGION["GC"], ctypes.byref(nb)) == 0 and nb.value == 1000 * 1024 * 4
    lib.gs_destroy(h)
    bad = make_config(1000, 65, DEFAULT_CFG, 0, 32)  # K > 64
    assert lib.gs_create(ctypes.byref(bad), ctypes.byref(h)) == -1


def test_window_layout_and_16_bit_tick_bounds():
    """Sampling windows: u32 sum|count + u16 last-report tick + state byte (+ u32 time of death); gs_create
    refuses configs under which a window silent for 2^15 ticks could still append an interval
    (max_interval >= 2^14 ticks) or still be alive (threshold x max(max_interval, prior) >= 2^15 ticks)."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.sim import make_config

    lib = _lib.load()
    h = ctypes.c_void_p()
    cfg = make_config(1000, 16, DEFAULT_CFG, _lib.GS_CANONICAL, 32)
    assert lib.gs_create(ctypes.byref(cfg), ctypes.byref(h)) == 0
    pairs = 1000 * 1024
    for name, per in (("FD", 4), ("FD_LAST", 2), ("FD_STATE", 1), ("FD_TOD", 4)):
        nb = ctypes.c_uint64()
        assert lib.gs_region_bytes(h, _lib.REGION[name], ctypes.byref(nb)) == 0 and nb.value == pairs * per, name
    nb = ctypes.c_uint64()
    assert lib.gs_region_bytes(h, _lib.REGION["LATEST"], ctypes.byref(nb)) == 0 and nb.value == 1000 * 16 * 4
    lib.gs_destroy(h)
    for over in ({"max_interval_s": 256.0}, {"phi_threshold": 200.0}, {"phi_threshold": 60.0, "max_interval_s": 9.0}):
        bad = make_config(1000, 16, dict(DEFAULT_CFG, **over), 0, 32)
        assert lib.gs_create(ctypes.byref(bad), ctypes.byref(h)) == -1, over
    ok = make_config(1000, 16, dict(DEFAULT_CFG, max_interval_s=255.0, phi_threshold=2.0, window=100), 0, 32)
    assert lib.gs_create(ctypes.byref(ok), ctypes.byref(h)) == 0
    lib.gs_destroy(h)


def test_sched_delay_rounding():
    from aiocluster_amd.sim import sched_delay_ticks

    assert sched_delay_ticks(86400.0) == 43200 * 64
    assert sched_delay_ticks(1 / 64) == 1  # 7812.5 us rounds half-even to 7812 -> 1 tick
    assert sched_delay_ticks(30.0) == 15 * 64


def test_slice_columns_and_region_sizes_without_gpu():
    """Owner-column slices (gs_config.n_shards/shard): the library and the host agree on the split."""
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    from aiocluster_amd.scenario import DEFAULT_CFG
    from aiocluster_amd.sim import make_config

    lib = _lib.load()
    n = 1000
    seen = []
    for g in range(3):
        c = make_config(n, 16, DEFAULT_CFG, _lib.GS_CANONICAL, 32)
        c.n_shards, c.shard = 3, g
        h = ctypes.c_void_p()
        assert lib.gs_create(ctypes.byref(c), ctypes.byref(h)) == 0
        lo, nc = ctypes.c_uint32(), ctypes.c_uint32()
        assert lib.gs_shard_columns(h, ctypes.byref(lo), ctypes.byref(nc)) == 0
        assert (lo.value, nc.value) == _lib.slice_columns(n, 3, g)
        seen.append((lo.value, nc.value))
        npad = (nc.value + 63) // 64 * 64
        nb = ctypes.c_uint64()
        assert lib.gs_region_bytes(h, _lib.REGION["HB"], ctypes.byref(nb)) == 0 and nb.value == n * npad * 2
        assert lib.gs_region_bytes(h, _lib.REGION["HIST"], ctypes.byref(nb)) == 0 and nb.value == nc.value * 32 * 16 * 8
        assert lib.gs_region_bytes(h, _lib.REGION["SLICE_BITS"], ctypes.byref(nb)) == 0
        assert nb.value == (n // 2) * 2 * (npad // 32) * 4
        lib.gs_destroy(h)
    assert seen == [(0, 384), (384, 384), (768, 232)]
    # slices need the canonical layout, and none may be empty
    c = make_config(n, 16, DEFAULT_CFG, 0, 32)
    c.n_shards, c.shard = 2, 0
    h = ctypes.c_void_p()
    assert lib.gs_create(ctypes.byref(c), ctypes.byref(h)) == -1
    c = make_config(100, 16, DEFAULT_CFG, _lib.GS_CANONICAL, 32)
    c.n_shards, c.shard = 3, 0
    assert lib.gs_create(ctypes.byref(c), ctypes.byref(h)) == -1
    with pytest.raises(ValueError):
        _lib.slice_columns(100, 3, 0)


def test_region_enum_matches_binding():
    src = open(_lib.HEADER).read()
    body = re.search(r"enum gs_region \{(.*?)GS_NUM_REGIONS", src, re.S).group(1)
    names = re.findall(r"^\s*GS_R_(\w+)", body, re.M)
    assert names == _lib.REGIONS
