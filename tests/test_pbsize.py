"""Closed-form protobuf sizes vs the reference's generated classes' ByteSize() (CPU)."""

import json
import os

from aiocluster_amd import pbsize

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pbsize.json")


def test_pbsize_matches_reference_bytesize():
    cases = json.load(open(GOLDEN))["cases"]
    assert len(cases) >= 100
    for c in cases:
        name, gen, host, port, tls = c["nid"]
        nid = pbsize.nodeid_size(name, gen, host, port, tls)
        assert nid == c["nid_size"], c
        kvs = [pbsize.kv_size(k, v, ver, st) for k, v, ver, st in c["kvs"]]
        assert kvs == c["kv_sizes"], c
        nd = pbsize.nodedelta_size(nid, c["from"], c["gc"], kvs, c["mv"])
        assert nd == c["nd_size"], c
        assert pbsize.delta_size([nd, nd]) == c["delta_size"], c


def test_varint_boundaries():
    assert [pbsize.vlen(x) for x in (0, 127, 128, 16383, 16384, (1 << 21) - 1, 1 << 21)] == [1, 1, 2, 2, 3, 3, 4]
    assert pbsize.u_field(0) == 0 and pbsize.s_field(0) == 0
