"""Host half of the wire-format emitter against the REAL reference's bytes (no GPU).

``tests/golden/wire_*.json.gz`` (``oracle/gen_wire_fixture.py``) hold the reference's
``_make_syn_msg().SerializeToString()`` for pairs of nodes of golden scenarios.  The host encodes
the NodeIdPb table the device copies into every NodeDigest / NodeDelta, and the PacketPb framing
around the device's DigestPb / DeltaPb; both must reproduce the reference's bytes exactly.
"""

import gzip
import json
import os

import pytest
from helpers import GOLDEN, load_scenario
from pbread import fields

from aiocluster_amd.pbsize import nodeid_size
from aiocluster_amd.scenario import scenario_node_ids
from aiocluster_amd.wire import frame, node_id_pb, packet, varint

NAMES = ["trunc8", "sched16", "fdgc12", "simple3", "cold64"]


def load_wire(name):
    with gzip.open(os.path.join(GOLDEN, f"wire_{name}.json.gz"), "rt") as f:
        return json.load(f)


@pytest.mark.parametrize("name", NAMES)
def test_syn_framing_and_node_ids_match_reference(name):
    scen = load_scenario(name)
    ids = scenario_node_ids(scen)
    nid = [node_id_pb(x) for x in ids]
    for x, b in zip(ids, nid):  # the device packer prices NodeIds with pbsize (GS_R_NID_SIZE)
        assert len(b) == nodeid_size(x.name, x.generation_id, *x.gossip_advertise_addr, x.tls_name)
    w = load_wire(name)
    assert w["cases"]
    for r, s, q, syn_hex, _ in w["cases"]:
        syn = bytes.fromhex(syn_hex)
        top = fields(syn)
        assert top[0] == (1, 2, b"default-cluster")
        assert [f[0] for f in top] == [1, 2]
        synpb = fields(top[1][2])
        assert [f[0] for f in synpb] == [2]
        digest = synpb[0][2]
        assert packet("default-cluster", "syn", digest=digest) == syn
        for num, wt, nd in fields(digest):
            assert (num, wt) == (1, 2)
            sub = fields(nd)
            assert sub[0][0] == 1 and sub[0][2] in nid  # NodeIdPb bytes of a known node
            assert [f[0] for f in sub] == sorted(f[0] for f in sub)  # field-number order
            assert all(f[2] != 0 for f in sub[1:])  # proto3: zero scalars are omitted


def test_delta_fixture_structure():
    """DeltaPb bodies of the fixture: NodeDeltaPb fields in number order, max_version always present
    (proto3 ``optional``), kvs in increasing version order (state.py:373-374)."""
    seen_trunc = False
    for name in NAMES:
        for _, _, _, _, dhex in load_wire(name)["cases"]:
            for num, _, nd in fields(bytes.fromhex(dhex)):
                assert num == 1
                sub = fields(nd)
                nums = [f[0] for f in sub]
                assert nums == sorted(nums) and nums[-1] == 5
                vers = [dict((g[0], g[2]) for g in fields(f[2])).get(3, 0) for f in sub if f[0] == 4]
                assert vers == sorted(vers)
                seen_trunc |= len(vers) == 0
    assert not seen_trunc  # a NodeDelta is only sent with at least one kv (state.py:403)


def test_packet_kinds_and_frame():
    d, e = b"\x0a\x01x", b"\x0a\x01y"
    assert packet("c", "synack", digest=d, delta=e) == b"\x0a\x01c" + b"\x1a" + varint(10) + b"\x12\x03" + d + b"\x1a\x03" + e
    assert packet("", "ack", delta=b"") == b"\x22\x02\x1a\x00"
    assert frame(b"abc") == b"\x00\x00\x00\x03abc"
