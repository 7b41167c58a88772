"""Wire-format emitter: real aiocluster protobuf bytes from the device state.

A simulated cluster can hand its messages to real ``Cluster`` nodes (``server.py:502-521`` frames
them as a 4-byte size + ``PacketPb``): the DigestPb and DeltaPb bodies are produced on the GPU
by ``gs_emit_digest`` / ``gs_emit_delta`` (``include/gossip_sim.h``); this module owns the string
tables those kernels read and the few bytes of ``PacketPb`` framing around them
(``messages.proto:3-26``), the part the reference's ``_make_syn_msg`` / ``_handle_syn_msg`` /
``_handle_synac_msg`` (``server.py:327-370``) build around the digest and delta.

Encodings follow protobuf's wire format as upb writes it: fields in field-number order, proto3
scalars and strings only when non-zero / non-empty, message fields whenever set (the reference
always sets ``SynPb.digest``, ``SynAckPb.digest/delta`` and ``AckPb.delta``, even when empty).
Pinned byte for byte to the reference's own ``SerializeToString`` output
(``tests/golden/wire_*.json.gz``, ``oracle/gen_wire_fixture.py``).
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .entities import NodeId


def varint(x: int) -> bytes:
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _len_field(tag: int, body: bytes) -> bytes:
    return bytes([tag]) + varint(len(body)) + body


def _str_field(tag: int, s: str) -> bytes:
    b = s.encode()
    return _len_field(tag, b) if b else b""


def _u_field(tag: int, x: int) -> bytes:
    return bytes([tag]) + varint(x) if x else b""


def node_id_pb(nid: NodeId) -> bytes:
    """``NodeId.to_pb().SerializeToString()`` (``entities.py:62-72``, ``messages.proto:39-44``):
    name, generation_id, gossip_advertise_addr {host, port} (always set), tls_name ("" when None)."""
    host, port = nid.gossip_advertise_addr
    addr = _str_field(0x0A, host) + _u_field(0x10, int(port))
    return (_str_field(0x0A, nid.name) + _u_field(0x10, int(nid.generation_id)) + _len_field(0x1A, addr)
            + _str_field(0x22, nid.tls_name or ""))


def packet(cluster_id: str, kind: str, digest: bytes | None = None, delta: bytes | None = None) -> bytes:
    """``PacketPb`` (``messages.proto:18-26``) around DigestPb / DeltaPb bodies: kind ``syn``
    (SynPb {digest = 2}), ``synack`` (SynAckPb {digest = 2, delta = 3}) or ``ack`` (AckPb {delta = 3})."""
    head = _str_field(0x0A, cluster_id)
    if kind == "syn":
        return head + _len_field(0x12, _len_field(0x12, digest))
    if kind == "synack":
        return head + _len_field(0x1A, _len_field(0x12, digest) + _len_field(0x1A, delta))
    if kind == "ack":
        return head + _len_field(0x22, _len_field(0x1A, delta))
    raise ValueError(kind)


def frame(pkt: bytes) -> bytes:
    """``add_msg_size``: the 4-byte big-endian size prefix of a TCP frame (``server.py:516-521``)."""
    return len(pkt).to_bytes(4, "big") + pkt


class WireEmitter:
    """Emits the wire bytes of a ``GossipSim``'s nodes from the device state.

    The node-id and key tables are uploaded once; the value table is re-uploaded when values were
    interned since the last call (values are host strings interned by ``GossipSim.intern``)."""

    def __init__(self, sim, cluster_id: str = "default-cluster", cap: int = 1 << 26):
        torch = sim.torch
        self.sim, self.torch, self.cluster_id = sim, torch, cluster_id
        if sim.node_ids is None:
            raise _lib.GsError("the wire emitter needs the NodeIds of the simulated nodes")
        dev = sim.device
        nid = [node_id_pb(x) for x in sim.node_ids]
        self._nid, self._nid_off = self._blob(nid, np.uint32)
        self._key, self._key_off = self._blob([k.encode() for k in sim.keys], np.uint32)
        self._nvals = -1
        self._val = self._val_off = None
        nb = C.c_uint64()
        sim._chk(sim.L.gs_emit_scratch_bytes(sim.h, C.byref(nb)), "gs_emit_scratch_bytes")
        self._scratch = torch.empty(int(nb.value), dtype=torch.uint8, device=dev)
        self._out = torch.empty(cap, dtype=torch.uint8, device=dev)
        self._w = _lib.GsWire()

    def _blob(self, items: list[bytes], off_dtype):
        torch = self.torch
        off = np.zeros(len(items) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(b) for b in items])
        data = np.frombuffer(b"".join(items) or b"\0", dtype=np.uint8).copy()
        d = torch.from_numpy(data).to(self.sim.device)
        o = torch.from_numpy(off.astype(off_dtype).view(np.int32 if off_dtype == np.uint32 else np.int64))
        return d, o.to(self.sim.device)

    def _tables(self):
        if self._nvals != len(self.sim.values):
            self._val, self._val_off = self._blob([v.encode() for v in self.sim.values], np.uint64)
            self._nvals = len(self.sim.values)
        w = self._w
        w.node_ids, w.node_id_off = self._nid.data_ptr(), self._nid_off.data_ptr()
        w.keys, w.key_off = self._key.data_ptr(), self._key_off.data_ptr()
        w.values, w.value_off = self._val.data_ptr(), self._val_off.data_ptr()
        return w

    def _emit(self, fn, name, *args) -> bytes:
        sim = self.sim
        sim._flush()
        n = C.c_uint64()
        w = self._tables()
        rc = fn(sim.h, C.byref(w), *args, C.c_void_p(self._out.data_ptr()), self._out.numel(), C.byref(n),
                C.c_void_p(self._scratch.data_ptr()))
        if rc == _lib.GS_E_INVALID and n.value > self._out.numel():  # grow the buffer and retry once
            self._out = self.torch.empty(int(n.value), dtype=self.torch.uint8, device=sim.device)
            rc = fn(sim.h, C.byref(w), *args, C.c_void_p(self._out.data_ptr()), self._out.numel(), C.byref(n),
                    C.c_void_p(self._scratch.data_ptr()))
        sim._chk(rc, name)
        return bytes(self._out[: n.value].cpu().numpy()) if n.value else b""

    def digest(self, observer: int, tick: int) -> bytes:
        """DigestPb of ``observer``'s ``compute_digest`` at ``tick`` (``state.py:324-331, 56-58``)."""
        return self._emit(self.sim.L.gs_emit_digest, "gs_emit_digest", int(observer), int(tick))

    def delta(self, sender: int, receiver: int, tick: int) -> bytes:
        """DeltaPb of ``sender``'s ``compute_partial_delta_respecting_mtu`` against ``receiver``'s digest at
        ``tick`` (``state.py:340-415, 98-99``), not applied."""
        return self._emit(self.sim.L.gs_emit_delta, "gs_emit_delta", int(sender), int(receiver), int(tick))

    def syn(self, observer: int, tick: int) -> bytes:
        """``_make_syn_msg().SerializeToString()`` (``server.py:327-332``)."""
        return packet(self.cluster_id, "syn", digest=self.digest(observer, tick))

    def synack(self, responder: int, initiator: int, tick: int) -> bytes:
        """The SynAck ``responder`` would answer ``initiator``'s Syn with, had it not yet merged that Syn's
        heartbeats (``server.py:339-348`` computes the digest after ``_report_heartbeat``)."""
        return packet(self.cluster_id, "synack", digest=self.digest(responder, tick),
                      delta=self.delta(responder, initiator, tick))
