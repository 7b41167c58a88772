"""Closed-form protobuf wire sizes for the messages that drive MTU packing.

The reference truncates deltas with ``DeltaPb(...).ByteSize()``
(``aiocluster/state.py:395,412``) over the proto3 schema in
``aiocluster/protos/messages.proto:39-74``.  Every field number there is < 16,
so each tag is one byte, and proto3 omits scalar fields equal to their default.
The only ``optional`` field, ``NodeDeltaPb.max_version`` (``messages.proto:65``),
is always set by the reference (``state.py:389``), so it is always present.

These functions are the host-side definition; the device computes the same
quantities in ``aiocluster_amd/csrc/gossip_kernels.hip`` (``pb_*`` helpers).
They are pinned against the reference's own ``ByteSize()`` by
``tests/golden/pbsize.json`` (see ``oracle/gen_golden.py``).
"""

from __future__ import annotations


def vlen(x: int) -> int:
    """Length of ``x`` as a base-128 varint."""
    n = 1
    while x >= 0x80:
        x >>= 7
        n += 1
    return n


def s_field(nbytes: int) -> int:
    """A ``string`` field holding ``nbytes`` UTF-8 bytes (absent when empty)."""
    return 0 if nbytes == 0 else 1 + vlen(nbytes) + nbytes


def u_field(x: int) -> int:
    """A ``uint32``/``uint64``/enum field (absent when zero)."""
    return 0 if x == 0 else 1 + vlen(x)


def msg_field(length: int) -> int:
    """An embedded message field whose body is ``length`` bytes (always present once set)."""
    return 1 + vlen(length) + length


def nodeid_size(name: str, generation_id: int, host: str, port: int, tls_name: str | None) -> int:
    """``NodeIdPb`` body size (``messages.proto:39-44``; built at ``entities.py:62-72``)."""
    addr = s_field(len(host.encode())) + u_field(port)
    return (
        s_field(len(name.encode()))
        + u_field(generation_id)
        + msg_field(addr)
        + s_field(len((tls_name or "").encode()))
    )


def kv_size(key: str, value: str, version: int, status: int) -> int:
    """``KeyValueUpdatePb`` body size (``messages.proto:53-58``)."""
    return s_field(len(key.encode())) + s_field(len(value.encode())) + u_field(version) + u_field(status)


def kv_size_from_lens(key_len: int, value_len: int, version: int, status: int) -> int:
    return s_field(key_len) + s_field(value_len) + u_field(version) + u_field(status)


def nodedelta_size(nid_size: int, from_version: int, last_gc: int, kv_sizes: list[int], max_version: int) -> int:
    """``NodeDeltaPb`` body size (``messages.proto:60-66``)."""
    return (
        msg_field(nid_size)
        + u_field(from_version)
        + u_field(last_gc)
        + sum(msg_field(k) for k in kv_sizes)
        + 1
        + vlen(max_version)
    )


def delta_size(nodedelta_sizes: list[int]) -> int:
    """``DeltaPb`` size (``messages.proto:72-74``)."""
    return sum(msg_field(n) for n in nodedelta_sizes)
