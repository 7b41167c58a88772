"""Data model of the batched gossip backend.

Mirrors the reference's public data model so code written against
``aiocluster.entities`` reads the same here:

* ``VersionStatusEnum``   -- ``aiocluster/entities.py:25-35``
* ``VersionedValue``      -- ``aiocluster/entities.py:38-49``
* ``NodeId``              -- ``aiocluster/entities.py:55-82``
* ``FailureDetectorConfig`` -- ``aiocluster/entities.py:85-91``
* ``NodeDigest``          -- ``aiocluster/entities.py:118-136``
* ``NodeState`` (read-only view materialised from device rows) --
  ``aiocluster/state.py:106-113``

Time is simulated: one *tick* is 1/64 s (15 625 us).  A tick is the finest
unit that is both a whole number of microseconds (what ``datetime`` holds in
the reference) and a dyadic fraction of a second, so every failure-detector
interval the reference stores as ``timedelta.total_seconds()`` is an exact
binary double and the running sums of ``BoundedArrayStats`` are exact.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime, timedelta, timezone
from enum import IntEnum

TICK_US = 15_625
TICKS_PER_SECOND = 64
#: simulated wall clock origin (tick 0)
EPOCH = datetime(2024, 1, 1, tzinfo=timezone.utc)


def tick_to_datetime(tick: int) -> datetime:
    return EPOCH + timedelta(microseconds=tick * TICK_US)


def seconds_to_ticks(seconds: float) -> int:
    """Exact conversion; refuses durations that are not whole ticks."""
    us = round(seconds * 1_000_000)
    if us % TICK_US:
        raise ValueError(f"{seconds}s is not a whole number of 1/64 s ticks")
    return us // TICK_US


class VersionStatusEnum(IntEnum):
    """``aiocluster/entities.py:25-28``."""

    SET = 0
    DELETED = 1
    DELETE_AFTER_TTL = 2


@dataclass
class VersionedValue:
    """``aiocluster/entities.py:38-49``.

    ``status_change_ts`` is the simulated tick (the reference keeps a
    ``datetime``; ``tick_to_datetime`` converts).  The device only tracks it for
    tombstones, the only entries whose timestamp the reference ever reads
    (``state.py:261-265``); for ``SET`` entries it is ``None``.
    """

    value: str
    version: int
    status: VersionStatusEnum
    status_change_ts: int | None = None

    def is_deleted(self) -> bool:
        return self.status in (VersionStatusEnum.DELETED, VersionStatusEnum.DELETE_AFTER_TTL)


@dataclass(frozen=True, eq=True, slots=True)
class NodeId:
    """``aiocluster/entities.py:55-82`` (generation id is explicit: Q11)."""

    name: str
    generation_id: int
    gossip_advertise_addr: tuple[str, int] = ("localhost", 7001)
    tls_name: str | None = None

    def long_name(self) -> str:
        host, port = self.gossip_advertise_addr
        return f"{self.name}-{self.generation_id}-{host}:{port}"


@dataclass(frozen=True, eq=True, slots=True)
class FailureDetectorConfig:
    """``aiocluster/entities.py:85-91``; durations in seconds."""

    phi_threshhold: float = 8.0
    sampling_window_size: int = 1_000
    max_interval: float = 10.0
    initial_interval: float = 5.0
    dead_node_grace_period: float = 24 * 3600.0


@dataclass(frozen=True, eq=True, slots=True)
class Config:
    """The slice of ``aiocluster/entities.py:94-115`` that parameterises the hot path."""

    marked_for_deletion_grace_period: int = 3600 * 2  # seconds
    failure_detector: FailureDetectorConfig = field(default_factory=FailureDetectorConfig)
    max_payload_size: int = 65_507
    gossip_count: int = 3


@dataclass(frozen=True, eq=True, slots=True)
class NodeDigest:
    """``aiocluster/entities.py:118-123``."""

    node_id: NodeId
    heartbeat: int
    last_gc_version: int
    max_version: int


@dataclass
class NodeState:
    """Observer-side view of one owner (``aiocluster/state.py:106-113``)."""

    node: NodeId
    heartbeat: int = 0
    key_values: dict[str, VersionedValue] = field(default_factory=dict)
    max_version: int = 0
    last_gc_version: int = 0

    def get(self, key: str) -> VersionedValue | None:
        v = self.key_values.get(key)
        if v is not None and v.is_deleted():
            return None
        return v

    def get_versioned(self, key: str) -> VersionedValue | None:
        return self.key_values.get(key)

    def digest(self) -> NodeDigest:
        return NodeDigest(self.node, self.heartbeat, self.last_gc_version, self.max_version)


@dataclass(frozen=True, slots=True)
class ClusterSnapshot:
    """``aiocluster/server.py:65-71`` (``Cluster.snapshot``, ``server.py:168-175``)."""

    cluster_id: str
    self_node_id: NodeId
    node_states: dict[NodeId, NodeState]
    live_nodes: list[NodeId]
    dead_nodes: list[NodeId]
