"""aiocluster_amd -- MI355X-native batched backend for aiocluster's gossip hot path.

Scuttlebutt anti-entropy (``aiocluster/state.py``) and phi failure detection
(``aiocluster/failure_detector.py``) for a whole simulated cluster at once, as
hand-written gfx950 HIP kernels behind the C ABI of ``include/gossip_sim.h``.
See DESIGN.md.
"""

from .entities import (  # noqa: F401
    Config,
    FailureDetectorConfig,
    NodeDigest,
    NodeId,
    NodeState,
    VersionedValue,
    VersionStatusEnum,
)

__all__ = [
    "Config",
    "FailureDetectorConfig",
    "GossipSim",
    "NodeDigest",
    "NodeId",
    "NodeState",
    "VersionedValue",
    "VersionStatusEnum",
]


def __getattr__(name):
    if name == "GossipSim":
        from .sim import GossipSim

        return GossipSim
    raise AttributeError(name)
