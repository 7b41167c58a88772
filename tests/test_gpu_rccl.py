"""The multi-GPU code on one GPU (GPU only): a world-1 RCCL communicator and a world-1 torch ``nccl``
process group drive the sliced phase path of a one-slice cluster (``GS_SLICED``).

RCCL refuses two ranks on one GPU, so the 8-GPU bench's collectives cannot be rehearsed with several
slices here; with one slice they are the same calls: ``gs_comm_id`` + ``gs_comm_init`` and
``gs_run_phase`` over ``ncclAllGather`` (the library driver, ``bench.py --native-comm``), and
``DistComm.gather`` over ``all_gather_into_tensor`` (``aiocluster_amd/shard.py``, the bench's default).
Each run is compared with one unsliced handle on the same workload: MTU truncation in most exchanges
(the overflow list is non-empty every phase), churn, 6 rounds.  Reference semantics:
``aiocluster/state.py:340-415`` (the MTU walk the slices split), ``server.py:327-376``.
"""

import socket

import numpy as np
import pytest
from helpers import compare_exports

from aiocluster_amd import driver
from aiocluster_amd.scenario import DEFAULT_CFG
from aiocluster_amd.shard import DistComm, ShardGroup
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec, key_names, synthetic_node_ids

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl_world1():
    import torch
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def _run(sims, drive, plans):
    for rd in plans:
        driver.begin(sims, rd)
        for a, b, n, t in rd["phases"]:
            if n:
                drive(t, a, b)
        driver.end(sims, rd)


@pytest.mark.parametrize("native", [True, False], ids=["gs_comm_init+ncclAllGather", "torch_nccl_all_gather"])
def test_world1_rccl_sliced_path_matches_one_handle(nccl_world1, native):
    import torch

    n, K, rounds = 4096, 8, 6
    cfg = dict(DEFAULT_CFG, mtu=1500)  # most deltas are cut: every phase lists overflowing slots
    spec = WorkloadSpec(n=n, k=K, fanout=3, seed=11, init="warm", write_frac=0.2, down_frac=0.05, down_rounds=3)
    kw = dict(init="warm", tombstones=False, fd_ring=False, hist_cap=16, initial_ops=driver.boot_ops(n, K),
              hb8=True, mv8=True)
    ids, keys = synthetic_node_ids(n), key_names(K)
    ref = GossipSim(ids, keys, cfg, **kw)
    one = GossipSim(ids, keys, cfg, sliced=True, **kw)
    group = ShardGroup([one], DistComm(), cfg["mtu"], native=native)  # native: gs_comm_id + gs_comm_init
    plans = driver.prepare(spec, rounds, torch, ref.device)
    _run([ref], lambda t, a, b: ref.run_phase_arrays(t, a, b), plans)
    _run([one], lambda t, a, b: group.run_phase_arrays(t, a, b), plans)
    c_ref, c_one = ref.check(), group.check()
    assert c_ref["truncated"] > 0 and c_ref["node_deltas"] > 0
    for k in ("exchanges", "node_deltas", "kvs_sent", "truncated", "delta_bytes", "hb_reports"):
        assert c_one[k] == c_ref[k], (k, c_one[k], c_ref[k])
    diff = compare_exports(one.export(), ref.export())
    assert diff is None, diff
    assert np.array_equal(one.phi_row(5), ref.phi_row(5), equal_nan=True)
    one.close()
    ref.close()
