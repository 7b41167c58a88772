"""The exact packer's heavy-slot kernel (k_pack_heavy, round 6) against the C oracle.

At the headline a slot goes to k_pack_heavy past 2,048 stale owners (a node back from an absence); the full-size
checks (tests/test_gpu_fullsize.py, bench.py's CPU-baseline sample) cover that.  Here the hand-off threshold is
lowered (env GS_HEAVY_T, read once per process: a child process) so that small clusters send most truncating
slots through the heavy kernel -- whole-fit prefix, parallel first-fit filter, sequential survivors, bitmap
continuation past a half's 1,024 records -- and every round must equal the oracle.  GPU only.
"""

import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

SCRIPT = r"""
import sys
sys.path[:0] = [%(here)r, %(repo)r, %(oracle)r]
from helpers import compare_exports, make_backend
from oracle import OracleSim
from aiocluster_amd.scenario import make_scenario, replay_round
from aiocluster_amd.sim import GossipSim
from aiocluster_amd.workload import WorkloadSpec

n, K, mtu, rounds = %(n)d, 16, %(mtu)d, %(rounds)d
spec = WorkloadSpec(n=n, k=K, fanout=3, seed=%(seed)d, init="warm", write_frac=0.3, down_frac=0.1, down_rounds=3)
scen = make_scenario("heavy%%d" %% n, spec, rounds, {"mtu": mtu})
gpu = make_backend(GossipSim, scen, tombstones=False, fd_ring=False, hb8=%(hb8)s, mv8=%(hb8)s)
orc = make_backend(OracleSim, scen)
for r in range(rounds):
    replay_round(gpu, scen, r)
    replay_round(orc, scen, r)
    d = compare_exports(gpu.export(), orc.export())
    assert d is None, "round %%d: %%s" %% (r, d)
c, s = gpu.check(), orc.stats()
assert c["node_deltas"] == s["node_deltas"] and c["truncated"] == s["truncated"] and c["delta_bytes"] == s["delta_bytes"]
print("ok heavy_slots %%d truncated %%d steps_max %%d" %% (c["heavy_slots"], c["truncated"], c["pack_steps_max"]))
"""


def _run(env_extra, **kw):
    code = SCRIPT % dict(here=HERE, repo=REPO, oracle=os.path.join(REPO, "oracle"), **kw)
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = r.stdout.strip().splitlines()[-1]
    assert line.startswith("ok"), line
    return dict(zip(line.split()[1::2], (int(x) for x in line.split()[2::2])))


@pytest.mark.parametrize("n,mtu,hb8", [(1024, 1500, True), (3000, 4000, True), (768, 1200, False)],
                         ids=["n1024-hb8", "n3000-hb8-bitmap", "n768-hb16"])
def test_heavy_slots_match_oracle(n, mtu, hb8):
    """GS_HEAVY_T=48: slots with more than 48 stale owners go through k_pack_heavy.  n = 3,000 puts more than 1,024
    stale owners in one row half of the nodes back from an absence (the bitmap continuation)."""
    st = _run({"GS_HEAVY_T": "48"}, n=n, mtu=mtu, rounds=10, seed=n, hb8=hb8)
    assert st["heavy_slots"] > 0 and st["truncated"] > 0, st


def test_heavy_kernel_off_matches_oracle():
    """GS_HEAVY=0 (the A/B switch): the round-5 walk in k_pack_slice alone, same oracle result, no hand-off."""
    st = _run({"GS_HEAVY": "0"}, n=1024, mtu=1500, rounds=6, seed=5, hb8=True)
    assert st["heavy_slots"] == 0 and st["truncated"] > 0, st
