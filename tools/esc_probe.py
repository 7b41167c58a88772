"""Escape-slot census under the device's peer selection (sizing tests/test_gpu_longrun.py): for each
(nodes, fanout, seeds) the number of owner columns the lag sweeps escaped to 16-bit slots and released, over
R rounds of the long-run test's workload.  GPU only; prints one line per configuration.
    python tools/esc_probe.py [rounds]"""

import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    from helpers import make_backend

    from aiocluster_amd.peers import PeerSelector
    from aiocluster_amd.scenario import make_scenario
    from aiocluster_amd.sim import GossipSim
    from aiocluster_amd.workload import WorkloadSpec, liveness_tick, phase_tick, round_tick

    R = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    for n, F, ns in [(2048, 3, 8), (2048, 1, 8), (2048, 2, 8), (2048, 1, 4), (4096, 1, 8), (4096, 3, 8)]:
        spec = WorkloadSpec(n=n, k=16, fanout=F, seed=7, init="warm", write_frac=0.05, down_frac=0.05, down_rounds=3)
        scen = make_scenario(f"p{n}", spec, R)
        gpu = make_backend(GossipSim, scen, tombstones=False, fd_ring=False, hb8=True, mv8=True)
        sel = PeerSelector(gpu, fanout=F, seeds=list(range(0, n, n // ns)), seed=7)
        first = None
        for r in range(R):
            rd = scen["rounds"][r]
            t = round_tick(r)
            up = np.asarray(rd["up"], dtype=np.uint8)
            for j, k, op, v in rd["writes"]:
                gpu.write(t, j, k, op, v)
            up_dev = gpu._dev(up, gpu.torch.uint8)
            gpu.begin_round(t, up_dev)
            sel.select(up_dev, r)
            phases, _, _ = sel.schedule(up_dev, r)
            for p, (a, b, _) in enumerate(phases):
                gpu.run_phase_arrays(phase_tick(r, p), a, b)
            gpu.update_node_liveness(liveness_tick(r, len(phases)), up_dev)
            c = gpu.counters()
            if first is None and c["hb_escapes"]:
                first = r
        gpu.check_heartbeat_lag()
        c = gpu.counters()
        print(f"n={n} F={F} seeds={ns}: escapes {c['hb_escapes']} releases {c['hb_releases']} first at round {first} "
              f"err_hb_lag {c['err_hb_lag']} sweeps {c['lag_sweeps']}", flush=True)
        gpu.close()


if __name__ == "__main__":
    main()
