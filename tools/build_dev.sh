#!/bin/bash
# Development build of the HIP library without the K > 16 kernel instantiations (about a tenth of the
# full build time): aiocluster_amd/lib/libgossip_sim_kw4.so, loaded with GS_LIB=<that path> for
# kernel A/B runs on K <= 16 workloads.  The product build is __graft_entry__.build().
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${OUT:-libgossip_sim_kw4.so}
hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -shared -DGS_KW4_ONLY \
  -o $R/aiocluster_amd/lib/$OUT $R/aiocluster_amd/csrc/gossip_sim.hip -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib "$@"
