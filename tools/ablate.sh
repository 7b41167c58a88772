#!/bin/bash
# Profiling-only A/B of k_exchange phases (GS_ABLATE makes results invalid; never used by default).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out/ablate
for A in 0 1 2 3; do
  GS_ABLATE=$A timeout -k 10 300 python3 $R/bench.py --steps 4 --warmup 3 --no-cpu-baseline > $R/gpurun_out/ablate/a$A.log 2>&1 || exit 1
done
