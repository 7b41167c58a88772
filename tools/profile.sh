#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun).
#   1. kernel trace + stats (per-kernel average duration)
#   2. PMC FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md, HBM section), for the bench
#      and for tools/fetch_calib.py's known-byte streams (the per-width calibration factors)
#   3. (SQ=1) SQ issue/stall counters in a pass of their own
# Usage: [SQ=1] tools/profile.sh <tag> [bench args...]; then python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
# the kernel-trace pass runs the driver's own round-end command by default (its line reproduces BENCH's); the PMC
# passes skip the CPU baseline and the peer-selected rounds (after the timed region: the marker window excludes them)
ARGS=${@:---gpus 1 --steps 20 --warmup 5}
PARGS=${PARGS:-$ARGS --no-cpu-baseline --peer-select-steps 0}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $R/bench.py $ARGS > $OUT/bench_kt.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/cal_fetch -o cal --output-format csv -- python3 $R/tools/fetch_calib.py > $OUT/cal_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/cal_write -o cal --output-format csv -- python3 $R/tools/fetch_calib.py > $OUT/cal_write.log 2>&1
timeout -s KILL 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_write.log 2>&1
if [ -n "$SQ" ]; then
  timeout -s KILL 400 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $OUT/sq -o sq --output-format csv -- python3 $R/bench.py $PARGS > $OUT/bench_sq.log 2>&1
fi
find $OUT -name "*.csv" | xargs ls -la
