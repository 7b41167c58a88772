# One rocprofv3 SQ counter pass over bench.py (8 SQ counters: the per-pass hardware limit)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/sq_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $OUT -o sq --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_sq.log 2>&1
