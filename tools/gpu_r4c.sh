set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_rccl.py tests/test_gpu_config4.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
L=aiocluster_amd/lib
TAG=r4c VARIANTS="base:GS_LIB=$L/libgossip_sim_kw4.so nt:GS_LIB=$L/libgossip_sim_nt.so w8a0:GS_LIB=$L/libgossip_sim_w8a0.so w5a2:GS_LIB=$L/libgossip_sim_w5a2.so" ARGS="--steps 10 --warmup 2 --no-cpu-baseline --peer-select-steps 0" bash tools/ab.sh || exit 1
for g in 1 2 8; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --peer-select-steps 0 --slices $g > $O/bench_s$g.log 2>&1 || { tail -20 $O/bench_s$g.log; exit 1; }
  tail -1 $O/bench_s$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('slices $g value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), v['launches']) for k,v in r['kernels'].items()})"
done
SQ=1 timeout -k 10 1200 bash tools/profile.sh r4c > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo done
