# sliced-path check: GPU tests, then bench with 1, 2 and 8 in-process owner-column slices
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for g in 1 2 8; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --slices $g > $O/bench_s$g.log 2>&1 || { tail -20 $O/bench_s$g.log; exit 1; }
  tail -1 $O/bench_s$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('slices $g value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), v['launches']) for k,v in r['kernels'].items()})"
done
