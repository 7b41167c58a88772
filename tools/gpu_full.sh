# GPU tests, smoke, a full bench line (CPU baseline + peer-selection rounds), then the rocprofv3 evidence
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), round(v.get('frac') or 0,3)) for k,v in r['kernels'].items()}, 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']), 'ps', d['peer_select'] and (round(d['peer_select']['value']), d['peer_select']['unscheduled_exchanges']))"
if [ -n "$PROFILE" ]; then bash tools/profile.sh $TAG > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }; fi
if [ -n "$PROBE" ]; then timeout -k 10 150 python -u tools/rccl_probe.py > $O/rccl_probe.log 2>&1; cat $O/rccl_probe.log; fi
echo done
