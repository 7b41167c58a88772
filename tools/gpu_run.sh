#!/bin/bash
# One GPU call (gpurun): [pytest selection] then [bench], each step under its own time limit.
#   TAG=<tag> [TESTS="<pytest args>"] [BENCH="<bench args>"] [PROFILE=1] bash tools/gpu_run.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -22 $O/gpu_tests.log
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 500 python -u bench.py $BENCH > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), round(v.get('frac') or 0,3)) for k,v in r['kernels'].items()}, 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']), 'ps', d['peer_select'] and (round(d['peer_select']['value']), d['peer_select']['phases_per_round'], d['peer_select']['unscheduled_exchanges']), 'c4', d.get('config4') and (d['config4'].get('one_gpu_share_exchanges_per_s') or d['config4']['value'], d['config4']['ms_per_step']), 'hz', d.get('exactness'))"
fi
if [ -n "$PROFILE" ]; then bash tools/profile.sh $TAG > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }; fi
echo done
