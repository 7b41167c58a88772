#!/bin/bash
# Round-4 GPU call (gpurun): optional membench, the GPU tests (TESTS, default all), the bench (BENCH args), an A/B
# bench with round 3's pass 1 (AB=1: env GS_P1=old), the heartbeat-lag census under the reference's peer selection
# (LAG=1).  Each step under its own limit; the first failure ends the call.
#   TAG=<tag> [MEMBENCH=1] [TESTS="<pytest args>"] [BENCH="<bench args>"] [AB=1] [LAG=1] bash tools/gpu_r4.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$MEMBENCH" ]; then
  timeout -k 10 180 ./tools/membench8 > $O/membench8.txt 2>&1 || { cat $O/membench8.txt; exit 1; }
  cat $O/membench8.txt
fi
if [ "${TESTS:-}" != "none" ]; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -18 $O/gpu_tests.log
fi
summ() {
  tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), round(v.get('frac') or 0,3)) for k,v in r['kernels'].items()}, 'copy', r['measured_copy_ceiling'] and round(r['measured_copy_ceiling']), 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']), 'ps', d['peer_select'] and (round(d['peer_select']['value']), d['peer_select']['phases_per_round'], d['peer_select']['exact']))"
}
if [ -n "$BENCH" ]; then
  timeout -k 10 500 python -u bench.py $BENCH > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  summ $O/bench.log
fi
if [ -n "$AB" ]; then
  GS_P1=old timeout -k 10 500 python -u bench.py ${BENCH:---steps 10 --warmup 2} --no-cpu-baseline > $O/bench_p1old.log 2>&1 || { tail -20 $O/bench_p1old.log; exit 1; }
  echo "GS_P1=old:"; summ $O/bench_p1old.log
fi
if [ -n "$LAG" ]; then
  timeout -k 10 400 python -u tools/hb_lag.py --peer-select --rounds ${LAG_ROUNDS:-60} --every 3 > $O/lag_ps.txt 2>&1 || { tail -5 $O/lag_ps.txt; exit 1; }
  tail -4 $O/lag_ps.txt
fi
echo done
