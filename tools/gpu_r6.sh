#!/bin/bash
# GPU call (gpurun): optional GPU tests, then named bench runs, each under its own limit; the first
# failure ends the call.
#   TAG=<tag> [TESTS="<pytest args>"] [KEXPR="<pytest -k expression>"] RUNS="name:ENV=V,ENV=V:<bench args>;name2::<bench args>" bash tools/gpu_r6.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -18 $O/gpu_tests.log
fi
summ() {
  tail -1 $1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('$2', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'step_frac', r.get('step_frac') and round(r['step_frac'],3),
      {k:(round(v['avg_launch_ms'],3), v['launches'], round(v.get('frac') or 0,3)) for k,v in r['kernels'].items()},
      'copy', r['measured_copy_ceiling'] and round(r['measured_copy_ceiling']),
      'cpu', d['cpu_baseline'] and (round(d['cpu_baseline']['value']), round(d['cpu_baseline']['single_core_value'])),
      'ps', d['peer_select'] and (round(d['peer_select']['value']), d['peer_select']['phases_per_round'], d['peer_select'].get('exact')),
      'c4', d.get('config4') and (round(d['config4']['ms_per_step'],2), d['config4']['kernel_ms_per_step']),
      'parity', d.get('parity_check') and [x['exact'] for x in d['parity_check']['per_slice']],
      'sched', {k: d['config'][k] for k in ('unscheduled_exchanges_all_rounds', 'max_phases_per_round', 'rounds_with_sub_phases') if k in d['config']},
      'extra', d.get('slice_stats'))"
}
IFS=';' read -ra RUNL <<< "$RUNS"
for v in "${RUNL[@]}"; do
  [ -z "$v" ] && continue
  name=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; args=${rest#*:}
  ( for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 ${RUN_LIMIT:-400} python -u bench.py $args > $O/bench_$name.log 2>&1 ) || { echo "$name failed"; tail -20 $O/bench_$name.log; exit 1; }
  summ $O/bench_$name.log $name
done
echo done
