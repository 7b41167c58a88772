#!/bin/bash
# A/B bench runs in one GPU call: each VARIANT is "name:ENV=VAL,ENV=VAL" (env for bench.py), run in turn
#   TAG=<tag> VARIANTS="base: fused:GS_PACK=fused" [ARGS="--steps 5 --warmup 2 --no-cpu-baseline"] bash tools/ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
ARGS=${ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline"}
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}
  ( for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 python -u bench.py $ARGS > $O/bench_$name.log 2>&1 ) || { echo "$name failed"; tail -20 $O/bench_$name.log; exit 1; }
  tail -1 $O/bench_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', 'value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), round(v.get('frac') or 0,3)) for k,v in r['kernels'].items()}, 'ps', d['peer_select'] and (round(d['peer_select']['value']), d['peer_select']['phases_per_round']), 'copy', round(r['measured_copy_ceiling']))"
done
echo done
