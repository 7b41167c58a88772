#!/bin/bash
# Round-4 GPU call: the GPU tests (TESTS), A/B libraries (VARIANTS, tools/ab.sh), sliced rehearsals (SLICES=1),
# the reference-selection bench (PS=1: --peer-select, 200+ selected rounds on the 8-bit layout), a profile
# (PROFILE=1: tools/profile.sh with SQ counters).  Each step under its own limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$SMOKE" ]; then  # the driver's round-end smoke()
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --durations=12 --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -14 $O/gpu_tests.log
fi
if [ -n "$BENCHFULL" ]; then  # the driver's bench command (cpu_baseline and peer_select legs included)
  timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
  tail -1 $O/bench_full.log | cut -c1-600
fi
if [ -n "$VARIANTS" ]; then
  ARGS=${ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline --peer-select-steps 0"} bash tools/ab.sh || exit 1
fi
if [ -n "$SLICES" ]; then
  for g in 1 2 8; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --peer-select-steps 0 --slices $g > $O/bench_s$g.log 2>&1 || { tail -20 $O/bench_s$g.log; exit 1; }
    tail -1 $O/bench_s$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('slices $g value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), v['launches']) for k,v in r['kernels'].items()})"
  done
fi
if [ -n "$NATIVE_SLICES" ]; then  # the library driver (gs_run_phase_group): no Python per slice and launch
  for g in 2 8; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --peer-select-steps 0 --slices $g --native-comm > $O/bench_n$g.log 2>&1 || { tail -20 $O/bench_n$g.log; exit 1; }
    tail -1 $O/bench_n$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('native slices $g value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), {k:(round(v['avg_launch_ms'],3), v['launches']) for k,v in r['kernels'].items()})"
  done
fi
if [ -n "$PS" ]; then
  timeout -k 10 400 python -u bench.py --peer-select --settle 190 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_ps.log 2>&1 || { tail -20 $O/bench_ps.log; exit 1; }
  tail -1 $O/bench_ps.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('peer-select value', round(d['value']), 'ms/step', round(d['ms_per_step'],2), 'counters', {k: d['counters'][k] for k in ('lag_sweeps','hb_escapes','hb_releases')}, 'exactness', d['exactness'])"
fi
if [ -n "$SLICETRACE" ]; then  # kernel trace of a sliced rehearsal (gaps between launches: tools/gaps.py)
  for g in $SLICETRACE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/st$g -o st --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --slices $g --steps 3 --warmup 1 --no-cpu-baseline --peer-select-steps 0 $STARGS > $GRAFT_REPO_ROOT/$O/st$g.log 2>&1) || { tail -20 $O/st$g.log; exit 1; }
  done
  echo slicetrace
fi
if [ -n "$PROFILE" ]; then
  SQ=1 timeout -k 10 1100 bash tools/profile.sh $TAG > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
  echo profiled
fi
echo done
