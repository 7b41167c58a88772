# chunked split-phase check + sweep: GPU tests (default build), then bench per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
for v in "c4::4" "c1::1" "c8::8" "w6:aiocluster_amd/lib/var/p1w6.so:4" "w8:aiocluster_amd/lib/var/p1w8.so:4"; do
  IFS=: read name lib ch <<< "$v"
  GS_LIB=$lib GS_CHUNKS=$ch timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_$name.log 2>&1 || exit 1
  tail -1 $O/bench_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', round(d['value']), round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],3))"
done
