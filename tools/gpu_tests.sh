#!/bin/bash
# GPU call (gpurun): the GPU tests (all of them, or $TESTS), each under pytest-timeout, the whole step under its own
# limit.  Test failures (rc 1) are reported; any other exit (a limit, a crash) ends the call there.
#   TAG=<tag> [TESTS="tests/..."] [KEXPR="..."] [LIMIT=1100] bash tools/gpu_tests.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 ${LIMIT:-1100} python -u -m pytest ${TESTS:-tests} ${KEXPR:+-k "$KEXPR"} -m gpu -v -rP --capture=sys --durations=25 --timeout 400 \
  --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/gpu_tests.log | grep -c PASSED
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -20
tail -40 $O/gpu_tests.log
exit $rc
