#!/bin/bash
# One GPU test under several env settings (A/B isolation of a parity failure), each in its own process:
#   T="tests/...::test_x[param]" CASES="base: old:GS_P1=old dbg8:GS_LIB=...,GS_ABLATE=8" bash tools/ab_test.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in $CASES; do
  name=${v%%:*}; envs=${v#*:}
  ( for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 150 python -u -m pytest "$T" -m gpu -x -q --timeout 120 --timeout-method thread > /tmp/ab_$name.log 2>&1 )
  rc=$?
  echo "$name rc=$rc $(grep -E 'passed|failed' /tmp/ab_$name.log | tail -1)"
  grep -m1 "AssertionError" /tmp/ab_$name.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
