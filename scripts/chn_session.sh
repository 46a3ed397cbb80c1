#!/bin/bash
# Churn list pass: parity tests, then config #3 timing with and without it.
set -u
OUT=${OUT:-gpurun_out/chn}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/rc.txt"
  tail -5 "$OUT/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $name: stopping"; exit $rc;; esac
  return 0
}
step chn_tests ${TESTS_SECS:-900} python -u -m pytest ${TEST_FILES:-tests/test_gpu_parity.py} -k "${TEST_K:-churn}" ${TEST_ARGS:--x} -v --timeout 300 --timeout-method thread
step c3_list 300 python -u scripts/c3_probe.py
step c3_push 300 env GS_CHURN_LIST=0 python -u scripts/c3_probe.py
echo "session done"
