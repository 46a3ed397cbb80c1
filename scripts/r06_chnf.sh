#!/bin/bash
# Churn with fragment groups on the list pass: the churn / non-lockstep tests
# and config #3's oracle tests.
set -u
OUT=gpurun_out/${OUTD:-r06cf}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "churn or nonlockstep or config3" > $OUT/tests_chn.log 2>&1
rc=$?; echo "churn tests rc=$rc"; grep -E "FAILED|Error|assert" $OUT/tests_chn.log | head -20; tail -3 $OUT/tests_chn.log
