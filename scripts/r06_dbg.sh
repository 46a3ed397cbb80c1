#!/bin/bash
set -u
OUT=gpurun_out/r06e
mkdir -p $OUT
export TMPDIR=/tmp
for pipe in 1; do
  GS_CHN_PIPE=$pipe GS_DEBUG_AHEAD=1 GS_DEBUG_DTOR=1 timeout -k 10 90 python -u -m pytest -x -v --timeout 60 --timeout-method thread -m gpu \
    "tests/test_gpu_parity.py::test_churn_time_varying_mesh[1-1-0-0]" > $OUT/t_pipe$pipe.log 2>&1
  rc=$?; echo "pipe=$pipe rc=$rc"; grep -E "PASSED|FAILED|Timeout|ah\]|dtor" $OUT/t_pipe$pipe.log | head -30
  case $rc in 0|1) ;; *) exit $rc;; esac
done
