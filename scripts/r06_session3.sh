#!/bin/bash
set -u
OUT=gpurun_out/r06d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "churn or nonlockstep" > $OUT/tests_churn.log 2>&1
rc=$?; echo "churn tests rc=$rc"; tail -3 $OUT/tests_churn.log
case $rc in 0) ;; *) exit $rc;; esac
for m in 1024 4096; do
  for pipe in 1 0; do
    echo "== C3_MSGS=$m GS_CHN_PIPE=$pipe" >> $OUT/c3.txt
    C3_MSGS=$m GS_CHN_PIPE=$pipe timeout -k 10 180 python -u scripts/c3_probe.py >> $OUT/c3.txt 2>&1
    rc=$?; echo "c3 $m $pipe rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
grep -E "==|c3 probe" $OUT/c3.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_comm_ops.py tests/test_gpu_partition.py > $OUT/tests_part.log 2>&1
rc=$?; echo "partition tests rc=$rc"; tail -3 $OUT/tests_part.log
