#!/bin/bash
set -u
OUT=gpurun_out/${OUTD:-r06w}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_partition.py tests/test_comm_ops.py > $OUT/tests_part.log 2>&1
rc=$?; echo "partition tests rc=$rc"; tail -3 $OUT/tests_part.log
