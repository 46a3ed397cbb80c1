#!/bin/bash
set -u
OUT=gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp
OUT=$OUT/xcd bash scripts/chain_xcd_sweep.sh || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_comm_ops.py tests/test_gpu_partition.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
case $rc in 0) ;; *) exit $rc;; esac
for route in 0 1; do
  GS_PART_ROUTE=$route timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 3 --warmup 1 --configs 0 \
    --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/peer8_route$route.log 2>&1
  rc=$?; echo "peer8 route=$route rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $OUT/peer8_route$route.log
  case $rc in 0) ;; *) exit $rc;; esac
done
