#!/bin/bash
set -u
OUT=gpurun_out/r06k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_partition.py tests/test_comm_ops.py -k "route or partitioned_list or local_comm or processes" > $OUT/tests_part.log 2>&1
rc=$?; echo "partition tests rc=$rc"; tail -2 $OUT/tests_part.log
case $rc in 0) ;; *) exit $rc;; esac
for route in 1 0; do
  GS_PART_ROUTE=$route timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 6 --warmup 2 --configs 0 \
    --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/peer8_route$route.log 2>&1
  rc=$?; echo "peer8 route=$route rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/peer8_route$route.log)"
  case $rc in 0) ;; *) exit $rc;; esac
done
GS_PART_ROUTE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/route_prof -o run --output-format csv -- \
  python -u bench.py --mode peer --parts 8 --steps 3 --warmup 1 --configs 0 --cpu-seconds 0 --also-peers 0 \
  --gossip-check 0 --output-steps 0 > $OUT/route_prof.log 2>&1
echo "route prof rc=$?"
