#!/bin/bash
# Partition tests + 8 loop-back parts at 1M x 1024: routed direct stores (the
# default), gathered, routed through copies; kernel trace of the default.
set -u
OUT=gpurun_out/${OUTD:-r06l}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_partition.py tests/test_comm_ops.py > $OUT/tests_part.log 2>&1
rc=$?; echo "partition tests rc=$rc"; tail -2 $OUT/tests_part.log
case $rc in 0) ;; *) exit $rc;; esac
for v in direct gather; do
  case $v in direct) E="";; gather) E="GS_PART_ROUTE=0";; copy) E="GS_PART_ROUTE=1 GS_PART_DIRECT=0";; esac
  env $E timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 6 --warmup 2 --configs 0 \
    --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/peer8_$v.log 2>&1
  rc=$?; echo "peer8 $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/peer8_$v.log)"
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/route_prof -o run --output-format csv -- \
  python -u bench.py --mode peer --parts 8 --steps 3 --warmup 1 --configs 0 --cpu-seconds 0 --also-peers 0 \
  --gossip-check 0 --output-steps 0 > $OUT/route_prof.log 2>&1
echo "route prof rc=$?"
