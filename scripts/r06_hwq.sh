#!/bin/bash
# 8 loop-back parts (routed, direct stores) with 4 / 8 / 16 hardware queues per process.
set -u
OUT=gpurun_out/${OUTD:-r06n}
mkdir -p $OUT
export TMPDIR=/tmp
for q in 8 16 4; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 6 --warmup 2 --configs 0 \
    --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/peer8_q$q.log 2>&1
  rc=$?; echo "peer8 hwq=$q rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/peer8_q$q.log)"
  case $rc in 0) ;; *) exit $rc;; esac
done
