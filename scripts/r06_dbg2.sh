#!/bin/bash
set -u
OUT=gpurun_out/r06m
mkdir -p $OUT
export TMPDIR=/tmp GS_PART_ROUTE=1 GS_PART_DIRECT=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/copy_prof -o run --output-format csv -- \
  python -u bench.py --mode peer --parts 8 --steps 2 --warmup 1 --configs 0 --cpu-seconds 0 --also-peers 0 \
  --gossip-check 0 --output-steps 0 > $OUT/copy_prof.log 2>&1
echo "copy prof rc=$?"
