#!/bin/bash
# Config #3's 1024 messages as 1 batch of 1024, 2 of 512, 4 of 256, 8 of 128
# (the chain ahead overlaps a batch's passes with the next batch's epochs).
set -u
OUT=gpurun_out/r06x
mkdir -p $OUT
for r in 1 2; do
  for b in 1024 512 256 128; do
    C3_BATCH=$b timeout -k 10 200 python -u scripts/c3_probe.py > $OUT/b${b}_$r.log 2>&1
    rc=$?; echo "batch $b round $r rc=$rc: $(grep -o 'c3 probe: [0-9.]* ms' $OUT/b${b}_$r.log)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
