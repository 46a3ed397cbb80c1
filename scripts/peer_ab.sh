#!/bin/bash
# Partitioned mode A/B: 8 loop-back parts at 1M peers, routed record exchange
# (GS_PART_ROUTE=1) vs every part's records to every part.
set -u
OUT=${OUT:-gpurun_out/peer_ab}
mkdir -p "$OUT"
ARGS="--mode peer --steps ${STEPS:-3} --warmup 1 --configs 0 --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0"
for v in routed gather routed gather; do
  if [ $v = routed ]; then export GS_PART_ROUTE=1; else unset GS_PART_ROUTE; fi
  timeout -k 10 300 python -u bench.py $ARGS --parts ${PARTS:-8} > "$OUT/$v.log" 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$v.log")" | tee -a "$OUT/ab.txt"
  [ $rc -eq 0 ] || exit $rc
done
