#!/bin/bash
# bench.py --mode peer on one GPU: an RCCL communicator of one rank, then
# loop-back P = 2 / 4 / 8 parts; one JSON line each into gpurun_out/peer_bench.jsonl.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
ARGS="--mode peer --steps ${STEPS:-3} --warmup 1 --configs 0 --cpu-seconds 0 --also-peers 0 --gossip-check 0 ${PEER_ARGS:-}"
for P in ${PARTS:-1 2 4 8}; do
  echo "== parts $P $(date +%T)" >> "$OUT/peer_bench.log"
  timeout -k 10 ${PEER_SECS:-300} python -u bench.py $ARGS --parts $P > "$OUT/peer_p$P.log" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/peer_bench.log"
  grep '^{' "$OUT/peer_p$P.log" >> "$OUT/peer_bench.jsonl" || true
  case $rc in 124|134|137|139) echo "fatal rc=$rc at parts $P"; exit $rc;; esac
done
cat "$OUT/peer_bench.log"
