#!/bin/bash
# Same-box A/B of the loop-back pass control: serial reads + host sync (RS1 EV0),
# overlapped reads + host sync (RS0 EV0), overlapped reads + event waits (RS0 EV1).
set -u
OUT=gpurun_out/${OUTD:-r06r}
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in "1 0" "0 0" "0 1"; do
    set -- $v
    GS_AB_RSER=$1 GS_AB_EVW=$2 timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 4 --warmup 1 --configs 0 \
      --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/ab_$1$2_$r.log 2>&1
    rc=$?; echo "rs=$1 ev=$2 round $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_$1$2_$r.log)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
