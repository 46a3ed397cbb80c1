#!/bin/bash
set -u
OUT=gpurun_out/r06g
mkdir -p $OUT
export TMPDIR=/tmp
OUT=$OUT/libab LIBS="ng8 ng8n ng2r4 base" bash scripts/lib_ab.sh || exit $?
for route in 1 0 1; do
  GS_PART_ROUTE=$route timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 6 --warmup 2 --configs 0 \
    --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/peer8_route$route.log 2>&1
  rc=$?; echo "peer8 route=$route rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/peer8_route$route.log)"
  case $rc in 0) ;; *) exit $rc;; esac
done
GS_PART_ROUTE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/route_prof -o run --output-format csv -- \
  python -u bench.py --mode peer --parts 8 --steps 3 --warmup 1 --configs 0 --cpu-seconds 0 --also-peers 0 \
  --gossip-check 0 --output-steps 0 > $OUT/route_prof.log 2>&1
echo "route prof rc=$?"
