#!/bin/bash
set -u
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_comm_ops.py tests/test_gpu_partition.py > $OUT/tests_part.log 2>&1
rc=$?; echo "partition tests rc=$rc"; tail -2 $OUT/tests_part.log
case $rc in 0|1) ;; *) exit $rc;; esac
while read -r envs; do
  echo "== $envs" >> $OUT/c3.txt
  env C3_MSGS=4096 $envs timeout -k 10 180 python -u scripts/c3_probe.py >> $OUT/c3.txt 2>&1
  rc=$?; echo "c3 [$envs] rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done <<'LIST'
GS_CHN_PIPE=1
GS_SIDE_XCDS=0
GS_SIDE_XCDS=0-1 GS_PASS_XCDS=2-7
GS_SIDE_XCDS=1 GS_PASS_XCDS=2-7
GS_SIDE_XCDS=1-2 GS_PASS_XCDS=3-7
LIST
grep -E "==|c3 probe" $OUT/c3.txt
for route in 0 1; do
  GS_PART_ROUTE=$route timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 3 --warmup 1 --configs 0 \
    --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/peer8_route$route.log 2>&1
  rc=$?; echo "peer8 route=$route rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $OUT/peer8_route$route.log
  case $rc in 0) ;; *) exit $rc;; esac
done
OUT=$OUT/libab LIBS="noskip base" bash scripts/lib_ab.sh
