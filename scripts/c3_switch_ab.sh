#!/bin/bash
# Config #3 A/B of the receiver/sender-centric gossip split (GS_GOSSIP_SWITCH):
# one 1024-message batch per setting (scripts/c3_probe.py), after the churn tests.
set -u
OUT=${OUT:-gpurun_out/c3ab}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "churn" -x -v --timeout 300 --timeout-method thread \
  > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
for sw in ${SWITCHES:-1000 4 5 3}; do
  GS_DEBUG_COUNTS=1 GS_GOSSIP_SWITCH=$sw timeout -k 10 300 python -u scripts/c3_probe.py > "$OUT/probe_$sw.log" 2>&1 || exit $?
  echo "switch $sw: $(grep 'c3 probe' $OUT/probe_$sw.log) $(grep 'gossip-listed' $OUT/probe_$sw.log | tail -1)"
done
