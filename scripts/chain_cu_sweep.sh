#!/bin/bash
# Config #3 probe (one timed 1024-message batch) with the epoch chain on a
# CU-masked stream of n CUs: how the serial chain's time depends on the CUs it gets.
set -u
OUT=${OUT:-gpurun_out/chain_cu}
mkdir -p "$OUT"
for cfg in "0 1" "256 1" "128 1" "64 1" "32 1" "32 8" "16 1"; do
  set -- $cfg
  echo "== GS_CHAIN_CUS=$1 GS_CU_STRIDE=$2" | tee -a "$OUT/sweep.txt"
  GS_CHAIN_CUS=$1 GS_CU_STRIDE=$2 timeout -k 10 120 python -u scripts/c3_probe.py >> "$OUT/sweep.txt" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/sweep.txt"
  case $rc in 0) ;; *) echo "stop rc=$rc"; exit $rc;; esac
done
grep -E "==|c3 probe" "$OUT/sweep.txt"
