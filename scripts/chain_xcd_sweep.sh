#!/bin/bash
# Config #3 probe: the epoch chain, the churn tables (side stream) and the
# passes on separate XCD sets (serial batch: the sum, each part's cost).
set -u
OUT=${OUT:-gpurun_out/chain_xcd}
mkdir -p "$OUT"
while read -r envs; do
  echo "== $envs" | tee -a "$OUT/sweep.txt"
  env $envs timeout -k 10 120 python -u scripts/c3_probe.py >> "$OUT/sweep.txt" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/sweep.txt"
  case $rc in 0) ;; *) echo "stop rc=$rc"; exit $rc;; esac
done <<'LIST'
GS_EV_SW=1
GS_CHAIN_XCDS=0 GS_PASS_XCDS=1-7
GS_CHAIN_XCDS=0 GS_PASS_XCDS=2-7
GS_CHAIN_XCDS=0 GS_PASS_XCDS=3-7
GS_CHAIN_XCDS=0 GS_PASS_XCDS=4-7
GS_CHAIN_XCDS=0 GS_SIDE_XCDS=1-2 GS_PASS_XCDS=3-7
GS_CHAIN_XCDS=0 GS_SIDE_XCDS=1 GS_PASS_XCDS=2-7
GS_CHAIN_XCDS=0 GS_SIDE_XCDS=1-7
LIST
grep -E "==|c3 probe" "$OUT/sweep.txt"
