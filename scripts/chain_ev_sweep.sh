#!/bin/bash
# Config #3 probe variants: event-step rows per block (GS_EV_SW), the chain on
# one XCD (GS_CHAIN_CUS=32 GS_CU_STRIDE=8) with the passes on the others
# (GS_PASS_SKIP=8), other CU subsets.
set -u
OUT=${OUT:-gpurun_out/chain_ev}
mkdir -p "$OUT"
while read -r envs; do
  echo "== $envs" | tee -a "$OUT/sweep.txt"
  env $envs timeout -k 10 120 python -u scripts/c3_probe.py >> "$OUT/sweep.txt" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/sweep.txt"
  case $rc in 0) ;; *) echo "stop rc=$rc"; exit $rc;; esac
done <<'LIST'
GS_EV_SW=1
GS_EV_SW=2
GS_EV_SW=4
GS_EV_SW=1 GS_CHAIN_CUS=32 GS_CU_STRIDE=8 GS_PASS_SKIP=8
GS_EV_SW=4 GS_CHAIN_CUS=32 GS_CU_STRIDE=8 GS_PASS_SKIP=8
GS_EV_SW=1 GS_CHAIN_CUS=16 GS_CU_STRIDE=16
GS_EV_SW=1 GS_CHAIN_CUS=64 GS_CU_STRIDE=4
GS_EV_SW=1 GS_CHAIN_CUS=8 GS_CU_STRIDE=32
LIST
grep -E "==|c3 probe" "$OUT/sweep.txt"
