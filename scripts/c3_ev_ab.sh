#!/bin/bash
# Config #3 with the event-driven mesh epochs: grid of the row steps
# (GS_EV_BLOCKS_PER_CU, 0 = one row per group) under rocprofv3 kernel stats.
set -u
OUT=${OUT:-gpurun_out/c3ev_ab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in ${BPCS:-0 8 32}; do
  GS_EV_BLOCKS_PER_CU=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/b$b" -o c3 -- python3 scripts/prof_c3.py > "$OUT/b$b.txt" 2>&1
  rc=$?
  case $rc in 0) ;; *) echo "rc=$rc at b=$b"; exit $rc;; esac
done
