#!/bin/bash
# Config #3 A/B over environment settings: one probe batch per setting
# (scripts/c3_probe.py), e.g. ENVS="GS_SIDE_PRIORITY=0 GS_SIDE_PRIORITY=1".
set -u
OUT=${OUT:-gpurun_out/c3env}
mkdir -p "$OUT"
for r in 1 2; do
  for e in ${ENVS}; do
    f="$OUT/probe_$(echo "$e" | tr '/=' '__')_$r.log"
    env $e timeout -k 10 300 python -u scripts/c3_probe.py > "$f" 2>&1 || exit $?
    echo "$e (round $r): $(grep 'c3 probe' "$f")"
  done
done
