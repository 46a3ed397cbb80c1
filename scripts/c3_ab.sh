#!/bin/bash
# Config #3 A/B on one box: default (fused churn epochs + tile-skipping gossip
# scan) vs per-epoch mesh launches (GS_MESH_FUSED=0) vs no tile skip
# (GS_RELAX_VARIANT=45). Each run under its own time limit; output goes
# straight to gpurun_out/c3_ab.txt.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
CASES=${CASES:-"default mesh_unfused no_tile_skip"}
for name in $CASES; do
  case $name in
    default) E="GS_X=1";;
    mesh_fused) E="GS_MESH_FUSED=1";;
    mesh_fused2) E="GS_MESH_FUSED=1 GS_EPOCH_BLOCKS_PER_CU=2";;
    mesh_unfused) E="GS_MESH_FUSED=0";;
    rows64) E="GS_ROW_GROUP=64";;
    no_tile_skip) E="GS_RELAX_VARIANT=45";;
    unfused_noskip) E="GS_MESH_FUSED=0 GS_RELAX_VARIANT=45";;
  esac
  echo "== $name ($E) $(date +%T)" >> "$OUT/c3_ab.txt"
  env $E timeout -k 10 ${C3_SECS:-150} python -u scripts/prof_c3.py ${C3_ARGS:-} >> "$OUT/c3_ab.txt" 2>&1
  rc=$?
  echo "rc=$rc" >> "$OUT/c3_ab.txt"
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $name"; cat "$OUT/c3_ab.txt"; exit $rc;; esac
done
cat "$OUT/c3_ab.txt"
