#!/bin/bash
# Kernel trace of one config #3 batch (scripts/c3_probe.py) and its per-bucket
# summary (scripts/c3_trace.py).
set -u
OUT=${OUT:-gpurun_out/c3prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- python -u scripts/c3_probe.py \
  > "$OUT/probe.log" 2>&1 || exit $?
python scripts/c3_trace.py $(ls "$OUT"/tr/*/run_kernel_trace.csv "$OUT"/tr/run_kernel_trace.csv 2>/dev/null | head -1) \
  > "$OUT/c3_trace_buckets.txt"
head -20 "$OUT/c3_trace_buckets.txt"
