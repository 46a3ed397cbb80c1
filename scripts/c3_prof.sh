#!/bin/bash
# Config #3 kernel trace (churn list pass): rocprofv3 kernel stats of scripts/c3_probe.py.
set -u
OUT=${OUT:-gpurun_out/c3prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 scripts/c3_probe.py > "$OUT/probe.log" 2>&1
echo "rc=$?"
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -30
