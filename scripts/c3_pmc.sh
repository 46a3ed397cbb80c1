#!/bin/bash
# Config #3 HBM traffic: two PMC passes (FETCH_SIZE, WRITE_SIZE) over one probe
# batch (after a warm-up batch), summarised per kernel by scripts/c3_pmc.py.
set -u
OUT=${OUT:-gpurun_out/c3pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python -u scripts/c3_probe.py \
  > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python -u scripts/c3_probe.py \
  > "$OUT/write.log" 2>&1 || exit $?
ALG=$(python -c "import ast,sys; l=[x for x in open('$OUT/fetch.log') if x.startswith('{')][-1]; print(ast.literal_eval(l)['bytes_alg'])")
python scripts/c3_pmc.py $(ls "$OUT"/fetch/*/run_counter_collection.csv "$OUT"/fetch/run_counter_collection.csv 2>/dev/null | head -1) \
  $(ls "$OUT"/write/*/run_counter_collection.csv "$OUT"/write/run_counter_collection.csv 2>/dev/null | head -1) $ALG \
  | tee "$OUT/c3_pmc_summary.txt"
