#!/bin/bash
# Kernel trace of a short bench run (per-dispatch durations -> scripts/trace_passes.py).
# VARIANTS: GS_RELAX_VARIANT values to trace (default: the library default only).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then unset GS_RELAX_VARIANT; else export GS_RELAX_VARIANT=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$v -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --cpu-seconds 0 --also-peers 0 --configs 0 ${BENCH_ARGS:-} > gpurun_out/prof_$v.log 2>&1 || exit $?
done
