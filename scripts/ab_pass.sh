#!/bin/bash
# A/B of the window-pass kernels on the bench workload: for each GS_RELAX_VARIANT
# in VARIANTS (default "45 109": k_pull over dense rows, k_lpull over candidate
# lists) a kernel trace of a short bench run, then the last batch's per-dispatch
# durations (scripts/last_batch.py). Runs on the GPU box.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS:-45 109}; do
  export GS_RELAX_VARIANT=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --also-peers 0 --configs 0 --gossip-check 0 \
    ${BENCH_ARGS:-} > gpurun_out/ab_$v.log 2>&1 || exit $?
  echo "== variant $v"
  python scripts/last_batch.py gpurun_out/ab_$v/run_kernel_trace.csv || exit $?
done
