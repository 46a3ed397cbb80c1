#!/bin/bash
# SQ counter passes over one kernel family (KRE) of a 1-step bench, one pass per
# counter group (never combined with tracing; each pass under its own kill timer).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
KRE=${KRE:-k_pull}
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for grp in ${GROUPS_PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" -d gpurun_out/pmc_sq$i -o run --output-format csv -- \
    python bench.py --steps 1 --warmup 0 --cpu-seconds 0 --also-peers 0 --configs 0 ${BENCH_ARGS:-} > gpurun_out/pmc_sq$i.log 2>&1
  echo "group $i rc=$?"
done
