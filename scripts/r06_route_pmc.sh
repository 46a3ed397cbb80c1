#!/bin/bash
# SQ counters of the routed record pack (8 loop-back parts, 1M x 1024) and its
# kernel trace, for wave lifetime vs kernel duration.
set -u
OUT=gpurun_out/${OUTD:-r06j}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--mode peer --parts 8 --steps 1 --warmup 0 --configs 0 --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA" \
           FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex k_lpack_route -d $OUT/pmc$i -o run --output-format csv -- \
    python bench.py $ARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "group $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
