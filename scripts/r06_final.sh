#!/bin/bash
# Round-6 final evidence: headline kernel stats + PMC + traffic + bench line,
# then config PMC passes for config #3 (single batch, 4 batches, 1.5 s delay)
# and the go preset. Outputs under gpurun_out/r06f (copied to profiles/r06_final).
set -u
export OUT=gpurun_out/r06f
mkdir -p $OUT
bash scripts/prof_session.sh || exit $?
CFGS="c3_100k_gossip_churn c3_100k_gossip_churn_4096 c3_100k_delay1500ms go_100k_idontwant" OUT=$OUT/cfg_pmc \
  bash scripts/config_pmc.sh || exit $?
echo "final session done"
