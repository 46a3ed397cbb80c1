#!/bin/bash
# Profile round: kernel stats + PMC FETCH/WRITE passes, the traffic summary,
# then the bench line that reads it. Outputs under gpurun_out/ (copy to profiles/).
set -u
OUT=${OUT:-gpurun_out}
STEPS="prof" bash scripts/gpu_session.sh || exit $?
# PMC passes with dense rows on the list pull path, so k_complete's known key
# stream calibrates the FETCH_SIZE read factor (scripts/pmc_summary.py)
GS_LPULL_DENSE=1 STEPS="pmc" bash scripts/gpu_session.sh || exit $?
python scripts/pmc_summary.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv \
  $OUT/pmc_summary.json --traffic-json $OUT/traffic_latest.json --peers 1000000 --batch 1024 > $OUT/pmc_summary.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --traffic-json $OUT/traffic_latest.json > $OUT/bench.log 2>&1
echo "bench rc=$?"
tail -1 $OUT/bench.log
