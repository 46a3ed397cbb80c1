#!/bin/bash
# The 4-batch config #3 under: no profiler, kernel trace, PMC with one stream
# (GS_CHN_PIPE=0), PMC as is (crashed once in the launch path under --pmc).
set -u
OUT=gpurun_out/r06g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/config_prof.py c3_100k_gossip_churn_4096 > $OUT/plain.log 2>&1; echo "plain rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python scripts/config_prof.py c3_100k_gossip_churn_4096 > $OUT/kt.log 2>&1; echo "ktrace rc=$?"
GS_CHN_PIPE=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o run --output-format csv -- python scripts/config_prof.py c3_100k_gossip_churn_4096 > $OUT/pmc1.log 2>&1; echo "pmc pipe0 rc=$?"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc2 -o run --output-format csv -- python scripts/config_prof.py c3_100k_gossip_churn_4096 > $OUT/pmc2.log 2>&1; echo "pmc rc=$?"
