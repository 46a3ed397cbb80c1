#!/bin/bash
# IDONTWANT with coarse final times: the IDONTWANT tests, then the go preset's
# time and FETCH/WRITE traffic (scripts/config_pmc.sh, one config).
set -u
OUT=gpurun_out/${OUTD:-r06i2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_gossip_list.py tests/test_gpu_configs.py tests/test_gpu_partition.py \
  -k "idontwant or node_presets or go" > $OUT/tests_idw.log 2>&1
rc=$?; echo "idw tests rc=$rc"; tail -3 $OUT/tests_idw.log
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  timeout -k 10 300 python scripts/config_prof.py go_100k_idontwant go_100k_idontwant_gossip_370ms > $OUT/go_$r.json 2>&1
  echo "go round $r rc=$?: $(python -c "import json,sys; d=json.loads(open('$OUT/go_$r.json').read().strip().splitlines()[-1]); print({k:(round(v['ms'],3)) for k,v in d.items()})")"
done
CFGS="go_100k_idontwant go_100k_idontwant_gossip_370ms" OUT=$OUT/cfg_pmc bash scripts/config_pmc.sh > $OUT/pmc.log 2>&1
echo "pmc rc=$?"
