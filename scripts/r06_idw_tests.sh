#!/bin/bash
set -u
OUT=gpurun_out/r06i5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_gossip_list.py tests/test_gpu_configs.py tests/test_gpu_partition.py \
  -k "idontwant or node_presets or go" > $OUT/tests_idw.log 2>&1
rc=$?; echo "idw tests rc=$rc"; tail -3 $OUT/tests_idw.log
