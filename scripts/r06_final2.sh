#!/bin/bash
# Final: the whole GPU suite, smoke, the default bench line.
set -u
OUT=gpurun_out/r06f2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 $OUT/tests_gpu.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 800 python bench.py > $OUT/bench.log 2>&1
echo "bench rc=$?"
