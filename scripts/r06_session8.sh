#!/bin/bash
# Full GPU suite + smoke, then the FETCH_SIZE calibration micro-benchmark.
set -u
OUT=gpurun_out/${OUTD:-r06t}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_gpu.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $OUT/tests_gpu.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 120 ./scripts/bin/ubench_fetch > $OUT/ubench_fetch.csv 2>&1
rc=$?; echo "ubench rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_pmc -o run --output-format csv -- ./scripts/bin/ubench_fetch > $OUT/ubench_fetch_pmc.log 2>&1
echo "fetch pmc rc=$?"
