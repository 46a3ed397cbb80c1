#!/bin/bash
# One gpurun session: GPU tests -> smoke -> bench -> rocprofv3 kernel trace -> PMC.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session
# (exit codes 124, 134, 137, 139), an ordinary test failure does not.
# PMC counters run in their own passes (FETCH_SIZE and WRITE_SIZE cannot share
# one pass on gfx950) and never together with tracing.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/rc.txt"
  tail -5 "$OUT/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $name: stopping"; exit $rc;; esac
  return 0
}
PROFARGS="--steps ${PROF_STEPS:-6} --warmup 2 --cpu-seconds 0 --also-peers 0 --configs 0 --gossip-check 0 --output-steps 0"
KRE="k_lpull|k_pull|k_scan|k_frontier|k_complete|k_lcomplete"
for s in ${STEPS:-tests smoke bench prof}; do
  case $s in
    tests) step gpu_tests ${TESTS_SECS:-1200} python -u -m pytest tests -m gpu ${TEST_ARGS:--x} -v --timeout 300 --timeout-method thread ;;
    probe) step rccl_probe 300 ./scripts/bin/rccl_p2p_probe ;;
    abbatch) step ab_batch 600 python -u scripts/ab_batch.py ${ABB_ARGS:-} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py $PROFARGS ;;
    ab) step ab_relax 600 python scripts/ab_relax.py ${AB_ARGS:-} ;;
    ubench) step ubench_mem 300 ./build_tools/ubench_mem ;;
    pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -d "$OUT/pmc_fetch" -o run --output-format csv -- python bench.py $PROFARGS ;
         step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -d "$OUT/pmc_write" -o run --output-format csv -- python bench.py $PROFARGS ;;
  esac
done
echo "session done"
