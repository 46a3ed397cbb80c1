#!/bin/bash
# Round-5 GPU session: full GPU suite, list-pass A/B, config timings, config #3 kernel trace.
# Every GPU step has its own limit; a failing step ends the session.
set -u
OUT=${OUT:-gpurun_out/r05}
mkdir -p "$OUT"
export TMPDIR=/tmp
export GS_CFG_MARK=1
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/rc.txt"
  tail -3 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping at $name rc=$rc"; exit $rc; }
}
for st in ${STEPS:-tests ab cfg c3}; do
  case $st in
    tests) run gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TEST_ARGS:-} ;;
    ab) run ab 300 python -u scripts/ab_batch.py --rounds ${AB_ROUNDS:-4} --configs ${AB_CONFIGS:-1024 1024:GS_LPULL_PUBW=0} ;;
    cfg) run cfg 400 python scripts/config_prof.py ${CFG_NAMES:-c1_1k_uniform_F1 c2_10k_F8 c3_100k_gossip_churn} ;;
    c3) mkdir -p "$OUT/c3prof" && run c3prof 300 env OUT="$OUT/c3prof" bash scripts/c3_prof.sh ;;
    trace) run trace 400 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv \
             -- python scripts/config_prof.py ${CFG_NAMES:-c2_10k_F8} ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 3 ;;
  esac
done
echo "session done"
