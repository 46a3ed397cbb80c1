#!/bin/bash
# rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes (separate runs: they cannot
# share one pass on gfx950) over bench.py's configs_1gpu, one process per
# config (scripts/config_prof.py) so that every counter file holds one config's
# kernels. Summarise on the CPU with scripts/config_traffic.py.
# A fault, abort or time limit ends the session.
set -u
OUT=${OUT:-gpurun_out/cfg_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
export GS_CFG_MARK=1
for cfg in ${CFGS:-c1_1k_uniform_F1 c2_10k_F8 go_100k_idontwant c4_1m_gossip_370ms c3_100k_gossip_churn}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    echo "== $cfg $ctr ($(date +%T))"
    timeout -k 10 ${PMC_SECS:-400} rocprofv3 --pmc $ctr -d "$OUT/${cfg}_$ctr" -o run --output-format csv \
      -- python scripts/config_prof.py $cfg > "$OUT/${cfg}_$ctr.log" 2>&1
    rc=$?
    echo "$cfg $ctr rc=$rc" | tee -a "$OUT/rc.txt"
    tail -2 "$OUT/${cfg}_$ctr.log"
    case $rc in 0) ;; *) echo "stopping at rc=$rc"; exit $rc;; esac
  done
done
echo "config pmc done"
