#!/bin/bash
# Same-box A/B of library builds on the 1M-peer bench workload, alternating
# processes, scripts/ab_batch.py (ms per 1024 messages and window-pass time) in
# each. LIBS: variant names (libgossipsim_<name>.so; "base" = libgossipsim.so).
set -u
OUT=${OUT:-gpurun_out/libab}
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in ${LIBS:-a base}; do
    lib=dst-libp2p-test-node_amd/libgossipsim_$v.so
    [ $v = base ] && lib=dst-libp2p-test-node_amd/libgossipsim.so
    GOSSIPSIM_LIB=$lib timeout -k 10 300 python -u scripts/ab_batch.py --configs ${ABCFG:-1024} --rounds 3 > "$OUT/ab_${v}_$r.log" 2>&1 || exit $?
    echo "$v round $r: $(tail -1 "$OUT/ab_${v}_$r.log")"
  done
done
