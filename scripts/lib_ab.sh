#!/bin/bash
# Same-box A/B of two library builds on the 1M-peer bench workload:
# libgossipsim_a.so (A) against libgossipsim.so (B), alternating processes,
# scripts/ab_batch.py (ms per 1024 messages and window-pass time) in each.
set -u
OUT=${OUT:-gpurun_out/libab}
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in a b; do
    lib=dst-libp2p-test-node_amd/libgossipsim.so
    [ $v = a ] && lib=dst-libp2p-test-node_amd/libgossipsim_a.so
    GOSSIPSIM_LIB=$lib timeout -k 10 300 python -u scripts/ab_batch.py --configs 1024 --rounds 3 > "$OUT/ab_${v}_$r.log" 2>&1 || exit $?
    echo "$v round $r: $(tail -1 "$OUT/ab_${v}_$r.log")"
  done
done
