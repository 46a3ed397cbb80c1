#!/bin/bash
# Same-box A/B of k_lcomplete's log loads (8 chunks in flight, next row's
# length ahead, publishers in LDS) against the previous commit: the 1M-peer
# batch (scripts/ab_batch.py) and 8 loop-back parts, alternating processes.
set -u
OUT=gpurun_out/r06y
mkdir -p $OUT
for r in 1 2 3; do
  for v in head base; do
    lib=dst-libp2p-test-node_amd/libgossipsim_$v.so
    [ $v = base ] && lib=dst-libp2p-test-node_amd/libgossipsim.so
    GOSSIPSIM_LIB=$lib timeout -k 10 300 python -u scripts/ab_batch.py --configs 1024 --rounds 3 > $OUT/ab_${v}_$r.log 2>&1 || exit $?
    echo "$v round $r: $(tail -n 1 $OUT/ab_${v}_$r.log)"
  done
done
for r in 1 2; do
  for v in head base; do
    lib=dst-libp2p-test-node_amd/libgossipsim_$v.so
    [ $v = base ] && lib=dst-libp2p-test-node_amd/libgossipsim.so
    GOSSIPSIM_LIB=$lib timeout -k 10 300 python -u bench.py --mode peer --parts 8 --steps 4 --warmup 1 --configs 0 \
      --cpu-seconds 0 --also-peers 0 --gossip-check 0 --output-steps 0 > $OUT/peer8_${v}_$r.log 2>&1 || exit $?
    echo "peer8 $v round $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/peer8_${v}_$r.log)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u scripts/ab_batch.py --configs 1024 --rounds 2 > $OUT/prof.log 2>&1
echo "prof rc=$?"
