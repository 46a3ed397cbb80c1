#!/bin/bash
# Same-box A/B of the record step's neighbour-group size on config #3 (churn
# list pass, ~22 CSR neighbours per row): base (NG 4) vs NG 8 / 8 x 1 chunk / 6.
set -u
OUT=gpurun_out/r06h2
mkdir -p $OUT
for r in 1 2 3; do
  for v in base ng8 ng8r1 ng6; do
    lib=dst-libp2p-test-node_amd/libgossipsim_$v.so
    [ $v = base ] && lib=dst-libp2p-test-node_amd/libgossipsim.so
    GOSSIPSIM_LIB=$lib timeout -k 10 200 python -u scripts/c3_probe.py > $OUT/${v}_$r.log 2>&1
    rc=$?; echo "$v round $r rc=$rc: $(grep -o 'c3 probe: [0-9.]* ms' $OUT/${v}_$r.log)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
