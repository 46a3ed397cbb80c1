#!/bin/bash
# Same-box A/B: the go preset with the coarse IDONTWANT times (base) against
# the previous commit (head), alternating processes.
set -u
OUT=gpurun_out/r06i4
mkdir -p $OUT
for r in 1 2 3; do
  for v in head base; do
    lib=dst-libp2p-test-node_amd/libgossipsim_$v.so
    [ $v = base ] && lib=dst-libp2p-test-node_amd/libgossipsim.so
    GOSSIPSIM_LIB=$lib timeout -k 10 300 python scripts/config_prof.py go_100k_idontwant go_100k_idontwant_gossip_370ms > $OUT/go_${v}_$r.json 2>&1 || exit $?
    echo "$v round $r: $(python -c "import json; d=json.loads(open('$OUT/go_${v}_$r.json').read().strip().splitlines()[-1]); print({k:(round(v['ms'],3), round(v['roofline']['pass_ms'],3)) for k,v in d.items()})")"
  done
done
