#!/bin/bash
# A/B builds: libgossipsim_<name>.so = the in-tree objects with gs_relax.hip
# recompiled under extra defines (SRC: another csrc directory, e.g. a git
# checkout of an older commit), e.g.  scripts/build_variant.sh ng8 -DGS_LP_NG=8 -DGS_LP_RCH=1
set -eu
name=$1; shift
cd "$(dirname "$0")/../dst-libp2p-test-node_amd"
make -s libgossipsim.so
mkdir -p build_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result "$@" \
  -I../include -c ${SRC:-csrc}/gs_relax.hip -o build_$name/gs_relax.o
objs=$(ls build/*.o | grep -v gs_relax.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libgossipsim_$name.so $objs build_$name/gs_relax.o -ldl
echo "built libgossipsim_$name.so"
