#!/bin/bash
# A/B builds: libgossipsim_<name>.so = the in-tree objects with gs_relax.hip
# recompiled under extra defines, e.g.  scripts/build_variant.sh ng8 -DGS_LP_NG=8 -DGS_LP_RCH=1
# SRC=<csrc dir> (e.g. a git archive of an older commit): every object is
# built from that tree (headers such as gs_internal.h may differ between the
# two builds, so objects of different trees never mix).
set -eu
name=$1; shift
cd "$(dirname "$0")/../dst-libp2p-test-node_amd"
make -s libgossipsim.so
mkdir -p build_$name
HIPCC="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result"
if [ -n "${SRC:-}" ]; then
  for f in gs_topology gs_mesh gs_relax gs_ctx gs_comm; do
    $HIPCC "$@" -c $SRC/$f.hip -o build_$name/$f.o &
  done
  g++ -O3 -std=c++17 -fPIC -c $SRC/gs_host.cpp -o build_$name/gs_host.o &
  wait
  objs=$(ls build_$name/*.o)
else
  $HIPCC "$@" -c csrc/gs_relax.hip -o build_$name/gs_relax.o
  objs="$(ls build/*.o | grep -v gs_relax.o) build_$name/gs_relax.o"
fi
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libgossipsim_$name.so $objs -ldl
echo "built libgossipsim_$name.so"
