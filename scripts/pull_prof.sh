#!/bin/bash
# Builds the GS_PULL_PROF diagnostic library into prof_build (on the CPU
# host, before gpurun) — run with "build" — or runs scripts/pull_prof.py on the GPU.
set -eu
cd "$(dirname "$0")/.."
if [ "${1:-run}" = build ]; then
  mkdir -p prof_build
  for f in gs_topology gs_mesh gs_relax gs_ctx gs_comm; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DGS_PULL_PROF -c dst-libp2p-test-node_amd/csrc/$f.hip -o prof_build/$f.o &
  done
  g++ -O3 -std=c++17 -fPIC -c dst-libp2p-test-node_amd/csrc/gs_host.cpp -o prof_build/gs_host.o
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o prof_build/libgossipsim.so prof_build/*.o -ldl
else
  mkdir -p gpurun_out
  timeout -k 10 300 python scripts/${PROF_SCRIPT:-pull_prof.py} ${PEERS:-1000000} > gpurun_out/pull_prof.txt 2>&1
fi
