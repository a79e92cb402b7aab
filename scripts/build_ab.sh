#!/bin/bash
# Builds an A/B variant of libpgcn.so with extra compile flags into parallel-gcn_amd/<dir>/
# (load it with PGCN_LIB=parallel-gcn_amd/<dir>/libpgcn.so).  usage: build_ab.sh <dir> <flags...>
set -eu
cd "$(dirname "$0")/../parallel-gcn_amd"
DIR=$1; shift
mkdir -p "$DIR/obj"
FL="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $*"
objs=()
for f in csrc/k_peer.hip csrc/k_graphsum.hip csrc/k_graphsum_ring.hip csrc/k_gemm.hip csrc/k_gemm_wide.hip csrc/k_xstream_lds.hip \
         csrc/k_sparse.hip csrc/k_elementwise.hip csrc/capi.cpp csrc/rng.cpp csrc/host/graph.cpp \
         csrc/host/ring.cpp csrc/host/data.cpp csrc/host/comm.cpp csrc/host/api.cpp \
         csrc/host/module.cpp csrc/host/gcn.cpp; do
  o="$DIR/obj/$(basename "$f").o"
  /opt/rocm/bin/hipcc $FL -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c "$f" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc $FL -shared -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib -o "$DIR/libpgcn.so" "${objs[@]}"
rm -rf "$DIR/obj"
echo "built $DIR/libpgcn.so"
