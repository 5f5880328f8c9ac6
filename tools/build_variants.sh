#!/bin/bash
# Builds tuning variants of libsm_hip.so that differ only in one source file's compile-time
# switches (default sm_cbca.hip; SRC=sm_kernels, SRC=sm_sgm, SRC=sm_capi (.cpp), ... for the others), for same-box A/B
# runs on one GPU box (tools/ab_inproc.py; tools/abvar/ travels with gpurun -- delete it after the A/B
# so that later pushes, the driver's included, do not carry it).
# usage: [SRC=sm_cbca] tools/build_variants.sh NAME "-DSWITCH=value ..." [NAME2 "DEFS2" ...]
set -e
SRC=${SRC:-sm_cbca}
cd "$(dirname "$0")/../mystereomatching_amd/csrc"
make -s
mkdir -p ../../tools/abvar build/var
rm -f build/var/*.o
EXT=hip; [ -f $SRC.cpp ] && EXT=cpp
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -Wno-unused-result -Wno-unused-value"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc $FLAGS $defs -c $SRC.$EXT -o build/var/${SRC}__$name.o &
done
wait
OBJS="build/sm_kernels.o build/sm_cbca.o build/sm_sgm.o build/sm_refine.o build/sm_pyramid.o build/sm_so.o build/sm_gf.o build/sm_gf_cv.o build/sm_nl.o build/sm_nl_mst.o build/sm_nl_walk.o build/sm_capi.o"
for o in build/var/${SRC}__*.o; do
  name=${o#build/var/${SRC}__}; name=${name%.o}
  objs=${OBJS/build\/$SRC.o/$o}
  # (linked to a temporary name and renamed: a gpurun snapshot never sees a half-written library)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/abvar/.tmp_$name.so $objs
  mv ../../tools/abvar/.tmp_$name.so ../../tools/abvar/libsm_hip_$name.so
  echo "built tools/abvar/libsm_hip_$name.so"
done
