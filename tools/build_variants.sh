#!/bin/bash
# Builds tuning variants of libsm_hip.so that differ only in sm_cbca.hip's compile-time tile
# shapes, for same-process-type A/B runs on one GPU box (select with SM_HIP_LIB=<path>).
# usage: tools/build_variants.sh NAME "-DSM_CB_T_NORM_H=14 ..." [NAME2 "DEFS2" ...]
set -e
cd "$(dirname "$0")/../mystereomatching_amd/csrc"
make -s
mkdir -p ../../tools/variants build/var
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -Wno-unused-result -Wno-unused-value"
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc $FLAGS $defs -c sm_cbca.hip -o build/var/sm_cbca_$name.o &
done
wait
for o in build/var/sm_cbca_*.o; do
  name=${o#build/var/sm_cbca_}; name=${name%.o}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libsm_hip_$name.so \
    build/sm_kernels.o $o build/sm_sgm.o build/sm_capi.o
  echo "built tools/variants/libsm_hip_$name.so"
done
