#!/bin/bash
# Round-3 GPU pass g: GPU suite on the split-prep variant, CBCA CPW variants' parity, same-process A/Bs
# (CPW V sweeps, NORM_SCAN T = 12, split vs three-kernel prep) at full resolution and Teddy x16.
set -o pipefail
O=gpurun_out/${1:-r3g}
mkdir -p $O
SM_HIP_LIB=$PWD/tools/abvar/libsm_hip_prepsplit.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in cpw2 cpw4nb; do
  SM_HIP_LIB=$PWD/tools/abvar/libsm_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_large_fixtures.py > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
# (six full-resolution instances of 2 pairs = 148 GB of HBM)
timeout -k 10 400 python tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep,cbca_v,step \
  base cpw2 cpw4nb > $O/fullres.txt 2>&1 && tail -4 $O/fullres.txt \
 && timeout -k 10 400 python tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep,cbca_v,step \
  cpw2b ns12:fuse_norm_scan=1 prepsplit > $O/fullres2.txt 2>&1 && tail -4 $O/fullres2.txt \
 && timeout -k 10 300 python tools/ab_inproc.py --workload teddy --rounds 8 --steps 10 --copies 2 --kernels prep,cbca_v \
  base cpw2 cpw2b cpw4n cpw4nb prepsplit > $O/teddy.txt 2>&1 && tail -7 $O/teddy.txt
