#!/bin/bash
# Round-3 GPU pass j: GPU suite on the split prep with generic quad fills (variant split; the
# default library now fuses CBCA NORM_SCAN at >= 256 MiB per pair with T = 12, PF = 3), then prep
# A/B against the three-kernel prep (base) and the byte-load fills (splitnq) at full resolution and
# Teddy x16, and the default library's own GPU suite.
set -o pipefail
O=gpurun_out/${1:-r3j}
mkdir -p $O
V=$PWD/tools/abvar
SM_HIP_LIB=$V/libsm_hip_split.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu_split.log 2>&1 \
  || { tail -40 $O/pytest_gpu_split.log; exit 1; }
tail -1 $O/pytest_gpu_split.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
A="timeout -k 10 400 python tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep,cbca_v,step base split splitnq > $O/fr_prep.txt 2>&1 && tail -4 $O/fr_prep.txt \
 && $A --workload teddy --rounds 8 --steps 10 --copies 2 --kernels prep base split splitnq > $O/teddy_prep.txt 2>&1 && tail -4 $O/teddy_prep.txt \
 && $A --workload kitti --rounds 8 --steps 5 --copies 2 --kernels prep base split > $O/kitti_prep.txt 2>&1 && tail -3 $O/kitti_prep.txt
