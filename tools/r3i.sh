#!/bin/bash
# Round-3 GPU pass i: split prep with paired chunked walks (sw2/sw4/sw8) and aligned quad fills
# (sw4nq without) — GPU suite on sw4, parity on sw8 — and A/B against the three-kernel prep (base)
# and the first split prep (sw0); NORM_SCAN tile / prefetch variants at full resolution, 1080p, Teddy.
set -o pipefail
O=gpurun_out/${1:-r3i}
mkdir -p $O
V=$PWD/tools/abvar
SM_HIP_LIB=$V/libsm_hip_sw4.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu_sw4.log 2>&1 \
  || { tail -40 $O/pytest_gpu_sw4.log; exit 1; }
tail -1 $O/pytest_gpu_sw4.log
SM_HIP_LIB=$V/libsm_hip_sw8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_parity_sw8.log 2>&1 \
  || { tail -40 $O/pytest_parity_sw8.log; exit 1; }
tail -1 $O/pytest_parity_sw8.log
A="timeout -k 10 400 python tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep,step base:fuse_norm_scan=0 sw0 sw4 > $O/fr_prep1.txt 2>&1 && tail -4 $O/fr_prep1.txt \
 && $A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep,step sw2 sw8 sw4nq > $O/fr_prep2.txt 2>&1 && tail -4 $O/fr_prep2.txt \
 && $A --workload teddy --rounds 8 --steps 10 --copies 2 --kernels prep base:fuse_norm_scan=0 sw0 sw2 sw4 sw8 sw4nq > $O/teddy_prep.txt 2>&1 && tail -7 $O/teddy_prep.txt \
 && $A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca_v,step ns12:fuse_norm_scan=1 ns16:fuse_norm_scan=1 ns12p3:fuse_norm_scan=1 > $O/fr_ns1.txt 2>&1 && tail -4 $O/fr_ns1.txt \
 && $A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca_v,step base:fuse_norm_scan=0 ns20:fuse_norm_scan=1 > $O/fr_ns2.txt 2>&1 && tail -3 $O/fr_ns2.txt \
 && $A --workload hd --rounds 5 --steps 3 --copies 2 --kernels cbca_v,step base:fuse_norm_scan=0 ns12:fuse_norm_scan=1 ns16:fuse_norm_scan=1 ns12p3:fuse_norm_scan=1 > $O/hd_ns.txt 2>&1 && tail -5 $O/hd_ns.txt \
 && $A --workload teddy --rounds 8 --steps 10 --copies 2 --kernels cbca_v,step base:fuse_norm_scan=0 ns12:fuse_norm_scan=1 ns16:fuse_norm_scan=1 ns12p3:fuse_norm_scan=1 ns20:fuse_norm_scan=1 > $O/teddy_ns.txt 2>&1 && tail -6 $O/teddy_ns.txt
