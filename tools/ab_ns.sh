#!/bin/bash
# CBCA NORM_SCAN A/B (same process, interleaved rounds): full resolution with the fused sweep's
# tile / prefetch variants (tools/abvar), then the 1080p and Teddy workloads fused vs unfused.
set -o pipefail
O=gpurun_out/${1:-ab_ns}
mkdir -p $O
timeout -k 10 400 python tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --kernels cbca_v,step \
  base base:fuse_norm_scan=1 ns_pf2:fuse_norm_scan=1 ns_pf3:fuse_norm_scan=1 ns_t6pf2:fuse_norm_scan=1 ns_t12pf2:fuse_norm_scan=1 > $O/fullres.txt 2>&1 \
 && tail -8 $O/fullres.txt \
 && timeout -k 10 300 python tools/ab_inproc.py --workload hd --rounds 5 --steps 3 --copies 2 --kernels cbca_v \
  base base:fuse_norm_scan=1 ns_pf2:fuse_norm_scan=1 > $O/hd.txt 2>&1 \
 && tail -4 $O/hd.txt \
 && timeout -k 10 300 python tools/ab_inproc.py --workload teddy --rounds 8 --steps 10 --copies 2 --kernels cbca_v \
  base base:fuse_norm_scan=1 ns_pf2:fuse_norm_scan=1 > $O/teddy.txt 2>&1 \
 && tail -4 $O/teddy.txt
