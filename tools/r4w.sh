#!/bin/bash
# Round-4 GPU pass w: H sweep tile / prefetch depths re-swept after the exact-vmcnt loops (h_scan:
# one tile ahead at T = 24 -> two ahead (hspf2), T = 16 two ahead (hst16); h_norm: T = 10 two ahead ->
# three ahead (hnpf3), T = 8 three ahead (hnt8)); same-process A/B with a bitwise map check.
set -o pipefail
O=gpurun_out/${1:-r4w}
mkdir -p $O
A="timeout -k 10 500 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca_h,step base:num_streams=1 hspf2:num_streams=1 hst16:num_streams=1 hnpf3:num_streams=1 hnt8:num_streams=1 > $O/ab_fr.txt 2>&1 && grep -E "maps|cbca" $O/ab_fr.txt | tail -20 \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels cbca_h,step base:num_streams=1 hspf2:num_streams=1 hst16:num_streams=1 hnpf3:num_streams=1 hnt8:num_streams=1 > $O/ab_teddy.txt 2>&1 && grep -E "maps|cbca" $O/ab_teddy.txt | tail -8 \
 && echo "r4w done"
