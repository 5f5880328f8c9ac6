#!/bin/bash
# Round-4 GPU pass y: ring depths only for the D = 256 one-line-per-wave passes (apf4f: pass A with
# four tiles; apbf: that plus pass B of the first pair with three segments), against base at full
# resolution (one stream, per-kernel) and in the default two-stream schedule, plus KITTI / Teddy
# checks that other shapes are unchanged.
set -o pipefail
O=gpurun_out/${1:-r4y}
mkdir -p $O
A="timeout -k 10 600 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 3 --kernels sgm_ck,step base:num_streams=1 apf4f:num_streams=1 apbf:num_streams=1 > $O/ab_fr.txt 2>&1 && grep -E "maps|sgm" $O/ab_fr.txt | tail -14 \
 && $A --workload fullres --rounds 5 --steps 3 --copies 3 --kernels step apbf base > $O/ab_fr2.txt 2>&1 && tail -3 $O/ab_fr2.txt \
 && $A --workload hd --rounds 4 --steps 2 --copies 2 --kernels sgm_ck,step base apbf > $O/ab_hd.txt 2>&1 && tail -3 $O/ab_hd.txt \
 && echo "r4y done"
