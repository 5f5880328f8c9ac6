#!/bin/bash
# Round-4 GPU pass v: checkpointed SGM pass A with 3 / 4 tiles in its register ring (apf3, apf4:
# two / three tiles of loads in flight instead of one), same-process A/B with a bitwise map check.
set -o pipefail
O=gpurun_out/${1:-r4v}
mkdir -p $O
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels sgm_ck_a,step base:num_streams=1 apf3:num_streams=1 apf4:num_streams=1 > $O/ab_fr.txt 2>&1 && grep -E "maps|sgm" $O/ab_fr.txt | tail -12 \
 && $A --workload kitti --rounds 5 --steps 5 --copies 2 --kernels sgm_ck_a,step base apf3 apf4 > $O/ab_kitti.txt 2>&1 && grep -E "maps|sgm" $O/ab_kitti.txt | tail -6 \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels sgm_ck_a,step base:num_streams=1 apf3:num_streams=1 apf4:num_streams=1 > $O/ab_teddy.txt 2>&1 && grep -E "maps|sgm" $O/ab_teddy.txt | tail -6 \
 && echo "r4v done"
