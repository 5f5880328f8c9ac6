#!/bin/bash
# Round-4 GPU pass x: the two candidates of r4v / r4w at more instances each (placement spread is
# 5-10 % per instance): pass A with four tiles in its ring (apf4) and the H scan two tiles ahead
# (hspf2), against base, full resolution, three instances per variant.
set -o pipefail
O=gpurun_out/${1:-r4x}
mkdir -p $O
A="timeout -k 10 600 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 3 --kernels sgm_ck_a,cbca_h_scan,step base:num_streams=1 apf4:num_streams=1 hspf2:num_streams=1 > $O/ab_fr.txt 2>&1 && grep -E "maps|sgm" $O/ab_fr.txt | tail -16 \
 && $A --workload fullres --rounds 5 --steps 3 --copies 3 --kernels step base apf4 hspf2 > $O/ab_fr2.txt 2>&1 && tail -4 $O/ab_fr2.txt \
 && echo "r4x done"
