#!/bin/bash
# Round-4 GPU pass j: stream stagger at full resolution and 1080p: the pairs as sub-batches on two
# streams, the next group starting after this group's CBCA (base) or after its first CBCA sweep
# (stg1: the next group's prep, cost and H scan beside this group's LDS-bound NORM_SCAN sweep).
set -o pipefail
O=gpurun_out/${1:-r4j}
mkdir -p $O
A="timeout -k 10 500 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels step base base:sub_batch=1,num_streams=2 stg1:sub_batch=1,num_streams=2 > $O/ab_fr.txt 2>&1 && tail -4 $O/ab_fr.txt \
 && $A --workload hd --rounds 4 --steps 2 --copies 1 --kernels step base base:sub_batch=2,num_streams=2 stg1:sub_batch=2,num_streams=2 stg1:sub_batch=1,num_streams=2 stg1:sub_batch=4,num_streams=2 > $O/ab_hd.txt 2>&1 && tail -6 $O/ab_hd.txt \
 && echo "r4j done"
