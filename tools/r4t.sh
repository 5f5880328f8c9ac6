#!/bin/bash
# Round-4 GPU pass t: prep tile heights (k_prep_h rows: h2 / base 4 / h8; k_prep_v rows: base 64 /
# v128), same-process A/B with a bitwise map check against the base library.
set -o pipefail
O=gpurun_out/${1:-r4t}
mkdir -p $O
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep,step base:num_streams=1 h8:num_streams=1 v128:num_streams=1 h2:num_streams=1 > $O/ab_fr.txt 2>&1 && grep -E "maps|prep" $O/ab_fr.txt | tail -14 \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels prep,step base h8 v128 h2 > $O/ab_teddy.txt 2>&1 && grep -E "maps|prep" $O/ab_teddy.txt | tail -14 \
 && echo "r4t done"
