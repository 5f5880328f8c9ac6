#!/bin/bash
# CBCA H scan with two / three tiles in flight (full resolution, same-process A/B).
set -o pipefail
O=gpurun_out/${1:-r3v}
mkdir -p $O
timeout -k 10 400 python tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca_h,step base hpf2 hpf3 > $O/fr.txt 2>&1 && tail -4 $O/fr.txt
