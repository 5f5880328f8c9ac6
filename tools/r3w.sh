#!/bin/bash
# Placement probe at allocation (best of 3 volume allocations) vs the first allocation (nocal):
# full resolution, same process, three instances each; the probe times go to stderr.
set -o pipefail
O=gpurun_out/${1:-r3w}
mkdir -p $O
SM_TRACE_ALLOC=1 timeout -k 10 500 python tools/ab_inproc.py --workload fullres --rounds 4 --steps 3 --copies 3 --kernels cbca_h_scan,sgm_path1,step base nocal > $O/fr.txt 2>&1 && grep -v "^round" $O/fr.txt | tail -12
