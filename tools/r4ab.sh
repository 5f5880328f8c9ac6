#!/bin/bash
# Round-4 GPU pass ab (diagnostic): six one-stream instances of the same library at full resolution
# with SM_TRACE_ALLOC=1, so the per-instance H scan / NsV / SGM times (the placement spread) can be
# set against where each instance's volume buffers landed.
set -o pipefail
O=gpurun_out/${1:-r4ab}
mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py --workload fullres --rounds 4 --steps 3 --copies 6 --kernels cbca,sgm_ck,step base:num_streams=1,SM_TRACE_ALLOC=1 > $O/ab_place.txt 2>&1 && grep -E "alloc|step=" $O/ab_place.txt | tail -16 && echo "r4ab done"
