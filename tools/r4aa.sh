#!/bin/bash
# Round-4 GPU pass aa: deep SGM rings only for D = 256 launches of <= 2048 lines (CK_DEEP): the whole
# GPU suite, A/B against no deep launches (nodeep) in the default schedule and on one stream at full
# resolution, then the final profiles (tools/r4_final.sh minus the suite).
set -o pipefail
O=gpurun_out/${1:-r4aa}
mkdir -p $O
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit 1
A="timeout -k 10 600 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 3 --kernels step nodeep base > $O/ab_fr.txt 2>&1 && grep -E "maps|step=" $O/ab_fr.txt | tail -10 \
 && $A --workload fullres --rounds 4 --steps 3 --copies 2 --kernels sgm_ck,step base:num_streams=1 nodeep:num_streams=1 > $O/ab_fr1.txt 2>&1 && grep -E "maps|step=" $O/ab_fr1.txt | tail -7 \
 && echo "r4aa done"
