#!/bin/bash
# Round-4 GPU pass s: checkpointed SGM pass A with registers for five waves per SIMD (wa5: A23's
# 6000 full-resolution lines in 1.17 rounds of resident waves instead of 1.46), parity + A/B.
set -o pipefail
O=gpurun_out/${1:-r4s}
mkdir -p $O
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_large_fixtures.py -k "checkpoint or auto or fixture" > $O/pytest_ck.log 2>&1
rc=$?; tail -2 $O/pytest_ck.log; grep -E "^FAILED" $O/pytest_ck.log | head; ok $rc || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels sgm,step base:num_streams=1 wa5:num_streams=1 > $O/ab_fr.txt 2>&1 && tail -3 $O/ab_fr.txt \
 && $A --workload kitti --rounds 5 --steps 5 --copies 2 --kernels sgm,step base wa5 > $O/ab_kitti.txt 2>&1 && tail -3 $O/ab_kitti.txt \
 && echo "r4s done"
