#!/bin/bash
# Round-4 GPU pass r: H sweeps with one load / two store descriptors per line (SM_CB_H_LINE_RSRC;
# parity, the whole suite, A/B against hlr0 = the per-tile descriptors), and the auto two-group
# schedule at Teddy x16 (base) against one stream.
set -o pipefail
O=gpurun_out/${1:-r4r}
mkdir -p $O
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $PT -m gpu tests/test_gpu_agg.py tests/test_gpu_batch.py tests/test_gpu_large_fixtures.py -k "cbca or CBCA or auto or fixture or stream" > $O/pytest_h.log 2>&1
rc=$?; tail -2 $O/pytest_h.log; grep -E "^FAILED" $O/pytest_h.log | head; ok $rc || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head -20; ok $rc || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca_h,step base:num_streams=1 hlr0:num_streams=1 > $O/ab_fr.txt 2>&1 && tail -3 $O/ab_fr.txt \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels cbca_h,step base base:num_streams=1 hlr0 > $O/ab_teddy.txt 2>&1 && tail -4 $O/ab_teddy.txt \
 && echo "r4r done"
